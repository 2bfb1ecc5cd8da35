"""ctypes front-end of the CPU oracle (oracle/tls_oracle.c).

TEST INFRASTRUCTURE ONLY.  Importable from tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never from tlslite_amd/ (the product).  The
oracle restates tlslite's record seal/open (tlslite/tlsrecordlayer.py:538-616,
:958-1044) and is pinned against tests/golden/records.json.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

CIPHER = {"aes128": 1, "aes256": 2, "rc4": 3, "3des": 4}
MAC = {"sha1": 1, "sha256": 2, "md5": 3}
FAULT = {None: 0, "badMAC": 1, "badPadding": 2}
ALERT_BAD_RECORD_MAC = -20
ALERT_DECRYPTION_FAILED = -21
ALERT_RECORD_OVERFLOW = -23
EFRAME = -6
EABRUPT = -7

# suite name -> (cipher, key len, iv len, mac, mac len); tlsrecordlayer.py:1063-1095
SUITES = {
    "AES128-SHA": ("aes128", 16, 16, "sha1", 20),
    "AES256-SHA": ("aes256", 32, 16, "sha1", 20),
    "AES128-SHA256": ("aes128", 16, 16, "sha256", 32),
    "AES256-SHA256": ("aes256", 32, 16, "sha256", 32),
    "RC4-SHA": ("rc4", 16, 0, "sha1", 20),
    "RC4-MD5": ("rc4", 16, 0, "md5", 16),
    "3DES-SHA": ("3des", 24, 8, "sha1", 20),
}


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _load():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    u8p = ctypes.c_char_p
    lib.ora_conn_size.restype = ctypes.c_size_t
    lib.ora_conn_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p,
                                  ctypes.c_uint64]
    lib.ora_seal.argtypes = [ctypes.c_void_p, ctypes.c_int, u8p, ctypes.c_size_t, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_size_t]
    lib.ora_seal.restype = ctypes.c_long
    lib.ora_seal_len.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.ora_seal_len.restype = ctypes.c_long
    lib.ora_open.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                             ctypes.POINTER(ctypes.c_size_t)]
    lib.ora_open.restype = ctypes.c_long
    lib.ora_cipher_encrypt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.ora_cipher_decrypt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.ora_hash.argtypes = [ctypes.c_int, u8p, ctypes.c_size_t, ctypes.c_void_p]
    lib.ora_hmac.argtypes = [ctypes.c_int, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_void_p]
    lib.ora_prf.argtypes = [ctypes.c_int, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                            ctypes.c_void_p, ctypes.c_size_t]
    lib.ora_conn_get_iv.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.ora_conn_get_seq.argtypes = [ctypes.c_void_p]
    lib.ora_conn_get_seq.restype = ctypes.c_uint64
    lib.ora_conn_get_rc4.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_int)]
    lib.ora_seal_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.ora_fill_pattern.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


class Conn:
    """One write (or read) connection state: _ConnectionState + encContext."""

    def __init__(self, cipher, mac, version, key, iv=b"", mac_key=b"", fixed_iv=None, seq=0):
        L = lib()
        self.buf = ctypes.create_string_buffer(L.ora_conn_size())
        fiv = bytes(fixed_iv) if fixed_iv else None
        rc = L.ora_conn_init(self.buf, CIPHER[cipher], MAC[mac], version[0], version[1], bytes(key), len(key),
                             bytes(iv), len(iv), bytes(mac_key), len(mac_key), fiv, seq)
        if rc != 0:
            raise ValueError("bad key/iv lengths")
        self.cipher, self.mac, self.version = cipher, mac, tuple(version)

    @classmethod
    def for_suite(cls, suite, version, key, iv, mac_key, fixed_iv=None, seq=0):
        c, _, _, m, _ = SUITES[suite]
        return cls(c, m, version, key, iv, mac_key, fixed_iv, seq)

    def copy(self):
        n = Conn.__new__(Conn)
        n.buf = ctypes.create_string_buffer(self.buf.raw, len(self.buf))
        n.cipher, n.mac, n.version = self.cipher, self.mac, self.version
        return n

    def seal(self, pt, ctype=23, fault=None):
        L = lib()
        cap = len(pt) + 128
        out = ctypes.create_string_buffer(cap)
        fl = fault if isinstance(fault, int) else FAULT[fault]
        n = L.ora_seal(self.buf, ctype, bytes(pt), len(pt), fl, out, cap)
        if n < 0:
            raise ValueError("seal error %d" % n)
        return out.raw[:n]

    def open(self, body, ctype=23):
        """Returns plaintext bytes, or raises ValueError with the alert code."""
        L = lib()
        b = ctypes.create_string_buffer(bytes(body), len(body))
        off = ctypes.c_size_t(0)
        n = L.ora_open(self.buf, ctype, b, len(body), ctypes.byref(off))
        if n < 0:
            return n, None
        return 0, b.raw[off.value: off.value + n]

    def encrypt(self, data):
        b = ctypes.create_string_buffer(bytes(data), len(data))
        if lib().ora_cipher_encrypt(self.buf, b, len(data)) != 0:
            raise AssertionError("length not a multiple of the block size")
        return b.raw[: len(data)]

    def decrypt(self, data):
        b = ctypes.create_string_buffer(bytes(data), len(data))
        if lib().ora_cipher_decrypt(self.buf, b, len(data)) != 0:
            raise AssertionError("length not a multiple of the block size")
        return b.raw[: len(data)]

    @property
    def iv(self):
        o = ctypes.create_string_buffer(16)
        lib().ora_conn_get_iv(self.buf, o)
        return o.raw[: (8 if self.cipher == "3des" else 16)]

    @property
    def seqnum(self):
        return lib().ora_conn_get_seq(self.buf)

    @property
    def rc4(self):
        S = ctypes.create_string_buffer(256)
        i, j = ctypes.c_int(), ctypes.c_int()
        lib().ora_conn_get_rc4(self.buf, S, ctypes.byref(i), ctypes.byref(j))
        return S.raw, i.value, j.value


def hash_(alg, data):
    out = ctypes.create_string_buffer(32)
    lib().ora_hash(MAC[alg], bytes(data), len(data), out)
    return out.raw[: {"sha1": 20, "sha256": 32, "md5": 16}[alg]]


def hmac_(alg, key, data):
    out = ctypes.create_string_buffer(32)
    lib().ora_hmac(MAC[alg], bytes(key), len(key), bytes(data), len(data), out)
    return out.raw[: {"sha1": 20, "sha256": 32, "md5": 16}[alg]]


def prf(version, secret, label, seed, length):
    """PRF / PRF_1_2 / PRF_SSL by version (mathtls.py:37-68)."""
    out = ctypes.create_string_buffer(max(1, length))
    rc = lib().ora_prf(tuple(version)[1], bytes(secret), len(secret), bytes(label), len(label), bytes(seed),
                       len(seed), out, length)
    if rc:
        raise ValueError("ora_prf: bad arguments")
    return out.raw[:length]


def master_secret(version, premaster, client_random, server_random):
    """calcMasterSecret (mathtls.py:70-82)."""
    return prf(version, premaster, b"master secret", bytes(client_random) + bytes(server_random), 48)


def key_block(version, suite, master, client_random, server_random):
    """_calcPendingStates key block (tlsrecordlayer.py:1097-1114) and its
    slices in Parser order (:1117-1126)."""
    _, kl, ivl, _, ml = SUITES[suite]
    kb = prf(version, master, b"key expansion", bytes(server_random) + bytes(client_random), 2 * (ml + kl + ivl))
    parts, pos = {}, 0
    for name, size in (("client_mac", ml), ("server_mac", ml), ("client_key", kl), ("server_key", kl),
                       ("client_iv", ivl), ("server_iv", ivl)):
        parts[name] = kb[pos:pos + size]
        pos += size
    return kb, parts


def fill_pattern(n, seed, start=0):
    a = np.empty(n, dtype=np.uint8)
    lib().ora_fill_pattern(a.ctypes.data, n, seed, start)
    return a


def seal_batch(protos, chain_begin, chain_count, pt, pt_off, pt_len, wire, wire_off, ctype=None, nthreads=1,
               update=False, flags=None):
    """Seal many chains in parallel threads.  protos: list of Conn (one per
    chain, copied -- the originals are advanced only with update=True).
    Returns wire_len array."""
    L = lib()
    sz = L.ora_conn_size()
    arr = ctypes.create_string_buffer(sz * len(protos))
    for i, c in enumerate(protos):
        ctypes.memmove(ctypes.addressof(arr) + i * sz, c.buf, sz)
    chain_begin = np.ascontiguousarray(chain_begin, dtype=np.uint32)
    chain_count = np.ascontiguousarray(chain_count, dtype=np.uint32)
    pt_off = np.ascontiguousarray(pt_off, dtype=np.uint64)
    pt_len = np.ascontiguousarray(pt_len, dtype=np.uint32)
    wire_off = np.ascontiguousarray(wire_off, dtype=np.uint64)
    wl = np.zeros(len(pt_len), dtype=np.int64)
    ct = None if ctype is None else np.ascontiguousarray(ctype, dtype=np.uint8)
    fl = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
    L.ora_seal_batch(arr, len(protos), chain_begin.ctypes.data, chain_count.ctypes.data, pt.ctypes.data,
                     pt_off.ctypes.data, pt_len.ctypes.data, None if ct is None else ct.ctypes.data,
                     None if fl is None else fl.ctypes.data, wire.ctypes.data, wire_off.ctypes.data, wl.ctypes.data, nthreads)
    if update:
        for i, c in enumerate(protos):
            ctypes.memmove(c.buf, ctypes.addressof(arr) + i * sz, sz)
    return wl


def frame(data):
    """_getNextRecord's record framing over one connection's received bytes
    (tlsrecordlayer.py:832-876; RecordHeader3.parse, messages.py:44-49), pure Python: every
    complete record as (content_type, (major, minor), body), stopping at an incomplete record
    (left for the next read), at a first header byte that is no content type (:850-857 --
    SyntaxError as soon as that byte arrives; SSLv2 headers are handshake-only and not
    framed here), at a header announcing more than 18432 body bytes (:871-873,
    record_overflow), or at a header announcing an empty body (the body loop's sock.recv(0)
    returns b"" and raises TLSAbruptCloseError, :877-889).  Returns (records, consumed,
    code): code 0, EFRAME, ALERT_RECORD_OVERFLOW or EABRUPT."""
    data = bytes(data)
    out, pos = [], 0
    while pos < len(data):
        if data[pos] not in (20, 21, 22, 23):  # ContentType.all
            return out, pos, EFRAME
        if len(data) - pos < 5:
            break
        length = (data[pos + 3] << 8) | data[pos + 4]
        if length > 18432:
            return out, pos, ALERT_RECORD_OVERFLOW
        if length == 0:
            return out, pos, EABRUPT
        if len(data) - pos - 5 < length:
            break
        out.append((data[pos], (data[pos + 1], data[pos + 2]), data[pos + 5:pos + 5 + length]))
        pos += 5 + length
    return out, pos, 0

"""Post-handshake plumbing around the GPU record path (config 1 harness).

  * key-block derivation exactly as `_calcPendingStates` performs it
    (tlslite/tlsrecordlayer.py:1061-1149) from a master secret
    (calcMasterSecret, tlslite/mathtls.py:70-82) with the TLS 1.0/1.1 PRF,
    the TLS 1.2 PRF_1_2 and SSL 3.0 PRF_SSL (mathtls.py:24-68).  This is
    per-connection control plane on the host (stdlib hmac/hashlib), not the
    hot path; `derive_pending_states_gpu` does the same for thousands of
    connections in one launch (tg_derive.h) and leaves the states in HBM.
  * `RecordLayer`: write()/read() over a socket with every record sealed and
    opened by the gfx950 kernels -- the shape of TLSRecordLayer.write/read
    (tlsrecordlayer.py:163-255) once the handshake is done.

The handshake itself (RSA/SRP/DH, certificates, Finished) is out of scope:
see DESIGN.md.
"""
import ctypes
import hashlib
import hmac
import os

import numpy as np

from . import _native as N
from .constants import SUITE_NAMES, ContentType, suite_primitives
from .recordlayer import BadRecordMAC, DecryptionFailed, open_records, parse_records, plan_write, seal
from .state import ConnectionState


def _p_hash(digest, secret, seed, length):
    out = bytearray()
    a = seed
    while len(out) < length:
        a = hmac.new(secret, a, digest).digest()
        out += hmac.new(secret, a + seed, digest).digest()
    return bytes(out[:length])


def prf(version, secret, label, seed, length):
    """TLS PRF for `version` (mathtls.py:37-50 PRF, :52-53 PRF_1_2)."""
    secret, seed = bytes(secret), bytes(label) + bytes(seed)
    if tuple(version) == (3, 3):
        return _p_hash(hashlib.sha256, secret, seed, length)
    half = (len(secret) + 1) // 2
    s1, s2 = secret[:half], secret[len(secret) // 2:]
    a = _p_hash(hashlib.md5, s1, seed, length)
    b = _p_hash(hashlib.sha1, s2, seed, length)
    return bytes(x ^ y for x, y in zip(a, b))


def prf_ssl(secret, seed, length):
    """SSL 3.0 key derivation (mathtls.py:55-68)."""
    out = bytearray()
    for i in range(26):
        label = bytes([ord("A") + i]) * (i + 1)
        out += hashlib.md5(bytes(secret) + hashlib.sha1(label + bytes(secret) + bytes(seed)).digest()).digest()
        if len(out) >= length:
            break
    return bytes(out[:length])


def master_secret(version, premaster, client_random, server_random):
    """calcMasterSecret (mathtls.py:70-82)."""
    version = tuple(version)
    if version == (3, 0):
        return prf_ssl(premaster, bytes(client_random) + bytes(server_random), 48)
    return prf(version, premaster, b"master secret", bytes(client_random) + bytes(server_random), 48)


def key_block(version, suite, master, client_random, server_random):
    """Key block + slicing of _calcPendingStates (tlsrecordlayer.py:1097-1126)."""
    cipher, mac, kl, ivl, ml = suite_primitives(suite)
    n = 2 * (ml + kl + ivl)
    seed = bytes(server_random) + bytes(client_random)
    if tuple(version) == (3, 0):
        kb = prf_ssl(master, seed, n)
    else:
        kb = prf(version, master, b"key expansion", seed, n)
    parts = {}
    pos = 0
    for name, size in (("client_mac", ml), ("server_mac", ml), ("client_key", kl), ("server_key", kl),
                       ("client_iv", ivl), ("server_iv", ivl)):
        parts[name] = kb[pos:pos + size]
        pos += size
    return kb, parts


def pending_states(version, suite, master, client_random, server_random, client, fixed_iv=None):
    """(write_state, read_state) for one side.  fixed_iv: this side's
    fixedIVBlock (random by default, tlsrecordlayer.py:1146-1149); it only
    affects the sender, the receiver strips the explicit IV."""
    _, kp = key_block(version, suite, master, client_random, server_random)
    cipher, mac, kl, ivl, ml = suite_primitives(suite)
    need_fiv = tuple(version) >= (3, 2) and ivl
    if fixed_iv is None and need_fiv:
        fixed_iv = os.urandom(ivl)
    me, peer = ("client", "server") if client else ("server", "client")
    w = ConnectionState(cipher, mac, version, kp[me + "_key"], kp[me + "_iv"], kp[me + "_mac"],
                        fixed_iv if need_fiv else None)
    r = ConnectionState(cipher, mac, version, kp[peer + "_key"], kp[peer + "_iv"], kp[peer + "_mac"],
                        bytes(ivl) if need_fiv else None)
    return w, r


class DerivedStates:
    """Result of `derive_pending_states_gpu`: this side's pending write and
    read states of n connections, resident in HBM (n * 2048 B each) where
    the seal/open kernels take them, plus per-connection status."""

    def __init__(self, n, write, read, master, key_block, status):
        self.n, self.write, self.read = n, write, read
        self.master, self.key_block, self.status = master, key_block, status

    def write_state_bytes(self, i):
        return bytes(self.write.download(N.CONN_STATE_BYTES, i * N.CONN_STATE_BYTES))

    def read_state_bytes(self, i):
        return bytes(self.read.download(N.CONN_STATE_BYTES, i * N.CONN_STATE_BYTES))


def derive_pending_states_gpu(conns, premaster=False, want_key_block=False, stream=None):
    """_calcPendingStates (tlsrecordlayer.py:1061-1149) for many connections
    at once on the GPU.  conns: iterable of dicts with `secret` (48-byte
    master secret, or premaster when premaster=True: calcMasterSecret
    mathtls.py:70-82 runs first), `client_random`, `server_random`, `suite`,
    `version`, `client` (bool) and optional `fixed_iv` (random when absent,
    as the reference's getRandomBytes).  Raises ValueError
    (the reference's AssertionError paths) if any connection has an
    unknown suite or version."""
    from .device import DeviceBuffer, synchronize

    conns = list(conns)
    n = len(conns)
    descs = (N.DeriveDesc * max(1, n))()
    for i, c in enumerate(conns):
        d = descs[i]
        for field, size in (("secret", 48), ("client_random", 32), ("server_random", 32)):
            v = bytes(c[field])
            if len(v) != size:
                raise ValueError("%s must be %d bytes" % (field, size))
            ctypes.memmove(ctypes.addressof(d) + getattr(N.DeriveDesc, field).offset, v, size)
        # the sender's fixedIVBlock is getRandomBytes(ivLength) (tlsrecordlayer.py:1146-1149)
        fiv = bytes(c.get("fixed_iv") or os.urandom(16))[:16]
        ctypes.memmove(ctypes.addressof(d) + N.DeriveDesc.fixed_iv.offset, fiv, len(fiv))
        suite = c["suite"]
        d.suite = SUITE_NAMES[suite] if isinstance(suite, str) else int(suite)
        d.ver_major, d.ver_minor = tuple(c["version"])
        d.client = 1 if c.get("client", True) else 0
        d.flags = N.DERIVE_PREMASTER if premaster else 0
    dd = DeviceBuffer(ctypes.sizeof(descs))
    dd.upload(bytes(descs))
    ws, rs = DeviceBuffer(n * N.CONN_STATE_BYTES), DeviceBuffer(n * N.CONN_STATE_BYTES)
    ms = DeviceBuffer(n * 48)
    kb = DeviceBuffer(n * N.KEY_BLOCK_MAX) if want_key_block else None
    st = DeviceBuffer(4 * max(1, n))
    N.call("tlsgpu_derive_states_dev", dd.ptr, n, ws.ptr, rs.ptr, ms.ptr, kb.ptr if kb else None, st.ptr,
           stream.handle if stream else None)
    if stream is None:
        synchronize()
    status = st.download(4 * n).view(np.int32)
    if (status != 0).any():
        bad = int(np.nonzero(status)[0][0])
        raise ValueError("key derivation failed for connection %d (suite/version)" % bad)
    master = ms.download(48 * n).reshape(n, 48)
    key_block = kb.download().reshape(n, N.KEY_BLOCK_MAX) if kb else None
    return DerivedStates(n, ws, rs, master, key_block, status)


class RecordLayer:
    """Application-data write()/read() over a connected socket, records sealed
    and opened on the GPU."""

    def __init__(self, sock, version, write_state, read_state):
        self.sock, self.version = sock, tuple(version)
        self._w, self._r = write_state, read_state
        self._inbuf = b""
        self._plain = bytearray()
        self.closed = False

    def write(self, data):
        """TLSRecordLayer.write: 16384-byte fragments, TLS<=1.0 block-cipher
        1/n-1 split (tlsrecordlayer.py:257-295, :543-550)."""
        if self.closed:
            raise ValueError("attempt to write to closed connection")
        payloads = plan_write(data, self.version, self._w.isBlockCipher)
        if payloads:
            wires = seal([self._w], [(0, p, ContentType.application_data) for p in payloads])
            self.sock.sendall(b"".join(wires))

    def _pump(self):
        chunk = self.sock.recv(1 << 16)
        if not chunk:
            return False
        self._inbuf += chunk
        recs, self._inbuf = parse_records(self._inbuf)
        if recs:
            res = open_records([self._r] * 1, [(0, ct, body) for ct, _, body in recs])
            for (ct, _, _), (st, p) in zip(recs, res):
                if st == N.ALERT_BAD_RECORD_MAC:
                    self.closed = True
                    raise BadRecordMAC("MAC failure (or padding failure)")
                if st == N.ALERT_DECRYPTION_FAILED:
                    self.closed = True
                    raise DecryptionFailed("decryption failed")
                if ct == ContentType.application_data:
                    self._plain += p
                elif ct == ContentType.alert:
                    self.closed = True  # nothing after an alert is delivered
                    self._inbuf = b""
                    break
        return True

    def read(self, max=None, min=1):
        """TLSRecordLayer.read (tlsrecordlayer.py:163-231): block until at
        least `min` bytes of application data are available."""
        while len(self._plain) < min and not self.closed:
            if not self._pump():
                break
        n = len(self._plain) if max is None else min_(max, len(self._plain))
        out = bytes(self._plain[:n])
        del self._plain[:n]
        return out

    def close(self):
        """Send a sealed close_notify alert (level warning=1, description 0)."""
        if not self.closed:
            wires = seal([self._w], [(0, b"\x01\x00", ContentType.alert)])
            self.sock.sendall(wires[0])
            self.closed = True


def min_(a, b):
    return a if a < b else b

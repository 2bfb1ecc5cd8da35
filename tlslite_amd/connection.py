"""Post-handshake plumbing around the GPU record path (config 1 harness).

  * key-block derivation exactly as `_calcPendingStates` performs it
    (tlslite/tlsrecordlayer.py:1061-1149) from a master secret
    (calcMasterSecret, tlslite/mathtls.py:70-82) with the TLS 1.0/1.1 PRF,
    the TLS 1.2 PRF_1_2 and SSL 3.0 PRF_SSL (mathtls.py:24-68).  This is
    per-connection control plane on the host (stdlib hmac/hashlib), not the
    hot path.
  * `RecordLayer`: write()/read() over a socket with every record sealed and
    opened by the gfx950 kernels -- the shape of TLSRecordLayer.write/read
    (tlsrecordlayer.py:163-255) once the handshake is done.

The handshake itself (RSA/SRP/DH, certificates, Finished) is out of scope:
see DESIGN.md.
"""
import hashlib
import hmac
import os

from . import _native as N
from .constants import ContentType, suite_primitives
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
                    self.closed = True
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

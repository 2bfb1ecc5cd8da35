"""Per-connection record state (one direction), the device-side counterpart of
tlslite's `_ConnectionState` + its macContext/encContext
(tlslite/tlsrecordlayer.py:27-37, :1061-1149).

The state is an opaque 2 KiB blob built by `tlsgpu_conn_state_init` (key
schedule, HMAC midstates, CBC residue, fixedIVBlock, RC4 S/i/j, seqnum) that
the kernels update in place, so consecutive batches behave like one long
tlslite connection.
"""
import ctypes

import numpy as np

from . import _native as N
from .constants import CIPHERS, MACS, suite_primitives

STATE_BYTES = N.CONN_STATE_BYTES


def _buf(b):
    return None if b is None else ctypes.c_char_p(bytes(b))


class ConnectionState:
    def __init__(self, cipher, mac, version, key, iv=b"", mac_key=b"", fixed_iv=None, seqnum=0):
        self.cipher, self.mac, self.version = cipher, mac, tuple(version)
        self.raw = bytearray(STATE_BYTES)
        cid = CIPHERS[cipher][0]
        mid = MACS[mac][0]
        buf = (ctypes.c_uint8 * STATE_BYTES).from_buffer(self.raw)
        fiv = bytes(fixed_iv) if fixed_iv is not None else None
        N.call("tlsgpu_conn_state_init", buf, cid, mid, self.version[0], self.version[1], _buf(key), len(key),
               _buf(iv), len(iv), _buf(mac_key), len(mac_key), _buf(fiv), len(fiv) if fiv else 0, seqnum)

    @classmethod
    def for_suite(cls, suite, version, key, iv, mac_key, fixed_iv=None, seqnum=0):
        cipher, mac, _, _, _ = suite_primitives(suite)
        return cls(cipher, mac, version, key, iv, mac_key, fixed_iv, seqnum)

    def _p(self):
        return (ctypes.c_uint8 * STATE_BYTES).from_buffer(self.raw)

    @property
    def variant(self):
        v = ctypes.c_uint32()
        N.call("tlsgpu_conn_state_variant", self._p(), ctypes.byref(v))
        return v.value

    @property
    def isBlockCipher(self):
        return self.cipher != "rc4"

    @property
    def seqnum(self):
        v = ctypes.c_uint64()
        N.call("tlsgpu_conn_state_get_seqnum", self._p(), ctypes.byref(v))
        return v.value

    @seqnum.setter
    def seqnum(self, value):
        N.call("tlsgpu_conn_state_set_seqnum", self._p(), int(value))

    @property
    def iv(self):
        out = ctypes.create_string_buffer(16)
        n = ctypes.c_size_t()
        N.call("tlsgpu_conn_state_get_iv", self._p(), out, 16, ctypes.byref(n))
        return out.raw[: n.value]

    @iv.setter
    def iv(self, value):
        N.call("tlsgpu_conn_state_set_iv", self._p(), _buf(value), len(value))

    @property
    def rc4(self):
        S = ctypes.create_string_buffer(256)
        i, j = ctypes.c_uint32(), ctypes.c_uint32()
        N.call("tlsgpu_conn_state_get_rc4", self._p(), S, ctypes.byref(i), ctypes.byref(j))
        return S.raw, i.value, j.value

    def wire_len(self, pt_len):
        v = ctypes.c_uint32()
        N.call("tlsgpu_seal_wire_len", self._p(), int(pt_len), ctypes.byref(v))
        return v.value

    def copy(self):
        c = ConnectionState.__new__(ConnectionState)
        c.cipher, c.mac, c.version = self.cipher, self.mac, self.version
        c.raw = bytearray(self.raw)
        return c


def cipher_state(cipher, key, iv):
    """Raw cipher-object context (no MAC / framing) -- the factory surface."""
    raw = bytearray(STATE_BYTES)
    buf = (ctypes.c_uint8 * STATE_BYTES).from_buffer(raw)
    N.call("tlsgpu_cipher_state_init", buf, CIPHERS[cipher][0], _buf(key), len(key), _buf(iv), len(iv))
    return raw


def pack_states(states):
    """list of ConnectionState -> contiguous numpy uint8 [n * 2048]."""
    a = np.empty(len(states) * STATE_BYTES, dtype=np.uint8)
    for i, s in enumerate(states):
        a[i * STATE_BYTES:(i + 1) * STATE_BYTES] = np.frombuffer(s.raw, dtype=np.uint8)
    return a


def unpack_states(arr, states):
    for i, s in enumerate(states):
        s.raw[:] = arr[i * STATE_BYTES:(i + 1) * STATE_BYTES].tobytes()

"""Shared engine of the "hip" cipher objects: one stateful context per
object, each encrypt/decrypt call is one kernel launch over the caller's
bytes (tlsgpu_cipher_dev), with the context blob carried on the host between
calls exactly like tlslite's objects carry `self.IV` / `S, i, j`
(python_aes.py:44, python_rc4.py:36-37)."""
import ctypes

import numpy as np

from .. import _native as N
from ..constants import CIPHERS
from ..device import DeviceBuffer, device_count, synchronize
from ..state import STATE_BYTES, cipher_state


def hip_available():
    return device_count() > 0


class _Workspace:
    """Grow-only device buffers reused across calls."""

    def __init__(self):
        self.cap = 0
        self.buf = self.state = self.span = None

    def ensure(self, n):
        if self.buf is None or n > self.cap:
            self.cap = max(n, 2 * self.cap, 4096)
            self.buf = DeviceBuffer(self.cap)
        if self.state is None:
            self.state = DeviceBuffer(STATE_BYTES)
            self.span = DeviceBuffer(ctypes.sizeof(N.Span))


_ws = _Workspace()


class HipCipherContext:
    def __init__(self, cipher, key, iv):
        self.cipher = cipher
        self.raw = cipher_state(cipher, bytes(key), bytes(iv))

    def run(self, data, decrypt):
        data = bytes(data)
        n = len(data)
        if n == 0:
            return bytearray()
        _ws.ensure(n)
        sp = N.Span(0, n, 0)
        _ws.buf.upload(np.frombuffer(data, dtype=np.uint8))
        _ws.state.upload(np.frombuffer(bytes(self.raw), dtype=np.uint8))
        _ws.span.upload(np.frombuffer(bytes(sp), dtype=np.uint8))
        N.call("tlsgpu_cipher_dev", _ws.span.ptr, 1, _ws.buf.ptr, _ws.buf.ptr, _ws.state.ptr,
               CIPHERS[self.cipher][0], 1 if decrypt else 0, None)
        synchronize()
        out = _ws.buf.download(n)
        self.raw[:] = _ws.state.download(STATE_BYTES).tobytes()
        return bytearray(out.tobytes())

    def iv(self):
        out = ctypes.create_string_buffer(16)
        ln = ctypes.c_size_t()
        buf = (ctypes.c_uint8 * STATE_BYTES).from_buffer(self.raw)
        N.call("tlsgpu_conn_state_get_iv", buf, out, 16, ctypes.byref(ln))
        return bytearray(out.raw[: ln.value])

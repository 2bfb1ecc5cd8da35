"""Device plumbing over the C ABI: device selection, HBM buffers, pinned host
buffers, streams and events.  No PyTorch: the product drives HIP directly
through libtlsgpu.so."""
import ctypes

import numpy as np

from . import _native as N


def device_count():
    n = ctypes.c_int(0)
    rc = N.lib.tlsgpu_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_device(ordinal):
    N.call("tlsgpu_set_device", ordinal)


def synchronize():
    N.call("tlsgpu_device_synchronize")


def current_device():
    d = ctypes.c_int(0)
    N.call("tlsgpu_get_device", ctypes.byref(d))
    return d.value


def cu_count(ordinal=None):
    """Compute units of `ordinal` (default: the current device)."""
    n = ctypes.c_int(0)
    N.call("tlsgpu_device_cu_count", current_device() if ordinal is None else ordinal, ctypes.byref(n))
    return n.value


def arch(ordinal=0):
    buf = ctypes.create_string_buffer(64)
    N.call("tlsgpu_device_arch", ordinal, buf, 64)
    return buf.value.decode()


class Stream:
    """A HIP stream of the library (tlsgpu_stream_create, the runtime's normal priority);
    high=True / False: created at the runtime's greatest / least priority level
    (tlsgpu_stream_create_priority; the least level is below normal) -- two streams whose
    kernels must overlap are only certain to get separate hardware queues at different
    priorities."""
    def __init__(self, default=False, high=None):
        self.handle = ctypes.c_void_p(None)
        self._own = not default
        if not default:
            if high is None:
                N.call("tlsgpu_stream_create", ctypes.byref(self.handle))
            else:
                N.call("tlsgpu_stream_create_priority", ctypes.byref(self.handle), 1 if high else 0)

    def synchronize(self):
        N.call("tlsgpu_stream_synchronize", self.handle)

    def close(self):
        if getattr(self, "_own", False) and self.handle:
            N.lib.tlsgpu_stream_destroy(self.handle)
            self.handle = ctypes.c_void_p(None)

    def __del__(self):
        self.close()


class Event:
    def __init__(self):
        self.handle = ctypes.c_void_p(None)
        N.call("tlsgpu_event_create", ctypes.byref(self.handle))

    def record(self, stream=None):
        N.call("tlsgpu_event_record", self.handle, stream.handle if stream else None)

    def synchronize(self):
        N.call("tlsgpu_event_synchronize", self.handle)

    def elapsed_ms(self, later):
        ms = ctypes.c_float(0)
        N.call("tlsgpu_event_elapsed_ms", ctypes.byref(ms), self.handle, later.handle)
        return ms.value

    def __del__(self):
        if getattr(self, "handle", None):
            N.lib.tlsgpu_event_destroy(self.handle)
            self.handle = None


class DeviceBuffer:
    """A byte buffer in HBM."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = ctypes.c_void_p(None)
        N.call("tlsgpu_malloc", ctypes.byref(self.ptr), max(1, self.nbytes))

    @property
    def addr(self):
        return self.ptr.value

    def at(self, offset):
        return ctypes.c_void_p(self.ptr.value + int(offset))

    def upload(self, src, offset=0, stream=None):
        """src: bytes / bytearray / numpy array (host memory)."""
        a = np.ascontiguousarray(np.frombuffer(src, dtype=np.uint8) if isinstance(src, (bytes, bytearray, memoryview))
                                 else src).view(np.uint8).reshape(-1)
        if offset + a.nbytes > self.nbytes:
            raise ValueError("upload out of range")
        N.call("tlsgpu_memcpy_h2d", self.at(offset), a.ctypes.data_as(ctypes.c_void_p), a.nbytes,
               stream.handle if stream else None)
        if stream is None:
            synchronize()

    def download(self, nbytes=None, offset=0, out=None, stream=None):
        nbytes = self.nbytes - offset if nbytes is None else int(nbytes)
        if out is None:
            out = np.empty(nbytes, dtype=np.uint8)
        N.call("tlsgpu_memcpy_d2h", out.ctypes.data_as(ctypes.c_void_p), self.at(offset), nbytes,
               stream.handle if stream else None)
        if stream is None:
            synchronize()
        return out

    def zero(self, stream=None):
        N.call("tlsgpu_memset", self.ptr, 0, self.nbytes, stream.handle if stream else None)

    def free(self):
        if self.ptr:
            N.lib.tlsgpu_free(self.ptr)
            self.ptr = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host buffer (hipHostMalloc) exposed as a numpy uint8 array,
    the staging area between socket buffers and HBM."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = ctypes.c_void_p(None)
        N.call("tlsgpu_host_alloc", ctypes.byref(self.ptr), max(1, self.nbytes))
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, self.nbytes)).from_address(self.ptr.value))

    def free(self):
        if self.ptr:
            self.array = None
            N.lib.tlsgpu_host_free(self.ptr)
            self.ptr = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def copy_h2d(dst, dst_off, src_ptr, nbytes, stream):
    N.call("tlsgpu_memcpy_h2d", dst.at(dst_off), ctypes.c_void_p(src_ptr), nbytes, stream.handle if stream else None)


def copy_d2h(dst_ptr, src, src_off, nbytes, stream):
    N.call("tlsgpu_memcpy_d2h", ctypes.c_void_p(dst_ptr), src.at(src_off), nbytes, stream.handle if stream else None)


def fill_pattern(buf, nbytes, seed, start=0, offset=0, stream=None):
    """Deterministic synthetic bytes (splitmix64 stream) written on the device."""
    N.call("tlsgpu_fill_pattern", buf.at(offset), int(nbytes), seed, start, stream.handle if stream else None)

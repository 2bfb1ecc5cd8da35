"""ctypes binding of libtlsgpu.so (include/tlsgpu.h).

There is no CPU fallback: if the HIP library is missing this module raises
ImportError, and every compute call goes to the gfx950 kernels.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# TLSGPU_LIB: an alternative build of the same library (A/B timing tools only)
LIB_PATH = os.environ.get("TLSGPU_LIB") or os.path.join(HERE, "lib", "libtlsgpu.so")

# constants mirrored from include/tlsgpu.h
CIPHER_AES128, CIPHER_AES256, CIPHER_RC4, CIPHER_3DES, CIPHER_AES192 = 1, 2, 3, 4, 5
MAC_SHA1, MAC_SHA256, MAC_MD5 = 1, 2, 3
FAULT_BAD_MAC, FAULT_BAD_PADDING = 1, 2
OK, EINVAL, EHIP, ENODEV, ETOOBIG, EMISMATCH, EFRAME, EABRUPT = 0, -1, -2, -3, -4, -5, -6, -7
ALERT_BAD_RECORD_MAC, ALERT_DECRYPTION_FAILED, ALERT_SKIPPED, ALERT_RECORD_OVERFLOW = -20, -21, -22, -23
CHAIN_STOP_ON_ALERT = 1
OPEN_SPLIT_AUTO, OPEN_SPLIT_CHAINS, OPEN_SPLIT_NONE, OPEN_SPLIT_BLOCKS = 0, 1, 2, 3
ABI_VERSION = 7
CONN_STATE_BYTES = 2048


def variant(cipher, mac, ssl3):
    return cipher | (mac << 8) | ((1 if ssl3 else 0) << 16)


class Record(ctypes.Structure):  # tlsgpu_record
    _fields_ = [("pt_off", ctypes.c_uint64), ("wire_off", ctypes.c_uint64), ("pt_len", ctypes.c_uint32),
                ("content_type", ctypes.c_uint8), ("flags", ctypes.c_uint8), ("reserved", ctypes.c_uint16)]


class Chain(ctypes.Structure):  # tlsgpu_chain
    _fields_ = [("state", ctypes.c_uint32), ("first", ctypes.c_uint32), ("count", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


class OpenRecord(ctypes.Structure):  # tlsgpu_open_record
    _fields_ = [("ct_off", ctypes.c_uint64), ("pt_off", ctypes.c_uint64), ("ct_len", ctypes.c_uint32),
                ("content_type", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3)]


class Span(ctypes.Structure):  # tlsgpu_span
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint32), ("state", ctypes.c_uint32)]


class DeriveDesc(ctypes.Structure):  # tlsgpu_derive_desc
    _fields_ = [("secret", ctypes.c_uint8 * 48), ("client_random", ctypes.c_uint8 * 32),
                ("server_random", ctypes.c_uint8 * 32), ("fixed_iv", ctypes.c_uint8 * 16),
                ("suite", ctypes.c_uint16), ("ver_major", ctypes.c_uint8), ("ver_minor", ctypes.c_uint8),
                ("client", ctypes.c_uint8), ("flags", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 2)]


DERIVE_PREMASTER = 1
KEY_BLOCK_MAX = 160
assert ctypes.sizeof(DeriveDesc) == 136
assert ctypes.sizeof(Record) == 24 and ctypes.sizeof(Chain) == 16
assert ctypes.sizeof(OpenRecord) == 24 and ctypes.sizeof(Span) == 16

# (name, restype, argtypes) for every symbol of include/tlsgpu.h
_vp, _u8p, _sz, _i, _u32, _u64 = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
SIGNATURES = [
    ("tlsgpu_abi_version", _i, []),
    ("tlsgpu_last_error", ctypes.c_char_p, []),
    ("tlsgpu_device_count", _i, [ctypes.POINTER(_i)]),
    ("tlsgpu_set_device", _i, [_i]),
    ("tlsgpu_get_device", _i, [ctypes.POINTER(_i)]),
    ("tlsgpu_device_synchronize", _i, []),
    ("tlsgpu_device_arch", _i, [_i, ctypes.c_char_p, _sz]),
    ("tlsgpu_device_cu_count", _i, [_i, ctypes.POINTER(_i)]),
    ("tlsgpu_malloc", _i, [ctypes.POINTER(_vp), _sz]),
    ("tlsgpu_free", _i, [_vp]),
    ("tlsgpu_host_alloc", _i, [ctypes.POINTER(_vp), _sz]),
    ("tlsgpu_host_free", _i, [_vp]),
    ("tlsgpu_memcpy_h2d", _i, [_vp, _vp, _sz, _vp]),
    ("tlsgpu_memcpy_d2h", _i, [_vp, _vp, _sz, _vp]),
    ("tlsgpu_memcpy_d2d", _i, [_vp, _vp, _sz, _vp]),
    ("tlsgpu_memset", _i, [_vp, _i, _sz, _vp]),
    ("tlsgpu_stream_create", _i, [ctypes.POINTER(_vp)]),
    ("tlsgpu_stream_create_priority", _i, [ctypes.POINTER(_vp), ctypes.c_int]),
    ("tlsgpu_stream_destroy", _i, [_vp]),
    ("tlsgpu_stream_synchronize", _i, [_vp]),
    ("tlsgpu_event_create", _i, [ctypes.POINTER(_vp)]),
    ("tlsgpu_event_destroy", _i, [_vp]),
    ("tlsgpu_event_record", _i, [_vp, _vp]),
    ("tlsgpu_event_synchronize", _i, [_vp]),
    ("tlsgpu_event_elapsed_ms", _i, [ctypes.POINTER(ctypes.c_float), _vp, _vp]),
    ("tlsgpu_conn_state_init", _i, [_vp, _i, _i, _i, _i, _u8p, _sz, _u8p, _sz, _u8p, _sz, _u8p, _sz, _u64]),
    ("tlsgpu_cipher_state_init", _i, [_vp, _i, _u8p, _sz, _u8p, _sz]),
    ("tlsgpu_conn_state_set_seqnum", _i, [_vp, _u64]),
    ("tlsgpu_conn_state_set_iv", _i, [_vp, _u8p, _sz]),
    ("tlsgpu_conn_state_get_seqnum", _i, [_vp, ctypes.POINTER(_u64)]),
    ("tlsgpu_conn_state_get_iv", _i, [_vp, _u8p, _sz, ctypes.POINTER(_sz)]),
    ("tlsgpu_conn_state_get_rc4", _i, [_vp, _u8p, ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    ("tlsgpu_conn_state_variant", _i, [_vp, ctypes.POINTER(_u32)]),
    ("tlsgpu_seal_wire_len", _i, [_vp, _u32, ctypes.POINTER(_u32)]),
    ("tlsgpu_seal_workspace_bytes", _sz, [_u32]),
    ("tlsgpu_release_workspaces", _i, []),
    ("tlsgpu_owned_workspace_count", _sz, []),
    ("tlsgpu_owned_stream_count", _sz, []),
    ("tlsgpu_seal_cipher_kernel", _i, [_u32, _u32, ctypes.c_char_p, _sz]),
    ("tlsgpu_seal_dev", _i, [_vp, _u32, _vp, _u32, _vp, _sz, _vp, _sz, _vp, _u32, _vp, _u32, _vp, _sz, _vp]),
    ("tlsgpu_pipeline_create", _i, [ctypes.POINTER(_vp), _u32]),
    ("tlsgpu_pipeline_destroy", _i, [_vp]),
    ("tlsgpu_pipeline_synchronize", _i, [_vp]),
    ("tlsgpu_pipeline_seal", _i, [_vp, _vp, _u32, _vp, _u32, _vp, _sz, _vp, _sz, _vp, _u32, _vp, _u32, _vp, _vp]),
    ("tlsgpu_host_pipeline_create", _i, [ctypes.POINTER(_vp), _sz, _i]),
    ("tlsgpu_host_pipeline_destroy", _i, [_vp]),
    ("tlsgpu_host_pipeline_seal", _i, [_vp, _vp, _u32, _vp, _u32, _vp, _sz, _vp, _sz, _vp, _u32, _vp, _u32]),
    ("tlsgpu_host_pipeline_d2h_path", _i, [_vp, _vp]),
    ("tlsgpu_host_store", _i, [_vp, _vp, _sz, _vp]),
    ("tlsgpu_host_pipeline_open", _i, [_vp, _vp, _sz, _vp, _u32, _u32, _vp, _sz, _vp, _u32, _u32, _vp, _u32, _vp, _vp,
                                       _vp, _vp, _vp]),
    ("tlsgpu_open_workspace_bytes", _sz, [_u32]),
    ("tlsgpu_open_dev", _i, [_vp, _u32, _vp, _u32, _vp, _sz, _vp, _sz, _vp, _u32, _vp, _u32, _vp, _sz, _vp]),
    ("tlsgpu_set_open_parts", _i, [_i, ctypes.c_int64]),
    ("tlsgpu_frame_workspace_bytes", _sz, [_u32]),
    ("tlsgpu_frame_dev", _i, [_vp, _sz, _vp, _u32, _vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _sz, _vp]),
    ("tlsgpu_cipher_dev", _i, [_vp, _u32, _vp, _vp, _vp, _i, _i, _vp]),
    ("tlsgpu_derive_states_dev", _i, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("tlsgpu_fill_pattern", _i, [_vp, _sz, _u64, _u64, _vp]),
]


class TLSGPUError(RuntimeError):
    def __init__(self, code, where):
        msg = last_error()
        super().__init__("%s failed (%d): %s" % (where, code, msg))
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libtlsgpu.so is not built (%s); run `python -c \"import __graft_entry__ as g; g.build()\"`"
                          % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        if os.environ.get("TLSGPU_LIB") and not hasattr(lib, name):
            continue  # an older A/B build may predate a symbol; the in-tree library must have all
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if not os.environ.get("TLSGPU_LIB") and lib.tlsgpu_abi_version() != ABI_VERSION:
        raise ImportError("libtlsgpu.so ABI %d, this binding expects %d: rebuild the library"
                          % (lib.tlsgpu_abi_version(), ABI_VERSION))
    return lib


lib = _load()


def last_error():
    s = lib.tlsgpu_last_error()
    return s.decode(errors="replace") if s else ""


def check(rc, where):
    if rc != 0:
        raise TLSGPUError(rc, where)
    return rc


def call(name, *args):
    return check(getattr(lib, name)(*args), name)

"""tlslite_amd -- MI355X-native TLS record-layer bulk crypto.

The hot path of tlslite (per-record MAC -> pad -> CBC/stream encrypt ->
header, tlslite/tlsrecordlayer.py:538-617) as hand-written gfx950 HIP kernels
behind a C ABI (include/tlsgpu.h, lib/libtlsgpu.so), with a tlslite-shaped
cipher-factory surface (utils/cipherfactory.py) and a batched record API
(recordlayer.py).  Importing fails if the HIP library is not built: there is
no CPU fallback.
"""
from . import _native  # noqa: F401  (raises ImportError when libtlsgpu.so is missing)
from .constants import CipherSuite, ContentType, Fault  # noqa: F401
from .state import ConnectionState  # noqa: F401
from .recordlayer import plan_write, seal, seal_write  # noqa: F401

__version__ = "0.1.0"

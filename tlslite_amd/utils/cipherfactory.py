"""Cipher factory with the tlslite signature (tlslite/utils/cipherfactory.py:31-102).

`implList` is walked in order and the first available implementation wins;
NotImplementedError if none is.  This package provides "hip" (gfx950
kernels).  The reference's own names ("openssl", "pycrypto", "python") are
recognised and skipped here -- they belong to tlslite itself; INTEGRATION.md
shows how tlslite's factory dispatches "hip" to this module.
"""
from . import hip_aes, hip_rc4, hip_tripledes
from ._hip_cipher import hip_available

IMPLEMENTATIONS = ["hip"]
tripleDESPresent = True  # handshakesettings.py:137-138 keys "3des" off this flag


def _pick(implList):
    if implList is None:
        implList = IMPLEMENTATIONS
    for impl in implList:
        if impl == "hip" and hip_available():
            return "hip"
    return None


def createAES(key, IV, implList=None):
    """AES-CBC object (key 16/24/32 bytes, IV 16 bytes)."""
    if _pick(implList) == "hip":
        return hip_aes.new(key, 2, IV)
    raise NotImplementedError()


def createRC4(key, IV, implList=None):
    """RC4 object (key 16..256 bytes; IV must be empty, cipherfactory.py:70-71)."""
    if len(IV) != 0:
        raise AssertionError()
    if _pick(implList) == "hip":
        return hip_rc4.new(key)
    raise NotImplementedError()


def createTripleDES(key, IV, implList=None):
    """3DES-EDE-CBC object (key 24 bytes, IV 8 bytes)."""
    if _pick(implList) == "hip":
        return hip_tripledes.new(key, 2, IV)
    raise NotImplementedError()

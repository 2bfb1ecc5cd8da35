"""3DES-EDE-CBC cipher object on the GPU (the "hip" counterpart of
tlslite/utils/openssl_tripledes.py; tlslite itself has no pure-Python 3DES)."""
from .tripledes import TripleDES
from ._hip_cipher import HipCipherContext


def new(key, mode, IV):
    return HIP_TripleDES(key, mode, IV)


class HIP_TripleDES(TripleDES):
    def __init__(self, key, mode, IV):
        TripleDES.__init__(self, key, mode, IV, "hip")
        self._ctx = HipCipherContext("3des", key, IV)

    @property
    def IV(self):
        return self._ctx.iv()

    def encrypt(self, plaintext):
        TripleDES.encrypt(self, plaintext)
        return self._ctx.run(plaintext, decrypt=False)

    def decrypt(self, ciphertext):
        TripleDES.decrypt(self, ciphertext)
        return self._ctx.run(ciphertext, decrypt=True)

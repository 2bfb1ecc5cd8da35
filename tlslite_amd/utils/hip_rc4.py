"""RC4 cipher object on the GPU (the "hip" counterpart of
tlslite/utils/python_rc4.py)."""
from .rc4 import RC4
from ._hip_cipher import HipCipherContext


def new(key):
    return HIP_RC4(key)


class HIP_RC4(RC4):
    def __init__(self, keyBytes):
        RC4.__init__(self, keyBytes, "hip")
        self._ctx = HipCipherContext("rc4", keyBytes, b"")

    def encrypt(self, plaintext):
        return self._ctx.run(plaintext, decrypt=False)

    def decrypt(self, ciphertext):
        return self._ctx.run(ciphertext, decrypt=True)

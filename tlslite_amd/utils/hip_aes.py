"""AES-CBC cipher object on the GPU (the "hip" counterpart of
tlslite/utils/python_aes.py / openssl_aes.py)."""
from .aes import AES
from ._hip_cipher import HipCipherContext


def new(key, mode, IV):
    return HIP_AES(key, mode, IV)


class HIP_AES(AES):
    def __init__(self, key, mode, IV):
        AES.__init__(self, key, mode, IV, "hip")
        self._ctx = HipCipherContext(self.name, key, IV)

    @property
    def IV(self):
        """CBC residue carried between calls (python_aes.py:44)."""
        return self._ctx.iv()

    def encrypt(self, plaintext):
        AES.encrypt(self, plaintext)
        return self._ctx.run(plaintext, decrypt=False)

    def decrypt(self, ciphertext):
        AES.decrypt(self, ciphertext)
        return self._ctx.run(ciphertext, decrypt=True)

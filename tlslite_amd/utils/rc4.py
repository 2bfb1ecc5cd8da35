"""Abstract RC4 cipher object (interface of tlslite/utils/rc4.py:6-19)."""


class RC4(object):
    def __init__(self, keyBytes, implementation):
        if not 16 <= len(keyBytes) <= 256:
            raise ValueError()
        self.isBlockCipher = False
        self.name = "rc4"
        self.implementation = implementation

    def encrypt(self, plaintext):
        raise NotImplementedError()

    def decrypt(self, ciphertext):
        raise NotImplementedError()

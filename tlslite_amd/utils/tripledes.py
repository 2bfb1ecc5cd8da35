"""Abstract 3DES-EDE-CBC cipher object (interface of tlslite/utils/tripledes.py:6-27)."""


class TripleDES(object):
    def __init__(self, key, mode, IV, implementation):
        if len(key) != 24 or mode != 2 or len(IV) != 8:
            raise ValueError()
        self.isBlockCipher = True
        self.block_size = 8
        self.implementation = implementation
        self.name = "3des"

    def encrypt(self, plaintext):
        assert len(plaintext) % 8 == 0

    def decrypt(self, ciphertext):
        assert len(ciphertext) % 8 == 0

"""Abstract AES cipher object (interface of tlslite/utils/aes.py:6-34)."""


class AES(object):
    _NAMES = {16: "aes128", 24: "aes192", 32: "aes256"}

    def __init__(self, key, mode, IV, implementation):
        # same argument contract as the reference: AssertionError on bad input
        if len(key) not in self._NAMES or mode != 2 or len(IV) != 16:
            raise AssertionError()
        self.isBlockCipher = True
        self.block_size = 16
        self.implementation = implementation
        self.name = self._NAMES[len(key)]

    def encrypt(self, plaintext):
        """CBC encrypt; returns the ciphertext (the input may be modified)."""
        assert len(plaintext) % 16 == 0

    def decrypt(self, ciphertext):
        """CBC decrypt; returns the plaintext (the input may be modified)."""
        assert len(ciphertext) % 16 == 0

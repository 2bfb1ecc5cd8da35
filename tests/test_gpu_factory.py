"""GPU: the cipher-factory surface ("hip" objects) vs the oracle / KATs,
including state carried across calls (python_aes.py:44, python_rc4.py:36)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _F():
    from tlslite_amd import device
    from tlslite_amd.utils import cipherfactory as F
    if device.device_count() < 1:
        pytest.fail("no GPU visible")
    return F


def test_aes_kats():
    F = _F()
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    for key, ct in [("000102030405060708090a0b0c0d0e0f", "69c4e0d86a7b0430d8cdb78070b4c55a"),
                    ("000102030405060708090a0b0c0d0e0f1011121314151617", "dda97ca4864cdfe06eaf70a0ec0d7191"),
                    ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
                     "8ea2b7ca516745bfeafc49904b496089")]:
        c = F.createAES(bytearray.fromhex(key), bytearray(16), ["hip"])
        assert c.implementation == "hip"
        assert bytes(c.encrypt(bytearray(pt))).hex() == ct
        d = F.createAES(bytearray.fromhex(key), bytearray(16), ["python", "hip"])
        assert bytes(d.decrypt(bytearray.fromhex(ct))) == pt


@pytest.mark.parametrize("cipher", ["aes128", "aes256", "rc4", "3des"])
def test_chunked_calls_match_oracle(cipher):
    from oracle import oracle as O
    F = _F()
    rng = np.random.default_rng(len(cipher))
    kl, ivl, bs = {"aes128": (16, 16, 16), "aes256": (32, 16, 16), "rc4": (16, 0, 1), "3des": (24, 8, 8)}[cipher]
    key, iv = rng.bytes(kl), rng.bytes(ivl)
    mk = {"aes128": F.createAES, "aes256": F.createAES, "rc4": F.createRC4, "3des": F.createTripleDES}[cipher]
    enc, dec = mk(bytearray(key), bytearray(iv), ["hip"]), mk(bytearray(key), bytearray(iv), ["hip"])
    oe = O.Conn(cipher, "sha1", (3, 1), key, iv, bytes(20))
    od = O.Conn(cipher, "sha1", (3, 1), key, iv, bytes(20))
    for n in [bs, 3 * bs, 64 * bs, bs, 1000 * bs]:
        data = rng.bytes(n)
        ct = bytes(enc.encrypt(bytearray(data)))
        assert ct == oe.encrypt(data)
        assert bytes(dec.decrypt(bytearray(ct))) == data == od.decrypt(ct)
    if cipher != "rc4":
        assert bytes(enc.IV) == oe.iv and bytes(dec.IV) == od.iv

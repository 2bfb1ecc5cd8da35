"""Suite / content-type identifiers of the record path.

Values are the IANA/TLS wire constants tlslite uses (tlslite/constants.py:
ContentType :38-44, CipherSuite :137-201).  The suite -> primitive table is
the one `_calcPendingStates` applies (tlslite/tlsrecordlayer.py:1063-1095).
"""
from . import _native as N


class ContentType:
    change_cipher_spec = 20
    alert = 21
    handshake = 22
    application_data = 23


class CipherSuite:
    TLS_RSA_WITH_3DES_EDE_CBC_SHA = 0x000A
    TLS_RSA_WITH_AES_128_CBC_SHA = 0x002F
    TLS_RSA_WITH_AES_256_CBC_SHA = 0x0035
    TLS_RSA_WITH_RC4_128_SHA = 0x0005
    TLS_RSA_WITH_RC4_128_MD5 = 0x0004
    TLS_DH_ANON_WITH_AES_128_CBC_SHA = 0x0034
    TLS_DH_ANON_WITH_AES_256_CBC_SHA = 0x003A
    TLS_RSA_WITH_AES_128_CBC_SHA256 = 0x003C
    TLS_RSA_WITH_AES_256_CBC_SHA256 = 0x003D
    TLS_SRP_SHA_WITH_3DES_EDE_CBC_SHA = 0xC01A
    TLS_SRP_SHA_WITH_AES_128_CBC_SHA = 0xC01D
    TLS_SRP_SHA_WITH_AES_256_CBC_SHA = 0xC020
    TLS_SRP_SHA_RSA_WITH_3DES_EDE_CBC_SHA = 0xC01B
    TLS_SRP_SHA_RSA_WITH_AES_128_CBC_SHA = 0xC01E
    TLS_SRP_SHA_RSA_WITH_AES_256_CBC_SHA = 0xC021


# cipher name -> (C-ABI id, key length, IV length)
CIPHERS = {
    "aes128": (N.CIPHER_AES128, 16, 16),
    "aes256": (N.CIPHER_AES256, 32, 16),
    "rc4": (N.CIPHER_RC4, 16, 0),
    "3des": (N.CIPHER_3DES, 24, 8),
    "aes192": (N.CIPHER_AES192, 24, 16),  # cipher objects only
}
# MAC name -> (C-ABI id, MAC length)
MACS = {"sha1": (N.MAC_SHA1, 20), "sha256": (N.MAC_SHA256, 32), "md5": (N.MAC_MD5, 16)}

_S = CipherSuite
# suite id -> (cipher name, MAC name)
SUITE_PRIMITIVES = {
    _S.TLS_RSA_WITH_3DES_EDE_CBC_SHA: ("3des", "sha1"),
    _S.TLS_SRP_SHA_WITH_3DES_EDE_CBC_SHA: ("3des", "sha1"),
    _S.TLS_SRP_SHA_RSA_WITH_3DES_EDE_CBC_SHA: ("3des", "sha1"),
    _S.TLS_RSA_WITH_AES_128_CBC_SHA: ("aes128", "sha1"),
    _S.TLS_DH_ANON_WITH_AES_128_CBC_SHA: ("aes128", "sha1"),
    _S.TLS_SRP_SHA_WITH_AES_128_CBC_SHA: ("aes128", "sha1"),
    _S.TLS_SRP_SHA_RSA_WITH_AES_128_CBC_SHA: ("aes128", "sha1"),
    _S.TLS_RSA_WITH_AES_256_CBC_SHA: ("aes256", "sha1"),
    _S.TLS_DH_ANON_WITH_AES_256_CBC_SHA: ("aes256", "sha1"),
    _S.TLS_SRP_SHA_WITH_AES_256_CBC_SHA: ("aes256", "sha1"),
    _S.TLS_SRP_SHA_RSA_WITH_AES_256_CBC_SHA: ("aes256", "sha1"),
    _S.TLS_RSA_WITH_AES_128_CBC_SHA256: ("aes128", "sha256"),
    _S.TLS_RSA_WITH_AES_256_CBC_SHA256: ("aes256", "sha256"),
    _S.TLS_RSA_WITH_RC4_128_SHA: ("rc4", "sha1"),
    _S.TLS_RSA_WITH_RC4_128_MD5: ("rc4", "md5"),
}

# short names used by tests / bench (OpenSSL-style)
SUITE_NAMES = {
    "AES128-SHA": _S.TLS_RSA_WITH_AES_128_CBC_SHA,
    "AES256-SHA": _S.TLS_RSA_WITH_AES_256_CBC_SHA,
    "AES128-SHA256": _S.TLS_RSA_WITH_AES_128_CBC_SHA256,
    "AES256-SHA256": _S.TLS_RSA_WITH_AES_256_CBC_SHA256,
    "RC4-SHA": _S.TLS_RSA_WITH_RC4_128_SHA,
    "RC4-MD5": _S.TLS_RSA_WITH_RC4_128_MD5,
    "3DES-SHA": _S.TLS_RSA_WITH_3DES_EDE_CBC_SHA,
}


def suite_primitives(suite):
    """suite id or short name -> (cipher, mac, key_len, iv_len, mac_len)."""
    if isinstance(suite, str):
        suite = SUITE_NAMES[suite]
    cipher, mac = SUITE_PRIMITIVES[suite]
    return cipher, mac, CIPHERS[cipher][1], CIPHERS[cipher][2], MACS[mac][1]


class Fault:
    """Record-layer fault injection codes (tlslite/constants.py:310-359)."""
    badMAC = 301
    badPadding = 302


FAULT_FLAGS = {None: 0, Fault.badMAC: N.FAULT_BAD_MAC, Fault.badPadding: N.FAULT_BAD_PADDING,
               "badMAC": N.FAULT_BAD_MAC, "badPadding": N.FAULT_BAD_PADDING}

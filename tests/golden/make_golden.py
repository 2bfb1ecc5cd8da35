#!/usr/bin/env python3
"""Generate golden TLS record vectors from the *reference* tlslite (run only in
the build container, where /root/reference exists).

Output: tests/golden/records.json (small, committed).  The GPU box never runs
this script and never reads /root/reference; it only reads the JSON.

How the reference is driven: `import tlslite` raises a
SyntaxError on Python 3.10 (`async` keyword at tlslite/tlsconnection.py:71), so a
namespace package stub is put in sys.modules and the record layer modules are
imported directly.  For every case we build a `TLSRecordLayer` on a fake socket,
install a `_ConnectionState` exactly the way `_calcPendingStates`
(tlslite/tlsrecordlayer.py:1061-1149) would, and call `_sendMsg`
(tlslite/tlsrecordlayer.py:538-660) or `writeAsync` (:257-295) to capture wire
bytes.

3DES: tlslite ships no pure-Python 3DES (tlslite/utils/cipherfactory.py:82-102);
its openssl backend calls M2Crypto `des_ede3_cbc` (openssl_tripledes.py:23).
M2Crypto is absent, so the 3DES encContext here is a `TripleDES` subclass that
calls OpenSSL 3's EVP_des_ede3_cbc through ctypes and carries the IV exactly
like openssl_tripledes.py:30-33.  Record framing still comes from tlslite.

Large plaintexts are not stored; they are regenerated from `pt_gen`
(SHA-256 counter stream, see `gen_bytes`) and the expected wire is stored as
SHA-256 + length + head/tail bytes.

Usage:  PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_golden.py
"""
import ctypes
import ctypes.util
import hashlib
import json
import os
import sys
import types

REF = "/root/reference/tlslite"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "records.json")

sys.dont_write_bytecode = True
pkg = types.ModuleType("tlslite")
pkg.__path__ = [REF]
sys.modules["tlslite"] = pkg

from tlslite.tlsrecordlayer import TLSRecordLayer, _ConnectionState  # noqa: E402
from tlslite.messages import ApplicationData  # noqa: E402
from tlslite.mathtls import createHMAC, createMAC_SSL  # noqa: E402
from tlslite.utils.cipherfactory import createAES, createRC4  # noqa: E402
from tlslite.utils.tripledes import TripleDES  # noqa: E402
from tlslite.constants import Fault, CipherSuite  # noqa: E402
from tlslite.mathtls import PRF, PRF_1_2, PRF_SSL, calcMasterSecret  # noqa: E402


def gen_bytes(seed, n):
    """Deterministic byte stream: SHA-256(seed || be32(counter)) concatenated."""
    out = bytearray()
    ctr = 0
    while len(out) < n:
        out += hashlib.sha256(seed.encode() + ctr.to_bytes(4, "big")).digest()
        ctr += 1
    return bytes(out[:n])


# ---------------------------------------------------------------- OpenSSL 3DES
_lc = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
_lc.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_lc.EVP_des_ede3_cbc.restype = ctypes.c_void_p
_lc.EVP_CipherInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
_lc.EVP_CipherUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                 ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
_lc.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lc.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]


def _evp_3des(key, iv, data, enc):
    ctx = _lc.EVP_CIPHER_CTX_new()
    assert _lc.EVP_CipherInit_ex(ctx, _lc.EVP_des_ede3_cbc(), None, bytes(key), bytes(iv), enc) == 1
    _lc.EVP_CIPHER_CTX_set_padding(ctx, 0)
    out = ctypes.create_string_buffer(len(data) + 16)
    outl = ctypes.c_int(0)
    assert _lc.EVP_CipherUpdate(ctx, out, ctypes.byref(outl), bytes(data), len(data)) == 1
    _lc.EVP_CIPHER_CTX_free(ctx)
    assert outl.value == len(data)
    return bytearray(out.raw[: outl.value])


class OpenSSL3_TripleDES(TripleDES):
    """Stand-in for tlslite/utils/openssl_tripledes.py (M2Crypto absent)."""

    def __init__(self, key, mode, IV):
        TripleDES.__init__(self, key, mode, IV, "openssl")
        self.key = bytes(key)
        self.IV = bytes(IV)

    def encrypt(self, plaintext):
        TripleDES.encrypt(self, plaintext)
        ct = _evp_3des(self.key, self.IV, plaintext, 1)
        self.IV = bytes(ct[-self.block_size:])
        return ct

    def decrypt(self, ciphertext):
        TripleDES.decrypt(self, ciphertext)
        pt = _evp_3des(self.key, self.IV, ciphertext, 0)
        self.IV = bytes(ciphertext[-self.block_size:])
        return pt


# ---------------------------------------------------------------- suites
SUITES = {
    # name: (cipher, keyLen, ivLen, mac, macLen)  -- tlsrecordlayer.py:1063-1095
    "AES128-SHA": ("aes128", 16, 16, "sha1", 20),
    "AES256-SHA": ("aes256", 32, 16, "sha1", 20),
    "AES128-SHA256": ("aes128", 16, 16, "sha256", 32),
    "AES256-SHA256": ("aes256", 32, 16, "sha256", 32),
    "RC4-SHA": ("rc4", 16, 0, "sha1", 20),
    "RC4-MD5": ("rc4", 16, 0, "md5", 16),
    "3DES-SHA": ("3des", 24, 8, "sha1", 20),
}
VERSIONS = [(3, 0), (3, 1), (3, 2), (3, 3)]
DIGEST = {"sha1": hashlib.sha1, "sha256": hashlib.sha256, "md5": hashlib.md5}


def valid(suite, ver):
    if SUITES[suite][3] == "sha256" and ver != (3, 3):
        return False  # constants.py:204-210 filterForVersion
    return True


class FakeSock:
    def __init__(self):
        self.out = bytearray()
        self.writes = []

    def close(self):
        pass

    def send(self, s):
        self.out += s
        self.writes.append(bytes(s))
        return len(s)


def make_layer(suite, ver, keys):
    cipher, kl, ivl, mac, ml = SUITES[suite]
    r = TLSRecordLayer(FakeSock())
    r.version = ver
    r.closed = False
    st = _ConnectionState()
    mk = bytes.fromhex(keys["mac_key"])
    if ver == (3, 0):
        st.macContext = createMAC_SSL(mk, digestmod=DIGEST[mac])
    else:
        st.macContext = createHMAC(mk, digestmod=DIGEST[mac])
    key = bytearray.fromhex(keys["key"])
    iv = bytearray.fromhex(keys["iv"])
    if cipher.startswith("aes"):
        st.encContext = createAES(key, iv, ["python"])
    elif cipher == "rc4":
        st.encContext = createRC4(key, iv, ["python"])
    else:
        st.encContext = OpenSSL3_TripleDES(key, 2, iv)
    st.seqnum = keys["seq"]
    r._writeState = st
    if ver >= (3, 2) and ivl:
        r.fixedIVBlock = bytearray.fromhex(keys["fixed_iv"])
    return r


def final_state(r, suite):
    st = r._writeState
    enc = st.encContext
    d = {"seqnum": st.seqnum}
    if SUITES[suite][0] == "rc4":
        d["rc4_i"] = enc.i
        d["rc4_j"] = enc.j
        d["rc4_S"] = bytes(enc.S).hex()
    else:
        d["cbc_iv"] = bytes(enc.IV).hex()
    return d


def mk_keys(tag, suite, seq=0):
    cipher, kl, ivl, mac, ml = SUITES[suite]
    return {
        "key": gen_bytes(tag + "/key", kl).hex(),
        "iv": gen_bytes(tag + "/iv", ivl).hex(),
        "mac_key": gen_bytes(tag + "/mac", ml).hex(),
        "fixed_iv": gen_bytes(tag + "/fiv", ivl).hex(),
        "seq": seq,
    }


INLINE_MAX = 2048


def pt_entry(tag, n):
    pt = gen_bytes(tag, n)
    if n <= INLINE_MAX:
        return pt, {"pt": pt.hex()}
    return pt, {"pt_gen": tag, "pt_len": n}


def wire_entry(w):
    w = bytes(w)
    if len(w) <= INLINE_MAX + 64:
        return {"wire": w.hex()}
    return {"wire_sha256": hashlib.sha256(w).hexdigest(), "wire_len": len(w),
            "wire_head": w[:48].hex(), "wire_tail": w[-48:].hex()}


def seal_records(r, pts, ctype=23, fault=None):
    """Call _sendMsg once per record; return the per-record wire bytes."""
    outs = []
    r.fault = fault
    for pt in pts:
        before = len(r.sock.out)
        msg = ApplicationData().create(bytearray(pt))
        msg.contentType = ctype
        for _ in r._sendMsg(msg, False):
            pass
        outs.append(bytes(r.sock.out[before:]))
    return outs


def main():
    cases = []
    sizes = [1, 15, 16, 17, 19, 31, 32, 47, 50, 51, 52, 55, 56, 63, 64, 65, 100, 127, 128,
             129, 255, 1000, 1434, 16384]
    # (i) single records, fresh state, per suite x version x size
    for suite in SUITES:
        for ver in VERSIONS:
            if not valid(suite, ver):
                continue
            for n in sizes:
                tag = "single/%s/%d.%d/%d" % (suite, ver[0], ver[1], n)
                keys = mk_keys(tag, suite, seq=n * 7919)
                pt, pte = pt_entry(tag + "/pt", n)
                r = make_layer(suite, ver, keys)
                outs = seal_records(r, [pt])
                cases.append({"kind": "records", "name": tag, "suite": suite,
                              "version": list(ver), **keys,
                              "records": [{**pte, "type": 23, **wire_entry(outs[0])}],
                              "final": final_state(r, suite)})
    # (ii) chained connections: several records on one state (residue/seq/RC4 carry),
    #      including an empty record (no output, no seqnum consumed: :553-556) and a
    #      non-application content type.
    chain_sizes = [5, 100, 0, 16384, 17, 3000, 64, 1]
    for suite in SUITES:
        for ver in VERSIONS:
            if not valid(suite, ver):
                continue
            tag = "chain/%s/%d.%d" % (suite, ver[0], ver[1])
            keys = mk_keys(tag, suite, seq=2 ** 40 + 5)
            r = make_layer(suite, ver, keys)
            recs = []
            pts = []
            for i, n in enumerate(chain_sizes):
                pt, pte = pt_entry("%s/pt%d" % (tag, i), n)
                pts.append(pt)
                recs.append({**pte, "type": 21 if i == 5 else 23})
            outs = []
            for pt, rc in zip(pts, recs):
                outs += seal_records(r, [pt], ctype=rc["type"])
            for rc, w in zip(recs, outs):
                rc.update(wire_entry(w))
            cases.append({"kind": "records", "name": tag, "suite": suite, "version": list(ver),
                          **keys, "records": recs, "final": final_state(r, suite)})
    # (iii) fault injection: badMAC (:585-586) / badPadding (:603-604)
    for suite in ["AES128-SHA", "AES256-SHA256", "RC4-SHA", "3DES-SHA"]:
        for ver in [(3, 1), (3, 3)]:
            if not valid(suite, ver):
                continue
            for fname, fault in [("badMAC", Fault.badMAC), ("badPadding", Fault.badPadding)]:
                tag = "fault/%s/%d.%d/%s" % (suite, ver[0], ver[1], fname)
                keys = mk_keys(tag, suite, seq=3)
                r = make_layer(suite, ver, keys)
                pts = [gen_bytes(tag + "/a", 33), gen_bytes(tag + "/b", 200)]
                outs = seal_records(r, pts, fault=fault)
                cases.append({"kind": "records", "name": tag, "suite": suite, "version": list(ver),
                              **keys, "fault": fname,
                              "records": [{"pt": p.hex(), "type": 23, **wire_entry(w)}
                                          for p, w in zip(pts, outs)],
                              "final": final_state(r, suite)})
    # (iv) write(): 16384-byte fragmentation + BEAST 1/n-1 split (:257-295, :543-550)
    for suite in ["AES128-SHA", "RC4-SHA", "3DES-SHA", "AES256-SHA"]:
        for ver in VERSIONS:
            if not valid(suite, ver):
                continue
            for n in [1, 2, 40000]:
                tag = "write/%s/%d.%d/%d" % (suite, ver[0], ver[1], n)
                keys = mk_keys(tag, suite, seq=11)
                r = make_layer(suite, ver, keys)
                data, de = pt_entry(tag + "/data", n)
                for _ in r.writeAsync(data):
                    pass
                writes = r.sock.writes
                cases.append({"kind": "write", "name": tag, "suite": suite, "version": list(ver),
                              **keys, **de,
                              "writes": [wire_entry(w) for w in writes],
                              "final": final_state(r, suite)})
    # (v) open: _decryptRecord (:958-1044) on one read state over a chain of valid,
    #     tampered and malformed bodies (empty, IV-only, not a block multiple, garbage).
    #     _sendError (:524-529) shuts the layer down after an alert; the batch API keeps
    #     going, so each body is opened on the SAME state object again (the alert only
    #     resets the layer's references, not the state the earlier records advanced).
    #     A writer with the same keys makes the valid bodies; before each one its
    #     seqnum / CBC residue / RC4 state is synced to the reader's, as a peer's would be.
    from tlslite.errors import TLSLocalAlert
    for suite in SUITES:
        for ver in VERSIONS:
            if not valid(suite, ver):
                continue
            tag = "open/%s/%d.%d" % (suite, ver[0], ver[1])
            keys = mk_keys(tag, suite, seq=77)
            w = make_layer(suite, ver, keys)
            r = make_layer(suite, ver, keys)
            rs = r._writeState  # becomes the reader's read state; alerts go out in the clear
            r._writeState = _ConnectionState()
            ws = w._writeState
            bs = 1 if SUITES[suite][0] == "rc4" else (8 if SUITES[suite][0] == "3des" else 16)
            plan = [("valid", 40), ("empty", 0), ("raw", bs), ("valid", 1), ("raw", 2 * bs + 1),
                    ("raw", 4 * bs if bs > 1 else 64), ("valid", 300), ("flip", 70), ("raw", 3),
                    ("valid", 17), ("flip", 1), ("valid", 1434)]
            bodies = []
            for i, (kind, n) in enumerate(plan):
                if kind in ("valid", "flip"):
                    ws.seqnum = rs.seqnum
                    if bs == 1:
                        ws.encContext.S = list(rs.encContext.S)
                        ws.encContext.i, ws.encContext.j = rs.encContext.i, rs.encContext.j
                    elif ver < (3, 2):
                        ws.encContext.IV = bytearray(rs.encContext.IV)
                    body = bytearray(seal_records(w, [gen_bytes("%s/pt%d" % (tag, i), n)])[0][5:])
                    if kind == "flip":
                        body[len(body) // 2] ^= 0x10
                else:
                    body = bytearray(gen_bytes("%s/raw%d" % (tag, i), n))
                entry = {"type": 23, "body": bytes(body).hex()}
                r.version, r.closed, r._readState, r._writeState = ver, False, rs, _ConnectionState()
                try:
                    out = None
                    for out in r._decryptRecord(23, bytearray(body)):
                        pass
                    entry["status"] = 0
                    entry["pt"] = bytes(out).hex()
                except TLSLocalAlert as e:
                    entry["status"] = e.description
                bodies.append(entry)
            enc = rs.encContext
            fin = {"seqnum": rs.seqnum}
            if bs == 1:
                fin.update(rc4_i=enc.i, rc4_j=enc.j, rc4_S=bytes(enc.S).hex())
            else:
                fin["cbc_iv"] = bytes(enc.IV).hex()
            cases.append({"kind": "open", "name": tag, "suite": suite, "version": list(ver), **keys,
                          "bodies": bodies, "final": fin})
    # (vi) key-block derivation as _calcPendingStates does it (tlsrecordlayer.py:1097-1126):
    #      master secret (mathtls.py:70-82) -> PRF/PRF_1_2/PRF_SSL key block -> slices
    suite_ids = {"AES128-SHA": CipherSuite.TLS_RSA_WITH_AES_128_CBC_SHA,
                 "AES256-SHA": CipherSuite.TLS_RSA_WITH_AES_256_CBC_SHA,
                 "AES128-SHA256": CipherSuite.TLS_RSA_WITH_AES_128_CBC_SHA256,
                 "RC4-SHA": CipherSuite.TLS_RSA_WITH_RC4_128_SHA,
                 "RC4-MD5": CipherSuite.TLS_RSA_WITH_RC4_128_MD5,
                 "3DES-SHA": CipherSuite.TLS_RSA_WITH_3DES_EDE_CBC_SHA}
    for suite, sid in suite_ids.items():
        for ver in VERSIONS:
            if not valid(suite, ver):
                continue
            tag = "keys/%s/%d.%d" % (suite, ver[0], ver[1])
            pms = bytearray(gen_bytes(tag + "/pms", 48))
            cr = bytearray(gen_bytes(tag + "/cr", 32))
            sr = bytearray(gen_bytes(tag + "/sr", 32))
            ms = calcMasterSecret(ver, pms, cr, sr)
            cipher, kl, ivl, mac, ml = SUITES[suite]
            n = 2 * (ml + kl + ivl)
            if ver == (3, 0):
                kb = PRF_SSL(ms, sr + cr, n)
            elif ver in ((3, 1), (3, 2)):
                kb = PRF(ms, b"key expansion", sr + cr, n)
            else:
                kb = PRF_1_2(ms, b"key expansion", sr + cr, n)
            cases.append({"kind": "keys", "name": tag, "suite": suite, "suite_id": sid, "version": list(ver),
                          "premaster": bytes(pms).hex(), "client_random": bytes(cr).hex(),
                          "server_random": bytes(sr).hex(), "master": bytes(ms).hex(), "key_block": bytes(kb).hex(),
                          "key": "", "iv": "", "mac_key": "", "fixed_iv": "", "seq": 0})
    doc = {"generator": "tests/golden/make_golden.py",
           "reference": "trevp/tlslite 0.4.9 at /root/reference (pure-Python path); "
                        "3DES cipher = OpenSSL 3 EVP_des_ede3_cbc",
           "pt_gen": "SHA-256(seed || be32(ctr)) stream, see gen_bytes()",
           "cases": cases}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)
    print("wrote %d cases to %s (%d bytes)" % (len(cases), OUT, os.path.getsize(OUT)))


if __name__ == "__main__":
    main()

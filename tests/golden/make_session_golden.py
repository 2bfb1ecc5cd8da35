#!/usr/bin/env python3
"""Golden config-1 sessions from the *reference* tlslite (run only in the build
container, where /root/reference exists; the GPU box only reads the JSON).

Output: tests/golden/sessions.json -- per session the SHA-256, length and record
lengths of the byte stream each side writes after the handshake, for the traffic
of tests/tlstest.py's Test 22 (testConnClient: random 1/10/100/1000-byte echoes,
tests/tlstest.py:66-78, TLS 1.0, aes128/aes256/rc4, :337-353) and Test 23's
b"hello"*10000 echo (:364-381), followed by the client's close_notify
(tlsrecordlayer.py:343-347).  Randoms, premaster secret and fixedIVBlock are
fixed (the reference draws them from getRandomBytes), so the streams are
deterministic; everything else is the reference's own code:
calcMasterSecret (mathtls.py:70-82), _calcPendingStates (tlsrecordlayer.py:
1061-1149), _changeWriteState/_changeReadState, writeAsync (:257-295, with the
TLS 1.0 1/n-1 BEAST split :543-550) and _sendMsg (:538-617) on a fake socket.
The handshake messages themselves are not part of the stream (out of scope).

Usage:  PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_session_golden.py
"""
import hashlib
import json
import os
import sys
import types

REF = "/root/reference/tlslite"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sessions.json")

sys.dont_write_bytecode = True
pkg = types.ModuleType("tlslite")
pkg.__path__ = [REF]
sys.modules["tlslite"] = pkg

from tlslite.tlsrecordlayer import TLSRecordLayer  # noqa: E402
from tlslite.messages import Alert  # noqa: E402
from tlslite.mathtls import calcMasterSecret  # noqa: E402
from tlslite.constants import AlertDescription, AlertLevel, CipherSuite  # noqa: E402


def gen_bytes(seed, n):
    """SHA-256(seed || be32(counter)) concatenated (the same stream as make_golden.py)."""
    out = bytearray()
    ctr = 0
    while len(out) < n:
        out += hashlib.sha256(seed.encode() + ctr.to_bytes(4, "big")).digest()
        ctr += 1
    return bytes(out[:n])


class FakeSock:
    def __init__(self):
        self.out = bytearray()
        self.records = []

    def send(self, s):
        self.out += s
        return len(s)


# (name, suite id, version): Test 22's three ciphers at TLS 1.0 and Test 23's default (TLS 1.2)
SESSIONS = [
    ("test22-aes128-tls10", CipherSuite.TLS_RSA_WITH_AES_128_CBC_SHA, (3, 1)),
    ("test22-aes256-tls10", CipherSuite.TLS_RSA_WITH_AES_256_CBC_SHA, (3, 1)),
    ("test22-rc4-tls10", CipherSuite.TLS_RSA_WITH_RC4_128_SHA, (3, 1)),
    ("test23-aes128-tls12", CipherSuite.TLS_RSA_WITH_AES_128_CBC_SHA, (3, 3)),
]


def messages(name):
    """testConnClient's echoes (random bytes of 1, 10, 100, 1000) + Test 23's 50,000 bytes."""
    return [gen_bytes("%s-msg-%d" % (name, n), n) for n in (1, 10, 100, 1000)] + [b"hello" * 10000]


def session_inputs(name):
    return {"premaster": gen_bytes(name + "-pms", 48), "client_random": gen_bytes(name + "-cr", 32),
            "server_random": gen_bytes(name + "-sr", 32), "client_fixed_iv": gen_bytes(name + "-cfiv", 16),
            "server_fixed_iv": gen_bytes(name + "-sfiv", 16)}


def side(client, suite, version, ms, inp):
    r = TLSRecordLayer(FakeSock())
    r._client = client
    r.version = version
    r.closed = False
    r._calcPendingStates(suite, ms, inp["client_random"], inp["server_random"], ["python"])
    if version >= (3, 2):
        r.fixedIVBlock = bytearray(inp["client_fixed_iv" if client else "server_fixed_iv"])
    r._changeWriteState()
    r._changeReadState()
    return r


def run(name, suite, version):
    inp = session_inputs(name)
    ms = calcMasterSecret(version, bytearray(inp["premaster"]), bytearray(inp["client_random"]),
                          bytearray(inp["server_random"]))
    c = side(True, suite, version, ms, inp)
    s = side(False, suite, version, ms, inp)
    c_lens, s_lens = [], []
    for m in messages(name):
        n0 = len(c.sock.out)
        for _ in c.writeAsync(bytearray(m)):
            pass
        c_lens.append(len(c.sock.out) - n0)
        n0 = len(s.sock.out)
        for _ in s.writeAsync(bytearray(m)):  # the server's echo
            pass
        s_lens.append(len(s.sock.out) - n0)
    n0 = len(c.sock.out)
    for _ in c._sendMsg(Alert().create(AlertDescription.close_notify, AlertLevel.warning)):
        pass
    c_lens.append(len(c.sock.out) - n0)
    return {"name": name, "suite": suite, "version": list(version), "master": bytes(ms).hex(),
            "inputs": {k: v.hex() for k, v in inp.items()},
            "client": {"sha256": hashlib.sha256(bytes(c.sock.out)).hexdigest(), "len": len(c.sock.out),
                       "write_lens": c_lens, "head": bytes(c.sock.out[:64]).hex()},
            "server": {"sha256": hashlib.sha256(bytes(s.sock.out)).hexdigest(), "len": len(s.sock.out),
                       "write_lens": s_lens, "head": bytes(s.sock.out[:64]).hex()}}


def main():
    out = {"generator": "tests/golden/make_session_golden.py", "sessions": [run(*spec) for spec in SESSIONS]}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT, len(out["sessions"]), "sessions")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Golden receive-framing cases from the *reference* tlslite (run only in the build container,
where /root/reference exists; the GPU box only reads the JSON).

Each case is one connection's received bytes, fed to the reference's
TLSRecordLayer._getNextRecord (tlsrecordlayer.py:823-956; RecordHeader3.parse,
messages.py:44-49) through a fake non-blocking socket with a null read state (no cipher, no
MAC: _decryptRecord returns the body as received).  Recorded: every record it returns
(content type, version, body length and SHA-256), the bytes consumed up to the start of the
record it stopped at, and how it stopped -- "more" (the socket would block: an incomplete
header or body), "syntax" (SyntaxError: a first header byte that is no content type,
:850-857) or "overflow" (TLSLocalAlert record_overflow, :871-873).  Content types 20, 21
and 23 only (22 would go on into handshake-message parsing, beyond the record layer's
framing), no SSLv2 headers (first byte 128, handshake-only: the device framing refuses them
as a syntax error).  Empty records are in (round 6): the reference's body loop calls
sock.recv(0), which a socket answers with b"" (the fake socket too), and raises
TLSAbruptCloseError (:877-889) -- recorded as stop "abrupt" at the empty record's header.

Output: tests/golden/frames.json (inputs as hex).
Usage:  PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_frame_golden.py
"""
import errno
import hashlib
import json
import os
import random
import socket
import sys
import types

REF = "/root/reference/tlslite"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "frames.json")

sys.dont_write_bytecode = True
pkg = types.ModuleType("tlslite")
pkg.__path__ = [REF]
sys.modules["tlslite"] = pkg

from tlslite.tlsrecordlayer import TLSRecordLayer  # noqa: E402
from tlslite.errors import TLSAbruptCloseError, TLSLocalAlert  # noqa: E402


class FakeSock:
    """recv() hands out the received bytes; past their end it would block (EWOULDBLOCK)."""

    def __init__(self, data):
        self.data, self.pos, self.sent = bytes(data), 0, bytearray()

    def recv(self, n):
        if n == 0:  # a socket's recv(0) returns b"" at once
            return b""
        if self.pos >= len(self.data):
            raise socket.error(errno.EWOULDBLOCK, "would block")
        s = self.data[self.pos:self.pos + n]
        self.pos += len(s)
        return s

    def send(self, s):
        self.sent += s
        return len(s)

    def sendall(self, s):
        self.sent += s

    def close(self):
        pass


def ref_frame(data):
    sock = FakeSock(data)
    rl = TLSRecordLayer(sock)
    recs, stop = [], None
    while stop is None:
        start = sock.pos
        try:
            got = None
            for res in rl._getNextRecord():
                if res in (0, 1):
                    stop = "more"
                    break
                got = res
                break
            if stop == "more":
                return recs, start, stop
            r, p = got
            body = bytes(p.bytes)
            recs.append({"type": r.type, "version": list(r.version), "len": len(body),
                         "sha256": hashlib.sha256(body).hexdigest()})
        except SyntaxError:
            return recs, start, "syntax"
        except TLSLocalAlert as e:
            assert e.description == 22, e  # record_overflow
            return recs, start, "overflow"
        except TLSAbruptCloseError:
            return recs, start, "abrupt"
    return recs, sock.pos, stop


def header(t, n, ver=(3, 3)):
    return bytes([t, ver[0], ver[1], n >> 8, n & 0xff])


def rec(rng, t, n, ver=(3, 3)):
    return header(t, n, ver) + bytes(rng.getrandbits(8) for _ in range(n))


def cases():
    rng = random.Random(20261018)
    out = []
    types_ = (20, 21, 23)
    # whole records of many sizes, then every kind of tail
    for n in (1, 5, 16, 100, 1434, 16384, 16389, 18432):
        out.append(("one_%d" % n, rec(rng, 23, n)))
    for k in range(12):
        data = b"".join(rec(rng, rng.choice(types_), rng.choice([1, 37, 300, 2000, 16384]),
                            rng.choice([(3, 0), (3, 1), (3, 2), (3, 3)])) for _ in range(rng.randint(1, 6)))
        tail = rng.choice(["", "hdr1", "hdr4", "body", "bad", "over", "over_partial"])
        if tail == "hdr1":
            data += bytes([23])
        elif tail == "hdr4":
            data += header(23, 50)[:4]
        elif tail == "body":
            data += rec(rng, 23, 200)[:100]
        elif tail == "bad":
            data += bytes([rng.choice([0, 19, 24, 127, 255])]) + b"junk"
        elif tail == "over":
            data += header(23, 18433) + b"x" * 10
        elif tail == "over_partial":
            data += header(21, 0xffff)
        out.append(("mix_%d_%s" % (k, tail), data))
    out.append(("empty", b""))
    out.append(("bad_first", bytes([0x16 + 2]) + b"\x03\x03\x00\x01x"))
    out.append(("bad_lone_byte", bytes([7])))
    out.append(("overflow_first", header(23, 18433)))
    out.append(("max_body_then_more", rec(rng, 23, 18432) + header(20, 1) ))
    # empty records (round 6): the connection ends at the first one
    out.append(("empty_record_first", header(23, 0) + rec(rng, 23, 10)))
    out.append(("records_then_empty", rec(rng, 23, 300) + rec(rng, 21, 2) + header(23, 0) + rec(rng, 23, 7)))
    out.append(("empty_record_last", rec(rng, 20, 1) + header(21, 0)))
    out.append(("empty_handshake_type", rec(rng, 23, 40) + header(20, 0, (3, 1))))
    return out


def main():
    res = []
    for name, data in cases():
        recs, consumed, stop = ref_frame(data)
        res.append({"name": name, "hex": data.hex(), "records": recs, "consumed": consumed, "stop": stop})
    with open(OUT, "w") as fh:
        json.dump({"source": "reference tlslite TLSRecordLayer._getNextRecord (tlsrecordlayer.py:823-956) "
                             "on a fake non-blocking socket; generated by tests/golden/make_frame_golden.py",
                   "cases": res}, fh, indent=0)
    print("%d cases -> %s" % (len(res), OUT))


if __name__ == "__main__":
    main()

"""Whole config-1 sessions pinned to the reference (tests/golden/sessions.json,
made by tests/golden/make_session_golden.py from tlslite's own writeAsync /
_sendMsg): the byte stream each side writes for Test 22's echoes
(tests/tlstest.py:66-78, :337-353: TLS 1.0, aes128/aes256/rc4, BEAST 1/n-1
split) and Test 23's 50,000-byte echo (:364-381, TLS 1.2), then the client's
close_notify.  A symmetric bug in seal and open would still round-trip in the
loopback test; comparing the wire bytes with the reference's catches it."""
import hashlib
import socket
import threading

import pytest

from tests.golden_io import load_json

_ID_TO_NAME = {0x002F: "AES128-SHA", 0x0035: "AES256-SHA", 0x0005: "RC4-SHA"}


def _sessions():
    return load_json("sessions.json")["sessions"]


def _messages(s):
    from tests.golden_io import gen_bytes
    return [gen_bytes("%s-msg-%d" % (s["name"], n), n) for n in (1, 10, 100, 1000)] + [b"hello" * 10000]


def _inputs(s):
    return {k: bytes.fromhex(v) for k, v in s["inputs"].items()}


def test_host_key_schedule_matches_sessions():
    from tlslite_amd.connection import master_secret
    for s in _sessions():
        inp = _inputs(s)
        ms = master_secret(tuple(s["version"]), inp["premaster"], inp["client_random"], inp["server_random"])
        assert ms.hex() == s["master"], s["name"]


def test_oracle_reproduces_reference_sessions():
    """The C oracle + the host write planner (plan_write) rebuild both sides' streams."""
    from oracle import oracle as O
    from tlslite_amd.recordlayer import plan_write
    for s in _sessions():
        v, suite = tuple(s["version"]), _ID_TO_NAME[s["suite"]]
        inp = _inputs(s)
        ms = bytes.fromhex(s["master"])
        _, kp = O.key_block(v, suite, ms, inp["client_random"], inp["server_random"])
        block = not suite.startswith("RC4")
        conns = {}
        for side in ("client", "server"):
            fiv = inp[side + "_fixed_iv"] if v >= (3, 2) and block else None
            conns[side] = O.Conn.for_suite(suite, v, kp[side + "_key"], kp[side + "_iv"], kp[side + "_mac"], fiv)
        streams = {"client": bytearray(), "server": bytearray()}
        lens = {"client": [], "server": []}
        for m in _messages(s):
            for side in ("client", "server"):
                n0 = len(streams[side])
                for p in plan_write(m, v, block):
                    streams[side] += conns[side].seal(p, 23)
                lens[side].append(len(streams[side]) - n0)
        n0 = len(streams["client"])
        streams["client"] += conns["client"].seal(b"\x01\x00", 21)  # close_notify, warning
        lens["client"].append(len(streams["client"]) - n0)
        for side in ("client", "server"):
            assert lens[side] == s[side]["write_lens"], (s["name"], side)
            assert hashlib.sha256(bytes(streams[side])).hexdigest() == s[side]["sha256"], (s["name"], side)


class _Tap:
    """A socket that keeps a copy of everything sent through it."""

    def __init__(self, sock):
        self.s, self.log = sock, bytearray()

    def sendall(self, b):
        self.log += b
        self.s.sendall(b)

    def recv(self, n):
        return self.s.recv(n)


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(4))
def test_gpu_session_matches_reference(idx):
    """The loopback echo with every record sealed and opened on the GPU: the client's
    and the server's wire bytes equal the reference session's, byte for byte."""
    from tlslite_amd import device
    from tlslite_amd.connection import RecordLayer, master_secret, pending_states
    if device.device_count() < 1:
        pytest.fail("no GPU visible")
    s = _sessions()[idx]
    v, suite = tuple(s["version"]), _ID_TO_NAME[s["suite"]]
    inp = _inputs(s)
    ms = master_secret(v, inp["premaster"], inp["client_random"], inp["server_random"])
    cw, crd = pending_states(v, suite, ms, inp["client_random"], inp["server_random"], client=True,
                             fixed_iv=inp["client_fixed_iv"])
    sw, srd = pending_states(v, suite, ms, inp["client_random"], inp["server_random"], client=False,
                             fixed_iv=inp["server_fixed_iv"])
    a, b = socket.socketpair()
    ta, tb = _Tap(a), _Tap(b)
    client, server = RecordLayer(ta, v, cw, crd), RecordLayer(tb, v, sw, srd)
    msgs = _messages(s)
    lens = {"client": [], "server": []}

    def serve():
        for m in msgs:
            got = server.read(min=len(m), max=len(m))
            n0 = len(tb.log)
            server.write(got)
            lens["server"].append(len(tb.log) - n0)

    t = threading.Thread(target=serve)
    t.start()
    try:
        for m in msgs:
            n0 = len(ta.log)
            client.write(m)
            lens["client"].append(len(ta.log) - n0)
            assert client.read(min=len(m), max=len(m)) == m
        n0 = len(ta.log)
        client.close()
        lens["client"].append(len(ta.log) - n0)
    finally:
        t.join(timeout=60)
        a.close()
        b.close()
    assert not t.is_alive()
    for side, tap in (("client", ta), ("server", tb)):
        assert lens[side] == s[side]["write_lens"], side
        assert bytes(tap.log[:64]).hex() == s[side]["head"], side
        assert hashlib.sha256(bytes(tap.log)).hexdigest() == s[side]["sha256"], side

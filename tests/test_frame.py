"""Receive framing (tlsrecordlayer.py:823-893, _getNextRecord's header parse; RecordHeader3.parse,
messages.py:44-49): the oracle restatement and the host parse_records against golden cases
captured from the reference (tests/golden/make_frame_golden.py -> frames.json), and the device
framing (tlsgpu_frame_dev) against both -- including what the goldens cannot hold (empty
records, which the reference cannot receive: its body loop calls recv(0), :880-889), the
max_records cut and the path from received bytes to opened plaintext on the GPU."""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "frames.json")))["cases"]


def _code(O, stop):
    return {"more": 0, "syntax": O.EFRAME, "overflow": O.ALERT_RECORD_OVERFLOW, "abrupt": O.EABRUPT}[stop]


def _random_stream(rng, nrec, tail):
    """nrec records (types 20-23, random versions, lengths 0..18432, mostly short) + a tail."""
    parts, recs = [], []
    for _ in range(nrec):
        t = int(rng.integers(20, 24))
        n = int(rng.choice([0, int(rng.integers(1, 64)), int(rng.integers(64, 2048)), int(rng.integers(2048, 18433))],
                           p=[0.1, 0.4, 0.4, 0.1]))
        body = rng.bytes(n)
        parts.append(bytes([t, 3, int(rng.integers(0, 4)), n >> 8, n & 0xff]) + body)
        recs.append((t, body))
    data = b"".join(parts)
    if tail == "hdr":
        data += bytes([23, 3, 3])[: int(rng.integers(1, 4))]
    elif tail == "body":
        data += bytes([22, 3, 3, 0, 40]) + rng.bytes(int(rng.integers(0, 40)))
    elif tail == "bad":
        data += bytes([int(rng.choice([0, 19, 24, 128, 255]))]) + rng.bytes(int(rng.integers(0, 8)))
    elif tail == "over":
        data += bytes([23, 3, 3, 0x48, int(rng.integers(1, 256))]) + rng.bytes(int(rng.integers(0, 8)))
    return data, recs


def test_oracle_frame_matches_reference_goldens():
    from oracle import oracle as O
    assert len(GOLD) >= 20
    for c in GOLD:
        data = bytes.fromhex(c["hex"])
        recs, consumed, code = O.frame(data)
        assert (consumed, code) == (c["consumed"], _code(O, c["stop"])), c["name"]
        assert [(t, list(v), len(b), hashlib.sha256(b).hexdigest()) for t, v, b in recs] == \
               [(r["type"], r["version"], r["len"], r["sha256"]) for r in c["records"]], c["name"]


def test_parse_records_matches_reference_goldens():
    from oracle import oracle as O
    from tlslite_amd.recordlayer import RecordAbruptClose, RecordOverflow, RecordSyntaxError, parse_records
    exc = {"syntax": RecordSyntaxError, "overflow": RecordOverflow, "abrupt": RecordAbruptClose}
    for c in GOLD:
        data = bytes.fromhex(c["hex"])
        if c["stop"] == "more":
            recs, rest = parse_records(data)
            assert len(recs) == len(c["records"]) and rest == data[c["consumed"]:], c["name"]
            assert [hashlib.sha256(b).hexdigest() for _, _, b in recs] == [r["sha256"] for r in c["records"]]
        else:
            with pytest.raises(exc[c["stop"]]):
                parse_records(data)
        assert O.frame(data)[2] == _code(O, c["stop"])


def _expected(O, recs, tail):
    """(records, consumed, code) the framing must give for a _random_stream: every record up
    to the first empty one, where the connection ends (TLSAbruptCloseError in the reference),
    else every record and the tail's code."""
    for i, (_, b) in enumerate(recs):
        if not b:
            return recs[:i], sum(5 + len(x) for _, x in recs[:i]), O.EABRUPT
    code = {"": 0, "hdr": 0, "body": 0, "bad": O.EFRAME, "over": O.ALERT_RECORD_OVERFLOW}[tail]
    return recs, sum(5 + len(x) for _, x in recs), code


def test_oracle_frame_random_streams_and_empty_records():
    """The oracle on streams with empty records and every kind of tail agrees with the host
    parse_records record for record; an empty record ends the connection."""
    from oracle import oracle as O
    from tlslite_amd.recordlayer import RecordAbruptClose, RecordOverflow, RecordSyntaxError, parse_records
    rng = np.random.default_rng(7)
    nabrupt = 0
    for k in range(200):
        tail = ["", "hdr", "body", "bad", "over"][k % 5]
        data, recs = _random_stream(rng, int(rng.integers(0, 6)), tail)
        got, consumed, code = O.frame(data)
        want, wcons, wcode = _expected(O, recs, tail)
        assert [(t, b) for t, _, b in got] == want and code == wcode
        assert consumed == wcons
        nabrupt += code == O.EABRUPT
        if code == 0:
            r2, rest = parse_records(data)
            assert [(t, b) for t, _, b in r2] == recs and rest == data[consumed:]
        else:
            exc = {O.EFRAME: RecordSyntaxError, O.ALERT_RECORD_OVERFLOW: RecordOverflow, O.EABRUPT: RecordAbruptClose}
            with pytest.raises(exc[code]):
                parse_records(data)
    assert nabrupt >= 10


def _check_device(O, streams, res, total, max_records=None):
    n_all = 0
    for data, (st, consumed, recs) in zip(streams, res):
        want, wcons, wcode = O.frame(data)
        room = len(want) if max_records is None else max(0, min(len(want), max_records - n_all))
        n_all += len(want) if max_records is None else room
        if room < len(want):  # cut by max_records: the first `room` records, no error seen yet
            assert st == room and recs == [(t, b) for t, _, b in want[:room]]
            assert consumed == sum(5 + len(b) for _, _, b in want[:room])
            continue
        assert recs == [(t, b) for t, _, b in want]
        assert consumed == wcons
        assert st == (wcode if wcode else len(want))
    assert total == n_all


@pytest.mark.gpu
def test_device_framing_matches_goldens():
    from oracle import oracle as O
    from tlslite_amd.recordlayer import frame_streams
    streams = [bytes.fromhex(c["hex"]) for c in GOLD]
    res, total = frame_streams(streams)
    for c, (st, consumed, recs) in zip(GOLD, res):
        code = _code(O, c["stop"])
        assert consumed == c["consumed"], c["name"]
        assert st == (code if code else len(c["records"])), c["name"]
        assert [(t, len(b), hashlib.sha256(b).hexdigest()) for t, b in recs] == \
               [(r["type"], r["len"], r["sha256"]) for r in c["records"]], c["name"]
    assert total == sum(len(c["records"]) for c in GOLD)


@pytest.mark.gpu
@pytest.mark.parametrize("cut", [None, 0.5, 0])
def test_device_framing_random_connections(cut):
    """3,000 connections of 0-7 records (empty ones included) with every kind of tail; with
    `cut`, max_records below the total: connections in order get their records until it
    runs out, the rest none."""
    from oracle import oracle as O
    from tlslite_amd.recordlayer import frame_streams
    rng = np.random.default_rng(zlib.crc32(repr(("frame", cut)).encode()))
    streams = [_random_stream(rng, int(rng.integers(0, 8)), ["", "", "hdr", "body", "bad", "over"][i % 6])[0]
               for i in range(3000)]
    full = sum(len(O.frame(d)[0]) for d in streams)
    maxr = None if cut is None else int(full * cut)
    res, total = frame_streams(streams, max_records=maxr)
    _check_device(O, streams, res, total, maxr)


@pytest.mark.gpu
def test_device_framing_refuses_spans_outside_the_arena():
    import ctypes
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, synchronize
    from tlslite_amd.recordlayer import frame_dev
    data = bytes([23, 3, 3, 0, 2]) + b"ok"
    arena = np.frombuffer(data + bytes(9), dtype=np.uint8)
    spans = (N.Span * 3)()
    for sp, (off, ln) in zip(spans, [(0, 7), (10, 7), (2 ** 40, 1)]):
        sp.off, sp.len, sp.state = off, ln, 0
    d_s, d_sp = DeviceBuffer(16), DeviceBuffer(ctypes.sizeof(spans))
    d_s.upload(arena)
    d_sp.upload(np.frombuffer(spans, dtype=np.uint8))
    d_r, d_c = DeviceBuffer(8 * ctypes.sizeof(N.OpenRecord)), DeviceBuffer(48)
    d_cons, d_st, d_tot = DeviceBuffer(12), DeviceBuffer(12), DeviceBuffer(16)
    frame_dev(d_s, d_sp, 3, d_r, 8, d_c, d_cons, d_st, d_tot)
    synchronize()
    assert list(d_st.download().view(np.int32)) == [1, N.EINVAL, N.EINVAL]
    assert list(d_cons.download().view(np.uint32)) == [7, 0, 0]
    assert int(d_tot.download()[:4].view(np.uint32)[0]) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 3)), ("3DES-SHA", (3, 1)), ("RC4-SHA", (3, 0))])
def test_received_bytes_to_plaintext_on_the_device(suite, version):
    """Received bytes -> tlsgpu_frame_dev -> tlsgpu_open_dev on the framed descriptors, with
    no host pass between: 400 connections' streams of sealed records (one tampered now and
    then, some streams ending in a partial record); every status and plaintext equals the
    oracle's reading the same bytes record by record."""
    import ctypes
    from oracle import oracle as O
    import tlslite_amd as T
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, synchronize
    from tlslite_amd.recordlayer import frame_dev, open_dev
    from tlslite_amd.state import STATE_BYTES, pack_states, unpack_states
    rng = np.random.default_rng(zlib.crc32(repr(("frame-open", suite, version)).encode()))
    cipher, kl, ivl, mac, ml = O.SUITES[suite]
    nconn = 400
    writers, readers, oreaders = [], [], []
    for _ in range(nconn):
        key, iv, mk, fiv = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml), (rng.bytes(ivl) if ivl else None)
        seq = int(rng.integers(0, 2 ** 40))
        writers.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        readers.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        oreaders.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
    plan = [(ci, rng.bytes(int(rng.integers(1, 3000)))) for ci in range(nconn) for _ in range(int(rng.integers(0, 4)))]
    wires = T.seal(writers, plan)
    streams = [bytearray() for _ in range(nconn)]
    for (ci, _), w in zip(plan, wires):
        w = bytearray(w)
        if rng.random() < 0.03:
            w[5 + int(rng.integers(0, len(w) - 5))] ^= 0x40
        streams[ci] += w
    for ci in range(0, nconn, 7):  # a partial record at the end of some streams
        streams[ci] += bytes([23, 3, version[1], 0, 64]) + b"\0" * 10
    offs, pos = [], 0
    for b in streams:
        offs.append(pos)
        pos += len(b) + (-len(b)) % 16
    arena = np.zeros(max(pos, 16), dtype=np.uint8)
    for o, b in zip(offs, streams):
        arena[o:o + len(b)] = np.frombuffer(bytes(b), dtype=np.uint8)
    spans = (N.Span * nconn)()
    for i, sp in enumerate(spans):
        sp.off, sp.len, sp.state = offs[i], len(streams[i]), i
    maxr = len(plan) + 8
    d_s, d_pt = DeviceBuffer(arena.nbytes), DeviceBuffer(arena.nbytes)
    d_sp = DeviceBuffer(ctypes.sizeof(spans))
    d_s.upload(arena)
    d_sp.upload(np.frombuffer(spans, dtype=np.uint8))
    d_r, d_c = DeviceBuffer(maxr * ctypes.sizeof(N.OpenRecord)), DeviceBuffer(16 * nconn)
    d_cons, d_fst, d_tot = DeviceBuffer(4 * nconn), DeviceBuffer(4 * nconn), DeviceBuffer(16)
    d_states, d_ost = DeviceBuffer(STATE_BYTES * nconn), DeviceBuffer(4 * maxr)
    d_states.upload(pack_states(readers))
    d_pt.zero()
    frame_dev(d_s, d_sp, nconn, d_r, maxr, d_c, d_cons, d_fst, d_tot)
    open_dev(d_c, nconn, d_r, maxr, d_s, d_pt, d_states, d_ost, readers[0].variant)
    synchronize()
    fst = d_fst.download().view(np.int32)
    ch = d_c.download().view(np.uint32).reshape(nconn, 4)
    recs = np.frombuffer(d_r.download(), dtype=np.uint8).reshape(-1, ctypes.sizeof(N.OpenRecord))
    ost = d_ost.download().view(np.int32)
    pt = d_pt.download()
    unpack_states(d_states.download(), readers)
    amap = {0: 0, O.ALERT_BAD_RECORD_MAC: N.ALERT_BAD_RECORD_MAC, O.ALERT_DECRYPTION_FAILED: N.ALERT_DECRYPTION_FAILED}
    for ci in range(nconn):
        want, _, code = O.frame(bytes(streams[ci]))
        assert code == 0 and fst[ci] == len(want) and ch[ci, 2] == len(want)
        stopped = False
        for k, (t, _, body) in enumerate(want):
            r = recs[ch[ci, 1] + k]
            st = int(ost[ch[ci, 1] + k])
            if stopped:
                assert st == N.ALERT_SKIPPED
                continue
            ocode, opt = oreaders[ci].open(body, t)
            if ocode == 0:  # status = the payload length
                assert st == len(opt), (ci, k)
                off = int(r[8:16].view(np.uint64)[0])
                assert pt[off:off + st].tobytes() == opt
            else:
                assert st == amap[ocode], (ci, k)
                stopped = True
        assert readers[ci].seqnum == oreaders[ci].seqnum

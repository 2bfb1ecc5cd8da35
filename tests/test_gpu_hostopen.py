"""The receive path from host socket buffers (tlsgpu_host_pipeline_open, ABI 7): connections'
received bytes in HOST memory -> H2D per sub-batch -> framing on the device -> open on the
device -> D2H of plaintext, descriptors and statuses -- against the CPU oracle reading the same
bytes as the reference's _getNextRecord / _decryptRecord would (tlsrecordlayer.py:832-893,
:958-1044): each connection's records framed by oracle.frame (stopping at a partial record,
a bad type byte, an overflowing header or an empty record), then opened one after another by
an oracle read state, the connection stopping at its first alert (TLSGPU_CHAIN_STOP_ON_ALERT:
later records ALERT_SKIPPED).  Pinned and pageable host arenas, one to three sub-batches in
flight, sub-batches of a few KiB to the whole call, and a max_records cut.  Test
infrastructure: the oracle checks, the HIP path runs."""
import ctypes
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _T():
    import tlslite_amd as T
    from tlslite_amd import device
    if device.device_count() < 1:
        pytest.fail("no GPU visible to libtlsgpu (the gpu tests need an MI355X)")
    return T


def _streams(T, O, suite, version, nconn, rng):
    """nconn connections' received bytes: 0-4 sealed records each (3 % tampered), and now and
    then a partial record, a bad type byte, an overflowing header or an empty record last."""
    cipher, kl, ivl, mac, ml = O.SUITES[suite]
    writers, readers, oreaders = [], [], []
    for _ in range(nconn):
        key, iv, mk, fiv = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml), (rng.bytes(ivl) if ivl else None)
        seq = int(rng.integers(0, 2 ** 40))
        writers.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        readers.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        oreaders.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
    plan = [(ci, rng.bytes(int(rng.choice([1, 17, 300, 1434, 4000, 16384]))))
            for ci in range(nconn) for _ in range(int(rng.integers(0, 5)))]
    wires = T.seal(writers, plan)
    streams = [bytearray() for _ in range(nconn)]
    for (ci, _), w in zip(plan, wires):
        w = bytearray(w)
        if rng.random() < 0.03:
            w[5 + int(rng.integers(0, len(w) - 5))] ^= 0x10
        streams[ci] += w
    for ci in range(nconn):
        u = rng.random()
        if u < 0.08:
            streams[ci] += bytes([23, 3, version[1], 0, 64]) + b"\0" * int(rng.integers(0, 60))
        elif u < 0.11:
            streams[ci] += bytes([int(rng.choice([0, 19, 24, 128]))]) + b"junk"
        elif u < 0.13:
            streams[ci] += bytes([23, 3, version[1], 0x48, 1]) + b"\0" * 8
        elif u < 0.15:
            streams[ci] += bytes([23, 3, version[1], 0, 0]) + bytes(wires[0][:40])
    return readers, oreaders, [bytes(b) for b in streams]


def _arena(streams, rng, pinned):
    """Every connection's bytes at a 1-byte-granular offset with gaps between them."""
    from tlslite_amd.device import PinnedBuffer
    offs, pos = [], 0
    for b in streams:
        pos += int(rng.integers(0, 40))
        offs.append(pos)
        pos += len(b)
    nbytes = max(pos + 64, 64)
    keep = []
    if pinned:
        rxb, ptb = PinnedBuffer(nbytes), PinnedBuffer(nbytes)
        rx, pt = rxb.array[:nbytes], ptb.array[:nbytes]
        keep = [rxb, ptb]
    else:
        rx, pt = np.zeros(nbytes, dtype=np.uint8), np.zeros(nbytes, dtype=np.uint8)
    rx[:] = 0
    pt[:] = 0xEE  # bytes the call must overwrite (inside the received ranges) or leave alone
    for o, b in zip(offs, streams):
        if b:
            rx[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return rx, pt, offs, keep


def _expect(O, streams, oreaders, max_records):
    """Per connection (frame status, consumed, [(content type, body offset in the stream,
    body length, open status, plaintext)]), as one framing over every connection in order
    with max_records records at most, then the oracle's open with stop-on-alert."""
    out, left = [], max_records
    for ci, data in enumerate(streams):
        recs, consumed, code = O.frame(data)
        if len(recs) > left:  # cut: the first `left` records, no error seen yet
            recs = recs[:left]
            consumed, code = sum(5 + len(b) for _, _, b in recs), None
        left -= len(recs)
        rows, pos, stopped = [], 0, False
        for t, _, body in recs:
            if stopped:
                rows.append((t, pos + 5, len(body), O.ALERT_SKIPPED if hasattr(O, "ALERT_SKIPPED") else -22, None))
            else:
                c, p = oreaders[ci].open(body, t)
                rows.append((t, pos + 5, len(body), len(p) if c == 0 else c, p))
                stopped = c != 0
            pos += 5 + len(body)
        st = len(recs) if code in (None, 0) else code
        out.append((st, consumed, rows))
    return out


@pytest.mark.parametrize("suite,version,pinned,depth,chunk,cut", [
    ("AES128-SHA", (3, 3), True, 3, 64 << 10, None),
    ("AES128-SHA", (3, 3), False, 3, 64 << 10, None),
    ("AES256-SHA256", (3, 3), True, 2, 16 << 10, 0.6),
    ("AES128-SHA", (3, 1), False, 1, 48 << 10, None),
    ("3DES-SHA", (3, 2), True, 3, 32 << 10, None),
    ("3DES-SHA", (3, 0), False, 2, 1 << 30, 0.5),
    ("RC4-SHA", (3, 1), True, 3, 24 << 10, None),
    ("RC4-MD5", (3, 0), False, 3, 64 << 10, 0.3),
])
@pytest.mark.parametrize("d2h", ["engine", "stores"])
def test_host_pipeline_open_vs_oracle(suite, version, pinned, depth, chunk, cut, d2h, monkeypatch):
    from oracle import oracle as O
    T = _T()
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer
    from tlslite_amd.recordlayer import HostSealPipeline
    from tlslite_amd.state import pack_states, unpack_states
    rng = np.random.default_rng(zlib.crc32(repr(("hostopen", suite, version, pinned, depth, chunk, cut)).encode()))
    nconn = 500
    readers, oreaders, streams = _streams(T, O, suite, version, nconn, rng)
    rx, pt, offs, keep = _arena(streams, rng, pinned)
    full = sum(len(O.frame(d)[0]) for d in streams)
    maxr = full + 3 if cut is None else int(full * cut)
    spans = (N.Span * nconn)()
    for i, sp in enumerate(spans):
        sp.off, sp.len, sp.state = offs[i], len(streams[i]), i
    d_states = DeviceBuffer(pack_states(readers).size)
    d_states.upload(pack_states(readers))
    want = _expect(O, streams, oreaders, maxr)
    monkeypatch.setenv("TLSGPU_HOST_D2H", "kernel" if d2h == "stores" else "engine")
    with HostSealPipeline(chunk, depth) as hp:
        res = hp.open(rx, spans, pt, d_states, readers[0].variant, max_records=maxr)
        assert hp.d2h_path == d2h
    assert res["total"] == sum(len(w[2]) for w in want) <= maxr
    recs = np.frombuffer(res["records"], dtype=np.uint8).reshape(-1, 24)
    ch = np.frombuffer(res["chains"], dtype=np.uint32).reshape(nconn, 4)
    amap = {0: 0, O.ALERT_BAD_RECORD_MAC: N.ALERT_BAD_RECORD_MAC,
            O.ALERT_DECRYPTION_FAILED: N.ALERT_DECRYPTION_FAILED, -22: N.ALERT_SKIPPED}
    covered = np.zeros(pt.size, dtype=bool)
    for ci, (fst, consumed, rows) in enumerate(want):
        assert int(res["frame_status"][ci]) == fst, (ci, int(res["frame_status"][ci]), fst)
        assert int(res["consumed"][ci]) == consumed, ci
        assert int(ch[ci, 0]) == ci and int(ch[ci, 2]) == len(rows), ci
        for k, (t, boff, blen, st, p) in enumerate(rows):
            r = int(ch[ci, 1]) + k
            ct_off = int(recs[r, 0:8].view(np.uint64)[0])
            assert ct_off == offs[ci] + boff and int(recs[r, 16:20].view(np.uint32)[0]) == blen, (ci, k)
            assert int(recs[r, 20]) == t
            got = int(res["status"][r])
            assert got == (st if st >= 0 else amap[st]), (ci, k, got, st)
            if st >= 0:
                assert pt[ct_off:ct_off + st].tobytes() == p, (ci, k)
                covered[ct_off:ct_off + st] = True
    # bytes outside every connection's received range are the caller's, untouched
    inside = np.zeros(pt.size, dtype=bool)
    for o, b in zip(offs, streams):
        inside[o:o + len(b)] = True
    if not inside.all():
        assert (pt[~inside & (np.arange(pt.size) < offs[0])] == 0xEE).all()
    unpack_states(d_states.download(), readers)
    for r, o in zip(readers, oreaders):
        assert r.seqnum == o.seqnum
        assert (r.rc4 == o.rc4) if O.SUITES[suite][0] == "rc4" else (r.iv == o.iv)
    for b in keep:
        b.free()


def test_host_store_copies_exactly():
    """tlsgpu_host_store (a D2H copy by the GPU's own stores, the host pipelines' other D2H path):
    every byte of ranges with ragged heads and tails lands, nothing around them is written, a
    destination that is not pinned or differs mod 16, or a source that is not device memory, is
    refused; and a fresh pipeline's first
    call chooses a path (calibration) without changing its results."""
    _T()
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, PinnedBuffer, Stream
    rng = np.random.default_rng(7)
    n = (3 << 20) + 77
    src = rng.integers(0, 256, n, dtype=np.uint8)
    d = DeviceBuffer(n)
    d.upload(src)
    h = PinnedBuffer(n)
    s = Stream()
    for off, ln in [(0, n), (1, 15), (5, 16), (11, 4096 + 3), (16, 1 << 20), (7, 0), (13, 2), (3, (2 << 20) + 1)]:
        h.array[:n] = 0xEE
        N.call("tlsgpu_host_store", h.ptr.value + off, d.addr + off, ln, s.handle)
        s.synchronize()
        got = h.array[:n]
        assert np.array_equal(got[off:off + ln], src[off:off + ln]), (off, ln)
        assert (got[:off] == 0xEE).all() and (got[off + ln:] == 0xEE).all(), (off, ln)
    with pytest.raises(N.TLSGPUError):
        N.call("tlsgpu_host_store", h.ptr.value + 1, d.addr, 64, s.handle)  # differ mod 16
    pageable = np.zeros(64, dtype=np.uint8)
    with pytest.raises(N.TLSGPUError):
        N.call("tlsgpu_host_store", pageable.ctypes.data, d.addr, 64, s.handle)
    with pytest.raises(N.TLSGPUError):  # the source must be device memory
        N.call("tlsgpu_host_store", h.ptr.value, h.ptr.value + 4096, 64, s.handle)
    d.free()
    h.free()


def test_host_pipeline_chooses_d2h_path(monkeypatch):
    """Without TLSGPU_HOST_D2H a pipeline has no D2H path until its first call, which times the
    copy engine against the device stores (32 MiB each) and keeps one; the call's results are
    the oracle's whichever it keeps."""
    from oracle import oracle as O
    T = _T()
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer
    from tlslite_amd.recordlayer import HostSealPipeline
    from tlslite_amd.state import pack_states
    monkeypatch.delenv("TLSGPU_HOST_D2H", raising=False)
    rng = np.random.default_rng(99)
    nconn = 64
    readers, oreaders, streams = _streams(T, O, "AES128-SHA", (3, 3), nconn, rng)
    rx, pt, offs, keep = _arena(streams, rng, True)
    spans = (N.Span * nconn)()
    for i, sp in enumerate(spans):
        sp.off, sp.len, sp.state = offs[i], len(streams[i]), i
    d_states = DeviceBuffer(pack_states(readers).size)
    d_states.upload(pack_states(readers))
    full = sum(len(O.frame(d)[0]) for d in streams)
    want = _expect(O, streams, oreaders, full + 3)
    with HostSealPipeline(16 << 10, 3) as hp:
        assert hp.d2h_path is None
        res = hp.open(rx, spans, pt, d_states, readers[0].variant, max_records=full + 3)
        assert hp.d2h_path in ("engine", "stores")
    ch = np.frombuffer(res["chains"], dtype=np.uint32).reshape(nconn, 4)
    recs = np.frombuffer(res["records"], dtype=np.uint8).reshape(-1, 24)
    for ci, (fst, consumed, rows) in enumerate(want):
        assert int(res["frame_status"][ci]) == fst
        for k, (t, boff, blen, st, p) in enumerate(rows):
            r = int(ch[ci, 1]) + k
            if st >= 0:
                ct_off = int(recs[r, 0:8].view(np.uint64)[0])
                assert pt[ct_off:ct_off + st].tobytes() == p, (ci, k)

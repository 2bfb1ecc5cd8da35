"""Degenerate sizes through the C-ABI on the GPU -- what the reference's record layer meets as
an empty write (tlsrecordlayer.py:257-295 sends no record) and an empty receive buffer
(:832-893 waits for more bytes):
  * every batch entry point called with no chains / records / spans / connections returns
    TLSGPU_OK and writes nothing, except tlsgpu_frame_dev's `total` and
    tlsgpu_host_pipeline_open's *total_host, which read 0 (nothing framed);
  * chains without records between chains with records: the seal and the open leave the empty
    chains' states byte-for-byte as they were and give the other chain what the CPU oracle
    gives (_sendMsg :538-617, _decryptRecord :958-1044)."""
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


def test_zero_sized_calls():
    T = _T()
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, Stream, synchronize
    from tlslite_amd.recordlayer import HostSealPipeline, SealPipeline
    st = T.ConnectionState.for_suite("AES128-SHA", (3, 3), bytes(16), bytes(16), bytes(20), bytes(16), 0)
    var = st.variant
    s = Stream()
    canary = DeviceBuffer(256)
    canary.upload(np.full(256, 0xA5, dtype=np.uint8))
    synchronize()
    c = canary.ptr
    # device batch calls: no chains (with and without arenas behind the pointers)
    N.call("tlsgpu_seal_dev", c, 0, c, 0, c, 256, c, 256, c, 0, c, var, None, 0, s.handle)
    N.call("tlsgpu_seal_dev", None, 0, None, 0, None, 0, None, 0, None, 0, None, var, None, 0, s.handle)
    N.call("tlsgpu_open_dev", c, 0, c, 0, c, 256, c, 256, c, 0, c, var, None, 0, s.handle)
    N.call("tlsgpu_open_dev", None, 0, None, 0, None, 0, None, 0, None, 0, None, var, None, 0, s.handle)
    N.call("tlsgpu_cipher_dev", None, 0, None, None, None, N.CIPHER_AES128, 0, s.handle)
    N.call("tlsgpu_cipher_dev", None, 0, None, None, None, N.CIPHER_AES128, 1, s.handle)
    N.call("tlsgpu_derive_states_dev", None, 0, None, None, None, None, None, s.handle)
    N.call("tlsgpu_fill_pattern", c, 0, 7, 0, s.handle)
    # framing of no connections: total = 0, nothing else written
    tot = DeviceBuffer(16)
    tot.upload(np.full(16, 0xFF, dtype=np.uint8))
    N.call("tlsgpu_frame_dev", c, 256, None, 0, None, 0, None, 0, None, None, tot.ptr, None, 0, s.handle)
    s.synchronize()
    t = tot.download()
    assert int(t[:4].view(np.uint32)[0]) == 0 and (t[4:] == 0xFF).all()
    # seal pipeline and host pipelines
    with SealPipeline(16) as p:
        p.seal(canary, 0, canary, 0, canary, canary, canary, canary, var, nstates=0)
        p.synchronize()
    with HostSealPipeline(1 << 20, 2) as hp:
        N.call("tlsgpu_host_pipeline_seal", hp.handle, None, 0, None, 0, None, 0, None, 0, None, 0, None, var)
        empty = np.zeros(0, dtype=np.uint8)
        r = hp.open(empty, (N.Span * 0)(), empty, canary, var, max_records=0, nstates=0)
        assert r["total"] == 0 and len(r["status"]) == 0
    synchronize()
    assert (canary.download() == 0xA5).all(), "a zero-sized call wrote device memory"
    for b in (canary, tot):
        b.free()


@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 3)), ("AES256-SHA256", (3, 3)), ("AES256-SHA", (3, 1)),
                                           ("3DES-SHA", (3, 2)),
                                           ("RC4-SHA", (3, 1)), ("RC4-MD5", (3, 0))])
def test_chains_without_records(suite, version):
    from oracle import oracle as O
    T = _T()
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, Stream
    from tlslite_amd.recordlayer import make_chains, make_open_records, make_records, open_dev, seal_dev, wire_offsets
    from tlslite_amd.state import STATE_BYTES, pack_states, unpack_states
    rng = np.random.default_rng(zlib.crc32(repr(("degenerate", suite, version)).encode()))
    _, kl, ivl, _, ml = O.SUITES[suite]
    states, ocs = [], []
    for _ in range(5):
        key, iv, mk = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml)
        fiv = rng.bytes(ivl) if ivl else None
        seq = int(rng.integers(0, 2 ** 40))
        states.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        ocs.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
    readers = [o.copy() for o in ocs]  # the peer's read side of every connection
    payloads = [rng.bytes(100), rng.bytes(3000), rng.bytes(16)]  # connection 1 (two) and 3 (one)
    owner = [1, 1, 3]
    # chains: state 0 empty, 1 two records, 2 empty, 3 one record, 4 empty (the last one's first
    # index is nrecords: an empty chain may start at the end of the descriptor array)
    chains = make_chains([0, 1, 2, 3, 4], [0, 0, 2, 2, 3], [0, 2, 0, 1, 0])
    pt_off, pos = [], 0
    for p in payloads:
        pt_off.append(pos)
        pos += len(p) + (-len(p)) % 16
    pt_host = np.zeros(pos, dtype=np.uint8)
    for o, p in zip(pt_off, payloads):
        pt_host[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    wl = [states[c].wire_len(len(p)) for c, p in zip(owner, payloads)]
    wire_off, wire_bytes = wire_offsets(wl)
    recs = make_records(pt_off, wire_off, [len(p) for p in payloads], 23, 0)
    s = Stream()
    st0 = pack_states(states)
    d_states, d_ostates = DeviceBuffer(st0.size), DeviceBuffer(st0.size)
    d_states.upload(st0, stream=s)
    d_ostates.upload(st0, stream=s)
    d_pt, d_wire, d_len = DeviceBuffer(pt_host.size), DeviceBuffer(wire_bytes), DeviceBuffer(4 * len(payloads))
    d_pt.upload(pt_host, stream=s)
    d_wire.zero(s)
    d_recs, d_ch = DeviceBuffer(24 * len(payloads)), DeviceBuffer(16 * 5)
    d_recs.upload(np.frombuffer(recs, dtype=np.uint8), stream=s)
    d_ch.upload(np.frombuffer(chains, dtype=np.uint8), stream=s)
    var = states[0].variant
    seal_dev(d_ch, 5, d_recs, len(payloads), d_pt, d_wire, d_states, d_len, var, stream=s)
    s.synchronize()
    lens = d_len.download().view(np.int32)
    wire = d_wire.download()
    expect = np.zeros(wire_bytes, dtype=np.uint8)
    for k, (c, p) in enumerate(zip(owner, payloads)):
        w = ocs[c].seal(p, 23)
        assert int(lens[k]) == len(w) == wl[k]
        expect[int(wire_off[k]):int(wire_off[k]) + len(w)] = np.frombuffer(w, dtype=np.uint8)
    assert np.array_equal(wire, expect)
    st1 = d_states.download()
    for c in (0, 2, 4):  # the empty chains' states: untouched, byte for byte
        assert np.array_equal(st1[c * STATE_BYTES:(c + 1) * STATE_BYTES], st0[c * STATE_BYTES:(c + 1) * STATE_BYTES])
    got = [x.copy() for x in states]
    unpack_states(st1, got)
    for c in (1, 3):
        assert got[c].seqnum == ocs[c].seqnum
        if suite.startswith("RC4"):
            assert (bytes(got[c].rc4[0]),) + tuple(got[c].rc4[1:]) == (bytes(ocs[c].rc4[0]),) + tuple(ocs[c].rc4[1:])
        else:
            assert got[c].iv == ocs[c].iv
    # open the sealed records with the same chain shape on copies of the initial states
    orecs = make_open_records([int(o) + 5 for o in wire_off], [int(o) + 5 for o in wire_off],
                              [w - 5 for w in wl], 23)
    ochains = make_chains([0, 1, 2, 3, 4], [0, 0, 2, 2, 3], [0, 2, 0, 1, 0], N.CHAIN_STOP_ON_ALERT)
    d_orecs, d_och = DeviceBuffer(24 * len(payloads)), DeviceBuffer(16 * 5)
    d_orecs.upload(np.frombuffer(orecs, dtype=np.uint8), stream=s)
    d_och.upload(np.frombuffer(ochains, dtype=np.uint8), stream=s)
    d_opt, d_ost = DeviceBuffer(wire_bytes), DeviceBuffer(4 * len(payloads))
    d_opt.zero(s)
    open_dev(d_och, 5, d_orecs, len(payloads), d_wire, d_opt, d_ostates, d_ost, var, stream=s)
    s.synchronize()
    status = d_ost.download().view(np.int32)
    opened = d_opt.download()
    for k, (c, p) in enumerate(zip(owner, payloads)):
        body = wire[int(wire_off[k]) + 5:int(wire_off[k]) + wl[k]].tobytes()
        rs, rp = readers[c].open(body, 23)
        assert rs == 0 and rp == p
        assert int(status[k]) == len(p), (k, int(status[k]))
        o = int(wire_off[k]) + 5
        assert opened[o:o + len(p)].tobytes() == p
    so = d_ostates.download()
    for c in (0, 2, 4):
        assert np.array_equal(so[c * STATE_BYTES:(c + 1) * STATE_BYTES], st0[c * STATE_BYTES:(c + 1) * STATE_BYTES])
    gr = [x.copy() for x in states]
    unpack_states(so, gr)
    for c in (1, 3):
        assert gr[c].seqnum == readers[c].seqnum
        if suite.startswith("RC4"):
            assert bytes(gr[c].rc4[0]) == bytes(readers[c].rc4[0])
        else:
            assert gr[c].iv == readers[c].iv
    for b in (d_states, d_ostates, d_pt, d_wire, d_len, d_recs, d_ch, d_orecs, d_och, d_opt, d_ost):
        b.free()

"""GPU parity: the HIP seal path (libtlsgpu.so via the C ABI) against the
reference golden vectors and the CPU oracle.  Bit-exact required."""
import zlib

import numpy as np
import pytest

from tests.golden_io import case_data, case_keys, rec_pt, wire_matches

pytestmark = pytest.mark.gpu

FAULTS = {None: 0, "badMAC": 1, "badPadding": 2}


def _T():
    import tlslite_amd as T
    from tlslite_amd import device
    if device.device_count() < 1:
        pytest.fail("no GPU visible to libtlsgpu (the gpu tests need an MI355X)")
    return T


def _state(T, case):
    key, iv, mk, fiv, seq = case_keys(case)
    return T.ConnectionState.for_suite(case["suite"], tuple(case["version"]), key, iv, mk, fiv, seq)


def _check_final(st, case):
    f = case["final"]
    assert st.seqnum == f["seqnum"], case["name"]
    if "cbc_iv" in f:
        assert st.iv.hex() == f["cbc_iv"], case["name"]
    else:
        S, i, j = st.rc4
        assert (S.hex(), i, j) == (f["rc4_S"], f["rc4_i"], f["rc4_j"]), case["name"]


def test_golden_records_one_batch(golden):
    """Every golden record case, all in one multi-variant batch (one chain per case)."""
    T = _T()
    cases = [c for c in golden if c["kind"] == "records"]
    states = [_state(T, c) for c in cases]
    recs, where = [], []
    for ci, c in enumerate(cases):
        for ri, r in enumerate(c["records"]):
            recs.append((ci, rec_pt(r), r["type"], FAULTS[c.get("fault")]))
            where.append((ci, ri))
    out = T.seal(states, recs)
    bad = [cases[ci]["name"] for (ci, ri), w in zip(where, out) if not wire_matches(cases[ci]["records"][ri], w)]
    assert not bad, "mismatching cases: %s" % bad[:10]
    for st, c in zip(states, cases):
        _check_final(st, c)


def test_golden_write_beast_split(golden):
    T = _T()
    for c in golden:
        if c["kind"] != "write":
            continue
        st = _state(T, c)
        out = T.seal_write(st, case_data(c))
        assert len(out) == len(c["writes"]), c["name"]
        for w, e in zip(out, c["writes"]):
            assert wire_matches(e, w), c["name"]
        _check_final(st, c)


def test_state_carries_across_batches(golden):
    """Sealing a chain record-by-record in separate launches == one launch."""
    T = _T()
    c = [x for x in golden if x["name"] == "chain/AES128-SHA/3.3"][0]
    st = _state(T, c)
    for r in c["records"]:
        (w,) = T.seal([st], [(0, rec_pt(r), r["type"])])
        assert wire_matches(r, w)
    _check_final(st, c)


@pytest.mark.parametrize("suite,version", [(s, v) for v in [(3, 0), (3, 1), (3, 2), (3, 3)]
                                           for s in ["AES128-SHA", "AES256-SHA256", "RC4-SHA", "3DES-SHA", "RC4-MD5"]
                                           if not (s.endswith("SHA256") and v != (3, 3))])  # SHA256: TLS 1.2 only
def test_random_lengths_vs_oracle(suite, version):
    from oracle import oracle as O
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr((suite, version)).encode()))
    cipher, kl, ivl, mac, ml = O.SUITES[suite]
    nconn = 40
    states, ocs, recs = [], [], []
    for ci in range(nconn):
        key, iv, mk, fiv = (rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml), rng.bytes(ivl) if ivl else None)
        seq = int(rng.integers(0, 2 ** 48))
        states.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        ocs.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
        for _ in range(int(rng.integers(1, 4))):
            n = int(rng.choice([0, 1, 13, 16, 51, 52, 63, 64, 65, 200, 1433, 4095, 16384]))
            recs.append((ci, rng.bytes(n), int(rng.choice([21, 22, 23])), int(rng.integers(0, 4))))
    out = T.seal(states, recs)
    for (ci, p, ct, fl), w in zip(recs, out):
        assert w == ocs[ci].seal(p, ct, fl), (suite, version, len(p), fl)


def _mixed_workload(n, pt_len, seed, suites=("AES128-SHA", "RC4-SHA")):
    """Two suites, 3 chained records per connection, records of both suites
    interleaved in the arenas (seeded shuffle)."""
    from tlslite_amd import workloads as W
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    h = n // 2
    groups = []
    for suite, nconn, version in ((suites[0], h, (3, 3)), (suites[1], n - h, (3, 1))):
        _, kl, ivl, _, ml = O.SUITES[suite]
        key, mk = rng.bytes(kl), rng.bytes(ml)
        fiv = [rng.bytes(ivl)] if ivl else None
        ivs = np.frombuffer(rng.bytes(ivl * nconn), dtype=np.uint8).reshape(nconn, ivl) if ivl else None
        groups.append(W.Group(suite, version, [key], ivs, [mk], fiv, np.arange(nconn, dtype=np.uint64), 3, pt_len))
    return W.Workload("mixed", groups, seed, rec_order=rng.permutation(3 * n))


@pytest.mark.parametrize("kind", ["cfg2", "mixed", "3des", "rc4_3des", "many"])
def test_pipeline_equals_sequential(kind):
    """tlsgpu_pipeline_seal: K successive batches (MAC phase of batch k+1
    overlapping the cipher phase of batch k) give the same wire bytes and final
    connection states as K sequential tlsgpu_seal_dev calls -- for AES, the
    3DES split path (prefix / MAC / tdes4_kernel), RC4 + 3DES mixes, and AES
    batches with more chains than one cipher-workgroup generation per CU (the
    throughput layout, tlsgpu_seal_cipher_kernel)."""
    _T()
    from tlslite_amd import workloads as W
    from tlslite_amd.device import DeviceBuffer, Stream
    from tlslite_amd.recordlayer import SealPipeline
    if kind == "cfg2":
        wl = W.cfg2(n=700, pt_len=5003, seed=11)
    elif kind == "mixed":
        wl = _mixed_workload(300, 2000, 12)
    elif kind == "3des":
        wl = _mixed_workload(300, 2003, 13, ("3DES-SHA", "3DES-SHA"))
    elif kind == "rc4_3des":
        wl = _mixed_workload(300, 1999, 14, ("3DES-SHA", "RC4-SHA"))
    else:
        wl = W.cfg3(n=_many_chains() + 1000, pt_len=300, seed=15)
    wl.to_device()
    K = 4
    s = Stream()

    def run(pipelined):
        wl.reset_states(s)
        s.synchronize()
        wires = [DeviceBuffer(wl.d_wire.nbytes) for _ in range(K)]
        lens = [DeviceBuffer(wl.d_len.nbytes) for _ in range(K)]
        for b in wires + lens:
            b.zero(s)
        s.synchronize()  # pipeline streams do not order after other streams: inputs ready first
        if pipelined:
            pipe = SealPipeline(wl.n_records)
            for k in range(K):
                for var, d_ch, nch in wl.launches:
                    pipe.seal(d_ch, nch, wl.d_recs, wl.n_records, wl.d_pt, wires[k], wl.d_states, lens[k], var)
            pipe.synchronize()
            pipe.close()
        else:
            from tlslite_amd.recordlayer import seal_dev
            for k in range(K):
                for var, d_ch, nch in wl.launches:
                    seal_dev(d_ch, nch, wl.d_recs, wl.n_records, wl.d_pt, wires[k], wl.d_states, lens[k], var,
                             stream=s)
            s.synchronize()
        out = ([(w.download().tobytes(), l.download().tobytes()) for w, l in zip(wires, lens)],
               wl.d_states.download().tobytes())
        for b in wires + lens:
            b.free()
        return out

    seq_out, seq_states = run(False)
    pipe_out, pipe_states = run(True)
    for k in range(K):
        assert pipe_out[k][1] == seq_out[k][1], k
        assert pipe_out[k][0] == seq_out[k][0], k
    assert pipe_states == seq_states
    # successive batches really chain: a later batch differs from the first
    assert seq_out[1][0] != seq_out[0][0]
    # and the first batch is the oracle's
    from tests.wl_oracle import oracle_seal
    wl.reset_states(s)
    s.synchronize()
    wire, lens, _ = oracle_seal(wl)
    assert np.frombuffer(seq_out[0][1], dtype=np.int32).tolist() == lens.tolist()
    assert seq_out[0][0] == wire.tobytes()
    wl.free()


@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 1)), ("AES256-SHA256", (3, 3)), ("AES128-SHA", (3, 0)),
                                           ("3DES-SHA", (3, 2))])
def test_chained_vs_oracle(suite, version):
    """The split seal path (seqnum prefix, per-record MAC, quad-lane CBC or
    8-lane 3DES) on chains of mixed record counts and lengths (incl. empty and
    sub-block records) equals the oracle, including the final CBC residue and
    seqnum."""
    from oracle import oracle as O
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr(("ilp", suite, version)).encode()))
    cipher, kl, ivl, mac, ml = O.SUITES[suite]
    states, ocs, recs = [], [], []
    for ci in range(300):
        key, iv, mk, fiv = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml), rng.bytes(ivl)
        seq = int(rng.integers(0, 2 ** 40))
        states.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        ocs.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
        for _ in range(int(rng.integers(0, 6))):
            n = int(rng.choice([0, 1, 7, 8, 15, 16, 17, 100, 1434, 4000, 16384]))
            recs.append((ci, rng.bytes(n), 23, 0))
    out = T.seal(states, recs)
    for (ci, p, ct, fl), w in zip(recs, out):
        assert w == ocs[ci].seal(p, ct, fl), (suite, version, len(p))
    for s, o in zip(states, ocs):
        assert s.seqnum == o.seqnum and s.iv == o.iv


def test_persistent_generations_vs_oracle():
    """More chains in one launch than CUs x 256: cbc_kernel's quads take a
    second chain generation (cid += gridDim.x * cpw).  71,000 AES256-SHA256
    chains in ONE launch -- single records of 37 B, 3-record chains of 100 B and
    2-record chains of 1,500 B -- plus 66,000 AES128-SHA TLS 1.1 chains; every
    wire byte, wire length and every chain's final CBC residue and seqnum equal
    the oracle's (python_aes.py:44, tlsrecordlayer.py:594-608)."""
    _T()
    from tlslite_amd import workloads as W
    from tests.wl_oracle import device_states, oracle_seal
    rng = np.random.default_rng(70000)

    def grp(suite, version, nconn, recs, n):
        from oracle import oracle as O
        _, kl, ivl, _, ml = O.SUITES[suite]
        ivs = np.frombuffer(rng.bytes(ivl * nconn), dtype=np.uint8).reshape(nconn, ivl)
        return W.Group(suite, version, [rng.bytes(kl)], ivs, [rng.bytes(ml)], [rng.bytes(ivl)],
                       rng.integers(0, 2 ** 40, nconn, dtype=np.uint64), recs, n)
    groups = [grp("AES256-SHA256", (3, 3), 50000, 1, 37), grp("AES256-SHA256", (3, 3), 15000, 3, 100),
              grp("AES256-SHA256", (3, 3), 6000, 2, 1500), grp("AES128-SHA", (3, 2), 66000, 1, 20)]
    wl = W.Workload("generations", groups, 71, rec_order=None)
    wl.to_device()
    assert max(n for _, _, n in wl.launches) > 256 * 256
    wl.launch()
    from tlslite_amd.device import synchronize
    synchronize()
    wire_gpu = wl.d_wire.download()
    lens_gpu = wl.d_len.download().view(np.int32)
    states = device_states(wl)
    wire, lens, conns = oracle_seal(wl, nthreads=16)
    assert lens_gpu.tolist() == lens.tolist()
    assert np.array_equal(wire_gpu, wire)
    bad = [c for c, (s, o) in enumerate(zip(states, conns)) if s.iv != o.iv or s.seqnum != o.seqnum]
    assert not bad, "chains with a wrong final state: %s" % bad[:10]
    wl.free()


@pytest.mark.parametrize("pt_shift,wire_shift", [(0, 0), (4, 4), (0, 4), (4, 0), (1, 0), (0, 1), (3, 7)])
@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 3)), ("AES128-SHA", (3, 1)), ("RC4-SHA", (3, 1)),
                                           ("3DES-SHA", (3, 3))])
def test_unaligned_arenas_vs_oracle(pt_shift, wire_shift, suite, version):
    """Record arenas off the 16-byte grid: every record's plaintext at
    pt_off % 16 == pt_shift and its body at (wire_off + 5) % 16 == wire_shift.
    The kernels pick 16-byte, dword or byte paths per record; output equals the
    oracle."""
    from oracle import oracle as O
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr(("unal", pt_shift, wire_shift, suite, version)).encode()))
    cipher, kl, ivl, mac, ml = O.SUITES[suite]
    states, ocs, recs = [], [], []
    for ci in range(64):
        key, iv, mk, fiv = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml), rng.bytes(ivl) if ivl else None
        seq = int(rng.integers(0, 2 ** 40))
        states.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        ocs.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
    for blk in range(16):
        n = int(rng.choice([1, 17, 64, 100, 1434, 4096, 5003, 16384]))
        for ci in range(4 * blk, 4 * blk + 4):
            recs.append((ci, rng.bytes(n), 23, 0))
    for _ in range(40):
        ci = int(rng.integers(0, 64))
        recs.append((ci, rng.bytes(int(rng.integers(0, 3000))), 23, 0))
    out = T.seal(states, recs, pt_shift=pt_shift, wire_shift=wire_shift)
    for (ci, p, ct, fl), w in zip(recs, out):
        assert w == ocs[ci].seal(p, ct, fl), (suite, version, len(p), pt_shift, wire_shift)
    for s, o in zip(states, ocs):
        assert s.seqnum == o.seqnum


@pytest.mark.parametrize("pt_shift,wire_shift,suite,version", [(8, 8, "AES128-SHA", (3, 3)),
                                                                (0, 8, "AES256-SHA", (3, 2)),
                                                                (4, 12, "AES128-SHA", (3, 1))])
def test_unaligned_arenas_pair_regime(pt_shift, wire_shift, suite, version):
    """The pair cipher kernel (>= 256 chains per CU) on arenas off the 16-byte grid: with
    8-byte-aligned bodies at (wire_off + 5) % 16 == 8 the two lanes of a chain must still
    agree on the head blocks before the line-aligned groups (round 5 found them computed from
    the lane's own column address, which differs across the pair there), and 4-byte-aligned
    arenas take the dword path.  Records of 1-3000 B, one connection each (one launch: one
    suite per case): every byte equals the oracle."""
    from oracle import oracle as O
    from tlslite_amd.device import cu_count
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr(("unal-pair", pt_shift, wire_shift, suite)).encode()))
    nconn = 256 * cu_count() + 999
    states, ocs, recs = [], [], []
    _, kl, ivl, _, ml = O.SUITES[suite]
    for ci in range(nconn):
        key, iv, mk, fiv = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml), rng.bytes(ivl)
        states.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, ci))
        ocs.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, ci))
        recs.append((ci, rng.bytes(int(rng.choice([1, 300, 2048, 2999]))), 23, 0))
    out = T.seal(states, recs, pt_shift=pt_shift, wire_shift=wire_shift)
    bad = [ci for (ci, p, ct, fl), w in zip(recs, out) if w != ocs[ci].seal(p, ct, fl)]
    assert not bad, "records differing from the oracle: %d, first %s" % (len(bad), bad[:5])


@pytest.mark.parametrize("kind", ["cfg2", "chained", "shuffled", "rc4", "3des"])
@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("d2h", ["engine", "stores"])
def test_host_pipeline_equals_device_path(kind, pinned, d2h, monkeypatch):
    """tlsgpu_host_pipeline_seal (records in host memory; sub-batches' H2D, seal and
    D2H overlapped on 3 streams, pageable buffers staged through pinned ones) gives
    the same wire arena, wire lengths and final states as the device-resident
    tlsgpu_seal_dev path -- with a small chunk so the batch is cut into many
    sub-batches, for a shuffled arena layout (one sub-batch), and for the RC4
    single-kernel branch and the 3DES split path (TLS 1.0 and 1.2 records); with the wire
    ranges copied D2H by the copy engine and by the GPU's own stores (TLSGPU_HOST_D2H)."""
    monkeypatch.setenv("TLSGPU_HOST_D2H", "kernel" if d2h == "stores" else "engine")
    _T()
    from tlslite_amd import workloads as W
    from tlslite_amd.constants import ContentType
    from tlslite_amd.device import PinnedBuffer, synchronize
    from tlslite_amd.recordlayer import HostSealPipeline, make_chains, make_records
    if kind == "cfg2":
        wl = W.cfg2(n=700, pt_len=5003, seed=21)
    elif kind == "chained":
        wl = W.cfg4(nconn=40, recs_per_conn=5, pt_len=3001, seed=22)
    elif kind in ("rc4", "3des"):
        suites = ("RC4-SHA", "RC4-SHA") if kind == "rc4" else ("3DES-SHA", "3DES-SHA")
        wl = W.Workload(kind, _mixed_workload(200, 4001, 24, suites).groups, 24)
    else:
        g = W.cfg2(n=300, pt_len=777, seed=23).groups
        wl = W.Workload("shuffled", g, 23, rec_order=np.random.default_rng(23).permutation(300))
    wl.to_device()
    wl.launch()
    synchronize()
    ref_wire, ref_states = wl.d_wire.download(), wl.d_states.download()
    var = wl.launches[0][0]
    recs = make_records(wl.pt_off, wl.wire_off, wl.pt_len, ContentType.application_data, 0)
    chains = make_chains(np.arange(wl.n_chains, dtype=np.uint32), wl.chain_first, wl.chain_count)
    bufs = []
    if pinned:
        bufs = [PinnedBuffer(wl.pt_bytes), PinnedBuffer(wl.wire_bytes)]
        pt_h, wire_h = bufs[0].array[: wl.pt_bytes], bufs[1].array[: wl.wire_bytes]
        wire_h[:] = 0
    else:
        pt_h, wire_h = np.empty(wl.pt_bytes, dtype=np.uint8), np.zeros(wl.wire_bytes, dtype=np.uint8)
    wl.d_pt.download(out=pt_h)
    lens = np.zeros(wl.n_records, dtype=np.int32)
    wl.reset_states()
    synchronize()
    with HostSealPipeline(chunk_bytes=64 << 10, depth=3) as hp:
        hp.seal(chains, recs, pt_h, wire_h, wl.d_states, lens, var)
        assert hp.d2h_path == d2h
    assert lens.tolist() == wl.wire_len.astype(np.int32).tolist()
    bad = np.nonzero(wire_h != ref_wire)[0]
    bad_recs = sorted(set(int(np.searchsorted(wl.wire_off.astype(np.int64), x, side="right")) - 1 for x in bad[:4096]))
    assert not len(bad), "%d bytes differ, records %s" % (len(bad), bad_recs[:20])
    assert np.array_equal(wl.d_states.download(), ref_states)
    for b in bufs:
        b.free()
    wl.free()


@pytest.mark.parametrize("suite", ["AES128-SHA", "RC4-SHA"])
def test_host_pipeline_undersized_wire_arena(suite):
    """A wire arena one byte shorter than the last record's sealed form: the kernels
    must not write past it.  A CBC record's size depends on the state's version (device
    state), so that record alone is refused (wire_len = TLSGPU_EINVAL, nothing written,
    its state untouched) and the others are sealed; RC4 sizes are known on the host, so
    the call fails with TLSGPU_EINVAL before anything runs."""
    T = _T()
    from tlslite_amd import _native as N
    from tlslite_amd import workloads as W
    from tlslite_amd.constants import ContentType
    from tlslite_amd.device import synchronize
    from tlslite_amd.recordlayer import HostSealPipeline, make_chains, make_records
    from oracle import oracle as O
    rng = np.random.default_rng(25)
    _, kl, ivl, _, ml = O.SUITES[suite]
    ivs = np.frombuffer(rng.bytes(ivl * 64), dtype=np.uint8).reshape(64, ivl) if ivl else None
    g = W.Group(suite, (3, 3) if ivl else (3, 1), [rng.bytes(kl)], ivs, [rng.bytes(ml)],
                [rng.bytes(ivl)] if ivl else None, np.arange(64, dtype=np.uint64), 1, 3001)
    wl = W.Workload(suite, [g], 25)  # one record per connection
    wl.to_device()
    wl.launch()
    synchronize()
    ref_wire, ref_states = wl.d_wire.download(), wl.d_states.download()
    var = wl.launches[0][0]
    recs = make_records(wl.pt_off, wl.wire_off, wl.pt_len, ContentType.application_data, 0)
    chains = make_chains(np.arange(wl.n_chains, dtype=np.uint32), wl.chain_first, wl.chain_count)
    last = int(np.argmax(wl.wire_off))
    end = int(wl.wire_off[last]) + int(wl.wire_len[last])
    pt_h = wl.d_pt.download()
    wire_h = np.zeros(end - 1, dtype=np.uint8)
    lens = np.zeros(wl.n_records, dtype=np.int32)
    wl.reset_states()
    synchronize()
    with HostSealPipeline(chunk_bytes=64 << 10, depth=2) as hp:
        if suite.startswith("RC4"):
            with pytest.raises(N.TLSGPUError) as ei:
                hp.seal(chains, recs, pt_h, wire_h, wl.d_states, lens, var)
            assert ei.value.code == N.EINVAL
            assert not wire_h.any()
            return
        hp.seal(chains, recs, pt_h, wire_h, wl.d_states, lens, var)
    want = wl.wire_len.astype(np.int32).copy()
    want[last] = N.EINVAL
    assert lens.tolist() == want.tolist()
    assert np.array_equal(wire_h[:int(wl.wire_off[last])], ref_wire[:int(wl.wire_off[last])])
    assert not wire_h[int(wl.wire_off[last]):].any()  # the refused record: nothing written
    st = wl.d_states.download().reshape(-1, N.CONN_STATE_BYTES)
    ref = ref_states.reshape(-1, N.CONN_STATE_BYTES)
    init = wl.host_states().reshape(-1, N.CONN_STATE_BYTES)
    owner = int(np.searchsorted(wl.chain_first.astype(np.int64), last, side="right")) - 1
    for c in range(wl.n_chains):
        assert np.array_equal(st[c], init[c] if c == owner else ref[c]), c
    wl.free()


def _many_chains():
    """Chains per call from which the cipher phase runs its throughput layout on every
    CU (a full 256-chain workgroup per CU and more: cfg2 / cfg3 shapes)."""
    from tlslite_amd import _native as N
    from tlslite_amd.device import cu_count
    return 256 * cu_count()


@pytest.mark.parametrize("suite,version", [("AES256-SHA256", (3, 3)), ("AES128-SHA", (3, 1)), ("AES128-SHA", (3, 0)),
                                           ("AES256-SHA", (3, 2))])
def test_many_chains_vs_oracle(suite, version):
    """A seal call with more chains than one cipher-workgroup generation per CU (the
    layout cfg2 / cfg3 run, tlsgpu_seal_cipher_kernel names it) plus a persistent second
    generation -- one-record connections of 1,434 B (cfg3's record), 3-record chains of
    100 B, 2-record chains of 5,003 B, chains of sub-block, block-sized and empty
    records, random content types and badMAC / badPadding faults on ~3 % of the records
    -- equals the oracle byte for byte, every wire length, and every chain's final CBC
    residue and seqnum (tlsrecordlayer.py:538-617, python_aes.py:44)."""
    _T()
    from tlslite_amd import workloads as W
    from tlslite_amd.device import synchronize
    from tests.wl_oracle import device_states, oracle_seal
    from oracle import oracle as O
    rng = np.random.default_rng(zlib.crc32(repr(("lane", suite, version)).encode()))
    _, kl, ivl, _, ml = O.SUITES[suite]

    def grp(nconn, recs, n):
        ivs = np.frombuffer(rng.bytes(ivl * nconn), dtype=np.uint8).reshape(nconn, ivl)
        return W.Group(suite, version, [rng.bytes(kl)], ivs, [rng.bytes(ml)], [rng.bytes(ivl)],
                       rng.integers(0, 2 ** 40, nconn, dtype=np.uint64), recs, n)
    nmin = _many_chains()
    small = [grp(20000, 3, 100), grp(6000, 2, 5003), grp(3000, 2, 0), grp(3000, 4, 15), grp(3000, 1, 16),
             grp(3000, 2, 63), grp(3000, 1, 64), grp(3000, 1, 65)]
    n_big = nmin + 9000 - sum(g.nconn for g in small)
    groups = [grp(n_big, 1, 1434)] + small
    nrec = sum(g.nconn * g.recs_per_conn for g in groups)
    ctype = rng.choice([21, 22, 23], nrec, p=[0.05, 0.05, 0.9])
    flags = np.where(rng.random(nrec) < 0.03, rng.integers(1, 4, nrec), 0)
    wl = W.Workload("many", groups, 72, rec_ctype=ctype, rec_flags=flags)
    wl.to_device()
    assert [n for _, _, n in wl.launches] == [wl.n_chains] and wl.n_chains > nmin
    wl.launch()
    synchronize()
    wire_gpu = wl.d_wire.download()
    lens_gpu = wl.d_len.download().view(np.int32)
    states = device_states(wl)
    wire, lens, conns = oracle_seal(wl, nthreads=16)
    assert lens_gpu.tolist() == lens.tolist()
    bad = np.nonzero(wire_gpu != wire)[0]
    bad_recs = sorted(set(int(np.searchsorted(wl.wire_off.astype(np.int64), x, side="right")) - 1 for x in bad[:4096]))
    assert not len(bad), "%d bytes differ, records %s" % (len(bad), bad_recs[:20])
    bad = [c for c, (s, o) in enumerate(zip(states, conns)) if s.iv != o.iv or s.seqnum != o.seqnum]
    assert not bad, "chains with a wrong final state: %s" % bad[:10]
    wl.free()


def test_library_workspaces_released_and_reallocated():
    """tlsgpu_seal_dev with a NULL workspace on several short-lived streams: destroying a
    stream frees the library-owned workspace of that stream (the count of owned buffers
    drops back; a later stream that gets the same handle value starts without one), and
    every batch equals the first (no state of a freed buffer leaks into a later call).
    tlsgpu_release_workspaces then frees whatever is left (the null stream's buffer)."""
    _T()
    from tlslite_amd import _native as N
    from tlslite_amd import workloads as W
    from tlslite_amd.device import Stream, synchronize
    from tlslite_amd.recordlayer import seal_dev
    wl = W.cfg2(n=300, pt_len=3001, seed=31)
    wl.to_device()
    var, d_ch, nch = wl.launches[0]
    N.call("tlsgpu_release_workspaces")
    assert N.lib.tlsgpu_owned_workspace_count() == 0
    outs = []
    for k in range(6):
        s = Stream()
        wl.reset_states(s)
        wl.d_wire.zero(s)
        seal_dev(d_ch, nch, wl.d_recs, wl.n_records, wl.d_pt, wl.d_wire, wl.d_states, wl.d_len, var, None, s)
        assert N.lib.tlsgpu_owned_workspace_count() == 1
        s.synchronize()
        outs.append((wl.d_wire.download().tobytes(), wl.d_len.download().tobytes(), wl.d_states.download().tobytes()))
        s.close()
        assert N.lib.tlsgpu_owned_workspace_count() == 0, "stream destroy left its workspace"
    assert all(o == outs[0] for o in outs)
    # the null stream's buffer lives until tlsgpu_release_workspaces
    wl.reset_states()
    seal_dev(d_ch, nch, wl.d_recs, wl.n_records, wl.d_pt, wl.d_wire, wl.d_states, wl.d_len, var, None, None)
    synchronize()
    assert wl.d_wire.download().tobytes() == outs[0][0]
    assert N.lib.tlsgpu_owned_workspace_count() == 1
    N.call("tlsgpu_release_workspaces")
    assert N.lib.tlsgpu_owned_workspace_count() == 0
    wl.free()


@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 3)), ("AES128-SHA", (3, 1)), ("AES128-SHA", (3, 0)),
                                           ("AES256-SHA", (3, 3)), ("AES256-SHA", (3, 1)), ("AES256-SHA", (3, 0))])
def test_one_generation_pair_kernel_vs_oracle(suite, version):
    """Exactly 256 chains per CU: the cfg2 cipher layout (cbc_pair_kernel with 8-block
    groups, one generation; tlsgpu_seal_cipher_kernel names it) on mixed records -- empty,
    sub-block, 15/16/17 blocks (around the 16-block group-alignment threshold), 2G +- 1
    blocks, 1,434 B, 5,003 B and 16 KiB -- with random content types, badMAC / badPadding
    faults on ~5 % of the records, and plaintext / wire offsets off the 128-B line so the
    head blocks before the first whole-line group vary.  Every byte, wire length and final
    CBC residue / seqnum equals the oracle (tlsrecordlayer.py:538-617, python_aes.py:44)."""
    _T()
    from tlslite_amd import _native as N
    from tlslite_amd import workloads as W
    from tlslite_amd.device import synchronize
    from tlslite_amd.recordlayer import seal_cipher_kernel
    from tests.wl_oracle import device_states, oracle_seal
    from oracle import oracle as O
    rng = np.random.default_rng(zlib.crc32(repr(("gen1", suite, version)).encode()))
    _, kl, ivl, _, ml = O.SUITES[suite]
    nmin = _many_chains()
    lens = [0, 1, 15, 16, 17, 15 * 16, 16 * 16, 17 * 16 + 3, 15 * 16 + 9, 31 * 16, 33 * 16 + 1, 1434, 5003, 16384,
            16 * 8 * 3, 100]
    groups = []
    left = nmin
    for i, n in enumerate(lens):
        nconn = left if i == len(lens) - 1 else nmin // (2 * len(lens))
        left -= nconn
        ivs = np.frombuffer(rng.bytes(ivl * nconn), dtype=np.uint8).reshape(nconn, ivl)
        recs = 2 if n < 4096 else 1
        groups.append(W.Group(suite, version, [rng.bytes(kl)], ivs, [rng.bytes(ml)], [rng.bytes(ivl)],
                              rng.integers(0, 2 ** 40, nconn, dtype=np.uint64), recs, n))
    nrec = sum(g.nconn * g.recs_per_conn for g in groups)
    ctype = rng.choice([21, 22, 23], nrec, p=[0.05, 0.05, 0.9])
    flags = np.where(rng.random(nrec) < 0.05, rng.integers(1, 4, nrec), 0)
    wl = W.Workload("gen1", groups, 77, rec_ctype=ctype, rec_flags=flags)
    wl.to_device()
    assert [n for _, _, n in wl.launches] == [nmin] == [wl.n_chains]
    var = wl.launches[0][0]
    assert seal_cipher_kernel(var, nmin).startswith("cbc_pair_kernel<%d, 8, 8>" % (10 if "128" in suite else 14))
    wl.launch()
    synchronize()
    wire_gpu = wl.d_wire.download()
    lens_gpu = wl.d_len.download().view(np.int32)
    states = device_states(wl)
    wire, lens_o, conns = oracle_seal(wl, nthreads=16)
    assert lens_gpu.tolist() == lens_o.tolist()
    bad = np.nonzero(wire_gpu != wire)[0]
    bad_recs = sorted(set(int(np.searchsorted(wl.wire_off.astype(np.int64), x, side="right")) - 1 for x in bad[:4096]))
    assert not len(bad), "%d bytes differ, records %s" % (len(bad), bad_recs[:20])
    bad = [c for c, (s, o) in enumerate(zip(states, conns)) if s.iv != o.iv or s.seqnum != o.seqnum]
    assert not bad, "chains with a wrong final state: %s" % bad[:10]
    wl.free()

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


@pytest.mark.parametrize("suite", ["AES128-SHA", "AES256-SHA256", "RC4-SHA", "3DES-SHA", "RC4-MD5"])
@pytest.mark.parametrize("version", [(3, 0), (3, 1), (3, 2), (3, 3)])
def test_random_lengths_vs_oracle(suite, version):
    from oracle import oracle as O
    T = _T()
    if suite.endswith("SHA256") and version != (3, 3):
        pytest.skip("SHA256 suites are TLS 1.2 only")
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


def _mixed_workload(n, pt_len, seed):
    from tlslite_amd import workloads as W
    rng = np.random.default_rng(seed)
    h = n // 2
    ka, mka, fiva = rng.bytes(16), rng.bytes(20), rng.bytes(16)
    kr, mkr = rng.bytes(16), rng.bytes(20)
    iva = np.frombuffer(rng.bytes(16 * h), dtype=np.uint8).reshape(h, 16)
    g1 = W.Group("AES128-SHA", (3, 3), [ka], iva, [mka], [fiva], np.arange(h, dtype=np.uint64), 3, pt_len)
    g2 = W.Group("RC4-SHA", (3, 1), [kr], None, [mkr], None, np.arange(n - h, dtype=np.uint64), 3, pt_len)
    return W.Workload("mixed", [g1, g2], seed, rec_order=rng.permutation(3 * n))


@pytest.mark.parametrize("kind", ["cfg2", "mixed"])
def test_pipeline_equals_sequential(kind):
    """tlsgpu_pipeline_seal: K successive batches (MAC phase of batch k+1
    overlapping the CBC phase of batch k) give the same wire bytes and final
    connection states as K sequential tlsgpu_seal_dev calls."""
    _T()
    from tlslite_amd import workloads as W
    from tlslite_amd.device import DeviceBuffer, Stream
    from tlslite_amd.recordlayer import SealPipeline
    wl = W.cfg2(n=700, pt_len=5003, seed=11) if kind == "cfg2" else _mixed_workload(300, 2000, 12)
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
    wl.free()


# AES seal kernel selections (environment switches read per launch by libtlsgpu)
AES_IMPLS = {
    "cbc1": {},                                   # default: cbc_kernel, column-word I/O, per-lane MAC loads
    "cbc1io16": {"TLSGPU_CBC_IO": "16"},          # cbc_kernel<NR, IO16>: 16-byte I/O + quad transposes
    "macquad": {"TLSGPU_MAC_LOAD": "quad"},       # mac_kernel<.., QL>: quad-cooperative loads
    "cbc2": {"TLSGPU_CBC_ILP": "2"},              # cbc2_kernel: two chains per quad
    "pair": {"TLSGPU_CBC_LAYOUT": "pair"},        # cbcp_kernel: two lanes per chain
    "fused": {"TLSGPU_SEAL_IMPL": "fused"},       # single fused quad kernel
    "lane": {"TLSGPU_SEAL_IMPL": "lane"},         # one lane per chain
}


@pytest.mark.parametrize("ilp", list(AES_IMPLS))
@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 1)), ("AES256-SHA256", (3, 3)), ("AES128-SHA", (3, 0))])
def test_cbc_variants_chained_vs_oracle(ilp, suite, version, monkeypatch):
    """Every AES seal kernel -- split path with cbc_kernel (one chain per quad;
    column-word or 16-byte I/O; per-lane or quad-cooperative MAC loads) or
    cbc2_kernel (two chains per quad, bulk interleaved, IV/tail blocks one chain
    at a time), the fused single-kernel path, the 1-lane kernel -- on chains of
    mixed record counts and lengths (incl. empty and sub-block records) equals
    the oracle, including the final CBC residue and seqnum."""
    from oracle import oracle as O
    for k, v in AES_IMPLS[ilp].items():
        monkeypatch.setenv(k, v)
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
            n = int(rng.choice([0, 1, 15, 16, 17, 100, 1434, 4000, 16384]))
            recs.append((ci, rng.bytes(n), 23, 0))
    out = T.seal(states, recs)
    for (ci, p, ct, fl), w in zip(recs, out):
        assert w == ocs[ci].seal(p, ct, fl), (ilp, suite, version, len(p))
    for s, o in zip(states, ocs):
        assert s.seqnum == o.seqnum and s.iv == o.iv


@pytest.mark.parametrize("impl", ["cbc1", "cbc1io16", "macquad"])
@pytest.mark.parametrize("pt_shift,wire_shift", [(0, 0), (4, 4), (0, 4), (4, 0), (1, 0), (0, 1), (3, 7)])
@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 3)), ("AES128-SHA", (3, 1)), ("RC4-SHA", (3, 1))])
def test_unaligned_arenas_vs_oracle(pt_shift, wire_shift, suite, version, impl, monkeypatch):
    """Record arenas off the 16-byte grid: every record's plaintext at
    pt_off % 16 == pt_shift and its body at (wire_off + 5) % 16 == wire_shift.
    The kernels pick 16-byte, dword or byte paths per record (and the MAC its
    per-lane loads when a quad is not 16-byte aligned); output equals the oracle.
    Equal-length records in runs of 4 so quad-cooperative MAC loads are taken
    whenever the alignment allows."""
    from oracle import oracle as O
    if suite.startswith("RC4") and impl != "cbc1":
        pytest.skip("AES kernel selections only")
    for k, v in AES_IMPLS[impl].items():
        monkeypatch.setenv(k, v)
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

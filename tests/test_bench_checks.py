"""bench.py's parity checkers on the CPU (no GPU): `oracle_check` (the `bit_exact` field) and
`oracle_timed_check` (`timed_oracle_exact`: the last of n successive seals, states carried)
accept an output equal to the oracle's and reject one changed byte or one wrong length, on
small batches of every BASELINE config's shape (tlsrecordlayer.py:538-617: the chain's CBC
residue / RC4 state and seqnum carry from seal to seal).  Test infrastructure only."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [("cfg2", {"n": 48, "pt_len": 1500}), ("cfg3", {"n": 64, "pt_len": 1434}),
          ("cfg4", {"nconn": 8, "recs_per_conn": 3, "pt_len": 3000}), ("cfg5", {"n": 40, "pt_len": 2000})]


def _sealed(wl, n_launches):
    """The wire arena and wire lengths after n_launches successive seals (the oracle)."""
    import bench
    from oracle import oracle as O
    protos = bench.oracle_protos(wl, np.arange(wl.n_chains))
    pt = wl.host_plaintext(O.fill_pattern)
    wire = np.zeros(wl.wire_bytes, dtype=np.uint8)
    lens = None
    for _ in range(n_launches):
        lens = O.seal_batch(protos, wl.chain_first, wl.chain_count, pt, wl.pt_off, wl.pt_len, wire, wl.wire_off,
                            nthreads=2, update=True)
    return wire, np.asarray(lens, dtype=np.int32)


def _record_byte(wl, r):
    return int(wl.wire_off[r]) + 5 + int(wl.wire_len[r] - 5) // 2


@pytest.mark.parametrize("name,kw", SHAPES)
def test_timed_check_accepts_oracle_and_rejects_changes(name, kw):
    import bench
    from tlslite_amd import workloads as W
    wl = W.CONFIGS[name](**kw)
    wire, lens = _sealed(wl, 3)
    ok, k = bench.oracle_timed_check(wl, wire, lens, 3, 2)
    assert ok and k == wl.n_chains  # a small batch: every chain sampled
    bad = wire.copy()
    bad[_record_byte(wl, wl.n_records // 2)] ^= 0x40
    assert not bench.oracle_timed_check(wl, bad, lens, 3, 2)[0]
    bad_len = lens.copy()
    bad_len[wl.n_records - 1] += 16
    assert not bench.oracle_timed_check(wl, wire, bad_len, 3, 2)[0]
    # the output of two seals is not the output of three (states carried: new IV / keystream / seqnum)
    wire2, lens2 = _sealed(wl, 2)
    assert not bench.oracle_timed_check(wl, wire2, lens2, 3, 2)[0]


@pytest.mark.parametrize("name,kw", SHAPES)
def test_oracle_check_accepts_oracle_and_rejects_a_change(name, kw):
    import bench
    from tlslite_amd import workloads as W
    wl = W.CONFIGS[name](**kw)
    wire, _ = _sealed(wl, 1)
    ok, _, nrec, nbytes, _, reps = bench.oracle_check(wl, wire, 2)
    assert ok and nrec == wl.n_records and reps == 1 and nbytes == int(wl.pt_len.sum())
    bad = wire.copy()
    bad[_record_byte(wl, 0)] ^= 1
    assert not bench.oracle_check(wl, bad, 2)[0]


def test_pmc_traffic_attached_only_to_the_same_workload(tmp_path):
    """bench.py prices roofline.traffic from a committed PMC summary only when the summary
    names the run's dominant kernel and was collected on the same workload and record count
    (a 4,096-connection PMC file once priced a 512-connection run at 8.1x)."""
    import json
    import bench
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"dominant_kernel": "cbc_kernel<10, true, 16>", "workload": "cfg4: 4096 conns",
                             "records": 1048576, "hbm_bytes_per_launch": 123, "seal_call_hbm_bytes": 456}))
    assert bench.pmc_traffic(str(p), "cfg4: 4096 conns", 1048576, "cbc_kernel<10, false>") == (123, 456)
    assert bench.pmc_traffic(str(p), "cfg4: 512 conns", 131072, "cbc_kernel<10, true>") == (None, None)
    assert bench.pmc_traffic(str(p), "cfg4: 4096 conns", 1048576, "cbc_pair_kernel<10, 8, 8>") == (None, None)
    assert bench.pmc_traffic(str(tmp_path / "missing.json"), "x", 1, "k") == (None, None)
    (tmp_path / "bad.json").write_text("{not json")
    assert bench.pmc_traffic(str(tmp_path / "bad.json"), "x", 1, "k") == (None, None)
    # the committed summaries name their workload and record count
    for cfg in ("cfg2", "cfg3", "cfg4", "cfg5"):
        pj = json.load(open(os.path.join(ROOT, "profiles", "pmc_%s.json" % cfg)))
        assert pj["workload"].startswith(cfg) and pj["records"] > 0 and pj["hbm_bytes_per_launch"] > 0


class _FakeRanks:
    """Two ranks' results as ShardGroup.gather_bytes / sum would return them on rank 0."""

    def __init__(self, results, nbytes):
        import json
        self._b = [json.dumps(r).encode() for r in results]
        self._n = nbytes

    def gather_bytes(self, b):
        return self._b

    def sum(self, x):
        return float(sum(self._n))


def test_open_leg_aggregated_over_ranks():
    """bench.py's open leg at N > 1 (open_over_ranks): the job's rate is all ranks' plaintext /
    the slowest rank's median call, roundtrip_exact the AND over ranks, a failing rank an
    error -- never a silently dropped rank."""
    import bench
    gib = bench.GIB
    a = {"value": 800.0, "unit": "GiB/s", "ms": 1.25, "roundtrip_exact": True, "method": "m"}
    b = {"value": 780.0, "unit": "GiB/s", "ms": 1.30, "roundtrip_exact": True, "method": "m"}
    r = bench.open_over_ranks(_FakeRanks([a, b], [gib, gib]), a, gib)
    assert r["value"] == round(2.0 / (1.30 / 1e3), 2) and r["ms"] == 1.3 and r["roundtrip_exact"] is True
    assert [x["value"] for x in r["ranks"]] == [800.0, 780.0]
    b2 = dict(b, roundtrip_exact=False)
    assert bench.open_over_ranks(_FakeRanks([a, b2], [gib, gib]), a, gib)["roundtrip_exact"] is False
    r = bench.open_over_ranks(_FakeRanks([a, {"error": "boom"}], [gib, gib]), a, gib)
    assert "error" in r and "rank(s) [1]" in r["error"]
    # wall-clock-timed concurrent runs on every rank: aggregated beside the headline, which
    # stays the per-call median as at N = 1 (one metric at every N)
    ac = dict(a, concurrent={"ms": 2.0, "roundtrip_exact": True})
    bc = dict(b, concurrent={"ms": 2.5, "roundtrip_exact": True})
    r = bench.open_over_ranks(_FakeRanks([ac, bc], [gib, gib]), ac, gib)
    assert r["ms"] == 1.3 and r["value"] == round(2.0 / (1.30 / 1e3), 2) and "median" in r["aggregate"]
    assert r["concurrent_value"] == round(2.0 / 0.0025, 2) and "wall time" in r["concurrent_aggregate"]
    bc2 = dict(bc, concurrent={"ms": 2.5, "roundtrip_exact": False})
    assert bench.open_over_ranks(_FakeRanks([ac, bc2], [gib, gib]), ac, gib)["roundtrip_exact"] is False


def test_derive_and_host_legs_aggregated_over_ranks():
    """The derive and host-inclusive legs at N > 1 (derive_over_ranks,
    host_inclusive_over_ranks): sums over ranks / the slowest rank, exactness ANDed."""
    import bench
    gib = bench.GIB
    d0 = {"connections": 4096, "ms": 0.8, "conns_per_s": 5120000, "key_blocks_exact_sample": True}
    d1 = dict(d0, ms=1.0, key_blocks_exact_sample=False)
    r = bench.derive_over_ranks(_FakeRanks([d0, d1], [0, 0]), d0)
    assert r["connections"] == 8192 and r["ms"] == 1.0 and r["conns_per_s"] == 8192000
    assert r["key_blocks_exact_sample"] is False
    h = {"value": 40.0, "pinned": {"value": 40.0, "ms": 25.0, "bit_exact": True},
         "pageable": {"value": 30.0, "ms": 33.0, "bit_exact": True}, "pcie_frac": 0.9}
    r = bench.host_inclusive_over_ranks(_FakeRanks([h, h], [gib, gib]), h, gib)
    assert r["value"] == round(2.0 / 0.025, 2) and r["bit_exact"] is True and "pcie_frac" not in r
    hb = {"value": 40.0, "pinned": {"value": 40.0, "ms": 25.0, "bit_exact": True},
          "pageable": {"value": 30.0, "ms": 33.0, "bit_exact": False}}
    assert bench.host_inclusive_over_ranks(_FakeRanks([h, hb], [gib, gib]), h, gib)["bit_exact"] is False
    assert "error" in bench.host_inclusive_over_ranks(_FakeRanks([h, None], [gib, gib]), h, gib)


def test_pinned_visibility_narrows_to_the_ranks_own_gpu():
    """pin_rank_device's choice: the local rank's entry of the list HIP already applies, or
    HIP_VISIBLE_DEVICES = local rank; nothing when the node lacks a GPU for the rank."""
    import bench
    pv = bench.pinned_visibility
    assert pv({}, 0, 8) == ("HIP_VISIBLE_DEVICES", "0")
    assert pv({}, 7, 8) == ("HIP_VISIBLE_DEVICES", "7")
    assert pv({}, 1, 1) is None
    assert pv({"HIP_VISIBLE_DEVICES": "4,5,6,7"}, 2, 4) == ("HIP_VISIBLE_DEVICES", "6")
    assert pv({"CUDA_VISIBLE_DEVICES": "3, 1"}, 1, 2) == ("CUDA_VISIBLE_DEVICES", "1")
    assert pv({"HIP_VISIBLE_DEVICES": "2", "CUDA_VISIBLE_DEVICES": "0,1"}, 0, 1) == ("HIP_VISIBLE_DEVICES", "2")
    assert pv({"HIP_VISIBLE_DEVICES": ""}, 1, 2) == ("HIP_VISIBLE_DEVICES", "1")
    assert pv({"HIP_VISIBLE_DEVICES": "0"}, 1, 2) is None


def test_event_steps_spread_over_the_timed_region():
    """The timed steps whose dominant kernel bench.py brackets with HIP events."""
    import bench
    assert bench.event_steps(20, 4) == [2, 6, 10, 14, 18]
    assert bench.event_steps(500, 4)[:3] == [2, 6, 10] and len(bench.event_steps(500, 4)) == 125
    assert bench.event_steps(10, 1) == list(range(10))
    assert bench.event_steps(1, 4) == [0]
    assert bench.event_steps(2, 4) == [1]


def test_hip_error_in_a_leg_fails_the_run():
    """A failed HIP call in a side leg (TLSGPU_EHIP: the context is dead after a fault) is
    marked in the leg's field and named by hip_failures, which makes bench.py exit non-zero;
    other leg errors (an unsupported shape, a refused argument) are reported, not fatal."""
    import bench
    from tlslite_amd import _native as N
    hip = bench.leg_error(N.TLSGPUError(N.EHIP, "tlsgpu_stream_synchronize"))
    inval = bench.leg_error(N.TLSGPUError(N.EINVAL, "tlsgpu_open_dev"))
    assert hip["hip_error"] and not inval["hip_error"]
    assert bench.hip_failures({"open": hip, "derive": None}) == ["open"]
    assert bench.hip_failures({"open": inval, "derive": {"ms": 1.0}}) == []
    # N > 1: a rank's failure nested in the aggregated leg
    agg = {"error": "open leg failed on rank(s) [1]", "ranks": [{"value": 1.0}, hip]}
    assert bench.hip_failures({"open": agg, "host_inclusive": None}) == ["open"]


def test_link_ceiling_takes_the_better_d2h_path():
    """The host legs price their PCIe ceiling with the better of the pipelines' two D2H paths
    (copy engine or device stores): the engine's rates when it is the
    faster one, the stores' in a process where the engine's D2H runs slow."""
    import bench
    good = {"h2d": 57.5, "d2h": 57.0, "both": 97.1, "d2h_stores": 54.6, "both_stores": 85.4}
    slow = {"h2d": 57.5, "d2h": 30.0, "both": 57.0, "d2h_stores": 54.7, "both_stores": 87.2}
    assert bench.link_best(good) == (57.0, 97.1)
    assert bench.link_best(slow) == (54.7, 87.2)
    assert bench.link_best({"h2d": 57.5, "d2h": 57.0, "both": 97.1}) == (57.0, 97.1)  # no stores probe


def test_gpu_warm_runs_until_its_time_or_call_budget():
    """The side legs' warm-up burst: calls in groups of four, each group synchronised, until
    min_ms have passed or max_calls were made."""
    import time
    import bench
    calls, syncs = [], []
    n = bench.gpu_warm(lambda: calls.append(1), lambda: syncs.append(1), min_ms=1e9, max_calls=12)
    assert n == 12 and len(calls) == 12 and len(syncs) == 3
    calls.clear()
    t0 = time.perf_counter()
    n = bench.gpu_warm(lambda: (calls.append(1), time.sleep(0.002)), lambda: None, min_ms=20.0, max_calls=400)
    assert 8 <= n <= 16 and (time.perf_counter() - t0) * 1e3 >= 20.0

#!/usr/bin/env python3
"""bench.py -- BASELINE.json headline: device-resident AES-128-CBC + HMAC-SHA1
TLS-record seal of 64 Ki x 16 KiB records (config 2), in plaintext GiB/s.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

With --gpus N > 1 and no launcher environment (WORLD_SIZE unset) bench.py starts the N
ranks itself: before any GPU call it spawns N child processes of itself with RANK =
LOCAL_RANK = i, WORLD_SIZE = N and a rendezvous address, waits for them, and exits
non-zero if any fails; rank 0 prints the line.  N above the visible devices is refused
unless --share-devices is given (ranks then share GPUs round-robin: a rehearsal of the
N-rank path on a smaller box, not a scaling measurement).

A step = one seal of the whole per-GPU batch (every record MAC'd, padded,
CBC-encrypted and framed; connection states carried from the previous step).
Multi-GPU is weak scaling: each rank owns its own batch on its own device
(connection sharding, no collective on the data path); the ranks meet only for
the start/stop barriers and the max-over-ranks time (tlslite_amd.shard: a small
TCP rendezvous, no PyTorch).  After the timed loop the same number of seals is
replayed sequentially from the initial states and the last step's wire arena,
wire lengths and final states are compared (`timed_bit_exact`: a pipeline-vs-sequential
consistency check), and a sample of chains is sealed the same number of times by the CPU
oracle and compared with the last step's output (`timed_oracle_exact`).

Prints ONE JSON line (rank 0) with roofline + cpu_baseline objects.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# LDS lookup ceiling: conflict-free ds_read_b32 = 64 lanes per 2 LDS cycles = 32 lookups
# per cycle per CU (MI355X_MICROARCH.md §LDS), 256 CUs, priced at the 2.4 GHz peak engine clock
LDS_PEAK_GLOOKUPS = 256 * 32 * 2.4
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--share-devices", action="store_true",
                    help="allow --gpus N above the visible device count (ranks share GPUs round-robin)")
    ap.add_argument("--extra-streams", type=int, default=0,
                    help="create this many idle HIP streams before the seal pipeline (diagnostic: the pipeline's "
                         "overlap must survive an application's other streams)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only (no GPU call): every rank reports its RANK / LOCAL_RANK / device, rank 0 "
                         "prints one JSON line; TLSGPU_DRYRUN_DEVICES stands in for the visible device count")
    ap.add_argument("--pt-align", type=int, default=16,
                    help="plaintext slot alignment of the workload (16: packed, as generic callers lay records out; "
                         "128: every record on a cache line)")
    # defaults: 500 + 500 steps (~1 s of GPU time for cfg2): sustained load, ~4 % above what a 5-step
    # warmup + 50-step run sees (profiles/r03/warmup_steps.txt; a fresh process's first seal steps run
    # slower and a short timed region pays the pipeline's fill: DESIGN.md section 4, profiles/r06/clock);
    # cfg4 (~0.12 s per step): 2 + 10.  Explicit --steps / --warmup are used as given.
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3", "cfg4", "cfg5"])
    ap.add_argument("--records", type=int, default=None, help="override record count (debug)")
    ap.add_argument("--no-cpu", action="store_true", help="skip cpu_baseline")
    ap.add_argument("--no-check", action="store_true", help="skip the full-batch parity check")
    ap.add_argument("--no-derive", dest="derive", action="store_false",
                    help="skip the batched key-derivation measurement")
    ap.add_argument("--no-open", dest="open", action="store_false", help="skip the open-path measurement")
    ap.add_argument("--open", dest="open", action="store_true", help="measure the open path (the default; after a "
                    "--no-open, e.g. in tools/pmc_kernels.sh's fixed arguments, turns it back on)")
    ap.add_argument("--no-host-inclusive", dest="host_inclusive", action="store_false", default=None,
                    help="skip the PCIe-inclusive measurement (profiling runs)")
    ap.add_argument("--host-inclusive", dest="host_inclusive", action="store_true",
                    help="measure the PCIe-inclusive rate (default: cfg2 only -- cfg4's 16 GiB arenas would "
                         "pin 32 GiB of host memory for it)")
    ap.add_argument("--open-split", default=None, choices=["auto", "chains", "none", "blocks"],
                    help="force the open path's split form (tlsgpu_set_open_parts; default: the library's choice)")
    ap.add_argument("--traffic", default=None, help="JSON with PMC-derived HBM bytes per launch")
    ap.add_argument("--kernel-events-every", type=int, default=None,
                    help="time the dominant kernel with HIP events on every M-th timed step (the steps k with "
                         "k %% M == M // 2): AES suites, the cipher kernel's own dispatch events (hipExtLaunchKernelGGL); "
                         "RC4 / 3DES-only batches, event records around the call (~25 us each pair, DESIGN.md "
                         "section 4).  Default 4 (cfg4, cfg5: 1)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="minimum CPU time of the cpu_baseline sample (the full batch, repeated)")
    a = ap.parse_args()
    if a.host_inclusive is None:
        a.host_inclusive = a.config == "cfg2"
    if a.steps is None:
        a.steps = 10 if a.config == "cfg4" else 500
    if a.warmup is None:
        a.warmup = 2 if a.config == "cfg4" else 500
    if a.kernel_events_every is None:
        # cfg4 (0.12 s steps) and cfg5 (its events span the whole 4.7-ms 3DES call, so a sampled
        # step would run longer than the average step): every step
        a.kernel_events_every = 1 if a.config in ("cfg4", "cfg5") else 4
    a.kernel_events_every = max(1, a.kernel_events_every)
    return a


def event_steps(steps, every):
    """The timed steps whose dominant kernel is bracketed by HIP events: k % every == every // 2
    (spread over the run, centred), at least one."""
    ks = [k for k in range(steps) if k % every == every // 2]
    return ks or [steps // 2]


# The reference's own pure-Python path (measured in the survey container through
# the namespace shim: TLSRecordLayer._sendMsg with the "python" cipher implementation, 16 KiB
# AES-128-CBC + HMAC-SHA1 records, TLS 1.2).  It cannot run on the GPU box (the reference does
# not travel), so it is quoted, labelled, beside the measured C-restatement baseline.
REFERENCE_PYTHON = {"value": round(4.03e6 / GIB, 6), "unit": "GiB/s", "cores": 8, "per_core": round(0.621e6 / GIB, 6),
                    "kind": "reference",
                    "where": "survey container, Intel Xeon 8 cores (multiprocessing.Pool(8)); BASELINE.md",
                    "what": "tlslite 0.4.9 TLSRecordLayer._sendMsg, pure-Python AES-128-CBC + HMAC-SHA1 (stdlib "
                            "hmac), 16 KiB records, TLS 1.2"}


def usable_cpus():
    """Host cores this job may use: the affinity mask, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS (the GPU box sets it to the CPU share of one GPU); -> (threads, note)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    note = ["affinity %d" % n, "os.cpu_count %d" % (os.cpu_count() or 0)]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            lim = max(1, int(int(q) // int(per)))
            note.append("cgroup quota %d" % lim)
            n = min(n, lim)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        note.append("OMP_NUM_THREADS %s" % omp)
        n = min(n, int(omp))
    return n, ", ".join(note)


def build_workload(name, rank, world, records=None, pt_align=16):
    from tlslite_amd import workloads as W
    if name == "cfg4":
        kw = {} if records is None else {"nconn": records}
        return W.cfg4(rank=rank, world=world, **kw)
    kw = {} if records is None else {"n": records}
    if name == "cfg3":
        # packed 16-B plaintext slots by default; --pt-align 128 puts every record on a line
        # (cfg2 / cfg5 records are 16 KiB: line-aligned either way)
        kw["pt_align"] = int(pt_align)
    return W.CONFIGS[name](**kw)


def oracle_protos(wl, idx_chains):
    """CPU-oracle connection states (initial) of the workload's chains idx_chains."""
    from oracle import oracle as O
    protos = []
    for c in idx_chains:
        g = wl.groups[wl.chain_group[c]]
        gi = c - int(np.searchsorted(wl.chain_group, wl.chain_group[c]))
        key = g.keys[gi % len(g.keys)]
        mk = g.mac_keys[gi % len(g.mac_keys)]
        fiv = g.fixed_ivs[gi % len(g.fixed_ivs)] if g.fixed_ivs is not None else None
        iv = bytes(g.ivs[gi]) if g.ivs is not None else b""
        protos.append(O.Conn.for_suite(g.suite, g.version, bytes(key), iv, bytes(mk),
                                       None if fiv is None else bytes(fiv), int(g.seq0[gi])))
    return protos


def oracle_timed_check(wl, wire_last, len_last, n_launches, nthreads, budget_bytes=384 << 20):
    """The last timed step's output against the CPU oracle on a sample of chains: each
    sampled chain is sealed n_launches times in succession from its initial state (states
    carried, as the GPU's successive steps carry them) and its records of the last pass
    must equal the GPU's final wire arena and wire lengths.  The sample is spread over
    the batch and sized to ~budget_bytes of oracle plaintext.  -> (ok, chains sampled)."""
    from oracle import oracle as O
    per_chain = np.array([int(wl.pt_len[int(wl.chain_first[c]):int(wl.chain_first[c] + wl.chain_count[c])].sum())
                          for c in range(wl.n_chains)], dtype=np.int64)
    avg = max(1, int(per_chain.mean()) * max(1, n_launches))
    k = int(min(wl.n_chains, max(2, budget_bytes // avg), 256))
    idx = np.unique(np.linspace(0, wl.n_chains - 1, k).astype(np.int64))
    protos = oracle_protos(wl, idx)
    # the sampled chains' plaintext only (the arena's other bytes are never read)
    pt = np.zeros(wl.pt_bytes, dtype=np.uint8)
    for c in idx:
        a, b = int(wl.chain_first[c]), int(wl.chain_first[c] + wl.chain_count[c]) - 1
        if b < a:
            continue
        off = int(wl.pt_off[a])
        n = int(wl.pt_off[b]) + int(wl.pt_len[b]) - off
        pt[off:off + n] = O.fill_pattern(n, wl.seed, int(wl.chain_stream_start[c]))
    wire = np.zeros(wl.wire_bytes, dtype=np.uint8)
    lens = None
    for _ in range(n_launches):
        lens = O.seal_batch(protos, wl.chain_first[idx], wl.chain_count[idx], pt, wl.pt_off, wl.pt_len, wire,
                            wl.wire_off, nthreads=nthreads, update=True)
    for c in idx:
        for r in range(int(wl.chain_first[c]), int(wl.chain_first[c] + wl.chain_count[c])):
            o, L = int(wl.wire_off[r]), int(wl.wire_len[r])
            if int(lens[r]) != int(len_last[r]) or not np.array_equal(wire[o:o + L], wire_last[o:o + L]):
                return False, len(idx)
    return True, len(idx)


def oracle_check(wl, wire_gpu, nthreads, sample=None, min_seconds=0.0):
    """Seal the same workload with the CPU oracle; returns (bit_exact, seconds,
    records, plaintext bytes, threads, repetitions).  After the first (checked)
    pass the batch is sealed again -- connection states carried on, as the GPU
    steps do -- until min_seconds have been timed in total."""
    from oracle import oracle as O
    idx_chains = np.arange(wl.n_chains) if sample is None else sample
    protos = oracle_protos(wl, idx_chains)
    pt = wl.host_plaintext(O.fill_pattern)
    wire = np.zeros(wl.wire_bytes, dtype=np.uint8)
    t0 = time.perf_counter()
    wl_len = O.seal_batch(protos, wl.chain_first[idx_chains], wl.chain_count[idx_chains], pt, wl.pt_off, wl.pt_len,
                          wire, wl.wire_off, nthreads=nthreads)
    dt = time.perf_counter() - t0
    wire_first = wire.copy() if dt < min_seconds else wire
    reps = 1
    scratch = np.zeros_like(wire) if dt < min_seconds else None  # touched before the timed passes
    while dt < min_seconds:
        t0 = time.perf_counter()
        O.seal_batch(protos, wl.chain_first[idx_chains], wl.chain_count[idx_chains], pt, wl.pt_off, wl.pt_len,
                     scratch, wl.wire_off, nthreads=nthreads)
        dt += time.perf_counter() - t0
        reps += 1
    wire = wire_first
    recs = np.concatenate([np.arange(wl.chain_first[c], wl.chain_first[c] + wl.chain_count[c]) for c in idx_chains])
    ok = True
    for r in recs:
        o, L = int(wl.wire_off[r]), int(wl.wire_len[r])
        if int(wl_len[r]) != L:
            ok = False
            break
    if ok:
        mask = np.zeros(wl.wire_bytes, dtype=bool)
        if sample is None:
            ok = bool(np.array_equal(wire, wire_gpu))
        else:
            for r in recs:
                o, L = int(wl.wire_off[r]), int(wl.wire_len[r])
                if not np.array_equal(wire[o:o + L], wire_gpu[o:o + L]):
                    ok = False
                    break
        del mask
    return ok, dt, len(recs), int(wl.pt_len[recs].sum()) * reps, nthreads, reps


def oracle_wire(wl, nthreads):
    """The whole batch sealed by the CPU oracle from the initial states (wire arena)."""
    from oracle import oracle as O
    protos = oracle_protos(wl, np.arange(wl.n_chains))
    pt = wl.host_plaintext(O.fill_pattern)
    wire = np.zeros(wl.wire_bytes, dtype=np.uint8)
    O.seal_batch(protos, wl.chain_first, wl.chain_count, pt, wl.pt_off, wl.pt_len, wire, wl.wire_off,
                 nthreads=nthreads)
    return wire


def shard_parity(D, wl, wire_gpu, min_seconds=0.0):
    """Every rank checks its WHOLE shard (the batch it sealed) against the CPU oracle, with
    its share of the job's host cores (usable_cpus() // LOCAL_WORLD_SIZE); `bit_exact` is the
    AND over the ranks (an all-gather of the per-rank results).  min_seconds > 0 (rank 0 at
    N = 1) also times the oracle for cpu_baseline.  -> (bit_exact, per-rank results, threads,
    oracle_check's timing tuple)."""
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", D.world) or 1)
    nthreads = max(1, usable_cpus()[0] // max(1, local_world))
    ok, dt, nrec, ptb, th, reps = oracle_check(wl, wire_gpu, nthreads, min_seconds=min_seconds)
    oks = [bool(json.loads(b.decode())) for b in D.gather_bytes(json.dumps(bool(ok)).encode())]
    return all(oks), oks, nthreads, (dt, nrec, ptb, th, reps)


def pmc_traffic(path, workload, n_records, dominant):
    """(HBM bytes per launch of the dominant kernel, HBM bytes of one seal call) from a PMC
    summary (tools/pmc_kernels.sh -> profiles/pmc_<cfg>.json), only when it names this kernel
    and was collected on this very workload (name and record count: a PMC run of another
    batch size must not price this one); (None, None) otherwise."""
    if not os.path.exists(path):
        return None, None
    try:
        pj = json.load(open(path))
    except (OSError, ValueError):
        return None, None

    # kernel stems compared up to the first template argument (cbc_kernel<10> is the same
    # kernel as cbc_kernel<10, false>: the second argument is the round's form)
    def _key(k):
        return (k or "").split(",")[0].rstrip(">")
    if (_key(pj.get("dominant_kernel")) == _key(dominant) and pj.get("workload") == workload
            and pj.get("records") == n_records):
        return pj.get("hbm_bytes_per_launch"), pj.get("seal_call_hbm_bytes")
    return None, None


PCIE_GBS = 63.0  # MI355X_MICROARCH.md: host link PCIe Gen5 x16, 63 GB/s per direction (spec)


def pcie_rates(nbytes=256 << 20):
    """Measured pinned copy rates on this box with the HIP runtime directly (ctypes on
    libamdhip64, the engines the host pipeline uses): H2D alone, D2H alone, and both
    at once on two streams (GB/s; the last is the total of both directions).  Same
    method as tools/pcie_probe.hip.  Plus the host pipelines' other D2H path, the GPU's own
    stores (tlsgpu_host_store): alone (d2h_stores) and beside an H2D copy (both_stores)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    h1, h2, d1, d2, s1, s2 = vp(), vp(), vp(), vp(), vp(), vp()
    for ptr in (h1, h2):
        if hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(nbytes), 0):
            return None
    for ptr in (d1, d2):
        if hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(nbytes)):
            return None
    hip.hipStreamCreateWithFlags(ctypes.byref(s1), 1)
    hip.hipStreamCreateWithFlags(ctypes.byref(s2), 1)
    hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    res = {}
    from tlslite_amd import _native as N
    for name, mode in (("warm", 3), ("h2d", 1), ("d2h", 2), ("both", 3), ("d2h_stores", 6), ("both_stores", 7)):
        best = None  # "warm": untimed first copies; mode bit 2: the D2H copy by device stores
        for _ in range(6 if name != "warm" else 2):
            hip.hipDeviceSynchronize()
            t0 = time.perf_counter()
            if mode & 1:
                hip.hipMemcpyAsync(d1, h1, nbytes, 1, s1)
            if mode & 2:
                if mode & 4:
                    N.call("tlsgpu_host_store", h2, d2, nbytes, s2)
                else:
                    hip.hipMemcpyAsync(h2, d2, nbytes, 2, s2)
            hip.hipStreamSynchronize(s1)
            hip.hipStreamSynchronize(s2)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        if name != "warm":
            res[name] = round(nbytes * (2 if mode & 1 and mode & 2 else 1) / best / 1e9, 1)
    for ptr in (h1, h2):
        hip.hipHostFree(ptr)
    for ptr in (d1, d2):
        hip.hipFree(ptr)
    hip.hipStreamDestroy(s1)
    hip.hipStreamDestroy(s2)
    return res


def link_best(link):
    """(D2H GB/s, both-directions GB/s) of the better D2H path in pcie_rates' measurements."""
    return (max(link["d2h"], link.get("d2h_stores") or 0.0), max(link["both"], link.get("both_stores") or 0.0))


def host_inclusive_rate(wl, chunk=64 << 20, depth=3):
    """Plaintext GiB/s with the records starting and ending in HOST memory, through the
    C host pipeline (tlsgpu_host_pipeline_seal: H2D of plaintext, seal, D2H of the
    wire arena per sub-batch on three streams, `depth` sub-batches in flight), for pinned host arenas and
    for pageable ones (staged through the library's pinned buffers).  The wire output
    of both is compared with the device-resident path's.  Never `value`."""
    from tlslite_amd import _native as N
    from tlslite_amd.constants import ContentType
    from tlslite_amd.device import PinnedBuffer, synchronize
    from tlslite_amd.recordlayer import HostSealPipeline, make_chains, make_records
    if len(wl.launches) != 1:
        return None
    var = wl.launches[0][0]
    recs = make_records(wl.pt_off, wl.wire_off, wl.pt_len, ContentType.application_data, 0)
    chains = make_chains(np.arange(wl.n_chains, dtype=np.uint32), wl.chain_first, wl.chain_count)
    # reference output: the device-resident path from the initial states
    wl.reset_states()
    wl.launch()
    synchronize()
    ref = wl.d_wire.download()
    pin_pt, pin_wire = PinnedBuffer(wl.pt_bytes), PinnedBuffer(wl.wire_bytes)
    wl.d_pt.download(out=pin_pt.array[: wl.pt_bytes])
    pag_pt, pag_wire = pin_pt.array[: wl.pt_bytes].copy(), np.zeros(wl.wire_bytes, dtype=np.uint8)
    lens = np.zeros(wl.n_records, dtype=np.int32)
    link = pcie_rates()
    if link:
        # both directions at once share the link: the copies need at least
        # max(H2D bytes / H2D rate, D2H bytes / D2H rate, all bytes / both-at-once rate),
        # the D2H rates the better of the pipeline's two D2H paths
        d2h, both = link_best(link)
        t_min = max(wl.pt_bytes / (link["h2d"] * 1e9), wl.wire_bytes / (d2h * 1e9),
                    (wl.pt_bytes + wl.wire_bytes) / (both * 1e9))
        how = "measured pinned copy rates on this box (pcie_measured_gbs; D2H: copy engine or device stores)"
    else:
        t_min = max(wl.pt_bytes, wl.wire_bytes) / (PCIE_GBS * 1e9)
        how = "63 GB/s per direction, full duplex (spec)"
    out = {"unit": "GiB/s", "chunk_bytes": chunk, "depth": depth,
           "bytes_h2d": int(wl.pt_bytes), "bytes_d2h": int(wl.wire_bytes),
           "pcie_measured_gbs": link,
           "pcie_ceiling": round(wl.plaintext_total / GIB / t_min, 2),
           "method": "tlsgpu_host_pipeline_seal: per sub-batch of ~chunk_bytes plaintext H2D copy, seal, D2H copy "
                     "of its wire range on four event-chained streams (H2D, MAC phase, cipher phase, D2H), `depth` "
                     "sub-batches in flight; wall time of "
                     "the synchronous call, best of 3; pcie_ceiling = plaintext / the copies' minimum time at " + how}
    with HostSealPipeline(chunk, depth) as hp:
        for name, pt_h, wire_h in (("pinned", pin_pt.array[: wl.pt_bytes], pin_wire.array[: wl.wire_bytes]),
                                   ("pageable", pag_pt, pag_wire)):
            progress("host-inclusive seal, %s arenas" % name)
            best = None
            for _rep in range(3):
                wl.reset_states()
                synchronize()
                t0 = time.perf_counter()
                hp.seal(chains, recs, pt_h, wire_h, wl.d_states, lens, var)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            exact = bool(np.array_equal(wire_h, ref)) and bool(np.array_equal(lens, wl.wire_len.astype(np.int32)))
            out[name] = {"value": round(wl.plaintext_total / GIB / best, 2), "ms": round(best * 1e3, 3),
                         "bit_exact": exact}
        out["d2h_path"] = hp.d2h_path
    out["value"] = out["pinned"]["value"]
    out["pcie_frac"] = round(out["value"] / out["pcie_ceiling"], 3)
    pin_pt.free()
    pin_wire.free()
    return out


def compact_rx(wl):
    """The sealed batch as connections' received bytes: each connection's wire records back to
    back (what its socket delivers) in one host arena, connections one after another.  ->
    (arena, per-connection offsets and lengths, per-record body offsets in the arena)."""
    lens = wl.wire_len.astype(np.int64)
    n_conn = wl.n_chains
    conn_bytes = np.array([int(lens[int(f):int(f) + int(c)].sum()) for f, c in zip(wl.chain_first, wl.chain_count)],
                          dtype=np.int64)
    conn_off = np.concatenate([[0], np.cumsum(conn_bytes)[:-1]]).astype(np.int64)
    rec_pos = np.empty(wl.n_records, dtype=np.int64)  # record r's header in the compact arena
    for c in range(n_conn):
        f, k = int(wl.chain_first[c]), int(wl.chain_count[c])
        rec_pos[f:f + k] = conn_off[c] + np.concatenate([[0], np.cumsum(lens[f:f + k])[:-1]])
    return conn_off, conn_bytes, rec_pos


def host_open_rate(wl, link=None, chunk=64 << 20, depth=3):
    """Open with the records starting in HOST socket buffers and the plaintext ending there
    (tlsgpu_host_pipeline_open: H2D of the received bytes, framing and open on the device, D2H
    of the plaintext, sub-batches of ~chunk bytes overlapped), pinned and pageable host arenas;
    every status and every record's plaintext checked.  Wall time of the synchronous call, best
    of 3.  One-variant batches only.  Never `value`."""
    from tlslite_amd import _native as N
    from tlslite_amd.device import PinnedBuffer, synchronize
    from tlslite_amd.recordlayer import HostSealPipeline
    if len(wl.launches) != 1:
        return None
    var = wl.launches[0][0]
    wl.reset_states()
    wl.launch()
    synchronize()
    wire = wl.d_wire.download()
    ref_pt = wl.d_pt.download()
    conn_off, conn_bytes, rec_pos = compact_rx(wl)
    nbytes = int(conn_bytes.sum())
    pin_rx, pin_pt = PinnedBuffer(nbytes), PinnedBuffer(nbytes)
    rx = pin_rx.array[:nbytes]
    lens = wl.wire_len.astype(np.int64)
    for r in range(wl.n_records):  # the received bytes: each record where its connection's stream has it
        a, w = int(rec_pos[r]), int(wl.wire_off[r])
        rx[a:a + lens[r]] = wire[w:w + lens[r]]
    del wire
    spans = (N.Span * wl.n_chains)()
    sp = np.frombuffer(spans, dtype=np.uint8).reshape(wl.n_chains, 16)
    sp[:, 0:8] = conn_off.astype(np.uint64).reshape(-1, 1).view(np.uint8)
    sp[:, 8:12] = conn_bytes.astype(np.uint32).reshape(-1, 1).view(np.uint8)
    sp[:, 12:16] = np.arange(wl.n_chains, dtype=np.uint32).reshape(-1, 1).view(np.uint8)
    link = link or pcie_rates()
    if link:
        d2h, both = link_best(link)
        t_min = max(nbytes / (link["h2d"] * 1e9), nbytes / (d2h * 1e9), 2 * nbytes / (both * 1e9))
        how = "measured pinned copy rates on this box (pcie_measured_gbs; D2H: copy engine or device stores)"
    else:
        t_min = nbytes / (PCIE_GBS * 1e9)
        how = "63 GB/s per direction, full duplex (spec)"
    out = {"unit": "GiB/s", "chunk_bytes": chunk, "depth": depth, "bytes_h2d": nbytes, "bytes_d2h": nbytes,
           "pcie_measured_gbs": link, "pcie_ceiling": round(wl.plaintext_total / GIB / t_min, 2),
           "method": "tlsgpu_host_pipeline_open: each connection's received records back to back in a host "
                     "arena; per sub-batch of ~chunk_bytes an H2D copy, framing (as tlsgpu_frame_dev) and open "
                     "(as tlsgpu_open_dev) on the device, a D2H copy of the plaintext range, descriptors and "
                     "statuses, `depth` sub-batches in flight; wall time of the synchronous call, best of 3; "
                     "pcie_ceiling = plaintext / the copies' minimum time at " + how}
    body = rec_pos + 5
    want_st = wl.pt_len.astype(np.int32)
    recs_out = {"records": (N.OpenRecord * (wl.n_records + 1))(), "status": np.zeros(wl.n_records + 1, np.int32)}
    with HostSealPipeline(chunk, depth) as hp:
        for name, rx_h, pt_h in (("pinned", rx, pin_pt.array[:nbytes]), ("pageable", rx.copy(), None)):
            if pt_h is None:
                pt_h = np.zeros(nbytes, dtype=np.uint8)
            progress("host-inclusive open, %s arenas" % name)
            best = None
            for _rep in range(3):
                N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, None)
                synchronize()
                t0 = time.perf_counter()
                res = hp.open(rx_h, spans, pt_h, wl.d_ostates, var, max_records=wl.n_records + 1, out=recs_out)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            exact = res["total"] == wl.n_records and bool(np.array_equal(res["status"], want_st))
            if exact:
                got = np.frombuffer(res["records"], dtype=np.uint8).reshape(-1, 24)[: wl.n_records]
                exact = bool(np.array_equal(got[:, 0:8].copy().view(np.uint64).ravel(), body.astype(np.uint64)))
            if exact:
                for r in range(wl.n_records):
                    a, b, k = int(body[r]), int(wl.pt_off[r]), int(wl.pt_len[r])
                    if not np.array_equal(pt_h[a:a + k], ref_pt[b:b + k]):
                        exact = False
                        break
            out[name] = {"value": round(wl.plaintext_total / GIB / best, 2), "ms": round(best * 1e3, 3),
                         "roundtrip_exact": exact}
        out["d2h_path"] = hp.d2h_path
    out["value"] = out["pinned"]["value"]
    out["pcie_frac"] = round(out["value"] / out["pcie_ceiling"], 3)
    pin_rx.free()
    pin_pt.free()
    return out


def gpu_warm(call, sync, min_ms=40.0, max_calls=400):
    """Untimed calls back to back (synchronised every 4) until min_ms of them have run: a side leg
    measured after seconds of host work would otherwise time a GPU waking from its idle clock
    ("Short runs")."""
    t0 = time.perf_counter()
    n = 0
    while n < max_calls and (time.perf_counter() - t0) * 1e3 < min_ms:
        for _ in range(4):
            call()
        n += 4
        sync()
    return n


def open_rate(wl, stream, steps):
    """Open path on the batch: seal once from the initial states, then open it
    with read states reset to the initial ones before every (timed) call."""
    from tlslite_amd import _native as N
    from tlslite_amd.device import Event, Stream
    wl.reset_states(stream)
    wl.launch([stream])
    wl.open_setup()
    wl.open_launch(stream)
    stream.synchronize()
    status = wl.d_ostatus.download().view(np.int32)
    ok = bool(np.array_equal(status, wl.pt_len.astype(np.int32)))
    if ok:
        ok = wl.opened_plaintext_matches()
    ms = []
    # RC4 / 3DES-only batches (cfg5): the variants open concurrently on two streams, as their
    # seal does; timed by the host clock around both streams (states reset beforehand)
    conc = None if wl.uses_split_pipeline() else [Stream(high=True), Stream(high=False)]  # separate HW queues

    def warm_call():
        N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, stream.handle)
        wl.open_launch(stream, reset=False)

    gpu_warm(warm_call, stream.synchronize)
    for _ in range(max(1, min(steps, 20))):
        N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, stream.handle)
        if conc:
            stream.synchronize()
            t0 = time.perf_counter()
            wl.open_launch(reset=False, streams=conc)
            for s_ in conc:
                s_.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
            continue
        a, b = Event(), Event()
        a.record(stream)
        wl.open_launch(stream, reset=False)
        b.record(stream)
        stream.synchronize()
        ms.append(a.elapsed_ms(b))
    if conc:  # the concurrent calls' output is checked too
        status = wl.d_ostatus.download().view(np.int32)
        ok = ok and bool(np.array_equal(status, wl.pt_len.astype(np.int32))) and wl.opened_plaintext_matches()
    t = float(np.median(ms))
    out = {"value": round(wl.plaintext_total / GIB / (t / 1e3), 2), "unit": "GiB/s", "ms": round(t, 4),
           "roundtrip_exact": ok,
           "method": "tlsgpu_open_dev over the sealed batch (AES / 3DES: block-parallel CBC decrypt, per-chain "
                     "padding/seqnum pass, per-record MAC verify; RC4: lane per connection); median of "
                     "HIP-event-timed calls (RC4/3DES-only batches: variants on two streams, host-timed)"}
    return out


def device_free_bytes():
    """Free memory of the current device (hipMemGetInfo), 0 if the call fails."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    if hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)):
        return 0
    return int(free.value)


def open_concurrent_rate(wl, calls, nstreams=2, D=None, ranks_per_device=1):
    """Successive independent open calls (each against its own copy of the initial read
    states: batches of different connections) issued round-robin on `nstreams` streams of
    different priorities, so one call's MAC pass can run beside the next call's decrypt;
    wall time from the first call to the last stream's synchronize.  Every call's status and
    each stream's plaintext arena are checked.  With D (N > 1 ranks) every rank must call it:
    the timed section is bracketed by barriers (each rank's wall time covers the same interval
    of the job), reached by every rank whatever fails (errors are reported, not raised)."""
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, Stream, synchronize
    from tlslite_amd.recordlayer import open_dev, open_workspace_bytes
    err, bufs = None, []
    try:
        # every call has its own copy of the read states: at most a quarter of this rank's
        # share of the free device memory (ranks sharing a GPU split it)
        budget = device_free_bytes() // max(1, ranks_per_device) // 4
        calls = max(nstreams, min(int(calls), max(nstreams, int(budget // max(1, wl.d_states0.nbytes)))))
        streams = [Stream(high=(i == 0)) for i in range(nstreams)]
        states = [DeviceBuffer(wl.d_states0.nbytes) for _ in range(calls)]
        for st in states:
            N.call("tlsgpu_memcpy_d2d", st.ptr, wl.d_states0.ptr, st.nbytes, None)
        pts = [wl.d_opt] + [DeviceBuffer(wl.d_opt.nbytes) for _ in range(nstreams - 1)]
        wss = [[DeviceBuffer(max(open_workspace_bytes(wl.n_records), 16)) for _ in wl.launches]
               for _ in range(nstreams)]
        stat = [DeviceBuffer(4 * wl.n_records) for _ in range(calls)]
        bufs = states + stat + pts[1:] + [w for ws in wss for w in ws]
        synchronize()
    except Exception as e:  # reported after the collective below
        err = e
    ready = (err is None) if D is None else D.sum(0.0 if err is None else 1.0) == 0.0
    if not ready:
        for b in bufs:
            b.free()
        return (leg_error(err) if err is not None else
                {"error": "another rank could not prepare the concurrent opens"})
    if err is None:  # untimed opens first (their outputs are overwritten by the timed calls)
        try:
            def warm_call():  # on fresh read states each time (a call on advanced ones would alert)
                N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, streams[0].handle)
                for j, (var, d_ch, nch) in enumerate(wl.launches):
                    open_dev(d_ch, nch, wl.d_orecs, wl.n_records, wl.d_wire, pts[0], wl.d_ostates, stat[0], var,
                             wss[0][j], streams[0])
            gpu_warm(warm_call, streams[0].synchronize)
            for _ in range(4):  # still running while the ranks meet below
                warm_call()
        except Exception as e:
            err = e
    if D is not None:
        D.barrier()
    for s_ in streams:
        s_.synchronize()
    t0 = time.perf_counter()
    try:
        for k in range(calls):
            if err is not None:
                break
            i = k % nstreams
            for j, (var, d_ch, nch) in enumerate(wl.launches):
                open_dev(d_ch, nch, wl.d_orecs, wl.n_records, wl.d_wire, pts[i], states[k], stat[k], var, wss[i][j],
                         streams[i])
        for s_ in streams:
            s_.synchronize()
    except Exception as e:
        err = e
    if D is not None:
        D.barrier()
    t = time.perf_counter() - t0
    ok = False
    if err is None:
        want = wl.pt_len.astype(np.int32)
        ok = all(bool(np.array_equal(x.download().view(np.int32), want)) for x in stat)
        saved = wl.d_opt
        try:
            for p_ in pts:
                wl.d_opt = p_
                ok = ok and wl.opened_plaintext_matches()
        finally:
            wl.d_opt = saved
    for b in bufs:
        b.free()
    if err is not None:
        return leg_error(err)
    ms = t / calls * 1e3
    return {"value": round(wl.plaintext_total / GIB / (ms / 1e3), 2), "ms": round(ms, 4), "calls": calls,
            "streams": nstreams, "roundtrip_exact": ok,
            "method": "independent opens of the sealed batch (each against its own copy of the read states) issued "
                      "round-robin on %d streams; wall time / calls%s" %
                      (nstreams, ", between barriers over all ranks" if D is not None else "")}


def frame_rate(wl, stream, steps):
    """Receive framing on the device (tlsgpu_frame_dev) for a batch of one-record connections
    (cfg2 / cfg3 shapes): each connection's received bytes are its wire record (header +
    body) in the sealed wire arena.  The framed descriptors must equal the batch's own (body
    offset, length, content type; one chain per connection); then the same batch is opened
    from them (status = every record's plaintext length).  Median of HIP-event-timed frame
    calls, and of frame + open calls.  None for other shapes."""
    import ctypes
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, Event
    from tlslite_amd.recordlayer import frame_dev, frame_workspace_bytes, open_dev
    if len(wl.launches) != 1 or not bool((wl.chain_count == 1).all()):
        return None
    var, _, nch = wl.launches[0]
    n = wl.n_chains
    first = wl.chain_first.astype(np.int64)
    spans = np.zeros((n, 2), dtype=np.uint64)
    spans[:, 0] = wl.wire_off[first]
    sp32 = spans.view(np.uint32).reshape(n, 4)
    sp32[:, 2] = wl.wire_len[first].astype(np.uint32)
    sp32[:, 3] = np.arange(n, dtype=np.uint32)
    d_sp = DeviceBuffer(spans.nbytes)
    d_sp.upload(spans.view(np.uint8).reshape(-1))
    d_r = DeviceBuffer(n * ctypes.sizeof(N.OpenRecord))
    d_c, d_cons, d_st, d_tot = DeviceBuffer(16 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(16)
    ws = DeviceBuffer(frame_workspace_bytes(n))
    d_ost, d_ows = DeviceBuffer(4 * n), DeviceBuffer(wl.d_ows[0].nbytes)
    fms, foms = [], []

    def warm_call():
        N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, stream.handle)
        frame_dev(wl.d_wire, d_sp, n, d_r, n, d_c, d_cons, d_st, d_tot, workspace=ws, s=stream)
        open_dev(d_c, n, d_r, n, wl.d_wire, wl.d_opt, wl.d_ostates, d_ost, var, d_ows, stream)

    gpu_warm(warm_call, stream.synchronize)
    for it in range(max(2, min(steps, 20)) + 1):
        a, b, c = Event(), Event(), Event()
        N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, stream.handle)
        a.record(stream)
        frame_dev(wl.d_wire, d_sp, n, d_r, n, d_c, d_cons, d_st, d_tot, workspace=ws, s=stream)
        b.record(stream)
        open_dev(d_c, n, d_r, n, wl.d_wire, wl.d_opt, wl.d_ostates, d_ost, var, d_ows, stream)
        c.record(stream)
        stream.synchronize()
        if it:
            fms.append(a.elapsed_ms(b))
            foms.append(a.elapsed_ms(c))
    recs = np.frombuffer(d_r.download(), dtype=np.uint8).reshape(n, ctypes.sizeof(N.OpenRecord))
    ct_off = recs[:, 0:8].copy().view(np.uint64).ravel()
    ct_len = recs[:, 16:20].copy().view(np.uint32).ravel()
    ch = d_c.download().view(np.uint32).reshape(n, 4)
    exact = (int(d_tot.download()[:4].view(np.uint32)[0]) == n
             and bool(np.array_equal(d_st.download().view(np.int32), np.ones(n, dtype=np.int32)))
             and bool(np.array_equal(ct_off, (wl.wire_off[first] + 5).astype(np.uint64)))
             and bool(np.array_equal(ct_len, (wl.wire_len[first] - 5).astype(np.uint32)))
             and bool(np.array_equal(recs[:, 20], wl.rec_ctype[first].astype(np.uint8) if np.ndim(wl.rec_ctype)
                                     else np.full(n, wl.rec_ctype, dtype=np.uint8)))
             and bool(np.array_equal(ch[:, 1], np.arange(n, dtype=np.uint32)))
             and bool(np.array_equal(ch[:, 2], np.ones(n, dtype=np.uint32))))
    opened = bool(np.array_equal(d_ost.download().view(np.int32), wl.pt_len[first].astype(np.int32)))
    for buf in (d_sp, d_r, d_c, d_cons, d_st, d_tot, ws, d_ost, d_ows):
        buf.free()
    tf, tfo = float(np.median(fms)), float(np.median(foms))
    return {"records": n, "ms": round(tf, 4), "records_per_s": round(n / (tf / 1e3)),
            "frame_exact": exact, "open_from_frames_ms": round(tfo, 4),
            "open_from_frames_value": round(wl.plaintext_total / GIB / (tfo / 1e3), 2), "open_from_frames_exact": opened,
            "method": "tlsgpu_frame_dev over each connection's received record in the sealed wire arena, then "
                      "tlsgpu_open_dev on the framed descriptors; medians of HIP-event-timed calls"}


def leg_error(e):
    """A side leg's failure as its JSON field.  hip_error marks a failed HIP call (TLSGPU_EHIP:
    a fault such as an illegal memory access leaves the device context dead): the run then
    ends with a non-zero exit status after its line is printed (hip_failures)."""
    from tlslite_amd import _native as N
    return {"error": str(e), "hip_error": getattr(e, "code", None) == N.EHIP}


def hip_failures(legs):
    """Names of the legs (dict name -> result) that hit a HIP error on any rank."""
    def bad(r):
        if isinstance(r, dict):
            return bool(r.get("hip_error")) or any(bad(v) for v in r.values())
        if isinstance(r, list):
            return any(bad(v) for v in r)
        return False
    return [k for k, r in legs.items() if bad(r)]


def _leg_ranks(D, res, leg):
    """Every rank's result of a side leg (rank order), or an error naming the failed ranks."""
    ranks = [json.loads(b.decode()) for b in D.gather_bytes(json.dumps(res).encode())]
    bad = [i for i, r in enumerate(ranks) if r is None or "error" in r]
    return ranks, ({"error": "%s leg failed on rank(s) %s" % (leg, bad), "ranks": ranks} if bad else None)


def open_over_ranks(D, res, plaintext_bytes, shared=False):
    """The open leg at N > 1: every rank opened its own shard (after a barrier, so at the
    same time); the job's rate is all ranks' plaintext / the slowest rank's median call time,
    `roundtrip_exact` the AND over ranks, and each rank's own figure is listed."""
    ranks, err = _leg_ranks(D, res, "open")
    total = D.sum(float(plaintext_bytes))
    if err:
        return err
    # One metric at every N: value = all ranks' plaintext / the slowest rank's
    # median call time, as at N = 1.  The wall-clock rate of successive concurrent calls
    # (open_concurrent_rate) is aggregated the same way into `concurrent_value`; on GPUs shared
    # by several ranks (--share-devices rehearsals) the per-call medians include the other
    # ranks' work, and the concurrent figure is the one that reads as the job's rate.
    t = max(float(r["ms"]) for r in ranks)
    wall = all("ms" in (r.get("concurrent") or {}) for r in ranks)
    out = dict(ranks[0])
    out.update({"value": round(total / GIB / (t / 1e3), 2), "ms": round(t, 4),
                "roundtrip_exact": all(bool(r["roundtrip_exact"]) and
                                       bool(r.get("concurrent", {}).get("roundtrip_exact", True)) for r in ranks),
                "ranks": [{"value": r["value"], "ms": r["ms"], "roundtrip_exact": r["roundtrip_exact"],
                           "concurrent_ms": (r.get("concurrent") or {}).get("ms")} for r in ranks],
                "aggregate": "sum of the ranks' plaintext bytes / the slowest rank's median call time (as at N = 1)"})
    if wall:
        tc = max(float(r["concurrent"]["ms"]) for r in ranks)
        out["concurrent_value"] = round(total / GIB / (tc / 1e3), 2)
        out["concurrent_aggregate"] = ("sum of the ranks' plaintext bytes / the slowest rank's wall time per call "
                                       "over its successive concurrent calls")
        if shared:
            # ranks sharing a GPU: their timed calls overlap only in part, so per-call medians
            # overstate the job's rate; the barrier-bracketed wall-clock runs are the job's rate
            out["per_call_value"] = out["value"]
            out["value"], out["ms"] = out["concurrent_value"], round(tc, 4)
            out["aggregate"] = "devices shared by ranks (a rehearsal): " + out["concurrent_aggregate"]
    return out


def derive_over_ranks(D, res, shared=False):
    """The derive leg at N > 1: every rank derived its own 4,096 connections at the same time;
    the job's rate is all ranks' connections / the slowest rank's median call time."""
    ranks, err = _leg_ranks(D, res, "derive")
    if err:
        return err
    t = max(float(r["ms"]) for r in ranks)
    n = sum(int(r["connections"]) for r in ranks)
    out = dict(ranks[0])
    out.update({"connections": n, "ms": round(t, 4), "conns_per_s": round(n / (t / 1e3)),
                "key_blocks_exact_sample": all(bool(r["key_blocks_exact_sample"]) for r in ranks),
                "ranks": [{"ms": r["ms"], "key_blocks_exact_sample": r["key_blocks_exact_sample"]} for r in ranks],
                "aggregate": "sum of the ranks' connections / the slowest rank's median call time"})
    if shared:
        # ranks sharing a GPU time their calls at different moments: the sum above overstates the
        # job's rate; the rate if the ranks' calls ran one after another is its lower bound
        out["conns_per_s_serialised"] = round(n / (sum(float(r["ms"]) for r in ranks) / 1e3))
        out["aggregate"] += " (devices shared by ranks, a rehearsal: an upper bound; conns_per_s_serialised is " \
                            "the lower bound)"
    return out


def host_inclusive_over_ranks(D, res, plaintext_bytes):
    """The host-inclusive leg at N > 1 (each rank's GPU on its own link): all ranks' plaintext /
    the slowest rank's best pinned call; bit_exact the AND over ranks and both arena kinds."""
    ranks, err = _leg_ranks(D, res, "host-inclusive")
    total = D.sum(float(plaintext_bytes))
    if err:
        return err
    t = max(float(r["pinned"]["ms"]) for r in ranks)
    out = dict(ranks[0])
    out.update({"value": round(total / GIB / (t / 1e3), 2),
                "bit_exact": all(bool(r[k]["bit_exact"]) for r in ranks for k in ("pinned", "pageable")),
                "ranks": [{"value": r["value"], "pinned_ms": r["pinned"]["ms"],
                           "bit_exact": bool(r["pinned"]["bit_exact"] and r["pageable"]["bit_exact"])} for r in ranks],
                "aggregate": "sum of the ranks' plaintext bytes / the slowest rank's best pinned call"})
    out.pop("pcie_frac", None)
    return out


def derive_rate(stream, nconn=4096, steps=10):
    """Batched _calcPendingStates (tlsgpu_derive_states_dev) for cfg4's 4096
    connections: master secret -> key block (TLS 1.2 PRF_1_2) -> pending
    write/read states in HBM.  A sample of key blocks is checked against
    the CPU oracle's PRF."""
    import ctypes
    from tlslite_amd import _native as N
    from tlslite_amd.constants import SUITE_NAMES
    from tlslite_amd.device import DeviceBuffer, Event
    rng = np.random.default_rng(4)
    descs = (N.DeriveDesc * nconn)()
    raw = np.frombuffer(descs, dtype=np.uint8).reshape(nconn, ctypes.sizeof(N.DeriveDesc))
    raw[:, :128] = rng.integers(0, 256, size=(nconn, 128), dtype=np.uint8)
    for d in descs:
        d.suite, d.ver_major, d.ver_minor, d.client = SUITE_NAMES["AES128-SHA"], 3, 3, 1
    dd = DeviceBuffer(ctypes.sizeof(descs))
    dd.upload(bytes(descs))
    ws, rs = DeviceBuffer(nconn * N.CONN_STATE_BYTES), DeviceBuffer(nconn * N.CONN_STATE_BYTES)
    kb, st = DeviceBuffer(nconn * N.KEY_BLOCK_MAX), DeviceBuffer(4 * nconn)
    ms = []
    gpu_warm(lambda: N.call("tlsgpu_derive_states_dev", dd.ptr, nconn, ws.ptr, rs.ptr, None, kb.ptr, st.ptr,
                            stream.handle), stream.synchronize)
    for it in range(steps + 1):
        a, b = Event(), Event()
        a.record(stream)
        N.call("tlsgpu_derive_states_dev", dd.ptr, nconn, ws.ptr, rs.ptr, None, kb.ptr, st.ptr, stream.handle)
        b.record(stream)
        stream.synchronize()
        if it:
            ms.append(a.elapsed_ms(b))
    status = st.download().view(np.int32)
    kbs = kb.download().reshape(nconn, N.KEY_BLOCK_MAX)
    exact = bool((status == 0).all())
    from oracle import oracle as O  # parity checker only
    for i in rng.choice(nconn, 16, replace=False):
        ref, _ = O.key_block((3, 3), "AES128-SHA", raw[i, :48].tobytes(), raw[i, 48:80].tobytes(),
                             raw[i, 80:112].tobytes())
        exact = exact and kbs[i, :len(ref)].tobytes() == ref
    t = float(np.median(ms))
    return {"connections": nconn, "ms": round(t, 4), "conns_per_s": round(nconn / (t / 1e3)),
            "key_blocks_exact_sample": exact,
            "method": "tlsgpu_derive_states_dev: TLS 1.2 PRF_1_2 key block + slicing + AES-128 key schedule + "
                      "HMAC-SHA1 midstates, one lane per connection; median of HIP-event-timed calls"}


def copy_rate(wl, stream, reps=5):
    """HBM copy rate of this GPU (GB/s, read + write bytes): device-to-device copies of
    the wire arena, HIP events on one stream, best of `reps` -- what a kernel that only
    streams its bytes could reach (the fraction of the measured copy rate
    beside the 8 TB/s spec fraction)."""
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, Event
    n = min(wl.wire_bytes, 1 << 30)
    dst = DeviceBuffer(n)
    best = None
    for _ in range(reps):
        a, b = Event(), Event()
        a.record(stream)
        N.call("tlsgpu_memcpy_d2d", dst.ptr, wl.d_wire.ptr, n, stream.handle)
        b.record(stream)
        stream.synchronize()
        ms = a.elapsed_ms(b)
        best = ms if best is None or ms < best else best
    dst.free()
    return 2.0 * n / (best / 1e3) / 1e9


def probe_device_count():
    """GPUs visible to libtlsgpu.so, counted in a child process so that this process
    touches no GPU before it spawns the ranks."""
    import subprocess
    code = "import sys; sys.path.insert(0, %r); from tlslite_amd.device import device_count; print(device_count())" % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise SystemExit("bench.py: device probe failed: %s" % r.stderr[-2000:])
    return int(r.stdout.strip().splitlines()[-1])


def pinned_visibility(env, local_rank, ndev):
    """The visibility setting that leaves a rank only its own GPU: (variable, value), the
    local_rank-th entry of the list HIP already applies (HIP_VISIBLE_DEVICES, else
    CUDA_VISIBLE_DEVICES, which HIP also honours), or HIP_VISIBLE_DEVICES = local_rank when
    neither is set.  None when the node has fewer GPUs than that rank needs."""
    if local_rank >= ndev:
        return None
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None and v.strip():
            ids = [x.strip() for x in v.split(",") if x.strip()]
            return (var, ids[local_rank]) if local_rank < len(ids) else None
    return ("HIP_VISIBLE_DEVICES", str(local_rank))


def pin_rank_device(args, D):
    """One process per GPU, each seeing only its own.  With N > 1 ranks on a node with a GPU
    for every local rank (no --share-devices), rank i narrows HIP's visible devices to the
    i-th one before this process makes any GPU call (the count comes from a child process),
    so every rank drives device 0 of its own view: the library's per-device state (LDS
    attributes, CU counts, owned workspaces, the split open's second streams) is only used on
    device 0, the configuration the one-GPU box tests.  TLSGPU_PIN_DEVICE=0 turns it off,
    =1 forces it at N = 1 too.  Returns "VAR=value" as set, or None."""
    force = os.environ.get("TLSGPU_PIN_DEVICE")
    if force == "0" or args.share_devices or os.environ.get("TLSGPU_SHARE_DEVICES") == "1":
        return None
    if D.world <= 1 and force != "1":
        return None
    pv = pinned_visibility(os.environ, D.local, probe_device_count())
    if pv is None:
        return None  # main() refuses the run (too few GPUs), as without pinning
    os.environ[pv[0]] = pv[1]
    return "%s=%s" % pv


def spawn_ranks(args):
    """--gpus N > 1 without a launcher: one child process per rank (RANK = LOCAL_RANK = i,
    WORLD_SIZE = N, a free rendezvous port on 127.0.0.1), started before this process
    makes any GPU call.  Returns the exit code: non-zero if any rank fails (the others are
    then terminated)."""
    import socket
    import subprocess
    ndev = int(os.environ.get("TLSGPU_DRYRUN_DEVICES", args.gpus)) if args.dry_run else probe_device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible to libtlsgpu.so")
    if args.gpus > ndev and not args.share_devices:
        raise SystemExit("bench.py: --gpus %d but only %d GPU(s) visible; pass --share-devices to run %d ranks on "
                         "them round-robin (a rehearsal, not a scaling measurement)" % (args.gpus, ndev, args.gpus))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    token = os.urandom(8).hex()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TLSGPU_RDZV_PORT=str(port), TLSGPU_RDZV_TOKEN=token)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    import time as _t
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print("bench.py: rank %d exited with %d; stopping the others" % (procs.index(p), code), file=sys.stderr)
                for q in live:
                    q.terminate()
        _t.sleep(0.05)
    return rc


def dry_run(args, D):
    """--dry-run: the N-rank plumbing without the GPU (CPU tests of the spawner).  With
    --records R every rank also runs the shard parity check (shard_parity) on an R-record
    cfg2-shaped batch whose "GPU output" is the oracle's own wire arena -- one byte of it
    flipped on the rank named by TLSGPU_DRYRUN_CORRUPT_RANK -- so the AND over ranks is
    exercised without a GPU."""
    from tlslite_amd.shard import device_for_rank
    ndev = int(os.environ.get("TLSGPU_DRYRUN_DEVICES", max(D.world, 1)))
    if D.world > ndev and not args.share_devices:
        raise SystemExit("bench.py: %d ranks but only %d GPU(s) visible" % (D.world, ndev))
    if os.environ.get("TLSGPU_DRYRUN_FAIL_RANK") == str(D.rank):
        sys.exit(3)
    me = {"rank": D.rank, "local_rank": D.local, "device": device_for_rank(D.local, ndev), "pid": os.getpid()}
    ranks = [json.loads(b) for b in D.gather_bytes(json.dumps(me).encode())]
    t = D.max(0.001 * (1 + D.rank))
    parity = None
    if args.records:
        from tlslite_amd import workloads as W
        wl = W.cfg2(n=int(args.records), pt_len=1500 + 16 * D.rank, seed=7 + D.rank)  # each rank its own batch
        wire = oracle_wire(wl, 1)
        if os.environ.get("TLSGPU_DRYRUN_CORRUPT_RANK") == str(D.rank):
            wire[int(wl.wire_off[len(wl.wire_off) // 2]) + 9] ^= 0x40
        ok, oks, nthreads, _ = shard_parity(D, wl, wire)
        parity = {"bit_exact": ok, "bit_exact_ranks": oks, "threads_per_rank": nthreads}
    if D.rank == 0:
        print(json.dumps({"metric": "dry-run", "n_gpus": D.world, "ranks": ranks, "t_max": t,
                          "devices_shared": D.world > ndev, "parity": parity}))
    D.close()


def progress(msg):
    """Phase markers on stderr: a long run (cfg4's 16 GiB oracle checks) keeps writing."""
    print("bench.py [%s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    from tlslite_amd.shard import ShardGroup, device_for_rank
    D = ShardGroup()
    if D.world != args.gpus:
        print("bench.py: WORLD_SIZE %d from the launcher, --gpus %d: running %d ranks" % (D.world, args.gpus, D.world),
              file=sys.stderr)
    if args.dry_run:
        return dry_run(args, D)
    pinned = pin_rank_device(args, D)  # before the first GPU call of this process
    from tlslite_amd import _native as N
    from tlslite_amd.device import Event, Stream, set_device, synchronize, device_count, arch
    ndev = device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible to libtlsgpu.so")
    shared = pinned is None and D.world > ndev
    if shared and not args.share_devices and os.environ.get("TLSGPU_SHARE_DEVICES") != "1":
        raise SystemExit("bench.py: %d ranks but only %d GPU(s) visible; pass --share-devices to share them "
                         "round-robin (a rehearsal, not a scaling measurement)" % (D.world, ndev))
    dev = 0 if pinned else device_for_rank(D.local, ndev)
    set_device(dev)
    dev_arch = arch(dev)
    progress("rank %d/%d on device %d%s: building %s" % (D.rank, D.world, dev,
                                                        " (%s)" % pinned if pinned else "", args.config))
    pins = D.gather_bytes((pinned or "").encode()) if D.world > 1 else [(pinned or "").encode()]
    wl = build_workload(args.config, D.rank, D.world, args.records, args.pt_align)
    stream = Stream()
    wl.to_device(stream)
    stream.synchronize()

    # ---- one launch for the parity check against the CPU oracle (every rank its full batch):
    # its output is parked in a second device buffer and downloaded, compared -- and the CPU
    # baseline timed -- after the timed region, so the GPU does not sit idle through the
    # download and seconds of CPU work right before it
    bit_exact = None
    bit_exact_ranks = None
    cpu = None
    wire_gpu = None
    d_hold = None
    if not args.no_check:
        from tlslite_amd.device import DeviceBuffer
        d_hold = DeviceBuffer(wl.wire_bytes)
        wl.launch([stream])
        N.call("tlsgpu_memcpy_d2d", d_hold.ptr, wl.d_wire.ptr, wl.wire_bytes, stream.handle)
        wl.reset_states(stream)

    # the seal pipeline (its streams, events and workspaces) is set up before the legs below, so
    # no host-side setup idles the GPU between their seals and the warmup steps
    from tlslite_amd.recordlayer import SealPipeline
    pipe = SealPipeline(wl.n_records)
    n_state_launches = 0  # seals applied to the connection states since the last reset
    # ---- one-call latency (no overlap between calls): seal_dev on one stream
    nlat = min(args.steps, 10)
    ev = [Event() for _ in range(nlat + 1)]
    wl.launch([stream])
    stream.synchronize()
    ev[0].record(stream)
    for k in range(nlat):
        wl.launch([stream])
        ev[k + 1].record(stream)
    stream.synchronize()
    n_state_launches += 1 + nlat
    call_ms = float(np.mean([ev[k].elapsed_ms(ev[k + 1]) for k in range(nlat)]))

    # HIP events around the dominant kernel on a spread sample of the timed steps (every M-th):
    # (AES suites: the events of the cipher kernel's own dispatch; event records of their own around
    # a call cost ~25 us of the stream each pair)
    ev_steps = event_steps(args.steps, args.kernel_events_every)
    kev = {k: (Event(), Event()) for k in ev_steps}
    # RC4 / 3DES-only batches (cfg5) have no phases to overlap: their per-variant seal
    # kernels run concurrently on two streams (disjoint connection states), each step's
    # launch ordered after the previous step's launch of the same variant
    conc = None if wl.uses_split_pipeline() else [Stream(high=True), Stream(high=False)]  # separate HW queues
    extra = [Stream() for _ in range(args.extra_streams)]  # noqa: F841 (kept alive through the run)
    progress("warmup %d + timed %d steps" % (args.warmup, args.steps))
    # ---- warmup + timed region: successive batches through the seal pipeline
    # (per-record MAC phase of batch k+1 overlaps the CBC phase of batch k); every stream, event
    # and buffer of the timed region exists before the warmup starts
    for _ in range(args.warmup):
        wl.launch(pipeline=pipe)
    n_state_launches += args.warmup
    # the ranks meet while their GPUs still run the warmup steps, then each waits for its own:
    # a barrier over TCP between two synchronisations would idle every GPU for its duration
    D.barrier()
    pipe.synchronize()
    synchronize()
    if conc:
        for _ in range(args.warmup):
            wl.launch(conc)
        n_state_launches += args.warmup
        for s_ in conc:
            s_.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        if conc:
            if k in kev:
                kev[k][0].record(conc[0])
            wl.launch(conc)
            if k in kev:
                kev[k][1].record(conc[0])
        else:
            wl.launch(pipeline=pipe, cipher_events=kev.get(k))
    pipe.synchronize()
    if conc:
        for s_ in conc:
            s_.synchronize()
    synchronize()
    wall = time.perf_counter() - t0
    D.barrier()
    n_state_launches += args.steps
    per_launch = [kev[k][0].elapsed_ms(kev[k][1]) for k in ev_steps]
    pipe.close()

    # ---- the timed output itself: replay the same number of seals one call at a time
    # (tlsgpu_seal_dev, one stream) from the initial states; the last step's wire arena,
    # wire lengths and the final states must equal the pipelined / concurrent run's
    timed_ok = timed_oracle = None
    timed_oracle_chains = 0
    progress("timed region done (%.1f ms); checking the timed output" % (wall * 1e3))
    if not args.no_check:
        got = (wl.d_wire.download(), wl.d_len.download(), wl.d_states.download())
        wl.reset_states(stream)
        for _ in range(n_state_launches):
            wl.launch([stream])
        stream.synchronize()
        ok = (np.array_equal(got[0], wl.d_wire.download()) and np.array_equal(got[1], wl.d_len.download())
              and np.array_equal(got[2], wl.d_states.download()))
        timed_ok = D.sum(0.0 if ok else 1.0) == 0.0
        # ... and the last step's output against the CPU oracle on a sample of chains
        oo, timed_oracle_chains = oracle_timed_check(wl, got[0], got[1].view(np.int32), n_state_launches,
                                                     usable_cpus()[0])
        del got
        timed_oracle = D.sum(0.0 if oo else 1.0) == 0.0
        timed_oracle_chains = int(D.sum(timed_oracle_chains))
    t_max = D.max(wall)
    total_pt = D.sum(wl.plaintext_total * args.steps)
    value = total_pt / GIB / t_max

    if d_hold is not None:
        progress("parity check against the CPU oracle and the CPU baseline")
        wire_gpu = d_hold.download()
        d_hold.free()
    if wire_gpu is not None:
        # every rank checks its whole shard (the AND over ranks is bit_exact); the CPU baseline
        # is timed on rank 0 at N = 1 only
        baseline = D.world == 1 and not args.no_cpu
        bit_exact, bit_exact_ranks, _, (dt, nrec, ptb, th, reps) = shard_parity(
            D, wl, wire_gpu, min_seconds=args.cpu_seconds if baseline else 0.0)
        del wire_gpu
        cpu_note = usable_cpus()[1]
        if baseline:
            cpu = {"value": round(ptb / GIB / dt, 4), "unit": "GiB/s", "cores": th,
                   "per_core": round(ptb / GIB / dt / th, 5), "kind": "port",
                   "sample": "full batch (%d records, %.1f MiB plaintext) sealed %d times in succession by "
                             "oracle/tls_oracle.c (C restatement of tlslite's _sendMsg path), %d pthreads, %.2f s"
                             % (nrec, ptb / reps / 2 ** 20, reps, th, dt),
                   "cores_note": "threads = the host cores this job may use (%s)" % cpu_note,
                   "reference_python": REFERENCE_PYTHON}

    # roofline of the dominant kernel (the CBC kernel for AES suites; the single
    # seal kernel otherwise), timed with events on the stream it runs on
    avg_ms = float(np.mean(per_launch))
    # read P + write 5+C per record of the records the timed kernel seals: the
    # whole batch, or in a mixed batch (cfg5) the first launch's variant (its 3DES leg)
    alg_bytes = wl.launch_alg_bytes[0]
    achieved = alg_bytes / (avg_ms / 1e3) / 1e9
    copy_gbs = copy_rate(wl, stream)
    # HBM bytes per launch of the same kernel from the committed PMC summary
    # (tools/pmc_kernels.sh -> profiles/pmc_<cfg>.json), only when it names this kernel and
    # was collected on this workload; otherwise traffic is null
    tpath = args.traffic or os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    traffic, seal_call_bytes = pmc_traffic(tpath, wl.name, wl.n_records, wl.dominant_kernel())
    state_bytes = wl.cipher_state_bytes()
    lookups = wl.aes_lookups() if wl.dominant_kernel().startswith(("cbc_kernel", "cbc_pair_kernel")) else None
    lds = None
    if lookups:
        g = lookups / (avg_ms / 1e3) / 1e9
        lds = {"bound": "lds", "achieved": round(g, 1), "peak": LDS_PEAK_GLOOKUPS, "unit": "G lookups/s",
               "frac": round(g / LDS_PEAK_GLOOKUPS, 4), "lookups_per_launch": lookups,
               "note": "AES T-table lookups (16 per round per block) / kernel time; peak = 256 CUs x 32 "
                       "conflict-free ds_read_b32 lanes per cycle x 2.4 GHz"}

    # ---- open direction (decrypt + padding + MAC verify) of one sealed batch:
    # round trip checked byte-for-byte against the plaintext arena
    progress("open / derive / host-inclusive legs")
    open_res = None
    if args.open:
        D.barrier()  # at N > 1 the ranks open their shards at the same time
        try:
            progress("open leg")
            if args.open_split:
                from tlslite_amd.recordlayer import set_open_parts
                set_open_parts({"auto": N.OPEN_SPLIT_AUTO, "chains": N.OPEN_SPLIT_CHAINS,
                                "none": N.OPEN_SPLIT_NONE, "blocks": N.OPEN_SPLIT_BLOCKS}[args.open_split], 0)
            open_res = open_rate(wl, stream, args.steps)
            if args.open_split:
                open_res["split"] = args.open_split
            fr = frame_rate(wl, stream, args.steps)
            if fr is not None:
                open_res["frame"] = fr
            if args.host_inclusive:
                hio = host_open_rate(wl)
                if hio is not None:
                    open_res["host_inclusive"] = hio
        except Exception as e:  # reported, never silently replaced
            open_res = leg_error(e)
        if wl.uses_split_pipeline():  # every rank calls it (collectives inside)
            conc_res = open_concurrent_rate(wl, max(4, min(args.steps, 20)), D=D if D.world > 1 else None,
                                            ranks_per_device=-(-D.world // ndev) if shared else 1)
            if open_res is not None and "error" not in open_res:
                open_res["concurrent"] = conc_res
        if D.world > 1:
            open_res = open_over_ranks(D, open_res, wl.plaintext_total, shared=shared)

    derive_res = None
    if args.derive:
        D.barrier()
        try:
            progress("derive leg")
            derive_res = derive_rate(stream)
        except Exception as e:  # reported, never silently replaced
            derive_res = leg_error(e)
        if D.world > 1:
            derive_res = derive_over_ranks(D, derive_res, shared=shared)

    host_inc = None
    if args.host_inclusive:
        D.barrier()
        try:
            host_inc = host_inclusive_rate(wl)
        except Exception as e:  # reported, never silently replaced
            host_inc = leg_error(e)
        if D.world > 1 and D.sum(0.0 if host_inc is None else 1.0) > 0:  # None: a multi-variant batch
            host_inc = host_inclusive_over_ranks(D, host_inc, wl.plaintext_total)

    if D.rank == 0:
        out = {
            "metric": "GiB/s device-resident AES-128-CBC+HMAC-SHA1 TLS-record encrypt, 16KiB records"
            if args.config == "cfg2" else "GiB/s device-resident TLS-record seal (%s)" % args.config,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": D.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            # cfg4 shards one fixed set of 4,096 connections over the ranks (total work fixed);
            # every other config gives each rank its own full batch
            "scaling": "strong" if args.config == "cfg4" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 plaintext, seeded keys/IVs)",
            "config": {"workload": wl.name, "records_per_gpu": wl.n_records,
                       "plaintext_bytes_per_gpu": wl.plaintext_total,
                       "parallelism": "connection-sharded x%d (no collective)" % D.world,
                       "devices_shared": shared,
                       "device": dev_arch,
                       # per rank: the visible-device setting it narrowed itself to (pin_rank_device)
                       "device_pinning": [p.decode() or None for p in pins]},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": wl.dominant_kernel(), "kernel_avg_ms": round(avg_ms, 4),
                         # the timed steps' kernel times in order: a short run's first steps run
                         # slower than later ones ("Short runs")
                         # the timed steps whose kernel the events bracket: k % every == every // 2
                         "kernel_events": {"every": args.kernel_events_every, "steps": len(ev_steps),
                                           "first": ev_steps[0], "last": ev_steps[-1],
                                           "span": ("the first variant's whole tlsgpu_seal_dev call on its stream "
                                                    "(prefix, MAC and cipher kernels: conservative for the "
                                                    "cipher kernel alone)") if conc else
                                                   "the cipher kernel alone (tlsgpu_pipeline_seal's cipher events: "
                                                   "the kernel dispatch's own start / end, hipExtLaunchKernelGGL)"},
                         "kernel_ms_steps": {"first": round(per_launch[0], 4),
                                             "median": round(float(np.median(per_launch)), 4),
                                             "last": round(per_launch[-1], 4),
                                             "min": round(min(per_launch), 4), "max": round(max(per_launch), 4)},
                         "alg_bytes_per_launch": alg_bytes,
                         "batch_alg_bytes": wl.plaintext_total + wl.wire_total,
                         "copy_measured": round(copy_gbs, 1),
                         "frac_of_copy": round(achieved / copy_gbs, 4),
                         "copy_note": "device-to-device copy of the wire arena on this GPU, (read + write) "
                                      "bytes / HIP-event time, best of 5: the practical HBM ceiling",
                         "traffic_ratio": round(traffic / alg_bytes, 3) if traffic else None,
                         "state_bytes_per_launch": state_bytes,
                         "traffic_ratio_with_state": round(traffic / (alg_bytes + state_bytes), 3) if traffic else None,
                         "seal_call_hbm_bytes": seal_call_bytes,
                         "seal_call_ratio": round(seal_call_bytes / alg_bytes, 3) if seal_call_bytes else None,
                         "traffic_note": "traffic / seal_call_hbm_bytes: PMC HBM bytes (reads from the "
                                         "request-size counters 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B, "
                                         "+ WRITE_SIZE) of the dominant kernel / of all kernels of one seal call "
                                         "(profiles/pmc_<cfg>.json); ratios against alg_bytes (P read + 5+C "
                                         "written) and against alg_bytes + the cipher's per-connection state",
                         "lds": lds},
            "ms_per_seal_call": round(call_ms, 4),
            "cpu_baseline": cpu,
            "bit_exact": bit_exact,
            "bit_exact_ranks": bit_exact_ranks,
            "bit_exact_check": "every rank's whole batch (as sealed by one tlsgpu_seal_dev call from the initial "
                               "states) against the CPU oracle on its share of the host cores; bit_exact = AND "
                               "over the ranks",
            "timed_bit_exact": timed_ok,
            "timed_check": "pipeline-vs-sequential consistency: the %d seals before the last step's output "
                           "replayed one tlsgpu_seal_dev call at a time from the initial states; last wire arena, "
                           "wire lengths and final states equal the pipelined run's" % n_state_launches,
            "timed_oracle_exact": timed_oracle,
            "timed_oracle_check": "%d sampled chains sealed %d times in succession by the CPU oracle from their "
                                  "initial states: their records equal the last timed step's wire arena and "
                                  "wire lengths" % (timed_oracle_chains, n_state_launches),
            "host_inclusive": host_inc,
            "open": open_res,
            "derive": derive_res,
        }
    # a HIP error in any leg (on any rank) fails the run: the device context is dead, and the
    # line must not read as a successful one
    failed = hip_failures({"open": open_res, "derive": derive_res, "host_inclusive": host_inc})
    if D.rank == 0:
        if failed:
            out["error"] = "HIP error in the %s leg(s); the run failed" % ", ".join(failed)
        print(json.dumps(out))
    D.close()
    if failed:
        progress("HIP error in the %s leg(s): exiting with status 1" % ", ".join(failed))
        sys.exit(1)


if __name__ == "__main__":
    main()

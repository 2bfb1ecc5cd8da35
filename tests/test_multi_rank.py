"""N>1 path on CPU: two ranks shard config-4-style connections exactly as
bench.py does (tlslite_amd.shard, its own TCP rendezvous -- no PyTorch), each
seals its shard (with the CPU oracle standing in for the GPU, this is a
sharding/aggregation test), and the gathered result must equal the
single-process run; the max/sum reductions used for the bench line are
exercised too."""
import hashlib
import json
import os
import socket

import multiprocessing as mp

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _seal_shard(wl):
    from oracle import oracle as O
    protos = []
    for c in range(wl.n_chains):
        g = wl.groups[0]
        protos.append(O.Conn.for_suite(g.suite, g.version, bytes(g.keys[c]), bytes(g.ivs[c]), bytes(g.mac_keys[c]),
                                       bytes(g.fixed_ivs[c]), int(g.seq0[c])))
    pt = wl.host_plaintext(O.fill_pattern)
    wire = np.zeros(wl.wire_bytes, dtype=np.uint8)
    O.seal_batch(protos, wl.chain_first, wl.chain_count, pt, wl.pt_off, wl.pt_len, wire, wl.wire_off, nthreads=2)
    # per-connection digests, keyed by global connection id
    out = {}
    for c in range(wl.n_chains):
        h = hashlib.sha256()
        for r in range(int(wl.chain_first[c]), int(wl.chain_first[c] + wl.chain_count[c])):
            o, L = int(wl.wire_off[r]), int(wl.wire_len[r])
            h.update(wire[o:o + L].tobytes())
        out[c] = h.hexdigest()
    return out


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from tlslite_amd import workloads as W
    from tlslite_amd.shard import ShardGroup, shard_indices
    g = ShardGroup()
    wl = W.cfg4(nconn=6, recs_per_conn=3, pt_len=700, rank=rank, world=world)
    mine = shard_indices(6, rank, world)
    digests = _seal_shard(wl)
    by_global = {int(mine[c]): d for c, d in digests.items()}
    allmaps = g.gather_bytes(json.dumps(sorted(by_global.items())).encode())
    t_max = g.max(1.0 + rank)
    total = g.sum(wl.plaintext_total)
    g.barrier()
    g.close()
    q.put((rank, allmaps, t_max, total))


def test_two_rank_sharding_matches_single_process():
    from tlslite_amd import workloads as W
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = _seal_shard(W.cfg4(nconn=6, recs_per_conn=3, pt_len=700, rank=0, world=1))
    for rank, allmaps, t_max, total in res:
        merged = {}
        for m in allmaps:
            merged.update({int(c): d for c, d in json.loads(m.decode())})
        assert merged == single
        assert t_max == 2.0
        assert total == 6 * 3 * 700


# ---------------------------------------------------------------- HIP path, 2 ranks
_GPU_WORKER = r'''
import hashlib, json, os, sys
sys.path.insert(0, os.environ["TG_ROOT"])
import numpy as np
from tlslite_amd import workloads as W
from tlslite_amd.device import Stream, device_count, set_device, synchronize
from tlslite_amd.recordlayer import SealPipeline, seal_dev
from tlslite_amd.shard import ShardGroup, device_for_rank, shard_indices
g = ShardGroup()
# one GPU per rank (LOCAL_RANK % devices): distinct devices on a multi-GPU node -- there rank 1
# drives device 1 of the full device list (unlike bench.py, which narrows each rank's visible
# devices to its own device 0), so this is a device != 0 run of the library, as are
# tests/test_gpu_multidevice.py's -- and both ranks on the one GPU of a single-GPU box
dev = device_for_rank(g.local, device_count())
set_device(dev)
print("DEVICE %d %d" % (g.rank, dev), file=sys.stderr)
wl = W.cfg4(nconn=64, recs_per_conn=4, pt_len=3000, rank=g.rank, world=g.world)
wl.to_device()
synchronize()
mine = shard_indices(64, g.rank, g.world)
def digests():
    wire = wl.d_wire.download()
    out = {}
    for c in range(wl.n_chains):
        h = hashlib.sha256()
        for r in range(int(wl.chain_first[c]), int(wl.chain_first[c] + wl.chain_count[c])):
            o, L = int(wl.wire_off[r]), int(wl.wire_len[r])
            h.update(wire[o:o + L].tobytes())
        out[int(mine[c])] = h.hexdigest()
    return out
# batch 1: tlsgpu_seal_dev with the library-owned workspace, on two streams in turn
s1, s2 = Stream(), Stream()
var, d_ch, nch = wl.launches[0]
seal_dev(d_ch, nch, wl.d_recs, wl.n_records, wl.d_pt, wl.d_wire, wl.d_states, wl.d_len, var, None, s1)
s1.synchronize()
b1 = digests()
# batch 2: the seal pipeline (states carried from batch 1)
pipe = SealPipeline(wl.n_records)
wl.launch(pipeline=pipe)
pipe.synchronize()
pipe.close()
b2 = digests()
allmaps = g.gather_bytes(json.dumps([b1, b2]).encode())
g.barrier()
g.close()
if g.rank == 0:
    merged = [{}, {}]
    for m in allmaps:
        for k, d in enumerate(json.loads(m.decode())):
            merged[k].update({int(a): b for a, b in d.items()})
    print("RESULT " + json.dumps([sorted(merged[0].items()), sorted(merged[1].items())]))
'''


@pytest.mark.gpu
def test_two_rank_hip_sharding_matches_oracle(tmp_path):
    """Two processes (RANK 0/1, the shard rendezvous, device LOCAL_RANK % count) each seal
    their round-robin shard of 64 chained connections through libtlsgpu.so --
    batch 1 with tlsgpu_seal_dev and the library-owned workspace, batch 2
    through the seal pipeline with the states batch 1 left -- and the merged
    per-connection digests equal a single-process CPU-oracle run of both
    batches (the connection is the shard unit: tlsrecordlayer.py:27-37,
    python_aes.py:44)."""
    import json
    import subprocess
    import sys
    from tlslite_amd import workloads as W
    from tests.wl_oracle import oracle_seal
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "worker.py"
    script.write_text(_GPU_WORKER)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TG_ROOT=root)
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=100) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    line = [l for l in outs[0][0].splitlines() if l.startswith("RESULT ")][0]
    got = [dict((int(a), b) for a, b in x) for x in json.loads(line[7:])]
    wl = W.cfg4(nconn=64, recs_per_conn=4, pt_len=3000, rank=0, world=1)
    wire1, _, conns = oracle_seal(wl)

    def dig(wire):
        out = {}
        for c in range(wl.n_chains):
            h = hashlib.sha256()
            for r in range(int(wl.chain_first[c]), int(wl.chain_first[c] + wl.chain_count[c])):
                o, L = int(wl.wire_off[r]), int(wl.wire_len[r])
                h.update(wire[o:o + L].tobytes())
            out[c] = h.hexdigest()
        return out
    from oracle import oracle as O
    pt = wl.host_plaintext(O.fill_pattern)
    wire2 = np.zeros(wl.wire_bytes, dtype=np.uint8)
    O.seal_batch(conns, wl.chain_first, wl.chain_count, pt, wl.pt_off, wl.pt_len, wire2, wl.wire_off, nthreads=4)
    assert got[0] == dig(wire1)
    assert got[1] == dig(wire2)
    assert got[0] != got[1]


def _rdzv_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from tlslite_amd.shard import ShardGroup, device_for_rank
    g = ShardGroup()
    out = {"max": g.max(10.0 - rank), "sum": g.sum(rank + 0.5),
           "gather": g.gather_bytes(bytes([rank]) * (rank + 1)), "dev": device_for_rank(g.local, 2)}
    for _ in range(5):
        g.barrier()
    g.close()
    q.put((rank, out))


def test_shard_rendezvous_three_ranks():
    """The bench's rank plumbing without PyTorch (tlslite_amd.shard): 3 ranks, max / sum of
    floats, an all-gather of different-length byte strings in rank order, repeated barriers,
    and the rank -> device map (LOCAL_RANK % devices)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rdzv_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(3):
        assert res[r]["max"] == 10.0
        assert res[r]["sum"] == 0.5 + 1.5 + 2.5
        assert res[r]["gather"] == [b"\x00", b"\x01\x01", b"\x02\x02\x02"]
        assert res[r]["dev"] == r % 2


def _token_rank0(port, q):
    os.environ.update(RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1),
                      TLSGPU_RDZV_TOKEN="job-a")
    from tlslite_amd.shard import ShardGroup
    g = ShardGroup(timeout=60)
    q.put(g.sum(1.0))
    g.close()


def _token_rank1(port, q):
    os.environ.update(RANK="1", WORLD_SIZE="2", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1),
                      TLSGPU_RDZV_TOKEN="job-a")
    from tlslite_amd.shard import ShardGroup
    g = ShardGroup(timeout=60)
    q.put(g.sum(2.0))
    g.close()


def test_shard_rendezvous_drops_foreign_peers():
    """Rank 0 of the shard rendezvous only admits peers that present the job's token
    (TLSGPU_RDZV_TOKEN): a foreign connection claiming rank 1 with another token and one
    that sends garbage are dropped, and the real rank 1 still joins."""
    import struct
    import time
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p0 = ctx.Process(target=_token_rank0, args=(port, q))
    p0.start()
    deadline = time.monotonic() + 60
    while True:
        try:
            s = socket.create_connection(("127.0.0.1", port), timeout=2)
            break
        except OSError:
            assert time.monotonic() < deadline
            time.sleep(0.05)
    s.sendall(struct.pack("<IB", 1, 5) + b"job-b")  # wrong token, claims rank 1
    s2 = socket.create_connection(("127.0.0.1", port), timeout=2)
    s2.sendall(b"\xff")  # truncated hello
    s2.close()
    p1 = ctx.Process(target=_token_rank1, args=(port, q))
    p1.start()
    res = sorted([q.get(timeout=120), q.get(timeout=120)])
    for p in (p0, p1):
        p.join(timeout=60)
        assert p.exitcode == 0
    s.close()
    assert res == [3.0, 3.0]


def test_job_token_sources():
    """The rendezvous token: the spawner's random token wins; torchrun's
    TORCHELASTIC_RUN_ID when it is a real id; for torchrun's default "none" on one node, a
    token from the master address/port and the launcher's PID (every local rank's parent)."""
    from tlslite_amd.shard import job_token
    assert job_token({"TLSGPU_RDZV_TOKEN": "abc", "TORCHELASTIC_RUN_ID": "x"}) == "abc"
    assert job_token({"TORCHELASTIC_RUN_ID": "run-7"}) == "run-7"
    env = {"TORCHELASTIC_RUN_ID": "none", "LOCAL_WORLD_SIZE": "2", "WORLD_SIZE": "2",
           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29533"}
    assert job_token(env, ppid=4242) == "127.0.0.1:29533:4242"
    assert job_token(env, ppid=4242) != job_token(env, ppid=4243)
    # several nodes: the launchers' PIDs differ, so the PID cannot be part of the token
    assert job_token(dict(env, WORLD_SIZE="4"), ppid=4242) == "none"
    assert job_token({}) == ""

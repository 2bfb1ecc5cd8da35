"""N>1 path on CPU: two gloo ranks shard config-4-style connections exactly
as bench.py does (tlslite_amd.shard), each seals its shard (with the CPU
oracle standing in for the GPU, this is a sharding/aggregation test), and the
gathered result must equal the single-process run; the max/sum reductions
used for the bench line are exercised too."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


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
    g = ShardGroup("gloo")
    wl = W.cfg4(nconn=6, recs_per_conn=3, pt_len=700, rank=rank, world=world)
    mine = shard_indices(6, rank, world)
    digests = _seal_shard(wl)
    by_global = {int(mine[c]): d for c, d in digests.items()}
    allmaps = g.gather_bytes(repr(sorted(by_global.items())).encode())
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
            merged.update(dict(eval(m.decode())))
        assert merged == single
        assert t_max == 2.0
        assert total == 6 * 3 * 700

"""GPU parity at the BASELINE configurations' full sizes (BASELINE.json configs[1..4]):
one seal call of the whole cfg2 / cfg3 / cfg5 batch, and of cfg4's 8-GPU shards (the
512 connections rank 0 and rank 7 of 8 seal), equals the CPU oracle byte for byte --
every wire byte, every wire length and every chain's final CBC residue / RC4 state and
seqnum (tlsrecordlayer.py:538-617, python_aes.py:44, python_rc4.py:31-41).  The bench
checks the same for the config it runs; these put every config into the GPU suite.
Test infrastructure: the oracle is the checker, the HIP path is what runs."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _wl(name):
    from tlslite_amd import workloads as W
    if name == "cfg4_n1":
        return W.cfg4()  # the whole N=1 batch: 4,096 connections x 256 records x 16 KiB, 16 GiB arenas
    if name.startswith("cfg4"):
        rank = int(name.split("_r")[1])
        return W.cfg4(rank=rank, world=8)  # 512 of the 4,096 connections x 256 records x 16 KiB
    return W.CONFIGS[name]()


@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg5", "cfg4_r0", "cfg4_r7"])
def test_full_size_vs_oracle(name):
    from tlslite_amd import device
    from tlslite_amd.device import synchronize
    from tests.wl_oracle import device_states, oracle_seal
    if device.device_count() < 1:
        pytest.fail("no GPU visible to libtlsgpu (the gpu tests need an MI355X)")
    wl = _wl(name)
    try:
        wl.to_device()
        wl.launch()
        synchronize()
        wire_gpu = wl.d_wire.download()
        lens_gpu = wl.d_len.download().view(np.int32)
        states = device_states(wl)
        wire, lens, conns = oracle_seal(wl, nthreads=min(16, os.cpu_count() or 1))
        assert np.array_equal(lens_gpu, np.asarray(lens, dtype=np.int32)), name
        if not np.array_equal(wire_gpu, wire):
            off = wl.wire_off.astype(np.int64)
            bad = [r for r in range(wl.n_records)
                   if not np.array_equal(wire_gpu[off[r]:off[r] + lens[r]], wire[off[r]:off[r] + lens[r]])]
            pytest.fail("%s: %d records differ, first %s" % (name, len(bad), bad[:10]))
        for c, (s, o) in enumerate(zip(states, conns)):
            assert s.seqnum == o.seqnum, (name, c)
            if o.cipher == "rc4":
                assert tuple(s.rc4) == tuple(o.rc4), (name, c)
            else:
                assert s.iv == o.iv, (name, c)
    finally:
        wl.free()


def _opened_equals(wl, opened, pt):
    """Record r's opened payload (opened[opt_off[r] : + pt_len[r]]) equals its plaintext
    (pt[pt_off[r] : + pt_len[r]]) for every record; -> indices of the records that differ."""
    n = wl.pt_len.astype(np.int64)
    a, b = wl.opt_off.astype(np.int64), wl.pt_off.astype(np.int64)
    bad = []
    for r, (x, y, k) in enumerate(zip(a.tolist(), b.tolist(), n.tolist())):
        if not np.array_equal(opened[x:x + k], pt[y:y + k]):
            bad.append(r)
    return bad


@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg5", "cfg4_r0", "cfg4_n1"])
def test_full_size_open_vs_oracle(name):
    """The open of the whole sealed batch (tlsgpu_open_dev, tlsrecordlayer.py:958-1044) at the
    BASELINE config's full size -- cfg4_n1 is the whole one-GPU cfg4 batch, 16 GiB arenas with
    offsets past 2^32 -- against the CPU oracle: the oracle seals the batch (its wire must be
    the device's), every record opens with status = its plaintext length, its opened payload
    equals the oracle's plaintext (host splitmix64 fill), every read state ends at the oracle's
    final residue / RC4 state and seqnum (a read state that opened a chain's records equals the
    write state that sealed them), and on a sample of chains the oracle's own open of the
    records gives the same plaintext."""
    from oracle import oracle as O
    from tlslite_amd import device
    from tlslite_amd.device import synchronize
    from tests.wl_oracle import device_states, oracle_seal
    if device.device_count() < 1:
        pytest.fail("no GPU visible to libtlsgpu (the gpu tests need an MI355X)")
    wl = _wl(name)
    try:
        wl.to_device()
        wl.launch()
        synchronize()
        wire, lens, conns = oracle_seal(wl, nthreads=min(16, os.cpu_count() or 1))
        assert np.array_equal(wl.d_len.download().view(np.int32), np.asarray(lens, dtype=np.int32)), name
        assert np.array_equal(wl.d_wire.download(), wire), "%s: sealed wire differs from the oracle's" % name
        wl.open_setup()
        wl.open_launch()
        synchronize()
        status = wl.d_ostatus.download().view(np.int32)
        bad = np.nonzero(status != wl.pt_len.astype(np.int32))[0]
        assert bad.size == 0, "%s: %d records with status != length, first %s: %s" % (
            name, bad.size, bad[:8].tolist(), status[bad[:8]].tolist())
        pt = wl.host_plaintext(O.fill_pattern)
        opened = wl.d_opt.download()
        diff = _opened_equals(wl, opened, pt)
        assert not diff, "%s: %d opened records differ, first %s" % (name, len(diff), diff[:10])
        saved = wl.d_states
        wl.d_states = wl.d_ostates
        try:
            rstates = device_states(wl)
        finally:
            wl.d_states = saved
        for c, (s, o) in enumerate(zip(rstates, conns)):
            assert s.seqnum == o.seqnum, (name, c)
            if o.cipher == "rc4":
                assert tuple(s.rc4) == tuple(o.rc4), (name, c)
            else:
                assert s.iv == o.iv, (name, c)
        # the oracle's own open (ora_open) of every record of a few chains, in chain order
        from tests.wl_oracle import oracle_conns
        fresh = oracle_conns(wl)
        for c in sorted({0, wl.n_chains // 2, wl.n_chains - 1}):
            f, k = int(wl.chain_first[c]), int(wl.chain_count[c])
            for r in range(f, f + k):
                w0 = int(wl.wire_off[r])
                code, got = fresh[c].open(wire[w0 + 5:w0 + int(lens[r])].tobytes(), int(wire[w0]))
                assert code == 0, (name, r, code)
                a = int(wl.opt_off[r])
                assert got == opened[a:a + len(got)].tobytes(), (name, r)
    finally:
        wl.free()

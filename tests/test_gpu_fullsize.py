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

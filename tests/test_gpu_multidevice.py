"""One process driving several GPUs through one libtlsgpu.so: the library keys its
per-device state -- the LDS-size attribute of each kernel, the CU count that sizes the grids,
the library-owned workspaces and the split open's second streams -- on the device of the stream
a call is given, not on the calling thread's current device.  bench.py pins every rank to its
own device 0, so these tests are where device != 0 runs: on every visible device a batch is
sealed (tlsgpu_seal_dev and the pipeline) and opened (tlsgpu_open_dev) with library-owned
workspaces and compared with the CPU oracle (tlsrecordlayer.py:538-617, :958-1044); and with
two or more devices, calls are issued on a device-1 stream while the thread's current device is
0 (and the other way round).  On a one-GPU box the first test runs device 0 only and the second
is skipped; on an 8-GPU node they cover devices 1-7."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _batch(dev, seed):
    """A chained cfg4-shaped batch (32 connections x 3 records of 3000 B) on device `dev`."""
    from tlslite_amd import workloads as W
    from tlslite_amd.device import Stream, set_device
    set_device(dev)
    wl = W.cfg4(nconn=32, recs_per_conn=3, pt_len=3000, seed=seed)
    s = Stream()
    wl.to_device(s)
    s.synchronize()
    wl.open_setup()
    return wl, s


def _check(wl, name):
    from oracle import oracle as O
    from tests.wl_oracle import device_states, oracle_seal
    wire, lens, conns = oracle_seal(wl, nthreads=min(8, os.cpu_count() or 1))
    got = wl.d_wire.download()
    assert np.array_equal(wl.d_len.download().view(np.int32), np.asarray(lens, dtype=np.int32)), name
    assert np.array_equal(got, wire), name
    for c, (s, o) in enumerate(zip(device_states(wl), conns)):
        assert s.seqnum == o.seqnum and s.iv == o.iv, (name, c)
    st = wl.d_ostatus.download().view(np.int32)
    assert np.array_equal(st, wl.pt_len.astype(np.int32)), name
    pt = wl.host_plaintext(O.fill_pattern)
    opened = wl.d_opt.download()
    for r in range(wl.n_records):
        a, b, n = int(wl.opt_off[r]), int(wl.pt_off[r]), int(wl.pt_len[r])
        assert np.array_equal(opened[a:a + n], pt[b:b + n]), (name, r)


def _seal_open(wl, s):
    from tlslite_amd import _native as N
    from tlslite_amd.recordlayer import open_dev, seal_dev
    var, d_ch, nch = wl.launches[0]
    # library-owned workspaces (keyed on the stream's device)
    seal_dev(d_ch, nch, wl.d_recs, wl.n_records, wl.d_pt, wl.d_wire, wl.d_states, wl.d_len, var, None, s)
    N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, s.handle)
    open_dev(d_ch, nch, wl.d_orecs, wl.n_records, wl.d_wire, wl.d_opt, wl.d_ostates, wl.d_ostatus, var, None, s)


def test_every_device_seals_and_opens_like_oracle():
    from tlslite_amd.device import device_count, set_device
    n = device_count()
    if n < 1:
        pytest.fail("no GPU visible to libtlsgpu (the gpu tests need an MI355X)")
    for dev in range(n):
        wl, s = _batch(dev, 40 + dev)
        _seal_open(wl, s)
        s.synchronize()
        _check(wl, "device %d" % dev)
        wl.free()
    set_device(0)


def test_calls_on_another_devices_stream():
    from tlslite_amd.device import device_count, set_device
    n = device_count()
    if n < 2:
        pytest.skip("one GPU visible: the cross-device case needs two")
    a, sa = _batch(0, 50)
    b, sb = _batch(1, 51)
    set_device(0)
    _seal_open(b, sb)  # device-1 stream, current device 0
    set_device(1)
    _seal_open(a, sa)  # device-0 stream, current device 1
    sa.synchronize()
    sb.synchronize()
    _check(a, "device 0 from device 1")
    _check(b, "device 1 from device 0")
    a.free()
    b.free()
    set_device(0)


def test_host_pipeline_on_another_device():
    """A host pipeline created on device 1 and called with device 0 current seals and opens on
    device 1 (its streams and buffers live there; tlsgpu_host_pipeline_* switch to it for the
    call and restore the caller's device), results equal to the device-resident path."""
    from tlslite_amd import _native as N
    from tlslite_amd.constants import ContentType
    import ctypes
    from tlslite_amd.device import PinnedBuffer, device_count, set_device, synchronize
    from tlslite_amd.recordlayer import HostSealPipeline, make_chains, make_records
    if device_count() < 2:
        pytest.skip("one GPU visible: the cross-device case needs two")
    wl, s = _batch(1, 61)
    wl.launch()
    synchronize()
    ref = wl.d_wire.download()
    var = wl.launches[0][0]
    recs = make_records(wl.pt_off, wl.wire_off, wl.pt_len, ContentType.application_data, 0)
    chains = make_chains(np.arange(wl.n_chains, dtype=np.uint32), wl.chain_first, wl.chain_count)
    pin_pt, pin_wire = PinnedBuffer(wl.pt_bytes), PinnedBuffer(wl.wire_bytes)
    wl.d_pt.download(out=pin_pt.array[: wl.pt_bytes])
    pin_wire.array[:] = 0
    lens = np.zeros(wl.n_records, dtype=np.int32)
    wl.reset_states()
    synchronize()
    hp = HostSealPipeline(64 << 10, 3)  # created with device 1 current
    set_device(0)
    hp.seal(chains, recs, pin_pt.array[: wl.pt_bytes], pin_wire.array[: wl.wire_bytes], wl.d_states, lens, var)
    cur = ctypes.c_int(-1)
    N.call("tlsgpu_get_device", ctypes.byref(cur))
    assert cur.value == 0
    assert np.array_equal(pin_wire.array[: wl.wire_bytes], ref)
    hp.close()
    pin_pt.free()
    pin_wire.free()
    set_device(1)
    wl.free()
    set_device(0)

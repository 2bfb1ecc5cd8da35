"""Timeline of open_fused_kernel on one config (GPU box), from the diagnostic library that
tools/build_open_trace.py builds: seal the config's batch, open it (warm-up + traced call),
read the stamps out of the open workspace and print, over the workgroups, when the decrypt
waves publish each stripe and when the MAC waves see it and finish hashing it (microseconds
from the workgroup's first stamp; median / max over workgroups).  Diagnostic tool only.
  TLSGPU_LIB=tools/ab/oftrace/libtlsgpu.so python tools/open_trace.py [cfg2]
"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    os.environ.setdefault("TLSGPU_LIB", os.path.join(R, "tools", "ab", "oftrace", "libtlsgpu.so"))
    import bench
    from tlslite_amd import _native as N
    from tlslite_amd.device import Stream, set_device
    set_device(0)
    wl = bench.build_workload(cfg, 0, 1)
    s = Stream()
    wl.to_device(s)
    wl.reset_states(s)
    wl.launch([s])
    wl.open_setup()
    for _ in range(3):
        N.call("tlsgpu_memcpy_d2d", wl.d_ostates.ptr, wl.d_states0.ptr, wl.d_ostates.nbytes, s.handle)
        wl.open_launch(s, reset=False)
    s.synchronize()
    status = wl.d_ostatus.download().view(np.int32)
    print("status exact:", bool(np.array_equal(status, wl.pt_len.astype(np.int32))))
    ws = wl.d_ows[0].download()
    base = wl.n_records * 48 + 256 * 256
    tr = ws[base:base + 256 * 16 * 64 * 8].view(np.uint64).reshape(256, 16, 64).astype(np.int64)
    used = tr[:, 0, 0] != 0
    tr = tr[used]
    t0 = tr[:, :, 0].min(axis=1)[:, None, None]
    us = np.where(tr != 0, (tr - t0) / 100.0, np.nan)  # 100 MHz -> microseconds
    print("workgroups traced:", len(tr))

    def row(name, v):
        v = v[~np.isnan(v)]
        if len(v):
            print("%-34s median %8.1f  min %8.1f  max %8.1f" % (name, np.median(v), v.min(), v.max()))

    dec, mac = us[:, :12], us[:, 12:]
    row("decrypt start", dec[:, :, 0].ravel())
    row("MAC start", mac[:, :, 0].ravel())
    for st in range(20):
        if np.isnan(dec[:, :, 1 + st]).all():
            break
        row("stripe %2d last publish" % st, np.nanmax(dec[:, :, 1 + st], axis=1))
        row("stripe %2d MAC sees it" % st, mac[:, :, 1 + st].ravel())
        row("stripe %2d MAC hashed" % st, mac[:, :, 21 + st].ravel())
    row("decrypt done (per wave)", dec[:, :, 62].ravel())
    row("decrypt done (workgroup)", np.nanmax(dec[:, :, 62], axis=1))
    row("MAC record done (per wave)", mac[:, :, 61].ravel())
    row("MAC done (workgroup)", np.nanmax(mac[:, :, 61], axis=1))


if __name__ == "__main__":
    main()

"""Open-path kernel times for small batches (the receive pipeline's sub-batches): n records of
16 KiB (AES128-SHA, TLS 1.2) sealed on the GPU, then opened device-resident with the
plaintext bodies at a 16-byte-aligned offset or shifted by `shift` bytes, timed by HIP
events; run under rocprofv3 --kernel-trace for per-kernel times.
Usage: python tools/open_mac_probe.py [--n 1024,4096,65536] [--shift 0,5]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1024,4096,65536")
    ap.add_argument("--shift", default="0,5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--bg", default="none", choices=["none", "h2d", "d2h", "both"],
                    help="pinned copies of 512 MiB running on other streams during each open")
    a = ap.parse_args()
    from tlslite_amd import workloads as W
    from tlslite_amd.device import DeviceBuffer, Event, Stream, synchronize
    from tlslite_amd.recordlayer import make_open_records, open_dev
    from tlslite_amd.device import PinnedBuffer, copy_d2h, copy_h2d
    s = Stream()
    bg_n = 512 << 20
    if a.bg != "none":
        hbuf, dbuf = PinnedBuffer(bg_n), DeviceBuffer(bg_n)
        sh, sd = Stream(high=True), Stream(high=True)

    def background():
        if a.bg in ("h2d", "both"):
            copy_h2d(dbuf, 0, hbuf.ptr.value, bg_n, sh)
        if a.bg in ("d2h", "both"):
            copy_d2h(hbuf.ptr.value, dbuf, 0, bg_n, sd)
    for n in [int(x) for x in a.n.split(",")]:
        wl = W.cfg2(n=n)
        wl.to_device()
        wl.launch()
        synchronize()
        body = (wl.wire_len - 5).astype(np.int64)
        for shift in [int(x) for x in a.shift.split(",")]:
            # opened bodies packed at 16-aligned slots + shift
            slot = (body + 31) // 16 * 16
            opt = (np.concatenate([[0], np.cumsum(slot)[:-1]]) + shift).astype(np.uint64)
            recs = make_open_records(wl.wire_off + 5, opt, body, 23)
            d_r = DeviceBuffer(24 * n)
            d_r.upload(np.frombuffer(recs, dtype=np.uint8))
            d_pt = DeviceBuffer(int(opt[-1]) + int(slot[-1]) + 64)
            d_st, d_os = DeviceBuffer(4 * n), DeviceBuffer(wl.d_states0.nbytes)
            var, d_ch, nch = wl.launches[0]
            ms = []
            for _ in range(a.reps):
                d_os.upload(np.frombuffer(wl.d_states0.download(), dtype=np.uint8), stream=s)
                e0, e1 = Event(), Event()
                s.synchronize()
                if a.bg != "none":
                    background()
                e0.record(s)
                open_dev(d_ch, nch, d_r, n, wl.d_wire, d_pt, d_os, d_st, var, stream=s)
                e1.record(s)
                s.synchronize()
                synchronize()
                ms.append(e0.elapsed_ms(e1))
            ok = bool((d_st.download().view(np.int32) == wl.pt_len.astype(np.int32)).all())
            print(json.dumps({"n": n, "shift": shift, "bg": a.bg, "ms": round(float(np.median(ms)), 4), "ok": ok}), flush=True)
            for b in (d_r, d_pt, d_st, d_os):
                b.free()
        wl.free()


if __name__ == "__main__":
    main()

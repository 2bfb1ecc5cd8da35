"""Seal the cfg2 batch through the seal pipeline back to back for --seconds (diagnostic for
tools/clock_watch.sh: clock and power under sustained load); prints GiB/s per --block steps (each block bracketed by synchronizations, as bench.py's timed region)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--block", type=int, default=200, help="steps between synchronizations")
    ap.add_argument("--pipe-first", action="store_true", help="create the pipeline before --pre's work")
    ap.add_argument("--alloc-between", type=int, default=0,
                    help="MiB to hipMalloc and free between blocks (0: none): does an allocation slow the next block?")
    ap.add_argument("--pre-n", type=int, default=40, help="seal_dev calls of --pre dev")
    ap.add_argument("--pre", default="none", choices=["none", "dev", "fill"],
                    help="before the loop: none; 'dev' 40 tlsgpu_seal_dev calls; 'fill' ~100 ms of an unrelated "
                         "kernel (fill_pattern over a 4 GiB buffer, 25 times)")
    a = ap.parse_args()
    from tlslite_amd import workloads as W
    from tlslite_amd.device import synchronize
    from tlslite_amd.recordlayer import SealPipeline
    wl = W.CONFIGS[a.config]()
    wl.to_device()
    synchronize()
    pipe = SealPipeline(wl.n_records) if a.pipe_first else None
    if a.pre == "dev":
        for _ in range(a.pre_n):
            wl.launch()
        synchronize()
    elif a.pre == "fill":
        from tlslite_amd import _native as N
        from tlslite_amd.device import DeviceBuffer
        buf = DeviceBuffer(4 << 30)
        for k in range(25):
            N.call("tlsgpu_fill_pattern", buf.ptr, buf.nbytes, k, 0, None)
        synchronize()
        buf.free()
    pipe = pipe or SealPipeline(wl.n_records)
    t_end = time.perf_counter() + a.seconds
    from tlslite_amd.device import DeviceBuffer
    nblk = 0
    while time.perf_counter() < t_end:
        if a.alloc_between and nblk % 4 == 3:
            DeviceBuffer(a.alloc_between << 20).free()
            print("-- allocated and freed %d MiB" % a.alloc_between, flush=True)
        nblk += 1
        t0 = time.perf_counter()
        for _ in range(a.block):
            wl.launch(pipeline=pipe)
        pipe.synchronize()
        synchronize()
        dt = time.perf_counter() - t0
        print("%.3f %.1f GiB/s" % (time.time(), a.block * wl.plaintext_total / (1 << 30) / dt), flush=True)
    pipe.close()
    wl.free()


if __name__ == "__main__":
    main()

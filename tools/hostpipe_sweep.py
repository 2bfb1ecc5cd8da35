"""Sub-batch size / depth sweep of the host pipelines on cfg2 (tlsgpu_host_pipeline_seal and
tlsgpu_host_pipeline_open): one JSON line per (direction, chunk, depth) with the pinned and
pageable wall times, the PCIe ceiling and the exactness flags (bench.py's host legs).
Usage: python tools/hostpipe_sweep.py [--chunks 8,16,32,64] [--depths 2,3,4] [--dir seal,open]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="8,16,32,64")
    ap.add_argument("--depths", default="2,3,4")
    ap.add_argument("--dir", default="seal,open")
    ap.add_argument("--config", default="cfg2")
    a = ap.parse_args()
    import bench
    from tlslite_amd import workloads as W
    from tlslite_amd.device import synchronize
    wl = W.CONFIGS[a.config]()
    wl.to_device()
    wl.open_setup()
    synchronize()
    link = bench.pcie_rates()
    for d in a.dir.split(","):
        for c in [int(x) for x in a.chunks.split(",")]:
            for dep in [int(x) for x in a.depths.split(",")]:
                if d == "seal":
                    r = bench.host_inclusive_rate(wl, chunk=c << 20, depth=dep)
                    ok = r["pinned"]["bit_exact"] and r["pageable"]["bit_exact"]
                else:
                    r = bench.host_open_rate(wl, link=link, chunk=c << 20, depth=dep)
                    ok = r["pinned"]["roundtrip_exact"] and r["pageable"]["roundtrip_exact"]
                print(json.dumps({"dir": d, "chunk_mib": c, "depth": dep, "pinned": r["pinned"]["value"],
                                  "pinned_ms": r["pinned"]["ms"], "pageable": r["pageable"]["value"],
                                  "ceiling": r["pcie_ceiling"], "frac": r["pcie_frac"], "exact": ok}), flush=True)
    wl.free()


if __name__ == "__main__":
    main()

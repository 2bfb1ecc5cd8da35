"""Host-buffer pipeline sweep on cfg2 (diagnostic tool): raw PCIe copy rates on this box
(H2D alone, D2H alone, both at once on two streams) and tlsgpu_host_pipeline_seal over
pinned arenas for a grid of (chunk_bytes, depth).  Prints one line per point."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from tlslite_amd import workloads as W  # noqa: E402
from tlslite_amd.constants import ContentType  # noqa: E402
from tlslite_amd.device import PinnedBuffer, synchronize  # noqa: E402
from tlslite_amd.recordlayer import HostSealPipeline, make_chains, make_records  # noqa: E402

GIB = 1 << 30


def raw_copies(nbytes):
    """Raw pinned copy rates through the HIP runtime (bench.py's pcie_rates)."""
    sys.path.insert(0, ".")
    from bench import pcie_rates
    res = pcie_rates(nbytes)
    print("raw pinned copies of %d MiB: H2D %.1f GB/s, D2H %.1f GB/s, both at once %.1f GB/s total"
          % (nbytes >> 20, res["h2d"], res["d2h"], res["both"]), flush=True)


def main():
    raw_copies(1 << 30)
    wl = W.cfg2()
    wl.to_device()
    var = wl.launches[0][0]
    recs = make_records(wl.pt_off, wl.wire_off, wl.pt_len, ContentType.application_data, 0)
    chains = make_chains(np.arange(wl.n_chains, dtype=np.uint32), wl.chain_first, wl.chain_count)
    pin_pt, pin_wire = PinnedBuffer(wl.pt_bytes), PinnedBuffer(wl.wire_bytes)
    wl.d_pt.download(out=pin_pt.array[: wl.pt_bytes])
    lens = np.zeros(wl.n_records, dtype=np.int32)
    grid = [(c << 20, d) for c in (16, 32, 64, 128) for d in (2, 3, 4, 6)]
    for chunk, depth in grid:
        with HostSealPipeline(chunk, depth) as hp:
            best = 1e9
            for _ in range(3):
                wl.reset_states()
                synchronize()
                t0 = time.perf_counter()
                hp.seal(chains, recs, pin_pt.array[: wl.pt_bytes], pin_wire.array[: wl.wire_bytes], wl.d_states,
                        lens, var)
                best = min(best, time.perf_counter() - t0)
        print("chunk %4d MiB depth %d: %6.2f GiB/s (%.2f ms)" % (chunk >> 20, depth, wl.plaintext_total / GIB / best,
                                                              best * 1e3), flush=True)


if __name__ == "__main__":
    main()

"""One host-pipeline configuration on cfg2, pinned arenas, 3 calls (for rocprofv3 traces)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from tlslite_amd import workloads as W  # noqa: E402
from tlslite_amd.constants import ContentType  # noqa: E402
from tlslite_amd.device import PinnedBuffer, synchronize  # noqa: E402
from tlslite_amd.recordlayer import HostSealPipeline, make_chains, make_records  # noqa: E402

chunk, depth = int(sys.argv[1]) << 20, int(sys.argv[2])
wl = W.cfg2()
wl.to_device()
var = wl.launches[0][0]
recs = make_records(wl.pt_off, wl.wire_off, wl.pt_len, ContentType.application_data, 0)
chains = make_chains(np.arange(wl.n_chains, dtype=np.uint32), wl.chain_first, wl.chain_count)
pin_pt, pin_wire = PinnedBuffer(wl.pt_bytes), PinnedBuffer(wl.wire_bytes)
wl.d_pt.download(out=pin_pt.array[: wl.pt_bytes])
lens = np.zeros(wl.n_records, dtype=np.int32)
with HostSealPipeline(chunk, depth) as hp:
    for _ in range(3):
        wl.reset_states()
        synchronize()
        t0 = time.perf_counter()
        hp.seal(chains, recs, pin_pt.array[: wl.pt_bytes], pin_wire.array[: wl.wire_bytes], wl.d_states, lens, var)
        print("%.2f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)

"""Debug: host pipeline vs device path on a chained workload (diagnostic tool)."""
import sys
import numpy as np
sys.path.insert(0, '.')
from tlslite_amd import workloads as W
from tlslite_amd.constants import ContentType
from tlslite_amd.device import PinnedBuffer, synchronize
from tlslite_amd.recordlayer import HostSealPipeline, make_chains, make_records
kind = sys.argv[1]
chunk = int(sys.argv[2])
wl = W.cfg4(nconn=40, recs_per_conn=5, pt_len=3001, seed=22) if kind == "chained" else W.cfg2(n=700, pt_len=5003, seed=21)
wl.to_device()
wl.launch()
synchronize()
ref = wl.d_wire.download()
var = wl.launches[0][0]
recs = make_records(wl.pt_off, wl.wire_off, wl.pt_len, ContentType.application_data, 0)
chains = make_chains(np.arange(wl.n_chains, dtype=np.uint32), wl.chain_first, wl.chain_count)
for pinned in (True, False):
    if pinned:
        b = [PinnedBuffer(wl.pt_bytes), PinnedBuffer(wl.wire_bytes)]
        pt_h, wire_h = b[0].array[: wl.pt_bytes], b[1].array[: wl.wire_bytes]
        wire_h[:] = 0
    else:
        pt_h, wire_h = np.empty(wl.pt_bytes, dtype=np.uint8), np.zeros(wl.wire_bytes, dtype=np.uint8)
    wl.d_pt.download(out=pt_h)
    lens = np.zeros(wl.n_records, dtype=np.int32)
    wl.reset_states()
    synchronize()
    with HostSealPipeline(chunk_bytes=chunk, depth=3) as hp:
        hp.seal(chains, recs, pt_h, wire_h, wl.d_states, lens, var)
    bad = np.nonzero(wire_h != ref)[0]
    print("pinned", pinned, "mismatch bytes", len(bad), flush=True)
    if len(bad):
        recs_bad = sorted(set(int(np.searchsorted(wl.wire_off.astype(np.int64), x, side="right")) - 1 for x in bad[:5000]))
        print(" records", recs_bad[:40], "first bytes", bad[:10], "wire_off", [int(wl.wire_off[r]) for r in recs_bad[:5]])
        r = recs_bad[0]
        o = int(wl.wire_off[r])
        print(" got", wire_h[o:o + 24].tobytes().hex(), "\n ref", ref[o:o + 24].tobytes().hex())

"""Open-path smoke on a cfg2-shaped batch of n records (diagnostic tool)."""
import sys

import numpy as np

sys.path.insert(0, '.')
from tlslite_amd import workloads as W, device  # noqa: E402
from tlslite_amd.device import Stream  # noqa: E402

n = int(sys.argv[1])
wl = W.cfg2(n=n).to_device()
s = Stream()
wl.launch([s])
s.synchronize()
wl.open_setup()
wl.open_launch(s)
s.synchronize()
st = wl.d_ostatus.download().view(np.int32)
print("status ok", bool(np.array_equal(st, wl.pt_len.astype(np.int32))), np.unique(st)[:4], flush=True)
print("pt eq", wl.opened_plaintext_matches(), "devices", device.device_count(), flush=True)

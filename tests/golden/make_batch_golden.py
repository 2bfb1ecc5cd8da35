#!/usr/bin/env python3
"""Whole-batch reference digests: small instances of the bench
workloads cfg2-cfg5 (tlslite_amd.workloads, same keys / IVs / layout / splitmix
plaintext as the device path) sealed record by record by the *reference* tlslite
`_sendMsg` (tlsrecordlayer.py:538-620), one `TLSRecordLayer` per connection so the CBC
residue / RC4 state / seqnum carry through each connection's records.

Output: tests/golden/batches.json -- per batch the SHA-256 of the concatenated wire
records (record order) and of the final per-connection states, plus the workload
parameters.  tests/test_batch_golden.py checks the C oracle (CPU) and the HIP path
(GPU) against these digests.  Run only in the build container (needs /root/reference);
the GPU box reads the JSON only.

Usage:  PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_batch_golden.py
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import make_golden as MG  # noqa: E402  (reference import shim, make_layer, seal_records)

from tlslite_amd import workloads as W  # noqa: E402

OUT = os.path.join(HERE, "batches.json")

# (name, constructor, kwargs): 4-8 MB each, so the pure-Python reference finishes in seconds
BATCHES = [
    ("cfg2_small", "cfg2", {"n": 256, "pt_len": 16384}),
    ("cfg3_small", "cfg3", {"n": 4096, "pt_len": 1434}),
    ("cfg4_small", "cfg4", {"nconn": 16, "recs_per_conn": 16, "pt_len": 16384}),
    ("cfg5_small", "cfg5", {"n": 512, "pt_len": 16384}),
]


def splitmix_fill(n, seed, start):
    """fill_kernel's byte stream (tg_kernels.hip): byte g = splitmix64(seed + g/8) >> 8(g%8)."""
    g0, g1 = start // 8, (start + n + 7) // 8
    z = (np.arange(g0, g1, dtype=np.uint64) + np.uint64(seed)) + np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    off = start - 8 * g0
    return b[off:off + n].copy()


def conn_keys(wl, c):
    """make_golden.make_layer's key dict for chain c (as tests/wl_oracle.oracle_conns)."""
    g = wl.groups[wl.chain_group[c]]
    gi = c - int(np.searchsorted(wl.chain_group, wl.chain_group[c]))
    fiv = g.fixed_ivs[gi % len(g.fixed_ivs)] if g.fixed_ivs is not None else b""
    return g, {"key": bytes(g.keys[gi % len(g.keys)]).hex(),
               "iv": bytes(g.ivs[gi]).hex() if g.ivs is not None else "",
               "mac_key": bytes(g.mac_keys[gi % len(g.mac_keys)]).hex(),
               "fixed_iv": bytes(fiv).hex(), "seq": int(g.seq0[gi])}


def state_digest_entry(suite, fin):
    """Canonical text of one connection's final state (shared with the tests)."""
    if "rc4_S" in fin:
        return "%s|%d|%d|%d|%s" % (suite, fin["seqnum"], fin["rc4_i"], fin["rc4_j"], fin["rc4_S"])
    return "%s|%d|%s" % (suite, fin["seqnum"], fin["cbc_iv"])


def main():
    doc = {"generator": "tests/golden/make_batch_golden.py",
           "reference": "trevp/tlslite 0.4.9 at /root/reference, TLSRecordLayer._sendMsg per record; "
                        "3DES cipher = OpenSSL 3 EVP_des_ede3_cbc (as make_golden.py)",
           "plaintext": "splitmix64 fill of tlslite_amd.workloads (fill_kernel)",
           "wire_digest": "SHA-256 over the wire bytes of every record, record index order",
           "state_digest": "SHA-256 over '\\n'.join(suite|seqnum|cbc_iv_hex or suite|seqnum|i|j|S_hex) per chain",
           "batches": []}
    for name, cfg, kw in BATCHES:
        t0 = time.time()
        wl = W.CONFIGS[cfg](**kw)
        pt = wl.host_plaintext(splitmix_fill)
        wires = [b""] * wl.n_records
        states = []
        for c in range(wl.n_chains):
            g, keys = conn_keys(wl, c)
            layer = MG.make_layer(g.suite, g.version, keys)
            first, count = int(wl.chain_first[c]), int(wl.chain_count[c])
            for r in range(first, first + count):
                off, n = int(wl.pt_off[r]), int(wl.pt_len[r])
                wires[r] = MG.seal_records(layer, [bytes(pt[off:off + n])])[0]
                assert len(wires[r]) == int(wl.wire_len[r]), (name, r)
            states.append(state_digest_entry(g.suite, MG.final_state(layer, g.suite)))
        doc["batches"].append({
            "name": name, "config": cfg, "kwargs": kw, "records": int(wl.n_records), "chains": int(wl.n_chains),
            "plaintext_bytes": int(wl.plaintext_total),
            "wire_sha256": hashlib.sha256(b"".join(wires)).hexdigest(),
            "state_sha256": hashlib.sha256("\n".join(states).encode()).hexdigest()})
        print("%s: %d records, %.1f s" % (name, wl.n_records, time.time() - t0), flush=True)
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()

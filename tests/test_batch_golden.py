"""Whole-batch parity against digests captured from the reference:
small cfg2-cfg5 workloads sealed by tlslite's own `_sendMsg` (tests/golden/
make_batch_golden.py -> tests/golden/batches.json).  The C oracle must reproduce every
digest (CPU), and so must the HIP path through `tlsgpu_seal_dev` (GPU): every wire byte
of every record and every connection's final CBC residue / RC4 state / seqnum."""
import hashlib
import json
import os

import numpy as np
import pytest

from tlslite_amd import workloads as W

HERE = os.path.dirname(os.path.abspath(__file__))
DOC = json.load(open(os.path.join(HERE, "golden", "batches.json")))
BATCHES = {b["name"]: b for b in DOC["batches"]}


def _workload(b):
    return W.CONFIGS[b["config"]](**b["kwargs"])


def _wire_digest(wl, wire, lens):
    h = hashlib.sha256()
    for r in range(wl.n_records):
        assert int(lens[r]) == int(wl.wire_len[r]), r
        o = int(wl.wire_off[r])
        h.update(wire[o:o + int(lens[r])].tobytes())
    return h.hexdigest()


def _state_digest(wl, seqnum, iv, rc4):
    rows = []
    for c in range(wl.n_chains):
        suite = wl.groups[wl.chain_group[c]].suite
        if suite.startswith("RC4"):
            S, i, j = rc4(c)
            rows.append("%s|%d|%d|%d|%s" % (suite, seqnum(c), i, j, bytes(S).hex()))
        else:
            rows.append("%s|%d|%s" % (suite, seqnum(c), bytes(iv(c)).hex()))
    return hashlib.sha256("\n".join(rows).encode()).hexdigest()


@pytest.mark.parametrize("name", sorted(BATCHES))
def test_oracle_matches_reference_batch(name):
    from tests.wl_oracle import oracle_seal
    b = BATCHES[name]
    wl = _workload(b)
    assert (wl.n_records, wl.n_chains) == (b["records"], b["chains"])
    wire, lens, conns = oracle_seal(wl)
    assert _wire_digest(wl, wire, lens) == b["wire_sha256"]
    assert _state_digest(wl, lambda c: conns[c].seqnum, lambda c: conns[c].iv,
                         lambda c: conns[c].rc4) == b["state_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BATCHES))
def test_hip_matches_reference_batch(name):
    from tlslite_amd.device import synchronize
    from tests.wl_oracle import device_states
    b = BATCHES[name]
    wl = _workload(b)
    wl.to_device()
    wl.launch()
    synchronize()
    wire = wl.d_wire.download()
    d_len = wl.d_len.download().view(np.int32)  # the device's own wire_len output
    assert d_len.tolist() == wl.wire_len.astype(np.int32).tolist()
    assert _wire_digest(wl, wire, d_len) == b["wire_sha256"]
    st = device_states(wl)
    assert _state_digest(wl, lambda c: st[c].seqnum, lambda c: st[c].iv, lambda c: st[c].rc4) == b["state_sha256"]
    wl.free()

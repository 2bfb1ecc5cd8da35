"""Test helper: seal a device workload (tlslite_amd.workloads.Workload) with
the CPU oracle, for full-arena parity checks of the HIP path.  Test
infrastructure only."""
import ctypes

import numpy as np


def oracle_conns(wl):
    """One oracle connection per chain of the workload, in chain order."""
    from oracle import oracle as O
    out = []
    for c in range(wl.n_chains):
        g = wl.groups[wl.chain_group[c]]
        gi = c - int(np.searchsorted(wl.chain_group, wl.chain_group[c]))
        key = g.keys[gi % len(g.keys)]
        mk = g.mac_keys[gi % len(g.mac_keys)]
        fiv = g.fixed_ivs[gi % len(g.fixed_ivs)] if g.fixed_ivs is not None else None
        iv = bytes(g.ivs[gi]) if g.ivs is not None else b""
        out.append(O.Conn.for_suite(g.suite, g.version, bytes(key), iv, bytes(mk),
                                    None if fiv is None else bytes(fiv), int(g.seq0[gi])))
    return out


def oracle_seal(wl, nthreads=8):
    """-> (wire arena, wire_len per record, oracle connections after the batch)."""
    from oracle import oracle as O
    conns = oracle_conns(wl)
    pt = wl.host_plaintext(O.fill_pattern)
    wire = np.zeros(wl.wire_bytes, dtype=np.uint8)
    lens = O.seal_batch(conns, wl.chain_first, wl.chain_count, pt, wl.pt_off, wl.pt_len, wire, wl.wire_off,
                        ctype=wl.rec_ctype, flags=wl.rec_flags, nthreads=nthreads, update=True)
    return wire, lens, conns


def device_states(wl):
    """Connection states of the workload as the device holds them, as
    tlslite_amd.ConnectionState-like accessors (iv, seqnum, rc4)."""
    from tlslite_amd.state import STATE_BYTES, ConnectionState
    raw = wl.d_states.download()
    out = []
    for c in range(wl.n_chains):
        st = ConnectionState.__new__(ConnectionState)
        g = wl.groups[wl.chain_group[c]]
        from tlslite_amd.constants import suite_primitives
        st.cipher, st.mac = suite_primitives(g.suite)[:2]
        st.version = g.version
        st.raw = bytearray(raw[c * STATE_BYTES:(c + 1) * STATE_BYTES].tobytes())
        out.append(st)
    return out

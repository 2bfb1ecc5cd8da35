"""ABI 6 bounds of the device-resident batch calls (tlsgpu_seal_dev, tlsgpu_pipeline_seal,
tlsgpu_open_dev): the descriptors live in device memory, so the kernels check every record
against the caller's arena sizes and every chain against the state count.  A batch of valid
records is mixed with records whose plaintext / wire / ciphertext range leaves its arena and
with a chain whose state index is past the states array; then
  * every valid record equals the CPU oracle (which seals / opens only the valid ones: a
    refused record consumes no seqnum and leaves the CBC residue / RC4 state alone),
  * every refused record reports TLSGPU_EINVAL,
  * the guard bytes around the plaintext and wire arenas and the guard states after the
    states array are untouched.
The reference refuses bad lengths at the object boundary (utils/aes.py:28-34,
codec.py:19-20); here the boundary is the batch descriptor."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

G = 4096          # guard bytes before and after each arena
GUARD = 0xA5      # guard pattern
NGUARD_STATES = 3


def _T():
    import tlslite_amd as T
    from tlslite_amd import device
    if device.device_count() < 1:
        pytest.fail("no GPU visible to libtlsgpu (the gpu tests need an MI355X)")
    return T


def _plan(rng, suite, version, nconn, T, O):
    """Connections (GPU state + oracle) and a record plan: per connection 1-5 records of
    1-2000 B; ~15 % of them are made invalid in one of four ways."""
    _, kl, ivl, _, ml = O.SUITES[suite]
    states, ocs = [], []
    for _ in range(nconn):
        key, iv, mk = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml)
        fiv = rng.bytes(ivl) if ivl else None
        seq = int(rng.integers(0, 2 ** 40))
        states.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        ocs.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
    plan = []  # (conn, payload, bad) in chain order
    for ci in range(nconn):
        for _ in range(int(rng.integers(1, 6))):
            u = rng.random()
            bad = None if u > 0.15 else ("pt_off", "pt_len", "wire_off", "wire_end")[int(rng.integers(0, 4))]
            plan.append((ci, rng.bytes(int(rng.integers(1, 2001))), bad))
    return states, ocs, plan


def _guarded(nbytes, fill=GUARD):
    """A device buffer of G + nbytes + G bytes, guards set to the pattern, the arena zero."""
    from tlslite_amd.device import DeviceBuffer
    h = np.full(G + nbytes + G, fill, dtype=np.uint8)
    h[G:G + nbytes] = 0
    d = DeviceBuffer(h.size)
    d.upload(h)
    return d, h


def _layout(plan, states):
    """Plaintext / wire offsets of the valid layout; the refused records' descriptors point
    past an arena edge (their arena space is not reserved)."""
    from tlslite_amd.recordlayer import wire_offsets
    pt_off, pos = [], 0
    for _, p, _ in plan:
        pt_off.append(pos)
        pos += len(p) + (-len(p)) % 16
    pt_bytes = max(pos, 16)
    wl = [states[ci].wire_len(len(p)) for ci, p, _ in plan]
    wire_off, wire_bytes = wire_offsets(wl)
    wire_off = [int(x) for x in wire_off]
    pt_len = [len(p) for _, p, _ in plan]
    for k, (_, p, bad) in enumerate(plan):
        if bad == "pt_off":        # starts past the plaintext arena
            pt_off[k] = pt_bytes + 16 * (k % 7)
        elif bad == "pt_len":      # runs past the plaintext arena's end
            pt_off[k] = pt_bytes - 16
            pt_len[k] = 64 + len(p) % 1500
        elif bad == "wire_off":    # header past the wire arena
            wire_off[k] = wire_bytes + 11 + 16 * (k % 5)
        elif bad == "wire_end":    # header inside, sealed record runs past the end
            wire_off[k] = wire_bytes - 5 - 8
    return pt_off, pt_len, wire_off, wl, pt_bytes, wire_bytes


@pytest.mark.parametrize("suite,version,path", [("AES128-SHA", (3, 3), "dev"), ("AES256-SHA256", (3, 3), "pipeline"),
                                                ("AES128-SHA", (3, 1), "pipeline"), ("3DES-SHA", (3, 2), "dev"),
                                                ("RC4-SHA", (3, 1), "dev"), ("RC4-MD5", (3, 0), "pipeline")])
def test_seal_refuses_out_of_range_records(suite, version, path):
    from oracle import oracle as O
    T = _T()
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, Stream, synchronize
    from tlslite_amd.recordlayer import SealPipeline, make_chains, make_records, seal_dev
    from tlslite_amd.state import STATE_BYTES, pack_states, unpack_states
    rng = np.random.default_rng(zlib.crc32(repr(("bounds-seal", suite, version, path)).encode()))
    nconn = 300
    states, ocs, plan = _plan(rng, suite, version, nconn, T, O)
    pt_off, pt_len, wire_off, wl, pt_bytes, wire_bytes = _layout(plan, states)
    # one chain per connection, plus the last connection's records again under a state index
    # past the array (a chain the kernels must refuse without reading its state)
    firsts, counts = [], []
    k = 0
    for ci in range(nconn):
        n = sum(1 for c, _, _ in plan if c == ci)
        firsts.append(k)
        counts.append(n)
        k += n
    chain_state = list(range(nconn))
    bad_state_first = len(plan)
    extra = [(nconn - 1, p, "state") for c, p, b in plan if c == nconn - 1 and b is None]
    for _, p, _ in extra:
        pt_off.append(0)
        pt_len.append(len(p))
        wire_off.append(11)
        wl.append(0)
    plan = plan + extra
    chain_state.append(nconn + 1)  # inside the guard states, past nstates
    firsts.append(bad_state_first)
    counts.append(len(extra))
    # host plaintext arena (valid records only; refused ones read nothing)
    pt_host = np.zeros(pt_bytes, dtype=np.uint8)
    for (ci, p, bad), o in zip(plan, pt_off):
        if bad is None:
            pt_host[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    d_pt, pt_full = _guarded(pt_bytes)
    pt_full[G:G + pt_bytes] = pt_host
    d_pt.upload(pt_full)
    d_wire, wire_full0 = _guarded(wire_bytes)
    st_host = np.concatenate([pack_states(states), np.full(NGUARD_STATES * STATE_BYTES, GUARD, dtype=np.uint8)])
    d_states = DeviceBuffer(st_host.size)
    d_states.upload(st_host)
    recs = make_records(pt_off, wire_off, pt_len, 23, 0)
    d_recs = DeviceBuffer(len(plan) * 24)
    d_recs.upload(np.frombuffer(recs, dtype=np.uint8))
    chains = make_chains(chain_state, firsts, counts)
    d_ch = DeviceBuffer(len(firsts) * 16)
    d_ch.upload(np.frombuffer(chains, dtype=np.uint8))
    d_len = DeviceBuffer(4 * len(plan))
    d_len.zero()
    synchronize()
    var = states[0].variant
    args = (d_ch, len(firsts), d_recs, len(plan), d_pt.at(G).value, d_wire.at(G).value, d_states, d_len, var)
    kw = dict(pt_bytes=pt_bytes, wire_bytes=wire_bytes, nstates=nconn)
    if path == "dev":
        s = Stream()
        seal_dev(*args, stream=s, **kw)
        s.synchronize()
    else:
        with SealPipeline(len(plan)) as pipe:
            pipe.seal(*args, **kw)
            pipe.synchronize()
    lens = d_len.download().view(np.int32)
    wire_full = d_wire.download()
    st_after = d_states.download()
    # guards
    assert (wire_full[:G] == GUARD).all() and (wire_full[G + wire_bytes:] == GUARD).all(), "wire guard written"
    assert (d_pt.download() == pt_full).all(), "plaintext arena or its guards written"
    assert (st_after[nconn * STATE_BYTES:] == GUARD).all(), "guard state touched"
    # refused records
    bad_idx = [k for k, (_, _, b) in enumerate(plan) if b is not None]
    assert bad_idx and any(plan[k][2] == "state" for k in bad_idx)
    for k in bad_idx:
        assert lens[k] == N.EINVAL, (k, plan[k][2], lens[k])
    # valid records: the oracle sealing only them, in chain order
    expect = np.zeros(wire_bytes, dtype=np.uint8)
    for k, (ci, p, bad) in enumerate(plan):
        if bad is not None:
            continue
        w = ocs[ci].seal(p, 23)
        assert lens[k] == len(w) == wl[k], (k, lens[k], len(w))
        expect[wire_off[k]:wire_off[k] + len(w)] = np.frombuffer(w, dtype=np.uint8)
    assert np.array_equal(wire_full[G:G + wire_bytes], expect), "wire arena differs from the oracle's valid records"
    got_states = [s.copy() for s in states]
    unpack_states(st_after[:nconn * STATE_BYTES], got_states)
    for st, oc in zip(got_states, ocs):
        assert st.seqnum == oc.seqnum
        if suite.startswith("RC4"):
            S, i, j = st.rc4
            oS, oi, oj = oc.rc4
            assert (bytes(S), i, j) == (bytes(oS), oi, oj)
        else:
            assert st.iv == oc.iv
    for b in (d_pt, d_wire, d_states, d_recs, d_ch, d_len):
        b.free()


@pytest.mark.parametrize("suite,version", [("AES128-SHA", (3, 3)), ("AES256-SHA", (3, 0)), ("3DES-SHA", (3, 1)),
                                           ("RC4-SHA", (3, 1))])
def test_open_refuses_out_of_range_records(suite, version):
    from oracle import oracle as O
    T = _T()
    from tlslite_amd import _native as N
    from tlslite_amd.device import DeviceBuffer, Stream
    from tlslite_amd.recordlayer import make_chains, make_open_records, open_dev
    from tlslite_amd.state import STATE_BYTES, pack_states, unpack_states
    rng = np.random.default_rng(zlib.crc32(repr(("bounds-open", suite, version)).encode()))
    nconn = 300
    writers, ows, plan = _plan(rng, suite, version, nconn, T, O)
    readers = [w.copy() for w in writers]
    oreaders = [o.copy() for o in ows]
    # the peer's records of each connection in order -- the valid ones only: a refused record
    # is as if it were not in the batch, so the next valid one follows the previous valid one
    # (seqnum, CBC residue / RC4 keystream); a refused record gets a random body of a valid size
    bs = 0 if suite.startswith("RC4") else (8 if suite.startswith("3DES") else 16)
    bodies = []
    for ci, p, bad in plan:
        if bad is None:
            bodies.append(ows[ci].seal(p, 23)[5:])
        else:
            n = len(p) + 40
            bodies.append(rng.bytes(n + ((-n) % bs if bs else 0)))
    ct_off, pos = [], 0
    for b in bodies:
        ct_off.append(pos)
        pos += len(b) + (-len(b)) % 16
    wire_bytes = pt_bytes = max(pos, 16)
    ct_len = [len(b) for b in bodies]
    pt_off = list(ct_off)
    for k, (_, _, bad) in enumerate(plan):
        if bad == "pt_off":
            pt_off[k] = pt_bytes + 16
        elif bad == "pt_len":           # its plaintext would run past the plaintext arena
            pt_off[k] = pt_bytes - 16
        elif bad == "wire_off":
            ct_off[k] = wire_bytes + 32
        elif bad == "wire_end":         # its ciphertext runs past the wire arena
            ct_off[k] = wire_bytes - 16
    firsts, counts, k = [], [], 0
    for ci in range(nconn):
        n = sum(1 for c, _, _ in plan if c == ci)
        firsts.append(k)
        counts.append(n)
        k += n
    chain_state = list(range(nconn))
    # a chain with a state index past the array, over the first connection's records
    firsts.append(firsts[0])
    counts.append(counts[0])
    chain_state.append(nconn)
    wire_host = np.zeros(wire_bytes, dtype=np.uint8)
    for k, b in enumerate(bodies):
        if plan[k][2] in (None, "pt_off", "pt_len"):
            wire_host[ct_off[k]:ct_off[k] + len(b)] = np.frombuffer(b, dtype=np.uint8)
    d_wire, wire_full = _guarded(wire_bytes)
    wire_full[G:G + wire_bytes] = wire_host
    d_wire.upload(wire_full)
    d_pt, _ = _guarded(pt_bytes)
    st_host = np.concatenate([pack_states(readers), np.full(NGUARD_STATES * STATE_BYTES, GUARD, dtype=np.uint8)])
    d_states = DeviceBuffer(st_host.size)
    d_states.upload(st_host)
    recs = make_open_records(ct_off, pt_off, ct_len, 23)
    d_recs = DeviceBuffer(len(plan) * 24)
    d_recs.upload(np.frombuffer(recs, dtype=np.uint8))
    d_st = DeviceBuffer(4 * len(plan))
    d_st.zero()
    s = Stream()
    var = readers[0].variant
    # the valid chains first, then (same call order on one stream) the bad-state chain over
    # records the first call already opened: its statuses must come back EINVAL
    ch = make_chains(chain_state[:nconn], firsts[:nconn], counts[:nconn], 0)
    d_ch = DeviceBuffer(nconn * 16)
    d_ch.upload(np.frombuffer(ch, dtype=np.uint8), stream=s)
    open_dev(d_ch, nconn, d_recs, len(plan), d_wire.at(G).value, d_pt.at(G).value, d_states, d_st, var, stream=s,
             wire_bytes=wire_bytes, pt_bytes=pt_bytes, nstates=nconn)
    s.synchronize()
    status = d_st.download().view(np.int32).copy()
    bad_ch = make_chains([nconn], [firsts[0]], [counts[0]], 0)
    d_bch = DeviceBuffer(16)
    d_bch.upload(np.frombuffer(bad_ch, dtype=np.uint8), stream=s)
    open_dev(d_bch, 1, d_recs, len(plan), d_wire.at(G).value, d_pt.at(G).value, d_states, d_st, var, stream=s,
             wire_bytes=wire_bytes, pt_bytes=pt_bytes, nstates=nconn)
    s.synchronize()
    status2 = d_st.download().view(np.int32)
    assert (status2[:counts[0]] == N.EINVAL).all(), "bad-state chain not refused"
    assert np.array_equal(status2[counts[0]:], status[counts[0]:])
    pt_full = d_pt.download()
    st_after = d_states.download()
    assert (pt_full[:G] == GUARD).all() and (pt_full[G + pt_bytes:] == GUARD).all(), "plaintext guard written"
    assert (d_wire.download() == wire_full).all(), "wire arena or its guards written"
    assert (st_after[nconn * STATE_BYTES:] == GUARD).all(), "guard state touched"
    got = pt_full[G:G + pt_bytes]
    for k, (ci, p, bad) in enumerate(plan):
        if bad is not None:
            assert status[k] == N.EINVAL, (k, bad, status[k])
            continue
        ost, opt = oreaders[ci].open(bodies[k], 23)
        assert ost == 0 and opt == p
        assert status[k] == len(p), (k, status[k])
        assert got[pt_off[k]:pt_off[k] + len(p)].tobytes() == p
    got_states = [r.copy() for r in readers]
    unpack_states(st_after[:nconn * STATE_BYTES], got_states)
    for st, oc in zip(got_states, oreaders):
        assert st.seqnum == oc.seqnum
        if not suite.startswith("RC4"):
            assert st.iv == oc.iv
    for b in (d_pt, d_wire, d_states, d_recs, d_ch, d_bch, d_st):
        b.free()

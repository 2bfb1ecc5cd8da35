"""Records at arena offsets past 2^31 and 2^32 (BASELINE cfg4's one-GPU arenas are 16 GiB).

Round 5's open decrypt rebuilt each record's 64-bit ct_off / pt_off from two wave lanes with a
plain (uint64_t) cast of __builtin_amdgcn_readlane's int result: a low word >= 2^31 was
sign-extended and the kernel read and wrote at 0xffffffff'xxxxxxxx (the illegal memory access
of round 5's cfg4 open leg).  Every GPU test then used arenas < 2 GiB, so none saw it.

Here one batch per suite lives in three 6.5 GiB device arenas (plaintext, wire, opened
plaintext) with its records placed around 2^31, across 2^32 and above it (low words with bit
31 set and clear).  The HIP seal (tlsgpu_seal_dev, and the pipeline for AES) must equal the CPU
oracle's seal (tlsrecordlayer.py:538-616), and the HIP open (tlsgpu_open_dev) of those wire
records must equal the oracle's open (:958-1044): status, plaintext, and the read states'
final CBC residue / RC4 state and seqnum.  Test infrastructure: the oracle checks, the HIP
path runs."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ARENA = (13 << 29) + (1 << 20)  # 6.5 GiB + 1 MiB
# placement bases, >= 1 MiB apart (a base takes up to 8 records of <= 16.5 KiB): low, across
# 2^31, bit 31 set, across 2^32, above 2^32 with bit 31 clear / set
BASES = [0x10, 0x7FFF_C000, 0x8010_0000, 0xFFFF_E000, 0x1_0010_0040, 0x1_8000_1000, 0x1_2000_0000]


def _T():
    import tlslite_amd as T
    from tlslite_amd import device
    if device.device_count() < 1:
        pytest.fail("no GPU visible to libtlsgpu (the gpu tests need an MI355X)")
    return T


def _place(sizes, shift):
    """Offsets of records of the given sizes: record k at the next free 16-byte slot after
    BASES[k % len(BASES)] + shift (records sharing a base are packed after each other)."""
    cur = [b + shift for b in BASES]
    out = []
    for k, n in enumerate(sizes):
        i = k % len(BASES)
        out.append(cur[i])
        cur[i] += n + (-n) % 16 + 16
    assert max(o + n for o, n in zip(out, sizes)) <= ARENA
    iv = sorted(zip(out, sizes))
    assert all(a + n <= b for (a, n), (b, _) in zip(iv, iv[1:])), "records overlap"
    return out


@pytest.mark.parametrize("suite,version,path", [("AES128-SHA", (3, 3), "dev"), ("AES128-SHA", (3, 3), "pipeline"),
                                                ("AES256-SHA256", (3, 3), "dev"), ("AES128-SHA", (3, 1), "dev"),
                                                ("3DES-SHA", (3, 2), "dev"), ("RC4-SHA", (3, 1), "dev")])
def test_offsets_past_4gib_seal_and_open_vs_oracle(suite, version, path):
    from oracle import oracle as O
    T = _T()
    from tlslite_amd.device import DeviceBuffer, Stream
    from tlslite_amd.recordlayer import (SealPipeline, make_chains, make_open_records, make_records, open_dev,
                                         open_workspace_bytes, seal_dev)
    from tlslite_amd.state import pack_states, unpack_states
    rng = np.random.default_rng(zlib.crc32(repr(("bigarena", suite, version, path)).encode()))
    _, kl, ivl, _, ml = O.SUITES[suite]
    nconn, per = 10, 5
    wst, rst, ow, orr = [], [], [], []
    for _ in range(nconn):
        key, iv, mk = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml)
        fiv = rng.bytes(ivl) if ivl else None
        seq = int(rng.integers(0, 2 ** 40))
        wst.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        rst.append(T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq))
        ow.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
        orr.append(O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq))
    # chain order: connection ci's records are [ci * per, (ci + 1) * per); consecutive records of
    # one chain land at different bases, so a chain walks across the 2^31 / 2^32 boundaries
    pts = [rng.bytes(int(rng.choice([1, 300, 1434, 4099, 16384]))) for _ in range(nconn * per)]
    pt_len = [len(p) for p in pts]
    wl = [wst[k // per].wire_len(n) for k, n in enumerate(pt_len)]
    pt_off = _place(pt_len, 0)
    wire_off = [o + 11 for o in _place(wl, 0x100)]  # body after the explicit IV at varied line offsets
    opt_off = _place([w - 5 for w in wl], 0x3000)  # the open writes the whole body after the IV
    s = Stream()
    d_pt, d_wire, d_opt = DeviceBuffer(ARENA), DeviceBuffer(ARENA), DeviceBuffer(ARENA)
    bufs = [d_pt, d_wire, d_opt]
    try:
        for p, o in zip(pts, pt_off):
            d_pt.upload(np.frombuffer(p, dtype=np.uint8), offset=o, stream=s)
        recs = make_records(pt_off, wire_off, pt_len, 23, 0)
        d_recs = DeviceBuffer(len(pts) * 24)
        d_recs.upload(np.frombuffer(recs, dtype=np.uint8), stream=s)
        ch = make_chains(list(range(nconn)), [c * per for c in range(nconn)], [per] * nconn, 0)
        d_ch = DeviceBuffer(nconn * 16)
        d_ch.upload(np.frombuffer(ch, dtype=np.uint8), stream=s)
        d_ws = DeviceBuffer(pack_states(wst).size)
        d_ws.upload(pack_states(wst), stream=s)
        d_len = DeviceBuffer(4 * len(pts))
        bufs += [d_recs, d_ch, d_ws, d_len]
        var = wst[0].variant
        s.synchronize()
        if path == "pipeline":
            with SealPipeline(len(pts)) as pipe:
                pipe.seal(d_ch, nconn, d_recs, len(pts), d_pt, d_wire, d_ws, d_len, var)
                pipe.synchronize()
        else:
            seal_dev(d_ch, nconn, d_recs, len(pts), d_pt, d_wire, d_ws, d_len, var, stream=s)
        s.synchronize()
        lens = d_len.download().view(np.int32)
        bodies = []
        for k, p in enumerate(pts):
            want = ow[k // per].seal(p, 23)
            assert int(lens[k]) == len(want), (suite, k, int(lens[k]), len(want), hex(wire_off[k]))
            got = d_wire.download(len(want), offset=wire_off[k]).tobytes()
            assert got == want, (suite, "seal", k, hex(wire_off[k]))
            bodies.append(want[5:])
        unpack_states(d_ws.download(), wst)
        for w, o in zip(wst, ow):
            assert w.seqnum == o.seqnum
            assert (w.rc4 == o.rc4) if O.SUITES[suite][0] == "rc4" else (w.iv == o.iv)
        # open the sealed records where they lie (ct at wire_off + 5) into a third arena
        orecs = make_open_records([o + 5 for o in wire_off], opt_off, [len(b) for b in bodies], 23)
        d_orecs = DeviceBuffer(len(pts) * 24)
        d_orecs.upload(np.frombuffer(orecs, dtype=np.uint8), stream=s)
        d_rs = DeviceBuffer(pack_states(rst).size)
        d_rs.upload(pack_states(rst), stream=s)
        d_st = DeviceBuffer(4 * len(pts))
        d_ows = DeviceBuffer(max(16, open_workspace_bytes(len(pts))))
        bufs += [d_orecs, d_rs, d_st, d_ows]
        open_dev(d_ch, nconn, d_orecs, len(pts), d_wire, d_opt, d_rs, d_st, var, d_ows, s)
        s.synchronize()
        status = d_st.download().view(np.int32)
        for k, b in enumerate(bodies):
            code, want = orr[k // per].open(b, 23)
            assert code == 0 and want == pts[k]
            assert int(status[k]) == len(want), (suite, "open", k, int(status[k]), hex(opt_off[k]))
            assert d_opt.download(len(want), offset=opt_off[k]).tobytes() == want, (suite, "open", k)
        unpack_states(d_rs.download(), rst)
        for r, o in zip(rst, orr):
            assert r.seqnum == o.seqnum
            assert (r.rc4 == o.rc4) if O.SUITES[suite][0] == "rc4" else (r.iv == o.iv)
    finally:
        for b in bufs:
            b.free()

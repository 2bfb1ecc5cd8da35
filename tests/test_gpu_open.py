"""GPU parity of the open path (decrypt + padding + MAC verify,
tlsrecordlayer.py:958-1044) against the CPU oracle and the golden vectors."""
import os
import zlib

import numpy as np
import pytest

from tests.golden_io import case_keys, rec_pt

pytestmark = pytest.mark.gpu

SUITES = ["AES128-SHA", "AES256-SHA", "AES128-SHA256", "AES256-SHA256", "RC4-SHA", "RC4-MD5", "3DES-SHA"]


def _valid(suites, versions):
    """(suite, version) pairs the reference accepts: SHA256 suites are TLS 1.2 only."""
    return [(s, v) for v in versions for s in suites if not (s.endswith("SHA256") and v != (3, 3))]


def _T():
    import tlslite_amd as T
    from tlslite_amd import device
    if device.device_count() < 1:
        pytest.fail("no GPU visible")
    return T


def _mk(T, O, suite, version, rng):
    cipher, kl, ivl, mac, ml = O.SUITES[suite]
    key, iv, mk, fiv = rng.bytes(kl), rng.bytes(ivl), rng.bytes(ml), (rng.bytes(ivl) if ivl else None)
    seq = int(rng.integers(0, 2 ** 40))
    mk_t = lambda: T.ConnectionState.for_suite(suite, version, key, iv, mk, fiv, seq)  # noqa: E731
    mk_o = lambda: O.Conn.for_suite(suite, version, key, iv, mk, fiv, seq)  # noqa: E731
    return mk_t, mk_o


@pytest.mark.parametrize("suite,version", _valid(SUITES, [(3, 0), (3, 1), (3, 2), (3, 3)]))
def test_seal_open_roundtrip_and_state(suite, version):
    from oracle import oracle as O
    from tlslite_amd.recordlayer import open_records
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr((suite, version)).encode()))
    writers, readers, oreaders, recs = [], [], [], []
    for ci in range(24):
        mk_t, mk_o = _mk(T, O, suite, version, rng)
        writers.append(mk_t())
        readers.append(mk_t())
        oreaders.append(mk_o())
        for _ in range(int(rng.integers(1, 4))):
            n = int(rng.choice([1, 15, 16, 17, 63, 64, 65, 300, 1434, 16384]))
            recs.append((ci, rng.bytes(n), int(rng.choice([21, 23]))))
    wires = T.seal(writers, recs)
    opened = open_records(readers, [(ci, w[0], w[5:]) for (ci, _, _), w in zip(recs, wires)])
    for (ci, p, ct), w, (st, got) in zip(recs, wires, opened):
        assert st == 0 and got == p, (suite, version, len(p))
        ost, opt = oreaders[ci].open(w[5:], w[0])
        assert ost == 0 and opt == p
    for r, o in zip(readers, oreaders):
        assert r.seqnum == o.seqnum
        if O.SUITES[suite][0] == "rc4":
            assert r.rc4 == o.rc4
        else:
            assert r.iv == o.iv


@pytest.mark.parametrize("suite", ["AES128-SHA", "AES256-SHA256", "RC4-SHA", "3DES-SHA"])
def test_tamper_detected_like_oracle(suite):
    """Flip one bit anywhere in the body: status must equal the oracle's
    (bad_record_mac, or decryption_failed for bad lengths), including the
    consumed-seqnum behaviour."""
    from oracle import oracle as O
    from tlslite_amd import _native as N
    from tlslite_amd.recordlayer import open_records
    T = _T()
    version = (3, 3)
    rng = np.random.default_rng(zlib.crc32(suite.encode()))
    cases = []
    for i in range(60):
        mk_t, mk_o = _mk(T, O, suite, version, rng)
        w = T.seal([mk_t()], [(0, rng.bytes(int(rng.integers(1, 400))))])[0]
        body = bytearray(w[5:])
        kind = i % 3
        if kind == 0:
            body[int(rng.integers(0, len(body)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1 and O.SUITES[suite][0] != "rc4":
            body = body[:-1]  # not a multiple of the block size
        cases.append((mk_t(), mk_o(), bytes(body)))
    res = open_records([c[0] for c in cases], [(i, 23, c[2]) for i, c in enumerate(cases)])
    for (t, o, body), (st, p) in zip(cases, res):
        ost, opt = o.open(body, 23)
        exp = {0: 0, O.ALERT_BAD_RECORD_MAC: N.ALERT_BAD_RECORD_MAC,
               O.ALERT_DECRYPTION_FAILED: N.ALERT_DECRYPTION_FAILED}[ost]
        assert st == exp
        if st == 0:
            assert p == opt
        assert t.seqnum == o.seqnum


def test_golden_fault_records_rejected(golden):
    """The reference's badMAC/badPadding records (constants.py Fault) must
    raise bad_record_mac on open."""
    from tlslite_amd import _native as N
    from tlslite_amd.recordlayer import open_records
    T = _T()
    states, recs, expect = [], [], []
    for c in golden:
        if not c.get("fault"):
            continue
        key, iv, mk, fiv, seq = case_keys(c)
        si = len(states)
        states.append(T.ConnectionState.for_suite(c["suite"], tuple(c["version"]), key, iv, mk, fiv, seq))
        effective = c["fault"] == "badMAC" or not c["suite"].startswith("RC4")
        for r in c["records"]:
            w = bytes.fromhex(r["wire"])
            recs.append((si, w[0], w[5:]))
            expect.append(N.ALERT_BAD_RECORD_MAC if effective else 0)
            if effective:
                break
    res = open_records(states, recs)
    assert [s for s, _ in res] == expect


def test_parse_records_overflow():
    from tlslite_amd.recordlayer import RecordOverflow, parse_records
    recs, rest = parse_records(b"\x17\x03\x03\x00\x02ab\x17\x03")
    assert recs == [(23, (3, 3), b"ab")] and rest == b"\x17\x03"
    with pytest.raises(RecordOverflow):
        parse_records(b"\x17\x03\x03\x48\x01" + bytes(10))


@pytest.mark.parametrize("suite,version", _valid(["AES128-SHA", "AES256-SHA256", "3DES-SHA", "RC4-MD5"],
                                                 [(3, 0), (3, 1), (3, 2), (3, 3)]))
def test_malformed_chains_like_oracle(suite, version):
    """Chains mixing valid records with empty, IV-only, random-garbage and
    non-block-multiple bodies (tlsrecordlayer.py:964-977: b[bs:] of a body no
    longer than one block is empty -> decryption_failed): every status and the
    final seqnum / CBC residue / RC4 state equal the oracle's."""
    from oracle import oracle as O
    from tlslite_amd import _native as N
    from tlslite_amd.recordlayer import open_records
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr(("malformed", suite, version)).encode()))
    bs = {"aes128": 16, "aes256": 16, "3des": 8, "rc4": 1}[O.SUITES[suite][0]]
    readers, oreaders, recs = [], [], []
    for ci in range(16):
        mk_t, mk_o = _mk(T, O, suite, version, rng)
        w_o = mk_o()
        readers.append(mk_t())
        oreaders.append(mk_o())
        for k in range(6):
            kind = int(rng.integers(0, 5))
            if kind == 0:
                body = b""
            elif kind == 1:
                body = rng.bytes(bs)
            elif kind == 2:
                body = rng.bytes(bs * int(rng.integers(2, 8)))
            elif kind == 3:
                body = rng.bytes(bs * 3 + (1 if bs > 1 else 0))
            else:
                body = w_o.seal(rng.bytes(int(rng.integers(1, 200))), 23)[5:]
            recs.append((ci, 23, body))
    res = open_records(readers, recs, stop_on_alert=False)
    amap = {0: 0, O.ALERT_BAD_RECORD_MAC: N.ALERT_BAD_RECORD_MAC,
            O.ALERT_DECRYPTION_FAILED: N.ALERT_DECRYPTION_FAILED}
    for (ci, ct, body), (st, p) in zip(recs, res):
        ost, opt = oreaders[ci].open(body, ct)
        assert st == amap[ost], (ci, len(body))
        if st == 0:
            assert p == opt
    for r, o in zip(readers, oreaders):
        assert r.seqnum == o.seqnum
        if O.SUITES[suite][0] == "rc4":
            assert r.rc4 == o.rc4
        else:
            assert r.iv == o.iv


def test_golden_open_chains(golden):
    """The reference's _decryptRecord statuses / plaintexts / final state over
    chains of valid, tampered and malformed bodies (tests/golden open cases:
    successive _decryptRecord calls that continue after an alert), all chains in
    one open_records call per variant, without stop-on-alert."""
    from tlslite_amd import _native as N
    from tlslite_amd.recordlayer import open_records
    T = _T()
    amap = {0: 0, 20: N.ALERT_BAD_RECORD_MAC, 21: N.ALERT_DECRYPTION_FAILED}
    states, recs, expect, cases = [], [], [], []
    for c in golden:
        if c["kind"] != "open":
            continue
        key, iv, mk, fiv, seq = case_keys(c)
        si = len(states)
        states.append(T.ConnectionState.for_suite(c["suite"], tuple(c["version"]), key, iv, mk, fiv, seq))
        cases.append(c)
        for b in c["bodies"]:
            recs.append((si, b["type"], bytes.fromhex(b["body"])))
            expect.append((amap[b["status"]], bytes.fromhex(b["pt"]) if b["status"] == 0 else None))
    assert len(cases) == 22
    res = open_records(states, recs, stop_on_alert=False)
    for (st, pt), (est, ept) in zip(res, expect):
        assert st == est
        if est == 0:
            assert pt == ept
    for s, c in zip(states, cases):
        f = c["final"]
        assert s.seqnum == f["seqnum"], c["name"]
        if "cbc_iv" in f:
            assert s.iv.hex() == f["cbc_iv"], c["name"]
        else:
            S, i, j = s.rc4
            assert (S.hex(), i, j) == (f["rc4_S"], f["rc4_i"], f["rc4_j"]), c["name"]


@pytest.mark.parametrize("suite,version", _valid(["AES128-SHA", "AES256-SHA256", "3DES-SHA", "RC4-SHA"],
                                                 [(3, 0), (3, 1), (3, 3)]))
def test_stop_on_alert_like_connection(suite, version):
    """Connection semantics (the default of open_records): a chain stops at its
    first alert -- the reference's _getMsg raises and _sendError closes the
    connection (tlsrecordlayer.py:1039-1042) -- so no plaintext after a tampered
    or dropped record is returned (ALERT_SKIPPED), and the state is the one the
    failing record left, equal to the oracle's after opening records up to and
    including the failing one."""
    from oracle import oracle as O
    from tlslite_amd import _native as N
    from tlslite_amd.recordlayer import open_records
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr(("stop", suite, version)).encode()))
    amap = {0: 0, O.ALERT_BAD_RECORD_MAC: N.ALERT_BAD_RECORD_MAC,
            O.ALERT_DECRYPTION_FAILED: N.ALERT_DECRYPTION_FAILED}
    readers, oreaders, recs, fail_at = [], [], [], []
    for ci in range(40):
        mk_t, mk_o = _mk(T, O, suite, version, rng)
        w_t = mk_t()
        readers.append(mk_t())
        oreaders.append(mk_o())
        n = int(rng.integers(3, 7))
        bad = int(rng.integers(0, n + 1)) if ci % 4 else n  # every 4th chain clean
        fail_at.append(bad)
        bodies = [w[5:] for w in T.seal([w_t], [(0, rng.bytes(int(rng.integers(1, 300))))
                                                for _ in range(n)])]
        for k, b in enumerate(bodies):
            if k == bad:
                b = bytearray(b)
                if ci % 3 == 0 and O.SUITES[suite][0] != "rc4":
                    b = b[:-1]  # decryption_failed
                else:
                    b[int(rng.integers(0, len(b)))] ^= 0x10
                b = bytes(b)
            recs.append((ci, 23, b))
    res = open_records(readers, recs)
    k_of = {}
    for (ci, ct, body), (st, p) in zip(recs, res):
        k = k_of.get(ci, 0)
        k_of[ci] = k + 1
        if k < fail_at[ci]:
            ost, opt = oreaders[ci].open(body, ct)
            assert (st, p) == (0, opt) and ost == 0
        elif k == fail_at[ci]:
            ost, _ = oreaders[ci].open(body, ct)
            assert ost < 0 and st == amap[ost] and p is None
        else:
            assert st == N.ALERT_SKIPPED and p is None
    for r, o in zip(readers, oreaders):
        assert r.seqnum == o.seqnum
        if O.SUITES[suite][0] == "rc4":
            assert r.rc4 == o.rc4
        else:
            assert r.iv == o.iv


@pytest.mark.parametrize("suite,version,mode", [("AES128-SHA", (3, 3), "chains"), ("AES256-SHA256", (3, 3), "chains"),
                                                ("3DES-SHA", (3, 1), "chains"), ("AES128-SHA", (3, 0), "chains"),
                                                ("AES128-SHA", (3, 3), "single"), ("AES256-SHA256", (3, 3), "single"),
                                                ("3DES-SHA", (3, 2), "single"), ("AES128-SHA", (3, 0), "single"),
                                                ("AES256-SHA", (3, 1), "single"), ("3DES-SHA", (3, 2), "blocks"),
                                                ("3DES-SHA", (3, 0), "blocks"), ("3DES-SHA", (3, 1), "blocks")])
def test_split_open_parts_like_oracle(suite, version, mode):
    """The open's forms (launch_open_split; tlsgpu_set_open_parts forces them on these small
    batches).  "chains": in parts on a second stream, the decrypt and padding pass of chain
    range h+1 beside the MAC pass of range h -- 6,000 connections of 1-6 records of 1-700 B.
    "single": one pass of each kernel on long records (the round-5 decrypt: next record's
    keys prefetched, DPP predecessors, wave priority rotation, byte-replicated inverse
    S-box) -- 900 connections of 1-4 records of 1 B-16 KiB.  "blocks" (3DES): the same records
    with every record's tail blocks and the padding pass first, then block range h+1 of every
    record beside the MAC of the payload ranges <= h produced, the hash state carried in the
    workspace, so records end in every part.  ~3 % of records tampered (a bit
    flipped anywhere: payload, MAC or padding) or truncated, connection (stop-on-alert)
    semantics: every status, plaintext and final state equals the oracle's, across the part
    boundaries (tlsrecordlayer.py:958-1044)."""
    from oracle import oracle as O
    from tlslite_amd import _native as N
    from tlslite_amd.device import cu_count
    from tlslite_amd.recordlayer import open_records, set_open_parts
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr(("parts", suite, version, mode)).encode()))
    amap = {0: 0, O.ALERT_BAD_RECORD_MAC: N.ALERT_BAD_RECORD_MAC,
            O.ALERT_DECRYPTION_FAILED: N.ALERT_DECRYPTION_FAILED}
    nconn, per, maxlen = (6000, 7, 701) if mode == "chains" else (900, 5, 16385)
    writers, readers, oreaders, plan = [], [], [], []
    for ci in range(nconn):
        mk_t, mk_o = _mk(T, O, suite, version, rng)
        writers.append(mk_t())
        readers.append(mk_t())
        oreaders.append(mk_o())
        for _ in range(int(rng.integers(1, per))):
            plan.append((ci, rng.bytes(int(rng.integers(1, maxlen))), int(rng.choice([21, 22, 23], p=[0.05, 0.05, 0.9]))))
    if mode == "chains":
        assert len(plan) >= 4 * 16 * cu_count(), "too few records for a part's decrypt to fill the chip"
    wires = T.seal(writers, plan)
    recs = []
    for (ci, _, ct), w in zip(plan, wires):
        body = bytearray(w[5:])
        u = rng.random()
        if u < 0.02:
            body[int(rng.integers(0, len(body)))] ^= 1 << int(rng.integers(0, 8))
        elif u < 0.03:
            body = body[:-1]
        recs.append((ci, ct, bytes(body)))
    set_open_parts({"chains": N.OPEN_SPLIT_CHAINS, "single": N.OPEN_SPLIT_NONE, "blocks": N.OPEN_SPLIT_BLOCKS}[mode], 1)
    try:
        res = open_records(readers, recs)
    finally:
        set_open_parts()
    stopped = set()
    for (ci, ct, body), (st, p) in zip(recs, res):
        if ci in stopped:
            assert st == N.ALERT_SKIPPED and p is None
            continue
        ost, opt = oreaders[ci].open(body, ct)
        assert st == amap[ost]
        if ost == 0:
            assert p == opt
        else:
            assert p is None
            stopped.add(ci)
    assert stopped, "no alerts exercised"
    for r, o in zip(readers, oreaders):
        assert r.seqnum == o.seqnum and r.iv == o.iv


@pytest.mark.parametrize("suites,version", [(["AES128-SHA"], (3, 3)), (["AES256-SHA256", "AES128-SHA"], (3, 3)),
                                            (["3DES-SHA", "RC4-SHA"], (3, 1)), (["AES128-SHA", "RC4-MD5"], (3, 0))])
def test_open_batches_closed_connections_like_oracle(suites, version):
    """Successive batches of the same connections opened with the states device-resident
    (open_batches: 5 batches, one open_dev call per batch and variant).  ~3 % of records
    tampered or truncated; a connection that alerts in batch k is closed in its state
    (ConnState.closed): it reports ALERT_SKIPPED for its later records in batch k AND in
    every later batch, and its state stays as the failing record left it.  Every status, plaintext and final state equals the oracle's reading the
    batches in order (tlsrecordlayer.py:958-1044, :1039-1042)."""
    from oracle import oracle as O
    from tlslite_amd import _native as N
    from tlslite_amd.recordlayer import open_batches
    T = _T()
    rng = np.random.default_rng(zlib.crc32(repr(("batches", suites, version)).encode()))
    amap = {0: 0, O.ALERT_BAD_RECORD_MAC: N.ALERT_BAD_RECORD_MAC,
            O.ALERT_DECRYPTION_FAILED: N.ALERT_DECRYPTION_FAILED}
    nconn, nbatch = 500, 5
    writers, readers, oreaders, suite_of = [], [], [], []
    for ci in range(nconn):
        suite = suites[ci % len(suites)]
        mk_t, mk_o = _mk(T, O, suite, version, rng)
        writers.append(mk_t())
        readers.append(mk_t())
        oreaders.append(mk_o())
        suite_of.append(suite)
    batches = []
    for _ in range(nbatch):
        plan = []
        for ci in range(nconn):
            for _ in range(int(rng.integers(0, 3))):
                n = int(rng.choice([int(rng.integers(1, 300)), int(rng.integers(300, 16385))]))
                plan.append((ci, rng.bytes(n), int(rng.choice([21, 22, 23], p=[0.05, 0.05, 0.9]))))
        wires = T.seal(writers, plan)
        recs = []
        for (ci, _, ct), w in zip(plan, wires):
            body = bytearray(w[5:])
            u = rng.random()
            if u < 0.02:
                body[int(rng.integers(0, len(body)))] ^= 1 << int(rng.integers(0, 8))
            elif u < 0.03 and O.SUITES[suite_of[ci]][0] != "rc4":
                body = body[:-1]
            recs.append((ci, ct, bytes(body)))
        batches.append(recs)
    res = open_batches(readers, batches)
    stopped = set()
    for recs, out in zip(batches, res):
        assert len(out) == len(recs)
        for (ci, ct, body), (st, p) in zip(recs, out):
            if ci in stopped:
                assert st == N.ALERT_SKIPPED and p is None
                continue
            ost, opt = oreaders[ci].open(body, ct)
            assert st == amap[ost]
            if ost == 0:
                assert p == opt
            else:
                assert p is None
                stopped.add(ci)
    assert stopped, "no alerts exercised"
    for ci, (r, o) in enumerate(zip(readers, oreaders)):
        assert r.seqnum == o.seqnum, ci
        if O.SUITES[suite_of[ci]][0] == "rc4":
            assert r.rc4 == o.rc4, ci
        else:
            assert r.iv == o.iv, ci

"""GPU parity of the open path (decrypt + padding + MAC verify,
tlsrecordlayer.py:958-1044) against the CPU oracle and the golden vectors."""
import zlib

import numpy as np
import pytest

from tests.golden_io import case_keys, rec_pt

pytestmark = pytest.mark.gpu

SUITES = ["AES128-SHA", "AES256-SHA", "AES128-SHA256", "AES256-SHA256", "RC4-SHA", "RC4-MD5", "3DES-SHA"]


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


@pytest.mark.parametrize("suite", SUITES)
@pytest.mark.parametrize("version", [(3, 0), (3, 1), (3, 2), (3, 3)])
def test_seal_open_roundtrip_and_state(suite, version):
    from oracle import oracle as O
    from tlslite_amd.recordlayer import open_records
    T = _T()
    if suite.endswith("SHA256") and version != (3, 3):
        pytest.skip("TLS 1.2 only")
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

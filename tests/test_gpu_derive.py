"""GPU: batched key derivation (tlsgpu_derive_states_dev, tg_derive.h) --
calcMasterSecret + _calcPendingStates (mathtls.py:24-82,
tlsrecordlayer.py:1061-1149) for many connections in one launch -- against
the reference-captured derivations and the CPU oracle's PRF, and the
derived device states against states built on the host from the oracle's
key-block slices (tlsgpu_conn_state_init): byte-identical 2 KiB blobs."""
import numpy as np
import pytest

from oracle import oracle as O
from tlslite_amd.constants import SUITE_NAMES

pytestmark = pytest.mark.gpu

# (suite, versions it may run at): SHA256 suites need TLS 1.2 (constants.py:204-210)
SUITE_VERSIONS = [(s, [(3, 0), (3, 1), (3, 2), (3, 3)]) for s in
                  ("AES128-SHA", "AES256-SHA", "RC4-SHA", "RC4-MD5", "3DES-SHA")] + \
                 [(s, [(3, 3)]) for s in ("AES128-SHA256", "AES256-SHA256")]


def _need_gpu():
    from tlslite_amd import device
    if device.device_count() < 1:
        pytest.fail("no GPU visible")


def _host_states(version, suite, master, cr, sr, client, fixed_iv):
    """pending write/read states as the host builds them from the oracle's
    key-block slices (same slicing as tlsrecordlayer.py:1117-1143)."""
    from tlslite_amd.state import ConnectionState
    cipher, kl, ivl, mac, ml = O.SUITES[suite]
    _, kp = O.key_block(version, suite, master, cr, sr)
    need_fiv = tuple(version) >= (3, 2) and ivl
    me, peer = ("client", "server") if client else ("server", "client")
    w = ConnectionState(cipher, mac, version, kp[me + "_key"], kp[me + "_iv"], kp[me + "_mac"],
                        fixed_iv[:ivl] if need_fiv else None)
    r = ConnectionState(cipher, mac, version, kp[peer + "_key"], kp[peer + "_iv"], kp[peer + "_mac"],
                        bytes(ivl) if need_fiv else None)
    return bytes(w.raw), bytes(r.raw)


def test_derive_golden_premaster(golden):
    """premaster -> master -> key block on the GPU equals the reference's."""
    _need_gpu()
    from tlslite_amd.connection import derive_pending_states_gpu
    cases = [c for c in golden if c["kind"] == "keys"]
    conns = []
    for k, c in enumerate(cases):
        conns.append({"secret": bytes.fromhex(c["premaster"]), "client_random": bytes.fromhex(c["client_random"]),
                      "server_random": bytes.fromhex(c["server_random"]), "suite": c["suite"],
                      "version": tuple(c["version"]), "client": k % 2 == 0,
                      "fixed_iv": bytes(range(16, 32))})
    d = derive_pending_states_gpu(conns, premaster=True, want_key_block=True)
    for k, c in enumerate(cases):
        assert bytes(d.master[k]).hex() == c["master"], c["name"]
        kbl = len(bytes.fromhex(c["key_block"]))
        assert bytes(d.key_block[k][:kbl]).hex() == c["key_block"], c["name"]
        assert not d.key_block[k][kbl:].any(), c["name"]
        w, r = _host_states(tuple(c["version"]), c["suite"], bytes.fromhex(c["master"]),
                            bytes.fromhex(c["client_random"]), bytes.fromhex(c["server_random"]), k % 2 == 0,
                            bytes(range(16, 32)))
        assert d.write_state_bytes(k) == w, c["name"]
        assert d.read_state_bytes(k) == r, c["name"]


def test_derive_random_batch_vs_oracle():
    """1,000 connections over every suite x version x side, random secrets."""
    _need_gpu()
    from tlslite_amd.connection import derive_pending_states_gpu
    rng = np.random.default_rng(77)
    combos = [(s, v) for s, vs in SUITE_VERSIONS for v in vs]
    conns = []
    for k in range(1000):
        s, v = combos[k % len(combos)]
        conns.append({"secret": rng.bytes(48), "client_random": rng.bytes(32), "server_random": rng.bytes(32),
                      "suite": SUITE_NAMES[s], "version": v, "client": bool(rng.integers(2)),
                      "fixed_iv": rng.bytes(16), "_suite": s})
    d = derive_pending_states_gpu(conns, want_key_block=True)
    ws = d.write.download().reshape(len(conns), -1)
    rs = d.read.download().reshape(len(conns), -1)
    for k, c in enumerate(conns):
        kb, _ = O.key_block(c["version"], c["_suite"], c["secret"], c["client_random"], c["server_random"])
        assert bytes(d.key_block[k][:len(kb)]) == kb, k
        assert bytes(d.master[k]) == c["secret"]
        w, r = _host_states(c["version"], c["_suite"], c["secret"], c["client_random"], c["server_random"],
                            c["client"], c["fixed_iv"])
        assert ws[k].tobytes() == w, (k, c["_suite"], c["version"])
        assert rs[k].tobytes() == r, (k, c["_suite"], c["version"])


def test_derive_bad_suite_or_version_raises():
    _need_gpu()
    from tlslite_amd.connection import derive_pending_states_gpu
    base = {"secret": bytes(48), "client_random": bytes(32), "server_random": bytes(32), "client": True}
    for suite, version in ((0x1234, (3, 3)), (SUITE_NAMES["AES128-SHA256"], (3, 1)),
                           (SUITE_NAMES["AES128-SHA"], (3, 4))):
        with pytest.raises(ValueError):
            derive_pending_states_gpu([dict(base, suite=suite, version=version)])


def test_derived_states_seal_like_host_states():
    """A record sealed with a GPU-derived write state equals the oracle's
    seal with the same key-block slices (the state is usable as-is)."""
    _need_gpu()
    from tlslite_amd.connection import derive_pending_states_gpu
    from tlslite_amd.recordlayer import seal
    from tlslite_amd.state import ConnectionState
    rng = np.random.default_rng(5)
    for suite, version in (("AES128-SHA", (3, 3)), ("RC4-SHA", (3, 1)), ("3DES-SHA", (3, 2)),
                           ("AES256-SHA256", (3, 3))):
        conn = {"secret": rng.bytes(48), "client_random": rng.bytes(32), "server_random": rng.bytes(32),
                "suite": suite, "version": version, "client": True, "fixed_iv": rng.bytes(16)}
        d = derive_pending_states_gpu([conn])
        cipher, kl, ivl, mac, ml = O.SUITES[suite]
        _, kp = O.key_block(version, suite, conn["secret"], conn["client_random"], conn["server_random"])
        fiv = conn["fixed_iv"][:ivl] if version >= (3, 2) and ivl else None
        st = ConnectionState(cipher, mac, version, bytes(kl), bytes(ivl), bytes(ml), fiv)
        st.raw[:] = d.write_state_bytes(0)  # the GPU-derived state, nothing from the host build
        pt = rng.bytes(1000)
        wire = seal([st], [(0, pt, 23), (0, pt[:17], 23)])
        oc = O.Conn(cipher, mac, version, kp["client_key"], kp["client_iv"], kp["client_mac"], fiv)
        assert bytes(wire[0]) == oc.seal(pt, 23), suite
        assert bytes(wire[1]) == oc.seal(pt[:17], 23), suite

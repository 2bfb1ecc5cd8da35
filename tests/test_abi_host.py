"""CPU-only checks of the drop-in boundary and host logic: the C-ABI library
loads and exports every symbol include/tlsgpu.h declares; connection-state
construction validates like the reference; record planning / framing /
layout logic.  No kernel launches here."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden_io import case_data, case_keys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _decls():
    src = open(os.path.join(ROOT, "include", "tlsgpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w[\w\s\*]*?\b(tlsgpu_\w+)\s*\(", src, re.M)))


def test_header_symbols_exported():
    from tlslite_amd import _native as N
    decls = _decls()
    assert len(decls) >= 30
    for name in decls:
        assert hasattr(N.lib, name), name
    bound = {n for n, _, _ in N.SIGNATURES}
    assert set(decls) == bound, set(decls) ^ bound


def test_binding_arity_matches_header():
    """Every ctypes signature has as many arguments as the header's prototype (a missing
    size argument would shift every later one: ABI 6 added the arena sizes)."""
    from tlslite_amd import _native as N
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "tlsgpu.h")).read(), flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(tlsgpu_\w+)\s*\(([^;{]*?)\)\s*;", src):
        args = m.group(2).strip()
        protos[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    for name, _, argtypes in N.SIGNATURES:
        assert name in protos, name
        assert len(argtypes) == protos[name], (name, len(argtypes), protos[name])


def test_abi_structs_and_constants():
    from tlslite_amd import _native as N
    src = open(os.path.join(ROOT, "include", "tlsgpu.h")).read()
    for name, val in [("TLSGPU_CIPHER_AES128", 1), ("TLSGPU_CIPHER_AES256", 2), ("TLSGPU_CIPHER_RC4", 3),
                      ("TLSGPU_CIPHER_3DES", 4), ("TLSGPU_MAC_SHA1", 1), ("TLSGPU_MAC_SHA256", 2),
                      ("TLSGPU_MAC_MD5", 3), ("TLSGPU_ALERT_BAD_RECORD_MAC", -20),
                      ("TLSGPU_ALERT_DECRYPTION_FAILED", -21), ("TLSGPU_ALERT_SKIPPED", -22),
                      ("TLSGPU_ALERT_RECORD_OVERFLOW", -23), ("TLSGPU_EFRAME", -6),
                      ("TLSGPU_EABRUPT", -7), ("TLSGPU_CONN_STATE_BYTES", 2048), ("TLSGPU_ABI_VERSION", 7)]:
        assert re.search(r"\b%s\s*=?\s*%d\b" % (name, val), src), name
    assert re.search(r"#define TLSGPU_CHAIN_STOP_ON_ALERT 1u", src)
    assert N.lib.tlsgpu_abi_version() == N.ABI_VERSION == 7
    assert (N.ALERT_SKIPPED, N.CHAIN_STOP_ON_ALERT) == (-22, 1)
    assert (N.ALERT_RECORD_OVERFLOW, N.EFRAME, N.EABRUPT) == (-23, -6, -7)
    # per connection a 32-bit count, per 256 connections a 64-bit sum (ABI 7)
    assert N.lib.tlsgpu_frame_workspace_bytes(1000) >= 4 * 1000 + 8 * 4
    assert ctypes.sizeof(N.Record) == 24 and ctypes.sizeof(N.Chain) == 16
    assert [f[0] for f in N.Chain._fields_] == ["state", "first", "count", "flags"]


def test_open_split_modes_match_header():
    """tlsgpu_set_open_parts: the header's TLSGPU_OPEN_SPLIT_* values equal the bindings'
    constants, every mode is accepted and anything else is refused with TLSGPU_EINVAL (host
    only: no GPU needed); the open workspace holds an OpenMeta and an OpenMacState per record."""
    from tlslite_amd import _native as N
    src = open(os.path.join(ROOT, "include", "tlsgpu.h")).read()
    for name, val in [("AUTO", N.OPEN_SPLIT_AUTO), ("CHAINS", N.OPEN_SPLIT_CHAINS), ("NONE", N.OPEN_SPLIT_NONE),
                      ("BLOCKS", N.OPEN_SPLIT_BLOCKS)]:
        assert re.search(r"\bTLSGPU_OPEN_SPLIT_%s\s*=\s*%d\b" % (name, val), src), name
    try:
        for m in (N.OPEN_SPLIT_AUTO, N.OPEN_SPLIT_CHAINS, N.OPEN_SPLIT_NONE, N.OPEN_SPLIT_BLOCKS):
            assert N.lib.tlsgpu_set_open_parts(m, 0) == 0, m
        for bad in (-1, 4, 99):
            assert N.lib.tlsgpu_set_open_parts(bad, 0) == N.EINVAL, bad
    finally:
        assert N.lib.tlsgpu_set_open_parts(N.OPEN_SPLIT_AUTO, -1) == 0
    assert N.lib.tlsgpu_open_workspace_bytes(1000) == 1000 * 96


def test_state_validation_mirrors_reference():
    from tlslite_amd import ConnectionState, _native as N
    ok = ConnectionState("aes128", "sha1", (3, 3), bytes(16), bytes(16), bytes(20), bytes(16))
    assert ok.variant == N.variant(N.CIPHER_AES128, N.MAC_SHA1, False)
    bad = [("aes128", "sha1", (3, 3), bytes(15), bytes(16), bytes(20), bytes(16)),   # aes.py:8
           ("aes128", "sha1", (3, 3), bytes(16), bytes(8), bytes(20), bytes(16)),    # aes.py:12
           ("3des", "sha1", (3, 1), bytes(16), bytes(8), bytes(20), None),           # tripledes.py:8
           ("rc4", "sha1", (3, 1), bytes(15), b"", bytes(20), None),                # rc4.py:9
           ("rc4", "sha1", (3, 1), bytes(16), bytes(1), bytes(20), None),           # cipherfactory.py:70
           ("aes128", "sha256", (3, 1), bytes(16), bytes(16), bytes(32), None),     # constants.py:204-210
           ("aes128", "sha1", (3, 2), bytes(16), bytes(16), bytes(20), None)]       # fixedIVBlock needed
    for args in bad:
        with pytest.raises(N.TLSGPUError):
            ConnectionState(*args)


@pytest.mark.parametrize("suite", sorted(O.SUITES))
@pytest.mark.parametrize("version", [(3, 0), (3, 1), (3, 2), (3, 3)])
def test_wire_len_matches_oracle(suite, version):
    from tlslite_amd import ConnectionState
    if suite.endswith("SHA256") and version != (3, 3):
        return
    c, kl, ivl, m, ml = O.SUITES[suite]
    st = ConnectionState.for_suite(suite, version, bytes(kl), bytes(ivl), bytes(ml), bytes(ivl) if ivl else None)
    oc = O.Conn.for_suite(suite, version, bytes(kl), bytes(ivl), bytes(ml), bytes(ivl) if ivl else None)
    for n in [0, 1, 15, 16, 17, 1434, 16384, 16385]:
        assert st.wire_len(n) == len(oc.copy().seal(bytes(n))) if n else st.wire_len(0) == 0


def test_plan_write_matches_golden(golden):
    from tlslite_amd.recordlayer import plan_write
    for c in golden:
        if c["kind"] != "write":
            continue
        data = case_data(c)
        parts = plan_write(data, tuple(c["version"]), not c["suite"].startswith("RC4"))
        assert len(parts) == len(c["writes"]), c["name"]
        assert b"".join(parts) == data


def test_wire_offsets_alignment():
    from tlslite_amd.recordlayer import wire_offsets
    offs, total = wire_offsets([16437, 37, 1493, 5])
    assert all((int(o) + 5) % 16 == 0 for o in offs)
    assert total >= int(offs[-1]) + 5


def test_workload_layout():
    from tlslite_amd import workloads as W
    wl = W.cfg2(n=256)
    assert wl.n_records == 256 and wl.plaintext_total == 256 * 16384
    assert all(int(o) % 16 == 0 for o in wl.pt_off)
    assert all((int(o) + 5) % 16 == 0 for o in wl.wire_off)
    assert int(wl.wire_len[0]) == 16437
    st = wl.host_states()
    assert st.nbytes == 256 * 2048
    w5 = W.cfg5(n=64)
    assert sorted(w5.slot_of.tolist()) == list(range(64))
    ends = sorted((int(o), int(o) + int(l)) for o, l in zip(w5.wire_off, w5.wire_len))
    assert all(a[1] <= b[0] for a, b in zip(ends, ends[1:]))  # no overlap


def test_factory_without_gpu_or_impl():
    from tlslite_amd.utils import cipherfactory as F
    from tlslite_amd.utils.aes import AES
    from tlslite_amd.utils.rc4 import RC4
    from tlslite_amd.utils.tripledes import TripleDES
    with pytest.raises(NotImplementedError):
        F.createAES(bytes(16), bytes(16), ["python"])
    with pytest.raises(NotImplementedError):
        F.createTripleDES(bytes(24), bytes(8), ["openssl", "pycrypto"])
    with pytest.raises(AssertionError):
        F.createRC4(bytes(16), bytes(1), ["hip"])
    with pytest.raises(AssertionError):
        AES(bytes(15), 2, bytes(16), "hip")
    with pytest.raises(AssertionError):
        AES(bytes(16), 1, bytes(16), "hip")
    assert AES(bytes(24), 2, bytes(16), "hip").name == "aes192"
    with pytest.raises(ValueError):
        RC4(bytes(10), "hip")
    with pytest.raises(ValueError):
        TripleDES(bytes(24), 2, bytes(7), "hip")
    assert F.tripleDESPresent


def test_oracle_fill_pattern_is_splitmix():
    a = O.fill_pattern(40, 7, 3)

    def sm(z):
        z = (z + 0x9E3779B97F4A7C15) & (2 ** 64 - 1)
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2 ** 64 - 1)
        return z ^ (z >> 31)
    exp = [(sm(7 + (g >> 3)) >> (8 * (g & 7))) & 0xff for g in range(3, 43)]
    assert a.tolist() == exp


def test_no_kernel_gets_lds_it_does_not_declare():
    """Static LDS of every kernel in the built gfx950 code object (AMDGPU metadata,
    .group_segment_fixed_size) is only what the sources declare with __shared__: the frame
    kernels' reduction scratch.  The AES / 3DES / RC4 kernels take their tables as dynamic LDS
    at launch, and the MAC kernels must take none: the seal pipeline runs a MAC workgroup on a
    CU beside the cipher kernel's 128 KiB of tables, and round 6 found the backend's
    promote-alloca pass had given the MAC kernels 19 KiB each (build.py now disables it)."""
    import re
    import shutil
    import subprocess
    import tempfile
    lib = os.path.join(ROOT, "tlslite_amd", "lib", "libtlsgpu.so")
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-objdump")):
        pytest.skip("no llvm-objdump in this image")
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(lib, d)
        subprocess.check_call([os.path.join(llvm, "llvm-objdump"), "--offloading", "libtlsgpu.so"], cwd=d,
                              stdout=subprocess.DEVNULL)
        co = [f for f in os.listdir(d) if "gfx950" in f]
        assert co, os.listdir(d)
        notes = subprocess.check_output([os.path.join(llvm, "llvm-readelf"), "--notes", co[0]], cwd=d, text=True)
    kernels = re.findall(r"\.group_segment_fixed_size:\s+(\d+).*?\.name:\s+(\S+)", notes, re.S)
    assert len(kernels) >= 40
    with_lds = {n for lds, n in kernels if int(lds) > 0}
    allowed = ("frame_count_kernel", "frame_scan_kernel", "frame_write_kernel")
    assert all(any(a in n for a in allowed) for n in with_lds), sorted(with_lds)
    assert any("mac_kernel" in n for _, n in kernels)

"""Build libtlsgpu.so in-tree (tlslite_amd/lib/) with hipcc for gfx950.

The shared library is the product: the C ABI of include/tlsgpu.h, the gfx950
kernels, and the host-side state construction.  It is git-ignored but travels
to the GPU box with the repository snapshot.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libtlsgpu.so")
ARCH = os.environ.get("TLSGPU_ARCH", "gfx950")

SOURCES = ["tg_kernels.hip", "tg_api.hip"]
HEADERS = ["tg_config.h", "tg_common.h", "tg_hash.h", "tg_device.h", "tg_quad.h", "tg_aes3.h", "tg_open3.h", "tg_frame.h", "tg_launch.h", "tg_keysched.h", "tg_derive.h"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, extra_flags=(), libdir=LIBDIR, overlay=None):
    """Compile libtlsgpu.so into libdir.  extra_flags / libdir / overlay: experiment builds
    of the same sources (tools/build_ab.sh): `overlay` is a directory searched before csrc
    for <tg_config.h>, so its tuning constants (with -D overrides) replace the product's.
    The product is the default build in tlslite_amd/lib, from csrc/tg_config.h."""
    lib = os.path.join(libdir, "libtlsgpu.so")
    os.makedirs(libdir, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(HERE, "..", "include", "tlsgpu.h")]
    objs = []
    hipcc = _hipcc()
    incs = (["-I" + overlay] if overlay else []) + ["-I" + CSRC]
    if overlay:
        deps += [os.path.join(overlay, f) for f in os.listdir(overlay)]
    # -disable-promote-alloca-to-lds: the AMDGPU backend may turn a kernel's private array into
    # static LDS (round 6: the MAC kernels' funnel-shift words became 19 KiB per workgroup), which
    # no source line shows and which takes the LDS the seal pipeline needs to run a MAC
    # workgroup beside the cipher kernel's 128 KiB of tables (cfg3 -4.5 %, the concurrent open
    # -18 %).  Kernels that want LDS declare it; tests/test_abi_host.py checks the code objects.
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall", "-Wno-unused-function",
             "-munsafe-fp-atomics", "-mllvm", "-disable-promote-alloca-to-lds"] + incs + list(extra_flags)
    if not force and not _stale(lib, deps):
        return lib
    for s in srcs:
        o = os.path.join(libdir, os.path.basename(s) + ".o")
        cmd = [hipcc] + flags + ["-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        objs.append(o)
    tmp = lib + ".tmp"
    cmd = [hipcc, "-shared", "--offload-arch=" + ARCH, "-o", tmp] + objs
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    # python tlslite_amd/build.py [--force] [--out DIR --overlay DIR] [-DFLAG ...]
    args = sys.argv[1:]
    out = LIBDIR
    overlay = None
    if "--out" in args:
        out = os.path.abspath(args[args.index("--out") + 1])
    if "--overlay" in args:
        overlay = os.path.abspath(args[args.index("--overlay") + 1])
    if (overlay or any(a.startswith("-D") for a in args)) and out == LIBDIR:
        sys.exit("build.py: experiment builds (--overlay / -D) go to --out DIR, never to the product lib/")
    flags = [a for a in args if a.startswith("-D")]
    print(build(force="--force" in args or bool(flags), verbose=True, extra_flags=flags, libdir=out, overlay=overlay))

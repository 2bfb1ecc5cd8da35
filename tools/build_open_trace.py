"""Diagnostic build: libtlsgpu.so whose open_fused_kernel stamps a timeline (s_memrealtime,
100 MHz) into the open workspace after the stripe counters, for tools/open_trace.py.

The product sources are copied under tools/ab/oftrace_src/ and patched there (the product tree
is never touched); the library goes to tools/ab/oftrace/.  Per workgroup and wave 64 stamps
of the workgroup's first generation:
  decrypt waves  [0] start (tables filled), [1 + s] stripe s published, [62] done
  MAC waves      [0] start, [1 + s] stripe s seen complete, [21 + s] stripe s hashed,
                 [61] record finished, [62] done
  python tools/build_open_trace.py          (CPU box; hipcc cross-compiles)
"""
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from tlslite_amd import build as B  # noqa: E402

SRC = os.path.join(R, "tools", "ab", "oftrace_src", "src", "csrc")  # ../../include resolves beside it
OUT = os.path.join(R, "tools", "ab", "oftrace")


def patch(path, pairs):
    s = open(path).read()
    for a, b in pairs:
        if a not in s:
            sys.exit(f"build_open_trace: anchor not found in {os.path.basename(path)}: {a[:60]!r}")
        s = s.replace(a, b, 1)
    open(path, "w").write(s)


def main():
    shutil.rmtree(os.path.join(R, "tools", "ab", "oftrace_src"), ignore_errors=True)
    shutil.copytree(B.CSRC, SRC)
    shutil.copytree(os.path.join(R, "include"), os.path.join(SRC, "..", "..", "include"))
    patch(os.path.join(SRC, "tg_kernels.hip"), [
        ("return (size_t)nrecords * sizeof(OpenMeta) + (size_t)OF_MAX_CTL * sizeof(OpenFusedCtl);",
         "return (size_t)nrecords * sizeof(OpenMeta) + (size_t)OF_MAX_CTL * sizeof(OpenFusedCtl) + "
         "(size_t)OF_MAX_CTL * 16 * 64 * 8;"),
    ])
    o3 = os.path.join(SRC, "tg_open3.h")
    patch(o3, [
        ("    OpenFusedCtl* C = ctl + blockIdx.x;\n",
         "    OpenFusedCtl* C = ctl + blockIdx.x;\n"
         "    uint64_t* TR = (uint64_t*)(ctl + OF_MAX_CTL) + ((size_t)blockIdx.x * 16 + wv) * 64;\n"
         "#define OFT(i) do { if (j == 0 && lane == 0) TR[i] = __builtin_amdgcn_s_memrealtime(); } while (0)\n"),
        # decrypt waves
        ("            g.load(recs, states, meta, nrecords, epoch, gen_base, wv);\n",
         "            g.load(recs, states, meta, nrecords, epoch, gen_base, wv);\n            OFT(0);\n"),
        ("                        for (uint32_t t = pub; t < s; t++)\n"
         "                            __hip_atomic_fetch_add(&C->cnt[par][t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n",
         "                        for (uint32_t t = pub; t < s; t++) {\n"
         "                            __hip_atomic_fetch_add(&C->cnt[par][t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
         "                            if (j == 0) TR[1 + t] = __builtin_amdgcn_s_memrealtime();\n"
         "                        }\n"),
        ("                for (uint32_t t = pub; t < (uint32_t)OF_MAX_STRIPES; t++)\n"
         "                    __hip_atomic_fetch_add(&C->cnt[par][t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n",
         "                for (uint32_t t = pub; t < (uint32_t)OF_MAX_STRIPES; t++) {\n"
         "                    __hip_atomic_fetch_add(&C->cnt[par][t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
         "                    if (j == 0) TR[1 + t] = __builtin_amdgcn_s_memrealtime();\n"
         "                }\n"
         "            OFT(62);\n"),
        # MAC waves
        ("        M mac;\n        if (act) mac.begin(st, mt.seq, R.content_type, n);\n",
         "        M mac;\n        OFT(0);\n        if (act) mac.begin(st, mt.seq, R.content_type, n);\n"),
        ("            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"agent\");",
         "            if (s < 20) OFT(1 + s);\n            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"agent\");"),
        ("                    done = ready;\n                }\n            }\n",
         "                    done = ready;\n                }\n            }\n            if (s < 20) OFT(21 + s);\n"),
        ("        status[r] = ((mt.flags & OM_PADOK) && macGood) ? (int32_t)n : TLSGPU_ALERT_BAD_RECORD_MAC;\n    }\n}\n",
         "        status[r] = ((mt.flags & OM_PADOK) && macGood) ? (int32_t)n : TLSGPU_ALERT_BAD_RECORD_MAC;\n"
         "        OFT(61);\n    }\n}\n"),
    ])
    os.makedirs(OUT, exist_ok=True)
    hipcc = B._hipcc()
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + B.ARCH, "-Wno-unused-function", "-I" + SRC]
    objs = []
    for s in B.SOURCES:
        o = os.path.join(OUT, s + ".o")
        subprocess.check_call([hipcc] + flags + ["-c", os.path.join(SRC, s), "-o", o])
        objs.append(o)
    subprocess.check_call([hipcc, "-shared", "--offload-arch=" + B.ARCH, "-o", os.path.join(OUT, "libtlsgpu.so")] + objs)
    print(os.path.join(OUT, "libtlsgpu.so"))


if __name__ == "__main__":
    main()

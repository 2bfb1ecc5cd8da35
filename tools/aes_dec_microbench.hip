// aes_dec_microbench.hip -- the open path's AES decrypt round loop (one lane per block,
// lane_aes_dec of tg_open3.h: 16 Td lookups per round in the lane, 32-copy LDS tables) with
// no global-memory traffic, to find what bounds open_aes_kernel (0.96 ms on cfg2 against a
// 0.62 ms LDS-array floor, lds_busy 0.55 in PMC).  Variants:
//   ILP   independent blocks per lane (1: the product; 2: two blocks' rounds interleaved)
//   KEYV  round keys in VGPRs (1) or wave-uniform SGPRs (0: the product)
//   W     waves per CU (16: the product's 1024-thread workgroup; 8)
// Every variant decrypts the same blocks with the same keys; the host checks that the
// outputs agree and prints cycles per block-round per CU, the LDS-array busy fraction it
// implies (160 lookups per block, 32 per cycle) and the cfg2-equivalent time
// (67.3 M blocks).  Diagnostic tool only.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Itlslite_amd/csrc tools/aes_dec_microbench.hip -o tools/aes_dec_mb.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>
#include "../tlslite_amd/csrc/tg_open3.h"

using namespace tg;
constexpr int NR = 10;

// GL: lookups served by the vector memory path (a 2 KiB table in global memory, L1-resident)
// instead of LDS, to spread the gather load over two pipes: 1 = the last round's inverse
// S-box (16 of 160 lookups per block), 2 = that and every round's Td3 lookups (56 of 160)
template <int NR, int GL>
__device__ __forceinline__ void lane_aes_dec_gl(const QuadAesDec& D, uint32_t s[4], const uint32_t* dk,
                                                const uint32_t* __restrict__ g) {
    const QuadAes& A = D.t;
    uint32_t s0 = s[0] ^ dk[0], s1 = s[1] ^ dk[1], s2 = s[2] ^ dk[2], s3 = s[3] ^ dk[3];
    auto t3 = [&](uint32_t x) -> uint32_t {
        if constexpr (GL >= 2) return g[x >> 24];
        else return A.look<3, 3>(x);
    };
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t* k = dk + 4 * r;
        const uint32_t t0 = bx3(bx3(A.look<0, 0>(s0), A.look<1, 1>(s3), A.look<2, 2>(s2)), t3(s1), k[0]);
        const uint32_t t1 = bx3(bx3(A.look<0, 0>(s1), A.look<1, 1>(s0), A.look<2, 2>(s3)), t3(s2), k[1]);
        const uint32_t t2 = bx3(bx3(A.look<0, 0>(s2), A.look<1, 1>(s1), A.look<2, 2>(s0)), t3(s3), k[2]);
        const uint32_t t3v = bx3(bx3(A.look<0, 0>(s3), A.look<1, 1>(s2), A.look<2, 2>(s1)), t3(s0), k[3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3v;
    }
    const uint32_t* k = dk + 4 * NR;
    const uint32_t* gi = g + 256;
    auto ib = [&](uint32_t x, int B) -> uint32_t { return gi[(x >> (8 * B)) & 0xffu]; };
    s[0] = QuadAesDec::col(ib(s0, 0), ib(s3, 1), ib(s2, 2), ib(s1, 3), k[0]);
    s[1] = QuadAesDec::col(ib(s1, 0), ib(s0, 1), ib(s3, 2), ib(s2, 3), k[1]);
    s[2] = QuadAesDec::col(ib(s2, 0), ib(s1, 1), ib(s0, 2), ib(s3, 3), k[2]);
    s[3] = QuadAesDec::col(ib(s3, 0), ib(s2, 1), ib(s1, 2), ib(s0, 3), k[3]);
}

// ROT: the 4 waves of a SIMD (w, w+4, w+8, w+12) rotate the top issue priority every
// iteration (s_setprio 3..0), against the age order that lets the oldest wave run ahead
template <int ILP, int KEYV, int W, int ROT = 0, int GL = 0>
__global__ void __launch_bounds__(64 * W, 1) dec_kernel(const uint32_t* __restrict__ dk_g, uint32_t* __restrict__ out,
                                                       uint64_t* __restrict__ cyc, int iters,
                                                       const uint32_t* __restrict__ gtab) {
    aes_lds_fill(nullptr, true);
    __syncthreads();
    QuadAesDec D;
    D.init();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t dk[4 * (NR + 1)];
    const uint32_t* dkp = dk_g;
    if constexpr (KEYV) {
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++) {
            dk[i] = dk_g[i];
            asm volatile("" : "+v"(dk[i]));  // keep the keys in VGPRs
        }
        dkp = dk;
    }
    uint32_t s[ILP][4];
#pragma unroll
    for (int i = 0; i < ILP; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) s[i][j] = (gid * ILP + i) * 0x9e3779b9u ^ (j * 0x85ebca6bu);
    const uint32_t slot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);  // 0..W/4-1: the wave's rank on its SIMD
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        if constexpr (ROT) {
            const uint32_t p = ((uint32_t)it + slot) & 3u;
            if (p == 0) __builtin_amdgcn_s_setprio(3);
            else if (p == 1) __builtin_amdgcn_s_setprio(2);
            else if (p == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            if constexpr (GL) lane_aes_dec_gl<NR, GL>(D, s[i], dkp, gtab);
            else lane_aes_dec<NR>(D, s[i], dkp);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < ILP; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) out[(gid * ILP + i) * 4 + j] = s[i][j];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * W + (threadIdx.x >> 6)] = t1 - t0;
}

struct R {
    std::vector<uint32_t> out;
};

static const uint32_t* g_gtab = nullptr;
template <int ILP, int KEYV, int W, int ROT = 0, int GL = 0>
static R run(const char* name, const uint32_t* d_dk, int cus, int iters_total, int lanes_per_cu) {
    auto kern = dec_kernel<ILP, KEYV, W, ROT, GL>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              AES_DEC_LDS_BYTES);
    // the same blocks in every variant: lanes_per_cu * iters_total blocks per CU, spread as
    // (64 W lanes x ILP) x iters
    const int iters = iters_total * lanes_per_cu / (64 * W * ILP);
    const size_t nout = (size_t)cus * 64 * W * ILP * 4;
    uint32_t* d_out;
    uint64_t* d_cyc;
    (void)hipMalloc(&d_out, nout * 4);
    (void)hipMalloc(&d_cyc, (size_t)cus * W * 8);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * W), AES_DEC_LDS_BYTES, 0, d_dk, d_out, d_cyc, 4, g_gtab);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * W), AES_DEC_LDS_BYTES, 0, d_dk, d_out, d_cyc, iters, g_gtab);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> cyc((size_t)cus * W);
    (void)hipMemcpy(cyc.data(), d_cyc, cyc.size() * 8, hipMemcpyDeviceToHost);
    double c = 0, cmin = 1e30, cmax = 0;
    for (size_t i = 0; i < cyc.size(); i++) {
        c += (double)cyc[i];
        cmin = (double)cyc[i] < cmin ? (double)cyc[i] : cmin;
        cmax = (double)cyc[i] > cmax ? (double)cyc[i] : cmax;
    }
    c /= cyc.size();
    const double blocks_cu = (double)iters * 64 * W * ILP;
    const double cyc_per_round = c / (blocks_cu * NR);  // per block-round, per CU
    const double lds_busy = (blocks_cu * 160.0 / 32.0) / c;
    const double cfg2_ms = ms * (67.3e6 / (blocks_cu * cus));
    printf("%-12s ILP %d keys %s waves/CU %2d  %7.3f ms  cfg2-equiv %.3f ms  per-wave loop (s_memtime cycles) min %.0f "
           "avg %.0f max %.0f (max/avg %.2f)\n", name, ILP, KEYV ? "VGPR" : "SGPR", W, ms, cfg2_ms, cmin, c, cmax,
           cmax / c);
    (void)cyc_per_round;
    (void)lds_busy;
    fflush(stdout);
    R r;
    r.out.resize(nout);
    (void)hipMemcpy(r.out.data(), d_out, nout * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return r;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 256;  // blocks per lane of the ILP 1 / 16-wave variant
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    uint32_t dk[4 * (NR + 1)];
    for (int i = 0; i < 4 * (NR + 1); i++) dk[i] = 0x01234567u * (i + 3) ^ (i << 20);
    uint32_t* d_dk;
    (void)hipMalloc(&d_dk, sizeof(dk));
    (void)hipMemcpy(d_dk, dk, sizeof(dk), hipMemcpyHostToDevice);
    printf("CUs %d\n", cus);
    {  // the global-memory tables of the GL variants: Td3 (= rotl(Td0, 24)) and the byte-replicated InvS
        constexpr tg::AesTables T;
        std::vector<uint32_t> h(512);
        for (int e = 0; e < 256; e++) {
            const uint32_t v = T.td0[e];
            h[e] = (v << 24) | (v >> 8);
            h[256 + e] = (uint32_t)T.inv_sbox[e] * 0x01010101u;
        }
        uint32_t* d;
        (void)hipMalloc(&d, 2048);
        (void)hipMemcpy(d, h.data(), 2048, hipMemcpyHostToDevice);
        g_gtab = d;
    }
    const int lanes = 1024;  // blocks in flight per CU of the reference variant
    std::vector<R> rs;
    rs.push_back(run<1, 0, 16>("product", d_dk, cus, iters, lanes));
    rs.push_back(run<1, 1, 16>("keysV", d_dk, cus, iters, lanes));
    rs.push_back(run<2, 0, 16>("ilp2", d_dk, cus, iters, lanes));
    rs.push_back(run<2, 1, 16>("ilp2-keysV", d_dk, cus, iters, lanes));
    rs.push_back(run<2, 0, 8>("ilp2-8w", d_dk, cus, iters, lanes));
    rs.push_back(run<1, 0, 8>("8w", d_dk, cus, iters, lanes));
    rs.push_back(run<1, 0, 16, 1>("product-rot", d_dk, cus, iters, lanes));
    rs.push_back(run<2, 0, 16, 1>("ilp2-rot", d_dk, cus, iters, lanes));
    rs.push_back(run<1, 0, 16, 1, 1>("rot-glisb", d_dk, cus, iters, lanes));
    rs.push_back(run<1, 0, 16, 1, 2>("rot-glT3", d_dk, cus, iters, lanes));
    // variants with the same blocks per CU (64 W x ILP lanes' blocks, decrypted the same number
    // of times) must agree word for word: product / keysV / ilp2-8w, and ilp2 / ilp2-keysV
    int bad = 0;
    if (rs[1].out != rs[0].out || rs[4].out != rs[0].out || rs[6].out != rs[0].out || rs[7].out != rs[2].out ||
        rs[8].out != rs[0].out || rs[9].out != rs[0].out) {
        printf("MISMATCH among the 1024-block variants\n");
        bad = 1;
    }
    if (rs[3].out != rs[2].out) {
        printf("MISMATCH among the 2048-block variants\n");
        bad = 1;
    }
    if (!bad) printf("all variants decrypt the same blocks\n");
    return bad;
}

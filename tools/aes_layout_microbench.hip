// aes_layout_microbench.hip -- AES chains at a fixed number of chains per CU
// (cfg2: 65,536 independent CBC chains on 256 CUs = 256 per CU), comparing lane
// layouts of the LDS T-table round with no global-memory traffic in the loop:
//   quad1   4 lanes/chain, column per lane, XOR tree dpp2(t2^dpp1(t3)) (tg_quad.h), 16 waves/CU
//   quad1b  4 lanes/chain, XOR tree ordered for the last lookup: ((k ^ dpp2 t2) ^ dpp3 t3) ^ t0 ^ dpp1 t1
//   quad2   4 lanes/chain, 2 chains per quad interleaved,                    8 waves/CU
//   quad2b  as quad2 with the quad1b XOR order
//   pair1   2 lanes/chain (2 columns per lane, 8 lookups, one DPP swap),     8 waves/CU
//   pair2   2 lanes/chain, 2 chains per lane pair,                           4 waves/CU
//   pairg1  pair1 with the two T3 lookups of a round from a 1 KiB table in global memory
//           (the vector L1 as a second gather port beside the LDS), 8 waves/CU
//   pairg2  pair1 with the T3 and T2 lookups (4 of 8) from global tables
//   lane1   1 lane/chain (16 lookups per lane),                              4 waves/CU
//   mixN    (argv[2] = "m") 32 N chains on N pair waves, the rest on quad waves (N = 4: half and
//           half, 12 waves/CU)
//   *@512   the same at 512 chains per CU (cfg3 has 4,096 per CU)
//   trace mode (argv[2] = "t", round 5): the product pair round at 256 chains per CU, every
//   wave time-stamping (s_memtime) the start of NS consecutive blocks; the host derives each
//   wave's round period and the phase of every same-CU wave pair within a round (do the 8
//   waves convoy -- issue their rounds together -- or spread?), with and without a
//   mac_kernel-shaped SHA-1 co-runner, and for start-staggered variants (waves delayed by
//   w/8 or (w&1)/2 of a round before the loop)
//   latency mode (argv[2] = "lat"): 2 and 16 chains per CU (cfg4 at 8 GPUs / 1 GPU):
//   the round is then one chain's dependent latency, reported in shader cycles;
//   quad1s = quad1b with ONE chain per wave (chains spread over the SIMDs)
// Every layout encrypts the same chains with the same round keys; the host checks
// that all final states agree.  Reports ns and shader cycles (s_memtime) per round,
// the LDS-array floor fraction (16 lookups x chains / 32 per cycle) and the
// cfg2-equivalent time of 1,027 blocks per chain.  Diagnostic tool only.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/aes_layout_microbench.hip -o tools/aes_layout_mb.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../tlslite_amd/csrc/tg_quad.h"
#include "../tlslite_amd/csrc/tg_hash.h"

using namespace tg;

constexpr int NR = 10;

__device__ __forceinline__ uint32_t pair_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);
}

// quad round with the XOR tree ordered for the lookup issue order (T2, T3, T0, T1):
// column q = k_q ^ T2(q+2) ^ T3(q+3) ^ T0(q) ^ T1(q+1); only one DPP XOR follows the
// last lookup.  kq = round-key column q (not pre-rotated).
struct QuadAesB : QuadAes {
    __device__ __forceinline__ uint32_t round_b(uint32_t x, uint32_t kq) const {
        const uint32_t t2 = look<2, 2>(x);
        const uint32_t t3 = look<3, 3>(x);
        const uint32_t t0 = look<0, 0>(x);
        const uint32_t t1 = look<1, 1>(x);
        const uint32_t a = kq ^ quad_dpp<0x4E>(t2);
        const uint32_t w = a ^ quad_dpp<0x93>(t3);
        const uint32_t y = t0 ^ w;
        return y ^ quad_dpp<0x39>(t1);
    }
    __device__ __forceinline__ uint32_t last_b(uint32_t x, uint32_t kq) const {
        const uint32_t s2 = look<0, 2>(x) & 0xff0000u;
        const uint32_t s3 = look<1, 3>(x) & 0xff000000u;
        const uint32_t s0 = look<2, 0>(x) & 0xffu;
        const uint32_t s1 = look<3, 1>(x) & 0xff00u;
        const uint32_t a = kq ^ quad_dpp<0x4E>(s2);
        const uint32_t w = a ^ quad_dpp<0x93>(s3);
        return (s0 ^ w) ^ quad_dpp<0x39>(s1);
    }
};

// 2 lanes per chain: the product's PairAes (tg_quad.h)

// T2 / T3 in global memory (the second gather port): T_t = rotl(T0, 8t) as aes_lds_fill
__device__ uint32_t g_t[2][256];
__global__ void fill_gtables() {
    const uint32_t e = threadIdx.x;
    const uint32_t v = c_aes.te0[e];
    g_t[0][e] = (v << 16) | (v >> 16);  // T2
    g_t[1][e] = (v << 24) | (v >> 8);   // T3
}
template <int NG>  // NG = 1: T3 from global; 2: T2 and T3
struct PairAesG : PairAes {
    template <int T, int B>
    __device__ __forceinline__ uint32_t lk(uint32_t s) const {
        if constexpr ((T == 3 && NG >= 1) || (T == 2 && NG >= 2)) {
            const uint32_t* g = g_t[T - 2];
            return g[(s >> (8 * B)) & 0xffu];
        } else {
            return look<T, B>(s);
        }
    }
    __device__ __forceinline__ void round(uint32_t& a, uint32_t& b, uint32_t ka, uint32_t kb) const {
        const uint32_t a2 = lk<2, 2>(a), b3 = lk<3, 3>(b), a1 = lk<1, 1>(a), b2 = lk<2, 2>(b);
        const uint32_t a0 = lk<0, 0>(a), b1 = lk<1, 1>(b), b0 = lk<0, 0>(b), a3 = lk<3, 3>(a);
        const uint32_t sa = __builtin_amdgcn_bitop3_b32(a2, b3, ka, 0x96);
        const uint32_t sb = __builtin_amdgcn_bitop3_b32(a1, b2, kb, 0x96);
        a = (a0 ^ b1) ^ swap(sa);
        b = (b0 ^ a3) ^ swap(sb);
    }
};

__device__ __forceinline__ void lane_round(const QuadAes& L, uint32_t s[4], const uint32_t* k) {
    uint32_t t[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        t[j] = L.look<0, 0>(s[j]) ^ L.look<1, 1>(s[(j + 1) & 3]) ^ L.look<2, 2>(s[(j + 2) & 3]) ^
               L.look<3, 3>(s[(j + 3) & 3]) ^ k[j];
#pragma unroll
    for (int j = 0; j < 4; j++) s[j] = t[j];
}
__device__ __forceinline__ void lane_last(const QuadAes& L, uint32_t s[4], const uint32_t* k) {
    uint32_t t[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        t[j] = ((L.look<2, 0>(s[j]) & 0xffu) | (L.look<3, 1>(s[(j + 1) & 3]) & 0xff00u) |
                (L.look<0, 2>(s[(j + 2) & 3]) & 0xff0000u) | (L.look<1, 3>(s[(j + 3) & 3]) & 0xff000000u)) ^ k[j];
#pragma unroll
    for (int j = 0; j < 4; j++) s[j] = t[j];
}

__device__ __forceinline__ uint32_t init_word(uint32_t chain, uint32_t col) {
    return (chain * 2654435761u) ^ (col * 0x9e3779b9u) ^ 0x5bd1e995u;
}

// LAYOUT: 4 = quad, 5 = quad with round_b, 6 = round_b with one chain per wave, 2 = pair,
// 1 = lane.  CPC = chains per CU.
// out[chain*4 + col] = final state; cyc[block] = s_memtime delta of wave 0
template <int LAYOUT, int ILP, int CPC>
__global__ void __launch_bounds__(1024) bench_kernel(const uint32_t* __restrict__ ek, uint32_t* __restrict__ out,
                                                     uint64_t* __restrict__ cyc, int blocks) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    __builtin_amdgcn_s_setprio(1);  // as cbc_kernel: win issue arbitration over the MAC waves
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if constexpr (LAYOUT == 9) {  // mix: chains [0, 32 PW) on PW pair waves, the rest on quad waves
        constexpr uint32_t PW = ILP;  // (ILP carries the pair-wave count for this layout)
        if (wave < PW) {
            PairAes P;
            P.init();
            const uint32_t h = lane & 1;
            const uint32_t ch = blockIdx.x * CPC + wave * 32 + (lane >> 1);
            const uint32_t ca = 2 * h, pa = 2 * (1 - h);
            const uint32_t kwa = ek[ca], kwb = ek[ca + 1];
            uint32_t ka[NR + 1], kb[NR + 1];
#pragma unroll
            for (int r = 1; r <= NR; r++) {
                ka[r] = ek[4 * r + pa];
                kb[r] = ek[4 * r + pa + 1];
            }
            uint32_t a = init_word(ch, ca), bb = init_word(ch, ca + 1);
            for (int b = 0; b < blocks; b++) {
                a ^= kwa;
                bb ^= kwb;
#pragma unroll
                for (int r = 1; r < NR; r++) P.round(a, bb, ka[r], kb[r]);
                P.last(a, bb, ka[NR], kb[NR]);
            }
            out[ch * 4 + ca] = a;
            out[ch * 4 + ca + 1] = bb;
        } else {
            QuadAes L;
            L.init();
            const uint32_t q = lane & 3;
            const uint32_t ch = blockIdx.x * CPC + 32 * PW + (wave - PW) * 16 + (lane >> 2);
            uint32_t k[NR + 1];
            QuadAes::round_keys<NR>(ek, q, k);
            uint32_t x = init_word(ch, q);
            for (int b = 0; b < blocks; b++) {
                x ^= k[0];
#pragma unroll
                for (int r = 1; r < NR; r++) x = L.template round<false>(x, k[r]);
                x = L.template last<false>(x, k[NR]);
            }
            out[ch * 4 + q] = x;
        }
    } else if constexpr (LAYOUT == 4 || LAYOUT == 5 || LAYOUT == 6) {  // quad: lane q = column q
        QuadAesB L;
        L.init();
        const uint32_t q = lane & 3;
        const uint32_t quad = LAYOUT == 6 ? wave : wave * 16 + (lane >> 2);
        if (LAYOUT == 6 && lane >= 4) return;
        uint32_t k[NR + 1];
        if constexpr (LAYOUT == 4) {
            QuadAes::round_keys<NR>(ek, q, k);
        } else {
#pragma unroll
            for (int r = 0; r <= NR; r++) k[r] = ek[4 * r + q];
        }
        uint32_t x[ILP];
        uint32_t ch[ILP];
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            ch[i] = blockIdx.x * CPC + quad * ILP + i;
            x[i] = init_word(ch[i], q);
        }
        for (int b = 0; b < blocks; b++) {
#pragma unroll
            for (int i = 0; i < ILP; i++) x[i] ^= k[0];
#pragma unroll
            for (int r = 1; r < NR; r++) {
                uint32_t y[ILP];
#pragma unroll
                for (int i = 0; i < ILP; i++) y[i] = LAYOUT == 4 ? L.template round<false>(x[i], k[r]) : L.round_b(x[i], k[r]);
#pragma unroll
                for (int i = 0; i < ILP; i++) x[i] = y[i];
            }
            uint32_t y[ILP];
#pragma unroll
            for (int i = 0; i < ILP; i++) y[i] = LAYOUT == 4 ? L.template last<false>(x[i], k[NR]) : L.last_b(x[i], k[NR]);
#pragma unroll
            for (int i = 0; i < ILP; i++) x[i] = y[i];
        }
#pragma unroll
        for (int i = 0; i < ILP; i++) out[ch[i] * 4 + q] = x[i];
    } else if constexpr (LAYOUT == 2 || LAYOUT == 7 || LAYOUT == 8) {  // pair: lane h = columns 2h, 2h+1
        PairAesG<LAYOUT == 7 ? 1 : LAYOUT == 8 ? 2 : 0> P;
        P.init();
        const uint32_t h = lane & 1;
        const uint32_t pr = wave * 32 + (lane >> 1);
        const uint32_t ca = 2 * h, pa = 2 * (1 - h);
        const uint32_t kwa = ek[ca], kwb = ek[ca + 1];
        uint32_t ka[NR + 1], kb[NR + 1];
#pragma unroll
        for (int r = 1; r <= NR; r++) {
            ka[r] = ek[4 * r + pa];
            kb[r] = ek[4 * r + pa + 1];
        }
        uint32_t a[ILP], bb[ILP], ch[ILP];
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            ch[i] = blockIdx.x * CPC + pr * ILP + i;
            a[i] = init_word(ch[i], ca);
            bb[i] = init_word(ch[i], ca + 1);
        }
        for (int b = 0; b < blocks; b++) {
#pragma unroll
            for (int i = 0; i < ILP; i++) {
                a[i] ^= kwa;
                bb[i] ^= kwb;
            }
#pragma unroll
            for (int r = 1; r < NR; r++) {
#pragma unroll
                for (int i = 0; i < ILP; i++) {
                    if constexpr (LAYOUT == 2) P.PairAes::round(a[i], bb[i], ka[r], kb[r]);
                    else P.round(a[i], bb[i], ka[r], kb[r]);
                }
            }
#pragma unroll
            for (int i = 0; i < ILP; i++) P.last(a[i], bb[i], ka[NR], kb[NR]);
        }
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            out[ch[i] * 4 + ca] = a[i];
            out[ch[i] * 4 + ca + 1] = bb[i];
        }
    } else {  // lane: one chain per lane
        QuadAes L;
        L.init();
        const uint32_t c = blockIdx.x * CPC + wave * 64 + lane;
        uint32_t s[4];
#pragma unroll
        for (int j = 0; j < 4; j++) s[j] = init_word(c, j);
        uint32_t k[4 * (NR + 1)];
#pragma unroll
        for (int j = 0; j < 4 * (NR + 1); j++) k[j] = ek[j];
        for (int b = 0; b < blocks; b++) {
#pragma unroll
            for (int j = 0; j < 4; j++) s[j] ^= k[j];
#pragma unroll
            for (int r = 1; r < NR; r++) lane_round(L, s, k + 4 * r);
            lane_last(L, s, k + 4 * NR);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) out[c * 4 + j] = s[j];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        cyc[2 * blockIdx.x] = t1 - t0;
        cyc[2 * blockIdx.x + 1] = rt1 - rt0;
    }
}

// Trace kernel (mode "t"): the pair layout of bench_kernel (LAYOUT 2, 256 chains per CU)
// with per-wave block-start time stamps.  STAGGER 0: no delay; 1: wave w waits w/8 of a
// round before its loop; 2: odd waves wait half a round; 3: no delay, but the two waves of a
// SIMD (w, w + 4) take turns at the higher issue priority, 8 blocks each (s_setprio 2 / 1),
// against the age order that otherwise lets the older wave run ahead.  round_cyc: the delay
// unit.
constexpr int TR_NS = 64;     // time-stamped blocks per wave
constexpr int TR_B0 = 200;    // first time-stamped block (the waves have settled by then)
template <int STAGGER>
__global__ void __launch_bounds__(512) trace_kernel(const uint32_t* __restrict__ ek, uint32_t* __restrict__ out,
                                                    uint64_t* __restrict__ trace, int blocks, int round_cyc) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    __builtin_amdgcn_s_setprio(1);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    PairAes P;
    P.init();
    const uint32_t h = lane & 1;
    const uint32_t ch = blockIdx.x * 256 + wave * 32 + (lane >> 1);
    const uint32_t ca = 2 * h, pa = 2 * (1 - h);
    const uint32_t kwa = ek[ca], kwb = ek[ca + 1];
    uint32_t ka[NR + 1], kb[NR + 1];
#pragma unroll
    for (int r = 1; r <= NR; r++) {
        ka[r] = ek[4 * r + pa];
        kb[r] = ek[4 * r + pa + 1];
    }
    uint32_t a = init_word(ch, ca), bb = init_word(ch, ca + 1);
    if (STAGGER == 1 || STAGGER == 2) {
        const uint64_t d = STAGGER == 1 ? (uint64_t)round_cyc * wave / 8 : (wave & 1) ? (uint64_t)round_cyc / 2 : 0;
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < d) {
        }
    }
    uint64_t* tr = trace + ((size_t)blockIdx.x * 8 + wave) * (TR_NS + 2);
    const uint64_t tl0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < blocks; b++) {
        if (b >= TR_B0 && b < TR_B0 + TR_NS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (lane == 0) tr[b - TR_B0] = t;
        }
        if (STAGGER == 3 && (b & 7) == 0) {
            if ((((uint32_t)b >> 3) + (wave >> 2)) & 1) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(1);
        }
        a ^= kwa;
        bb ^= kwb;
#pragma unroll
        for (int r = 1; r < NR; r++) P.round(a, bb, ka[r], kb[r]);
        P.last(a, bb, ka[NR], kb[NR]);
    }
    const uint64_t tl1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        tr[TR_NS] = tl0;
        tr[TR_NS + 1] = tl1;
    }
    out[ch * 4 + ca] = a;
    out[ch * 4 + ca + 1] = bb;
}

// VALU co-runner shaped like mac_kernel: one lane per "record", SHA-1 compressions
// on register data, one 256-thread block per CU (one wave per SIMD).
__global__ void __launch_bounds__(256) sha_corun(uint32_t* out, int iters) {
    uint32_t h[8] = {1, 2, 3, 4, 5, 0, 0, 0};
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = threadIdx.x * 31 + i;
    __builtin_amdgcn_s_setprio(0);
    for (int i = 0; i < iters; i++) {
        Hash<TLSGPU_MAC_SHA1>::compress(h, w);
        w[i & 15] ^= h[0];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
}

struct Res {
    const char* name;
    int cpc;
    float ms;
    double cyc;
    std::vector<uint32_t> out;
};

static hipStream_t g_side = nullptr;
static uint32_t* g_side_out = nullptr;

template <int LAYOUT, int ILP, int CPC>
static Res run(const char* name, const uint32_t* d_ek, int cus, int blocks, int corun = 0) {
    const int lanes_per_chain = LAYOUT == 6 ? 64 : (LAYOUT == 7 || LAYOUT == 8) ? 2 : LAYOUT >= 4 ? 4 : LAYOUT;
    const int threads = LAYOUT == 9 ? 4 * CPC - 64 * ILP : CPC * lanes_per_chain / ILP;
    auto kern = bench_kernel<LAYOUT, ILP, CPC>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              AES_LDS_BYTES);
    uint32_t* d_out;
    uint64_t* d_cyc;
    (void)hipMalloc(&d_out, (size_t)cus * CPC * 16);
    (void)hipMalloc(&d_cyc, cus * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), AES_LDS_BYTES, 0, d_ek, d_out, d_cyc, 20);
    (void)hipDeviceSynchronize();
    if (corun) hipLaunchKernelGGL(sha_corun, dim3(cus), dim3(256), 0, g_side, g_side_out, corun);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), AES_LDS_BYTES, 0, d_ek, d_out, d_cyc, blocks);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    Res r;
    r.name = name;
    r.cpc = CPC;
    (void)hipEventElapsedTime(&r.ms, e0, e1);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> cyc(2 * cus);
    (void)hipMemcpy(cyc.data(), d_cyc, cus * 16, hipMemcpyDeviceToHost);
    double s = 0, rt = 0;
    for (int i = 0; i < cus; i++) {
        s += (double)cyc[2 * i];
        rt += (double)cyc[2 * i + 1];
    }
    r.cyc = s / cus;
    const double ghz = s / (rt * 10.0);  // s_memrealtime ticks at 100 MHz
    r.out.resize((size_t)cus * CPC * 4);
    (void)hipMemcpy(r.out.data(), d_out, r.out.size() * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    const double rounds = (double)blocks * NR;
    const double floor_cyc = CPC * 16.0 / 32.0;  // LDS-array cycles per round
    const double ns = r.ms * 1e6 / rounds;
    // loop cycles (s_memtime of wave 0 around the block loop, table fill excluded)
    printf("%-7s chains/CU=%3d waves/CU=%2d%s  %7.2f ns/round  %6.1f loop-cyc/round  clock %.2f GHz  %5.1f G lookups/s/CU  "
           "LDS-floor frac %.2f  cfg2-equiv %.3f ms\n",
           name, CPC, (threads + 63) / 64, corun ? " +sha" : "     ", ns, r.cyc / rounds, ghz, CPC * 16.0 / ns,
           floor_cyc / (ns * ghz), r.ms * (256.0 / CPC) * 1027.0 / blocks);
    fflush(stdout);
    return r;
}

static int compare(const std::vector<Res>& rs) {
    int bad = 0;
    for (size_t i = 1; i < rs.size(); i++)
        if (rs[i].out != rs[0].out) {
            printf("MISMATCH: %s differs from %s\n", rs[i].name, rs[0].name);
            bad = 1;
        }
    return bad;
}

// mode "t": run trace_kernel<STAGGER> (+ optional co-runner), print per-wave round periods and
// the same-CU pair phase histogram
template <int STAGGER>
static std::vector<uint32_t> trace_run(const char* name, const uint32_t* d_ek, int cus, int blocks, int corun,
                                       int round_cyc) {
    auto kern = trace_kernel<STAGGER>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              AES_LDS_BYTES);
    uint32_t* d_out;
    uint64_t* d_tr;
    const size_t ntr = (size_t)cus * 8 * (TR_NS + 2);
    (void)hipMalloc(&d_out, (size_t)cus * 256 * 16);
    (void)hipMalloc(&d_tr, ntr * 8);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(512), AES_LDS_BYTES, 0, d_ek, d_out, d_tr, TR_B0 + TR_NS + 8, round_cyc);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    if (corun) hipLaunchKernelGGL(sha_corun, dim3(cus), dim3(256), 0, g_side, g_side_out, corun);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(512), AES_LDS_BYTES, 0, d_ek, d_out, d_tr, blocks, round_cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> tr(ntr);
    (void)hipMemcpy(tr.data(), d_tr, ntr * 8, hipMemcpyDeviceToHost);
    std::vector<uint32_t> out((size_t)cus * 256 * 4);
    (void)hipMemcpy(out.data(), d_out, out.size() * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_tr);
    // per wave: round period over the stamped blocks; loop cycles per round
    double per_sum = 0, loop_sum = 0, loop_min = 1e30, loop_max = 0;
    int hist[10] = {0};
    int npairs = 0;
    double spread_sum = 0;  // per CU and block: max - min block-start over the 8 waves, in rounds
    int nspread = 0;
    for (int c = 0; c < cus; c++) {
        double per[8];
        for (int w = 0; w < 8; w++) {
            const uint64_t* t = &tr[((size_t)c * 8 + w) * (TR_NS + 2)];
            per[w] = (double)(t[TR_NS - 1] - t[0]) / ((TR_NS - 1) * NR);
            per_sum += per[w];
            const double lc = (double)(t[TR_NS + 1] - t[TR_NS]) / ((double)blocks * NR);
            loop_sum += lc;
            loop_min = lc < loop_min ? lc : loop_min;
            loop_max = lc > loop_max ? lc : loop_max;
        }
        for (int b = 0; b < TR_NS; b++) {
            uint64_t lo = ~0ull, hi = 0;
            for (int w = 0; w < 8; w++) {
                const uint64_t x = tr[((size_t)c * 8 + w) * (TR_NS + 2) + b];
                lo = x < lo ? x : lo;
                hi = x > hi ? x : hi;
            }
            spread_sum += (double)(hi - lo) / per[0];
            nspread++;
        }
        // phase of wave w' relative to wave w within a round, sampled at every stamped block
        for (int w = 0; w < 8; w++)
            for (int v = w + 1; v < 8; v++)
                for (int b = 0; b < TR_NS; b += 4) {
                    const double P = 0.5 * (per[w] + per[v]);
                    const double d = (double)(int64_t)(tr[((size_t)c * 8 + v) * (TR_NS + 2) + b] -
                                                       tr[((size_t)c * 8 + w) * (TR_NS + 2) + b]);
                    double f = d / P - __builtin_floor(d / P);
                    int k = (int)(f * 10.0);
                    k = k < 0 ? 0 : (k > 9 ? 9 : k);
                    hist[k]++;
                    npairs++;
                }
    }
    const double nw = cus * 8.0;
    printf("%-10s%s  %7.3f ms (cfg2-equiv %.3f)  round period %6.1f cyc (stamped blocks), loop %6.1f cyc/round "
           "(waves: min %.1f max %.1f)  block-start spread over the CU's 8 waves %.2f rounds\n  pair phase within a "
           "round (10 bins, %% of %d):",
           name, corun ? " +sha" : "     ", ms, ms * 1027.0 / blocks, per_sum / nw, loop_sum / nw, loop_min, loop_max,
           spread_sum / nspread, npairs);
    for (int k = 0; k < 10; k++) printf(" %4.1f", 100.0 * hist[k] / npairs);
    printf("\n");
    fflush(stdout);
    return out;
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 1027;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    printf("CUs %d, %d blocks per chain\n", cus, blocks);
    uint32_t ek[4 * (NR + 1)];
    for (int i = 0; i < 4 * (NR + 1); i++) ek[i] = 0x01234567u * (i + 3) ^ (i << 20);
    uint32_t* d_ek;
    (void)hipMalloc(&d_ek, sizeof(ek));
    (void)hipMemcpy(d_ek, ek, sizeof(ek), hipMemcpyHostToDevice);
    (void)hipStreamCreateWithFlags(&g_side, hipStreamNonBlocking);
    (void)hipMalloc(&g_side_out, (size_t)cus * 256 * 4);
    if (argc > 2 && argv[2][0] == 't') {  // trace: do the pair waves convoy?
        std::vector<std::vector<uint32_t>> o;
        const int rc = 192;  // the measured round period (cycles) the stagger variants delay by
        o.push_back(trace_run<0>("pair1", d_ek, cus, blocks, 0, rc));
        o.push_back(trace_run<1>("pair1-st8", d_ek, cus, blocks, 0, rc));
        o.push_back(trace_run<2>("pair1-st2", d_ek, cus, blocks, 0, rc));
        o.push_back(trace_run<3>("pair1-alt", d_ek, cus, blocks, 0, rc));
        o.push_back(trace_run<0>("pair1", d_ek, cus, blocks, 2 * blocks, rc));
        o.push_back(trace_run<1>("pair1-st8", d_ek, cus, blocks, 2 * blocks, rc));
        o.push_back(trace_run<2>("pair1-st2", d_ek, cus, blocks, 2 * blocks, rc));
        o.push_back(trace_run<3>("pair1-alt", d_ek, cus, blocks, 2 * blocks, rc));
        int bad = 0;
        for (size_t i = 1; i < o.size(); i++) bad |= o[i] != o[0];
        printf(bad ? "MISMATCH between trace variants\n" : "all trace variants agree\n");
        return bad;
    }
    if (argc > 2 && argv[2][0] == 'l') {  // latency regime (cfg4)
        std::vector<Res> l2, l16;
        l2.push_back(run<4, 1, 2>("quad1", d_ek, cus, blocks));
        l2.push_back(run<5, 1, 2>("quad1b", d_ek, cus, blocks));
        l2.push_back(run<6, 1, 2>("quad1s", d_ek, cus, blocks));
        l2.push_back(run<2, 1, 2>("pair1", d_ek, cus, blocks));
        l2.push_back(run<1, 1, 2>("lane1", d_ek, cus, blocks));
        l16.push_back(run<4, 1, 16>("quad1", d_ek, cus, blocks));
        l16.push_back(run<5, 1, 16>("quad1b", d_ek, cus, blocks));
        l16.push_back(run<6, 1, 16>("quad1s", d_ek, cus, blocks));
        l16.push_back(run<2, 1, 16>("pair1", d_ek, cus, blocks));
        l16.push_back(run<1, 1, 16>("lane1", d_ek, cus, blocks));
        const int bad = compare(l2) | compare(l16);
        if (!bad) printf("all layouts agree\n");
        return bad;
    }
    hipLaunchKernelGGL(fill_gtables, dim3(1), dim3(256), 0, 0);
    (void)hipDeviceSynchronize();
    if (argc > 2 && argv[2][0] == 'm') {  // mixed layout: half the chains on pair waves, half on quad waves
        std::vector<Res> m;
        m.push_back(run<2, 1, 256>("pair1", d_ek, cus, blocks));
        m.push_back(run<4, 1, 256>("quad1", d_ek, cus, blocks));
        m.push_back(run<9, 2, 256>("mix2", d_ek, cus, blocks));
        m.push_back(run<9, 3, 256>("mix3", d_ek, cus, blocks));
        m.push_back(run<9, 4, 256>("mix4", d_ek, cus, blocks));
        m.push_back(run<9, 5, 256>("mix5", d_ek, cus, blocks));
        m.push_back(run<9, 6, 256>("mix6", d_ek, cus, blocks));
        m.push_back(run<2, 1, 256>("pair1", d_ek, cus, blocks, 2 * blocks));
        m.push_back(run<9, 3, 256>("mix3", d_ek, cus, blocks, 2 * blocks));
        m.push_back(run<9, 4, 256>("mix4", d_ek, cus, blocks, 2 * blocks));
        m.push_back(run<9, 5, 256>("mix5", d_ek, cus, blocks, 2 * blocks));
        const int bad = compare(m);
        if (!bad) printf("all layouts agree\n");
        return bad;
    }
    if (argc > 2 && argv[2][0] == 'g') {  // second gather port: pair with T3 (T2) lookups from global
        std::vector<Res> g;
        g.push_back(run<2, 1, 256>("pair1", d_ek, cus, blocks));
        g.push_back(run<7, 1, 256>("pairg1", d_ek, cus, blocks));
        g.push_back(run<8, 1, 256>("pairg2", d_ek, cus, blocks));
        g.push_back(run<2, 1, 256>("pair1", d_ek, cus, blocks, 2 * blocks));
        g.push_back(run<7, 1, 256>("pairg1", d_ek, cus, blocks, 2 * blocks));
        g.push_back(run<8, 1, 256>("pairg2", d_ek, cus, blocks, 2 * blocks));
        const int bad = compare(g);
        if (!bad) printf("all layouts agree\n");
        return bad;
    }
    std::vector<Res> a;
    a.push_back(run<4, 1, 256>("quad1", d_ek, cus, blocks));
    a.push_back(run<5, 1, 256>("quad1b", d_ek, cus, blocks));
    a.push_back(run<4, 2, 256>("quad2", d_ek, cus, blocks));
    a.push_back(run<5, 2, 256>("quad2b", d_ek, cus, blocks));
    a.push_back(run<2, 1, 256>("pair1", d_ek, cus, blocks));
    a.push_back(run<2, 2, 256>("pair2", d_ek, cus, blocks));
    a.push_back(run<1, 1, 256>("lane1", d_ek, cus, blocks));
    std::vector<Res> b;
    b.push_back(run<5, 2, 512>("quad2b", d_ek, cus, blocks));
    b.push_back(run<4, 2, 512>("quad2", d_ek, cus, blocks));
    b.push_back(run<2, 2, 512>("pair2", d_ek, cus, blocks));
    b.push_back(run<2, 1, 512>("pair1", d_ek, cus, blocks));
    b.push_back(run<1, 1, 512>("lane1", d_ek, cus, blocks));
    // beside a mac_kernel-shaped VALU load (about 1.5x the AES kernel's duration)
    std::vector<Res> c;
    c.push_back(run<4, 1, 256>("quad1", d_ek, cus, blocks, 2 * blocks));
    c.push_back(run<5, 1, 256>("quad1b", d_ek, cus, blocks, 2 * blocks));
    c.push_back(run<2, 1, 256>("pair1", d_ek, cus, blocks, 2 * blocks));
    c.push_back(run<4, 1, 256>("quad1", d_ek, cus, blocks, blocks / 3));
    c.push_back(run<2, 1, 256>("pair1", d_ek, cus, blocks, blocks / 3));
    // many chains (cfg3: 4,096 per CU): one lane per chain at 12 / 16 waves, and at 8 waves
    // beside the mac_kernel-shaped load
    std::vector<Res> d;
    d.push_back(run<1, 1, 512>("lane1", d_ek, cus, blocks, 2 * blocks));
    d.push_back(run<2, 1, 512>("pair1", d_ek, cus, blocks, 2 * blocks));
    run<1, 1, 768>("lane1", d_ek, cus, blocks);
    run<1, 1, 1024>("lane1", d_ek, cus, blocks);
    const int bad = compare(a) | compare(b) | compare(c) | compare(d);
    if (!bad) printf("all layouts agree\n");
    return bad;
}

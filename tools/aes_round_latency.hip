// aes_round_latency.hip -- the pieces of the dependent AES round for a LONE wave per CU
// (the cfg4 regime: 2-16 chains per CU), diagnostic tool.  Each kernel runs
// one wave per CU over a dependent chain of one kind of step; s_memtime (shader clock)
// around the loop gives cycles per step:
//   valu      v_xor_b32 -> v_xor_b32                 (dependent VALU latency)
//   bitop3    v_bitop3_b32 chain
//   perm      v_perm_b32 chain
//   dpp       v_xor_b32_dpp quad_perm chain            (DPP + its read-after-write wait states)
//   lds       addr = bitop3(x, 0xff00, base); x = ds_read_b32(addr)   (address op + LDS latency)
//   lds4      4 independent ds_read_b32 per step, XOR-combined        (the round's 4 lookups)
//   quad_thr  QuadAes::round<false> (cbc_kernel throughput form), 4 lanes per chain
//   quad_lat  QuadAes::round<true>  (cbc_kernel latency form, cfg4)
//   pair      PairAes::round (cbc_pair_kernel), 2 lanes per chain
//   hexa      16 lanes per chain, one lookup per lane (candidate latency layout)
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/aes_round_latency.hip -o tools/bin/aes_round_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../tlslite_amd/csrc/tg_quad.h"

using namespace tg;

constexpr int ITERS = 4096;

template <int KIND>
__global__ void __launch_bounds__(64) lat_kernel(const uint32_t* __restrict__ ek, uint32_t* __restrict__ out,
                                                 uint64_t* __restrict__ cyc) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    const uint32_t lane = threadIdx.x;
    uint32_t x = lane * 0x9E3779B9u + blockIdx.x;
    QuadAes Q;
    Q.init();
    PairAes P;
    P.init();
    const uint32_t m8 = vconst(0xff00u), base = (lane & 31) * 4;
    const uint32_t k0 = ek[lane & 3], k1 = ek[4 + (lane & 3)];
    uint32_t y = x ^ 0x5bd1e995u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
        if constexpr (KIND == 0) {
#pragma unroll
            for (int u = 0; u < 8; u++) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(k0));
        } else if constexpr (KIND == 1) {
#pragma unroll
            for (int u = 0; u < 8; u++) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(k0), "v"(k1));
        } else if constexpr (KIND == 2) {
#pragma unroll
            for (int u = 0; u < 8; u++) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k0), "v"(k1));
        } else if constexpr (KIND == 3) {
#pragma unroll
            for (int u = 0; u < 8; u++) x = x ^ quad_dpp<0x39>(x);
        } else if constexpr (KIND == 4) {
#pragma unroll
            for (int u = 0; u < 8; u++) x = lds_read32(__builtin_amdgcn_bitop3_b32(x, m8, base, 0xEA));
        } else if constexpr (KIND == 5) {
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t a = lds_read32(__builtin_amdgcn_bitop3_b32(x, m8, base, 0xEA));
                const uint32_t b = lds_read32(__builtin_amdgcn_bitop3_b32(x >> 8, m8, base, 0xEA) + 128);
                const uint32_t c = lds_read32(__builtin_amdgcn_bitop3_b32(x << 8, m8, base | 0x10000u, 0xEA));
                const uint32_t d = lds_read32(__builtin_amdgcn_bitop3_b32(x >> 16, m8, base | 0x10000u, 0xEA) + 128);
                x = a ^ b ^ c ^ d;
            }
        } else if constexpr (KIND == 6) {
#pragma unroll
            for (int u = 0; u < 8; u++) x = Q.round<false>(x, k1);
        } else if constexpr (KIND == 7) {
#pragma unroll
            for (int u = 0; u < 8; u++) x = Q.round<true>(x, k1);
        } else if constexpr (KIND == 8) {
#pragma unroll
            for (int u = 0; u < 8; u++) P.round(x, y, k0, k1);
        } else if constexpr (KIND == 9) {
            // 16 lanes per chain: lane 4b + c looks up table b for byte b of column (c + b) & 3 (its
            // own copy of the state word it needs), the 4 terms of column c are XOR-reduced across
            // the row's 4 quads (row_ror 4 / 8), then quad b's lanes rotate their column by b so
            // that lane 4b + c again holds column (c + b) & 3 -- one lookup per lane per round.
            const uint32_t b = (lane >> 2) & 3;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                uint32_t t;
                if (b == 0) t = Q.look<0, 0>(x);
                else if (b == 1) t = Q.look<1, 1>(x);
                else if (b == 2) t = Q.look<2, 2>(x);
                else t = Q.look<3, 3>(x);
                t ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x124, 0xf, 0xf, true);  // row_ror:4
                t ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x128, 0xf, 0xf, true);  // row_ror:8
                t ^= k1;
                // quad b takes column (c + b) & 3 from lane 4b + ((c + b) & 3) of its own quad
                const uint32_t r1 = quad_dpp<0x39>(t), r2 = quad_dpp<0x4E>(t), r3 = quad_dpp<0x93>(t);
                x = b == 0 ? t : b == 1 ? r1 : b == 2 ? r2 : r3;
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = x ^ y;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char* name, const uint32_t* d_ek, int cus, double steps_per_iter) {
    auto kern = lat_kernel<KIND>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              AES_LDS_BYTES);
    uint32_t* d_out;
    uint64_t* d_cyc;
    (void)hipMalloc(&d_out, (size_t)cus * 64 * 4);
    (void)hipMalloc(&d_cyc, (size_t)cus * 8);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(64), AES_LDS_BYTES, 0, d_ek, d_out, d_cyc);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(kern, dim3(cus), dim3(64), AES_LDS_BYTES, 0, d_ek, d_out, d_cyc);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> c(cus);
    (void)hipMemcpy(c.data(), d_cyc, (size_t)cus * 8, hipMemcpyDeviceToHost);
    std::vector<uint64_t> s(c);
    std::sort(s.begin(), s.end());
    const double med = (double)s[cus / 2];
    printf("%-9s %7.1f shader cycles per step (median over %d CUs, min %.1f)\n", name,
           med / (ITERS * 8.0 * steps_per_iter), cus, (double)s[0] / (ITERS * 8.0 * steps_per_iter));
    fflush(stdout);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t ek[44];
    for (int i = 0; i < 44; i++) ek[i] = 0x01234567u * (i + 3) ^ (i << 20);
    uint32_t* d_ek;
    (void)hipMalloc(&d_ek, sizeof(ek));
    (void)hipMemcpy(d_ek, ek, sizeof(ek), hipMemcpyHostToDevice);
    run<0>("valu", d_ek, cus, 1);
    run<1>("bitop3", d_ek, cus, 1);
    run<2>("perm", d_ek, cus, 1);
    run<3>("dpp", d_ek, cus, 1);
    run<4>("lds", d_ek, cus, 1);
    run<5>("lds4", d_ek, cus, 1);
    run<6>("quad_thr", d_ek, cus, 1);
    run<7>("quad_lat", d_ek, cus, 1);
    run<8>("pair", d_ek, cus, 1);
    run<9>("hexa", d_ek, cus, 1);
    return 0;
}

// des_layout_microbench.hip -- 3DES-EDE CBC chains at cfg5's 128 chains per CU
// (32,768 3DES records on 256 CUs), comparing lane layouts of the Feistel round
// with no global-memory traffic in the loop (diagnostic tool only):
//   d8     8 lanes/chain, one SP box per lane, 3 DPP XOR steps (round 1's tdes8_kernel)
//   d8x2   d8 with two chains interleaved per 8-lane group
//   d4     4 lanes/chain, two SP boxes per lane (even + odd half), 2 DPP XOR steps (tdes4_kernel)
//   d4x2   d4 with two chains interleaved per 4-lane group
//   d4b    d4 with the next round's key-side address part computed a round early
//   d2     2 lanes/chain, four SP boxes per lane, 1 DPP XOR step
//   d1     1 lane/chain, all eight SP boxes, no DPP
// All layouts run the same 48 rounds with the same per-round key words and must end
// in the same (l, r) per chain.  Reports ns and loop cycles per Feistel round and the
// fraction of the LDS floor (8 lookups per round per chain, 32 lanes per cycle).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/des_layout_microbench.hip -o tools/des_layout_mb.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <type_traits>
#include "../tlslite_amd/csrc/tg_aes3.h"

using namespace tg;

constexpr int CPC = 128;

__device__ __forceinline__ uint32_t rotl4(uint32_t x) { return (x << 4) | (x >> 28); }
// per-round key words: the even and the odd word of round g (synthetic, same for all layouts)
__device__ __forceinline__ uint32_t kev(uint32_t chain, int g) { return (chain * 0x9E3779B9u) ^ (g * 0x85EBCA6Bu); }
__device__ __forceinline__ uint32_t kod(uint32_t chain, int g) { return (chain * 0xC2B2AE35u) ^ (g * 0x27D4EB2Fu) ^ 0x5bd1e995u; }

// 8 lanes per chain (the round-1 product layout): lane j evaluates ONE SP-box term and
// three DPP XOR steps sum the eight
struct Des8 {
    uint32_t base, sa;
    bool odd;
    __device__ __forceinline__ void init() {
        const uint32_t lane = __lane_id(), j = lane & 7;
        const uint32_t K = j < 4 ? 7 - 2 * j : 6 - 2 * (j - 4);
        base = (lane & 31) * 4 + K * 8192;
        odd = j >= 4;
        sa = ((odd ? 4u : 0u) + 8 * (j & 3) + 25u) & 31u;
    }
    __device__ __forceinline__ uint32_t key(uint32_t even, uint32_t oddw) const {
        return odd ? ((oddw << 4) | (oddw >> 28)) : even;
    }
    __device__ __forceinline__ uint32_t f(uint32_t t) const {
        const uint32_t u = __builtin_amdgcn_alignbit(t, t, sa);
        uint32_t v = lds_read32((u & 0x1f80u) | base);
        v ^= quad_dpp<0xB1>(v);
        v ^= quad_dpp<0x4E>(v);
        v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, true);  // row_half_mirror
        return v;
    }
    __device__ __forceinline__ void block(uint32_t& hi, uint32_t& lo, const uint32_t* kw) const {
        uint32_t l = hi, r = lo;
        des_ip(l, r);
        uint32_t t = r ^ kw[0];
#pragma unroll
        for (int g = 0; g < 48; g++) {
            const uint32_t fv = f(t);
            const uint32_t rn = l ^ fv;
            if (g % 16 != 15) {
                if (g + 1 < 48) t = __builtin_amdgcn_bitop3_b32(l, fv, kw[g + 1], 0x96);
                l = r;
                r = rn;
            } else {
                l = rn;
                if (g + 1 < 48) t = r ^ kw[g + 1];
            }
        }
        des_fp(l, r);
        hi = l;
        lo = r;
    }
};

// Round 2's tdes4_kernel round (two lookups per lane on the 32-copy SP tables, des_lds_fill);
// the product kernel moved to one lookup per lane on combined tables in round 3 (Des4C, tg_aes3.h).
struct Des4 {
    uint32_t be, bo, se, so, m;
    __device__ __forceinline__ void init() {
        const uint32_t lane = __lane_id(), j = lane & 3;
        m = vconst(0x1f80u);
        be = (lane & 31) * 4 + (7 - 2 * j) * 8192;
        bo = (lane & 31) * 4 + (6 - 2 * j) * 8192;
        // rotate so that the lane's 6 index bits (bit 8j of w, bit 8j+4 of t_odd) land at bits 7..12
        se = (8 * j + 25u) & 31u;
        so = (8 * j + 29u) & 31u;
    }
    // Feistel f of te = r ^ k_even, to = r ^ rotl4(k_odd), summed over the quad
    __device__ __forceinline__ uint32_t f(uint32_t te, uint32_t to) const {
        const uint32_t ue = __builtin_amdgcn_alignbit(te, te, se);
        const uint32_t uo = __builtin_amdgcn_alignbit(to, to, so);
        // (u & 0x1f80) | base as an all-VGPR v_bitop3 (2 cycles) rather than v_and_or_b32 (4)
        uint32_t v = lds_read32(__builtin_amdgcn_bitop3_b32(ue, m, be, 0xEA)) ^
                     lds_read32(__builtin_amdgcn_bitop3_b32(uo, m, bo, 0xEA));
        v ^= quad_dpp<0xB1>(v);
        v ^= quad_dpp<0x4E>(v);
        return v;
    }
    // block as two big-endian words; ke/ko[16p + i] = even / pre-rotated odd key word of
    // pass p, round i.  The next round's key XORs take l ^ f ^ k in one 3-input XOR each.
    __device__ __forceinline__ void block(uint32_t& hi, uint32_t& lo, const uint32_t* ke, const uint32_t* ko) const {
        uint32_t l = hi, r = lo;
        des_ip(l, r);
        uint32_t te = r ^ ke[0], to = r ^ ko[0];
#pragma unroll
        for (int g = 0; g < 48; g++) {
            const uint32_t fv = f(te, to);
            const uint32_t rn = l ^ fv;
            if (g % 16 != 15) {
                if (g + 1 < 48) {
                    te = __builtin_amdgcn_bitop3_b32(l, fv, ke[g + 1], 0x96);
                    to = __builtin_amdgcn_bitop3_b32(l, fv, ko[g + 1], 0x96);
                }
                l = r;
                r = rn;
            } else {  // end of a DES pass: (l, r) = (R16, L16) feeds the next pass
                l = rn;
                if (g + 1 < 48) {
                    te = r ^ ke[g + 1];
                    to = r ^ ko[g + 1];
                }
            }
        }
        des_fp(l, r);
        hi = l;
        lo = r;
    }
    // CBC on LE words (TdesCbc::enc_block): c = E(p ^ iv), iv = c
    __device__ __forceinline__ void cbc(uint32_t d0, uint32_t d1, uint32_t& iv0, uint32_t& iv1,
                                        const uint32_t* ke, const uint32_t* ko) const {
        uint32_t hi = bswap32(d0 ^ iv0), lo = bswap32(d1 ^ iv1);
        block(hi, lo, ke, ko);
        iv0 = bswap32(hi);
        iv1 = bswap32(lo);
    }
};

// 4 lanes per chain: Des4 above.  2 and 1 lanes per chain: DesG,
// lane j does the 8/LPC lookups of bytes [4j/LPC, 4(j+1)/LPC) of w and v.
template <int LPC>
struct DesG {
    static constexpr int NB = 4 / LPC;
    uint32_t be[NB], bo[NB], se[NB], so[NB];
    __device__ __forceinline__ void init() {
        const uint32_t lane = __lane_id(), j = lane & (LPC - 1);
#pragma unroll
        for (int i = 0; i < NB; i++) {
            const uint32_t b = j * NB + i;
            be[i] = (lane & 31) * 4 + (7 - 2 * b) * 8192;
            bo[i] = (lane & 31) * 4 + (6 - 2 * b) * 8192;
            se[i] = (8 * b + 25u) & 31u;
            so[i] = (8 * b + 29u) & 31u;
        }
    }
    __device__ __forceinline__ uint32_t f(uint32_t te, uint32_t to) const {
        uint32_t t[2 * NB];
#pragma unroll
        for (int i = 0; i < NB; i++) {
            t[2 * i] = lds_read32((__builtin_amdgcn_alignbit(te, te, se[i]) & 0x1f80u) | be[i]);
            t[2 * i + 1] = lds_read32((__builtin_amdgcn_alignbit(to, to, so[i]) & 0x1f80u) | bo[i]);
        }
#pragma unroll
        for (int w = 1; w < 2 * NB; w *= 2)
#pragma unroll
            for (int i = 0; i + w < 2 * NB; i += 2 * w) t[i] ^= t[i + w];
        uint32_t v = t[0];
        if constexpr (LPC == 2) v ^= quad_dpp<0xB1>(v);
        return v;
    }
};

// d4b: Des4 with the next round's address split into a part known one round early,
// A = (rotr(l ^ k, s) & M) | base, and the part from f: addr = A ^ (rotr(f, s) & M) -- one
// v_alignbit + one v_bitop3 between f and the LDS read instead of bitop3, alignbit, and_or.
__device__ __forceinline__ void d4b_rounds(const Des4& D, uint32_t& L, uint32_t& R, const uint32_t* ke,
                                           const uint32_t* ko) {
    const uint32_t M = D.m;  // 0x1f80 in a VGPR: the bitop3 forms stay 2-cycle
    uint32_t ae = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(R ^ ke[0], R ^ ke[0], D.se), M, D.be, 0xEA);
    uint32_t ao = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(R ^ ko[0], R ^ ko[0], D.so), M, D.bo, 0xEA);
#pragma unroll
    for (int g = 0; g < 48; g++) {
        uint32_t v = lds_read32(ae) ^ lds_read32(ao);
        // the next round's key-side address part, off the critical path (l is known)
        uint32_t ne = 0, no = 0;
        const uint32_t lx = (g % 16 != 15) ? L : R;  // the word f is XORed onto for the next round's input
        if (g + 1 < 48) {
            const uint32_t te = lx ^ ke[g + 1], to = lx ^ ko[g + 1];
            ne = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(te, te, D.se), M, D.be, 0xEA);
            no = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(to, to, D.so), M, D.bo, 0xEA);
        }
        v ^= quad_dpp<0xB1>(v);
        v ^= quad_dpp<0x4E>(v);
        const uint32_t rn = L ^ v;
        if (g % 16 != 15) {
            if (g + 1 < 48) {
                ae = __builtin_amdgcn_bitop3_b32(ne, __builtin_amdgcn_alignbit(v, v, D.se), M, 0x78);
                ao = __builtin_amdgcn_bitop3_b32(no, __builtin_amdgcn_alignbit(v, v, D.so), M, 0x78);
            }
            L = R;
            R = rn;
        } else {
            L = rn;
            ae = ne;
            ao = no;
        }
    }
}

template <int LAYOUT, int ILP>  // LAYOUT 8 or 4 lanes per chain
__global__ void __launch_bounds__(1024) bench_kernel(uint32_t* __restrict__ out, uint64_t* __restrict__ cyc,
                                                     int blocks) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    des_lds_fill(lds);
    __syncthreads();
    __builtin_amdgcn_s_setprio(1);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint32_t lane = threadIdx.x & 63;
    constexpr int LPC = LAYOUT == 5 ? 4 : LAYOUT;
    const uint32_t grp = threadIdx.x / LPC;
    const uint32_t j = lane & (LPC - 1);
    uint32_t ch[ILP], l[ILP], r[ILP];
#pragma unroll
    for (int i = 0; i < ILP; i++) {
        ch[i] = blockIdx.x * CPC + grp * ILP + i;
        l[i] = ch[i] * 2654435761u;
        r[i] = ch[i] ^ 0xdeadbeefu;
    }
    if constexpr (LAYOUT == 5) {
        Des4 D;
        D.init();
        uint32_t ke[48], ko[48];
#pragma unroll
        for (int g = 0; g < 48; g++) {
            ke[g] = kev(ch[0], g);
            ko[g] = rotl4(kod(ch[0], g));
        }
        for (int b = 0; b < blocks; b++) {
            uint32_t L = l[0], R = r[0];
            des_ip(L, R);
            d4b_rounds(D, L, R, ke, ko);
            des_fp(L, R);
            l[0] = L;
            r[0] = R;
        }
    } else if constexpr (LAYOUT == 8) {
        Des8 D;
        D.init();
        uint32_t kw[ILP][48];
#pragma unroll
        for (int i = 0; i < ILP; i++)
#pragma unroll
            for (int g = 0; g < 48; g++) kw[i][g] = D.key(kev(ch[i], g), kod(ch[i], g));
        for (int b = 0; b < blocks; b++) {
#pragma unroll
            for (int i = 0; i < ILP; i++) D.block(l[i], r[i], kw[i]);
        }
    } else {
        typename std::conditional<LAYOUT == 4, Des4, DesG<LAYOUT == 4 ? 1 : LAYOUT>>::type D;
        D.init();
        uint32_t ke[ILP][48], ko[ILP][48];
#pragma unroll
        for (int i = 0; i < ILP; i++)
#pragma unroll
            for (int g = 0; g < 48; g++) {
                ke[i][g] = kev(ch[i], g);
                ko[i][g] = rotl4(kod(ch[i], g));
            }
        for (int b = 0; b < blocks; b++) {
            uint32_t L[ILP], R[ILP], te[ILP], to[ILP];
#pragma unroll
            for (int i = 0; i < ILP; i++) {
                L[i] = l[i];
                R[i] = r[i];
                des_ip(L[i], R[i]);
                te[i] = R[i] ^ ke[i][0];
                to[i] = R[i] ^ ko[i][0];
            }
#pragma unroll
            for (int g = 0; g < 48; g++) {
#pragma unroll
                for (int i = 0; i < ILP; i++) {
                    const uint32_t fv = D.f(te[i], to[i]);
                    const uint32_t rn = L[i] ^ fv;
                    if (g % 16 != 15) {
                        if (g + 1 < 48) {
                            te[i] = __builtin_amdgcn_bitop3_b32(L[i], fv, ke[i][g + 1], 0x96);
                            to[i] = __builtin_amdgcn_bitop3_b32(L[i], fv, ko[i][g + 1], 0x96);
                        }
                        L[i] = R[i];
                        R[i] = rn;
                    } else {
                        L[i] = rn;
                        if (g + 1 < 48) {
                            te[i] = R[i] ^ ke[i][g + 1];
                            to[i] = R[i] ^ ko[i][g + 1];
                        }
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < ILP; i++) {
                des_fp(L[i], R[i]);
                l[i] = L[i];
                r[i] = R[i];
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (j == 0)
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            out[2 * ch[i]] = l[i];
            out[2 * ch[i] + 1] = r[i];
        }
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

struct Res {
    const char* name;
    std::vector<uint32_t> out;
};

template <int LAYOUT, int ILP>
static Res run(const char* name, int cus, int blocks) {
    const int threads = CPC * (LAYOUT == 5 ? 4 : LAYOUT) / ILP;
    auto kern = bench_kernel<LAYOUT, ILP>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              DES_LDS_BYTES);
    uint32_t* d_out;
    uint64_t* d_cyc;
    (void)hipMalloc(&d_out, (size_t)cus * CPC * 8);
    (void)hipMalloc(&d_cyc, cus * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), DES_LDS_BYTES, 0, d_out, d_cyc, 4);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), DES_LDS_BYTES, 0, d_out, d_cyc, blocks);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> cyc(cus);
    (void)hipMemcpy(cyc.data(), d_cyc, cus * 8, hipMemcpyDeviceToHost);
    double c = 0;
    for (int i = 0; i < cus; i++) c += (double)cyc[i];
    c /= cus;
    Res r;
    r.name = name;
    r.out.resize((size_t)cus * CPC * 2);
    (void)hipMemcpy(r.out.data(), d_out, r.out.size() * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    const double rounds = (double)blocks * 48;
    const double ns = ms * 1e6 / rounds;
    const double floor_cyc = CPC * 8.0 / 32.0;
    printf("%-5s chains/CU=%d waves/CU=%2d  %7.2f ns/round  %6.1f loop-cyc/round  LDS-floor frac %.2f  "
           "cfg5-equiv %.2f ms\n",
           name, CPC, threads / 64, ns, c / rounds, floor_cyc / (c / rounds), ns * 2052 * 48 / 1e6);
    fflush(stdout);
    return r;
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 256;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    printf("CUs %d, %d blocks per chain\n", cus, blocks);
    std::vector<Res> rs;
    rs.push_back(run<8, 1>("d8", cus, blocks));
    rs.push_back(run<8, 2>("d8x2", cus, blocks));
    rs.push_back(run<4, 1>("d4", cus, blocks));
    rs.push_back(run<4, 2>("d4x2", cus, blocks));
    rs.push_back(run<5, 1>("d4b", cus, blocks));
    rs.push_back(run<2, 1>("d2", cus, blocks));
    rs.push_back(run<1, 1>("d1", cus, blocks));
    int bad = 0;
    for (size_t i = 1; i < rs.size(); i++)
        if (rs[i].out != rs[0].out) {
            printf("MISMATCH: %s differs from %s\n", rs[i].name, rs[0].name);
            bad = 1;
        }
    if (!bad) printf("all layouts agree\n");
    return bad;
}

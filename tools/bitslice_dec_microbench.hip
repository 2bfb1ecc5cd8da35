// bitslice_dec_microbench.hip -- is a bitsliced AES decrypt worth running beside the open path's
// T-table decrypt?  
//
// No global-memory traffic in the loops.  Waves of two kinds, in two kernels:
//   T  the product's lane-per-block decrypt round loop (lane_aes_dec, tg_open3.h: 16 Td lookups
//      per round from the 32-copy LDS tables), round keys wave-uniform (SGPRs)
//   B  a bitsliced decrypt: 32 blocks of one record per lane, 128 planes (tools/bs_aes_inv.h,
//      generated and checked by tools/bitslice_gen.py), the round key applied as conditional
//      NOTs (SGPR masks); two rounds per loop iteration so InvShiftRows stays a renaming
//      (ping-pong plane arrays; one kernel cannot hold both kinds: its VGPR allocation is the
//      larger one for every wave)
// Modes: T alone (16 waves per CU, the product's shape), B alone (4, 8, 12 waves per CU), and
// both at once on two streams (the B waves take the wave slots and VGPRs the T workgroup leaves).
// The host prints each kind's rate in block-rounds per second and the total, and checks the B
// waves' output against a host run of the same bitsliced code and a plain AES inverse round.
// Diagnostic tool only (not in the product):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Itlslite_amd/csrc -mllvm -disable-promote-alloca-to-lds \
//         tools/bitslice_dec_microbench.hip -o tools/bs_dec_mb.bin
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../tlslite_amd/csrc/tg_open3.h"
#include "bs_aes_inv.h"

using namespace tg;
constexpr int NR = 10;

// InvShiftRows: output byte 4c + r takes input byte 4((c - r) & 3) + r (FIPS-197 5.3.1)
__host__ __device__ constexpr int isr(int o) { return 4 * (((o >> 2) - (o & 3)) & 3) + (o & 3); }

// one bitsliced inverse round: dst = InvMixColumns(InvSubBytes(InvShiftRows(src)) ^ key);
// key word k[i] holds bytes 4i..4i+3 of the round key (little-endian), the same for all 32 blocks
template <bool MIX>
__host__ __device__ __forceinline__ void bs_round(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                  const uint32_t* __restrict__ k) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t sb[32];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int o = 4 * c + r;
            bs_inv_sbox(src + 8 * isr(o), sb + 8 * r);
#pragma unroll
            for (int b = 0; b < 8; b++) sb[8 * r + b] ^= 0u - ((k[o >> 2] >> (8 * (o & 3) + b)) & 1u);
        }
        if constexpr (MIX) {
            bs_inv_mix_column(sb, dst + 32 * c);
        } else {
#pragma unroll
            for (int i = 0; i < 32; i++) dst[32 * c + i] = sb[i];
        }
    }
}

// T waves: the product's decrypt round loop; one 1,024-thread workgroup per CU (the LDS tables
// take 160 KiB of the CU's 160 KiB)
__global__ void __launch_bounds__(1024, 1) t_kernel(const uint32_t* __restrict__ dk, uint32_t* __restrict__ out,
                                                   uint64_t* __restrict__ cyc, int iters, uint32_t* __restrict__ done) {
    aes_lds_fill(nullptr, true);
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    QuadAesDec D;
    D.init();
    uint32_t s[4];
#pragma unroll
    for (int j = 0; j < 4; j++) s[j] = gid * 0x9e3779b9u ^ (j * 0x85ebca6bu);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) lane_aes_dec<NR>(D, s, dk);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int j = 0; j < 4; j++) out[gid * 4 + j] = s[j];
    if ((threadIdx.x & 63) == 0) {
        cyc[gid >> 6] = t1 - t0;
        __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);  // a vector atomic
    }
}

// B waves: one-wave workgroups, no LDS.  The round keys rotate with the iteration (as a record's
// ten differ), so their masks are computed per round by the scalar unit, not hoisted.
__device__ __host__ __forceinline__ const uint32_t* bs_key(const uint32_t* dk, int it, int half) {
    return dk + 4 * (1 + half + (it & 7));
}
// With stop != 0 a wave also leaves once *done reaches stop (every T wave finished): the B waves'
// iterations then measure what they got while the T kernel ran.  Every wave reaches an exit: the
// iteration cap, or the T kernel's last wave.
__global__ void __launch_bounds__(64) b_kernel(const uint32_t* __restrict__ dk, uint32_t* __restrict__ out,
                                               uint64_t* __restrict__ cyc, int iters, const uint32_t* done,
                                               uint32_t stop, uint32_t* __restrict__ iters_done) {
    const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
    uint32_t p[128], q[128];
#pragma unroll
    for (int i = 0; i < 128; i++) p[i] = (gid * 0x2545f491u) ^ (i * 0x9e3779b9u) ^ 0x5bd1e995u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    int it = 0;
    for (; it < iters; it++) {
        if (stop && __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= stop) break;
        bs_round<true>(p, q, bs_key(dk, it, 0));
        bs_round<true>(q, p, bs_key(dk, it, 1));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 128; i++) out[(size_t)gid * 128 + i] = p[i];
    if (threadIdx.x == 0) {
        cyc[blockIdx.x] = t1 - t0;
        iters_done[blockIdx.x] = (uint32_t)it;
    }
}

// 32 x 32 bit transpose of a[0..31] in place (out[k] bit j = in[j] bit k): the 16- and 8-bit stages
// as byte permutes (one v_perm per word), the 4-, 2- and 1-bit stages as shift + select pairs.
// Transposing blocks' word w gives planes 32w + 8 * (byte in word) + bit = 8 * (state byte) + bit,
// the layout bs_round uses.  The transpose is its own inverse.
__host__ __device__ __forceinline__ uint32_t bs_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint8_t b[8] = {(uint8_t)lo, (uint8_t)(lo >> 8), (uint8_t)(lo >> 16), (uint8_t)(lo >> 24),
                          (uint8_t)hi, (uint8_t)(hi >> 8), (uint8_t)(hi >> 16), (uint8_t)(hi >> 24)};
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) r |= (uint32_t)b[(sel >> (8 * i)) & 7] << (8 * i);
    return r;
#endif
}
template <int S>
__host__ __device__ __forceinline__ void bs_swap_stage(uint32_t* a) {  // rows k and k + S, bit blocks of S
    constexpr uint32_t m = S == 4 ? 0x0f0f0f0fu : S == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int k = 0; k < 32; k++) {
        if (k & S) continue;
        const uint32_t x = a[k], y = a[k + S];
        a[k] = (x & m) | ((y << S) & ~m);
        a[k + S] = ((x >> S) & m) | (y & ~m);
    }
}
__host__ __device__ __forceinline__ void bs_transpose32(uint32_t* a) {
#pragma unroll
    for (int k = 0; k < 16; k++) {  // halves: a[k] keeps its low half, gains a[k+16]'s low half
        const uint32_t x = a[k], y = a[k + 16];
        a[k] = bs_perm(y, x, 0x05040100u);
        a[k + 16] = bs_perm(y, x, 0x07060302u);
    }
#pragma unroll
    for (int k = 0; k < 32; k++) {  // bytes, rows k and k + 8
        if (k & 8) continue;
        const uint32_t x = a[k], y = a[k + 8];
        a[k] = bs_perm(y, x, 0x06020400u);
        a[k + 8] = bs_perm(y, x, 0x07030501u);
    }
    bs_swap_stage<4>(a);
    bs_swap_stage<2>(a);
    bs_swap_stage<1>(a);
}

// B waves on real data: a bitsliced CBC decrypt, 32 consecutive blocks per lane (512 B), from
// global memory and back: load, transpose, 10 rounds, transpose back, XOR the predecessor
// ciphertext blocks (reloaded: an L2 hit), store.  rk[0..10] the encryption round keys,
// wave-uniform (the record's).  Rounds 9..2 as pairs in a loop (two rounds of code, ~45 KB), the
// last two after it.
// STRIDED: lane l of a wave takes blocks base + l + 64 j (each load / store instruction moves one
// contiguous KiB) instead of base + 32 l + j (each lane its own 512 B)
template <bool STRIDED>
__global__ void __launch_bounds__(64) bcbc_kernel(const uint32_t* __restrict__ rk, const uint4* __restrict__ ct,
                                                  uint4* __restrict__ pt, uint64_t* __restrict__ cyc, int iters,
                                                  const uint32_t* done, uint32_t stop, uint32_t* __restrict__ iters_done) {
    const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
    const size_t b0 = STRIDED ? (size_t)blockIdx.x * 2048 + threadIdx.x : (size_t)gid * 32;
    constexpr size_t BS = STRIDED ? 64 : 1;  // block stride between a lane's blocks
    const uint4* c = ct + b0;
    uint4* o = pt + b0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    int it = 0;
    for (; it < iters; it++) {
        if (stop && __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= stop) break;
        uint32_t p[128], q[128];
        // the block addresses are loop-invariant: kept opaque per iteration, or the compiler
        // hoists all 96 of them (strided layout: 1-KiB steps, no immediate offsets) into VGPRs
        uintptr_t cb = reinterpret_cast<uintptr_t>(c), ob = reinterpret_cast<uintptr_t>(o);
        asm volatile("" : "+v"(cb), "+v"(ob));
        const uint4* c = reinterpret_cast<const uint4*>(cb);
        uint4* o = reinterpret_cast<uint4*>(ob);
        // word w of the 32 blocks XOR the last round key's word w (the transpose is linear, and
        // plane masks of a loop-invariant key would be hoisted into 128 VGPRs), then its transpose
        {
            const uint32_t* cw = reinterpret_cast<const uint32_t*>(c);
#pragma unroll
            for (int w = 0; w < 4; w++) {
#pragma unroll
                for (int j = 0; j < 32; j++) p[32 * w + j] = cw[4 * BS * j + w] ^ rk[40 + w];  // round-10 key, pre-transpose
                __builtin_amdgcn_sched_barrier(0);
                bs_transpose32(p + 32 * w);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll 1
        for (int r = 9; r >= 3; r -= 2) {
            bs_round<true>(p, q, rk + 4 * r);
            bs_round<true>(q, p, rk + 4 * (r - 1));
        }
        bs_round<true>(p, q, rk + 4);
        bs_round<false>(q, p, rk);
        __builtin_amdgcn_sched_barrier(0);  // keep the reloads below from rising into the rounds
#pragma unroll
        for (int w = 0; w < 4; w++) {
            bs_transpose32(p + 32 * w);
            __builtin_amdgcn_sched_barrier(0);  // one 32 x 32 transpose at a time (VGPRs)
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 32; j++) {
            const size_t blk = b0 + BS * j;  // predecessor block blk - 1 (block 0: a zero IV)
            const uint4 v = blk ? c[(ptrdiff_t)(BS * j) - 1] : make_uint4(0, 0, 0, 0);
            o[BS * j] = make_uint4(p[j] ^ v.x, p[32 + j] ^ v.y, p[64 + j] ^ v.z, p[96 + j] ^ v.w);
            if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // at most 8 reloads in flight
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        cyc[blockIdx.x] = t1 - t0;
        iters_done[blockIdx.x] = (uint32_t)it;
    }
}

// host reference: plain AES inverse round on bytes (InvShiftRows, InvSubBytes, AddRoundKey, InvMixColumns)
static uint8_t gm(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}
static void ref_round(uint8_t st[16], const uint32_t k[4], const uint8_t* isbox) {
    uint8_t t[16];
    for (int o = 0; o < 16; o++) t[o] = isbox[st[isr(o)]] ^ (uint8_t)(k[o >> 2] >> (8 * (o & 3)));
    for (int c = 0; c < 4; c++) {
        const uint8_t* a = t + 4 * c;
        st[4 * c + 0] = gm(a[0], 14) ^ gm(a[1], 11) ^ gm(a[2], 13) ^ gm(a[3], 9);
        st[4 * c + 1] = gm(a[0], 9) ^ gm(a[1], 14) ^ gm(a[2], 11) ^ gm(a[3], 13);
        st[4 * c + 2] = gm(a[0], 13) ^ gm(a[1], 9) ^ gm(a[2], 14) ^ gm(a[3], 11);
        st[4 * c + 3] = gm(a[0], 11) ^ gm(a[1], 13) ^ gm(a[2], 9) ^ gm(a[3], 14);
    }
}

// The two streams every mode uses.  Created once: a process gets four hardware queues
// (GPU_MAX_HW_QUEUES), and streams beyond them share queues -- two such streams serialise.
static hipStream_t sa = nullptr, sb = nullptr;
static void streams() {
    if (sa) return;
    (void)hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(t_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              AES_DEC_LDS_BYTES);
}

static std::vector<uint64_t> fetch64(const uint64_t* d, int n) {
    std::vector<uint64_t> h(n);
    (void)hipMemcpy(h.data(), d, (size_t)n * 8, hipMemcpyDeviceToHost);
    return h;
}

// t: whether the T kernel runs; bsw: B waves per CU (0: none).  Both launched back to back on two
// streams, so with both the B waves take the SIMDs' spare wave slots beside the T workgroup and
// stop when its last wave ends: their iterations are what they got during it.
static void run(const char* name, bool t, int bsw, const uint32_t* d_dk, int cus, int it_t, int it_b,
                const uint32_t* h_dk, const uint8_t* isbox, bool check) {
    streams();
    const int nt = t ? cus * 16 : 0, nb = cus * bsw;
    uint32_t *t_out = nullptr, *b_out = nullptr, *done = nullptr, *b_it = nullptr;
    uint64_t *t_cyc = nullptr, *b_cyc = nullptr;
    (void)hipMalloc(&done, 256);  // one 128-byte line per pass
    if (nt) {
        (void)hipMalloc(&t_out, (size_t)nt * 64 * 16);
        (void)hipMalloc(&t_cyc, (size_t)nt * 8);
    }
    if (nb) {
        (void)hipMalloc(&b_out, (size_t)nb * 64 * 512);
        (void)hipMalloc(&b_cyc, (size_t)nb * 8);
        (void)hipMalloc(&b_it, (size_t)nb * 4);
    }
    const uint32_t stop = (nt && nb) ? (uint32_t)nt : 0u;
    const int b_cap = stop ? 100 * it_b : it_b; // with the T kernel: until it ends (the cap a bound only)
    hipEvent_t e0, ea, eb;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&ea);
    (void)hipEventCreate(&eb);
    for (int pass = 0; pass < 2; pass++) {  // pass 0 warms up (code, tables)
        (void)hipMemset(done, 0, 256);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, sa);
        (void)hipStreamWaitEvent(sb, e0, 0);
        if (nt) hipLaunchKernelGGL(t_kernel, dim3(cus), dim3(1024), AES_DEC_LDS_BYTES, sa, d_dk, t_out, t_cyc,
                                   pass ? it_t : 2, done + 32 * pass);
        if (nb) hipLaunchKernelGGL(b_kernel, dim3(nb), dim3(64), 0, sb, d_dk, b_out, b_cyc, pass ? b_cap : 1,
                                   (const uint32_t*)(done + 32 * pass), stop, b_it);
        (void)hipEventRecord(ea, sa);
        (void)hipEventRecord(eb, sb);
        (void)hipDeviceSynchronize();
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        printf("%s: HIP error %s\n", name, hipGetErrorString(err));
        exit(1);
    }
    float ma = 0, mb = 0;
    (void)hipEventElapsedTime(&ma, e0, ea);
    (void)hipEventElapsedTime(&mb, e0, eb);
    std::vector<uint32_t> its(nb);
    if (nb) (void)hipMemcpy(its.data(), b_it, (size_t)nb * 4, hipMemcpyDeviceToHost);
    double b_iters = 0;
    for (uint32_t v : its) b_iters += v;
    const double br_t = (double)nt * 64 * it_t * NR;  // block-rounds
    const double br_b = b_iters * 64 * 32 * 2;
    // with both kernels the B work is what was done inside the T kernel's window (the B waves stop
    // at its end); otherwise each kind over its own kernel time
    const double sec_t = ma * 1e-3, sec_b = (stop ? ma : mb) * 1e-3;
    double tt = 0, tb = 0;  // mean s_memtime ticks per wave in the loop
    if (nt) for (uint64_t v : fetch64(t_cyc, nt)) tt += (double)v / nt;
    if (nb) for (uint64_t v : fetch64(b_cyc, nb)) tb += (double)v / nb;
    const double rt = nt ? br_t / sec_t / 1e9 : 0, rb = nb ? br_b / sec_b / 1e9 : 0;
    printf("%-6s T: %7.3f ms %8.0f ticks/wave %7.2f G block-rounds/s | B %2d/CU: %7.3f ms %8.0f ticks/wave "
           "%6.1f it/wave %7.2f G block-rounds/s | sum %7.2f G block-rounds/s = %6.2f GiB/s of AES-128 decrypt\n",
           name, nt ? ma : 0.f, tt, rt, bsw, nb ? (stop ? ma : mb) : 0.f, tb, nb ? b_iters / nb : 0.0, rb, rt + rb,
           (rt + rb) * 1e9 / NR * 16 / (1u << 30));
    fflush(stdout);
    if (check && nb) {  // lane 0 of B wave 0 against the host, over the iterations it did
        std::vector<uint32_t> o(128);
        (void)hipMemcpy(o.data(), b_out, 512, hipMemcpyDeviceToHost);
        uint32_t p[128], q[128];
        for (int i = 0; i < 128; i++) p[i] = (i * 0x9e3779b9u) ^ 0x5bd1e995u;
        uint8_t st[32][16];
        for (int j = 0; j < 32; j++)
            for (int by = 0; by < 16; by++) {
                uint8_t v = 0;
                for (int b = 0; b < 8; b++) v |= (uint8_t)(((p[8 * by + b] >> j) & 1u) << b);
                st[j][by] = v;
            }
        for (int it = 0; it < (int)its[0]; it++) {
            bs_round<true>(p, q, bs_key(h_dk, it, 0));
            bs_round<true>(q, p, bs_key(h_dk, it, 1));
            for (int j = 0; j < 32; j++) {
                ref_round(st[j], bs_key(h_dk, it, 0), isbox);
                ref_round(st[j], bs_key(h_dk, it, 1), isbox);
            }
        }
        bool ok_dev = true, ok_ref = true;
        for (int i = 0; i < 128; i++) ok_dev = ok_dev && o[i] == p[i];
        for (int j = 0; j < 32; j++)
            for (int by = 0; by < 16; by++)
                for (int b = 0; b < 8; b++) ok_ref = ok_ref && (((p[8 * by + b] >> j) & 1u) == ((st[j][by] >> b) & 1u));
        printf("  check (%u iterations): GPU planes == host bitsliced run: %s; host bitsliced == plain AES inverse "
               "rounds: %s\n", its[0], ok_dev ? "yes" : "NO", ok_ref ? "yes" : "NO");
        if (!ok_dev || !ok_ref) exit(1);
    }
    (void)hipFree(done);
    if (nt) { (void)hipFree(t_out); (void)hipFree(t_cyc); }
    if (nb) { (void)hipFree(b_out); (void)hipFree(b_cyc); (void)hipFree(b_it); }
}

static void ref_last(uint8_t st[16], const uint32_t k[4], const uint8_t* isbox) {
    uint8_t t[16];
    for (int o = 0; o < 16; o++) t[o] = isbox[st[isr(o)]] ^ (uint8_t)(k[o >> 2] >> (8 * (o & 3)));
    for (int o = 0; o < 16; o++) st[o] = t[o];
}
// FIPS-197 5.2 key expansion (AES-128), words little-endian (byte 0 = the key's first byte)
static void expand128(const uint8_t key[16], uint32_t rk[44], const uint8_t* sbox) {
    for (int i = 0; i < 4; i++) rk[i] = key[4 * i] | key[4 * i + 1] << 8 | key[4 * i + 2] << 16 | (uint32_t)key[4 * i + 3] << 24;
    uint8_t rc = 1;
    for (int i = 4; i < 44; i++) {
        uint32_t t = rk[i - 1];
        if (i % 4 == 0) {
            t = (t >> 8) | (t << 24);
            t = sbox[t & 255] | sbox[(t >> 8) & 255] << 8 | sbox[(t >> 16) & 255] << 16 | (uint32_t)sbox[t >> 24] << 24;
            t ^= rc;
            rc = (uint8_t)((rc << 1) ^ ((rc & 0x80) ? 0x1b : 0));
        }
        rk[i] = rk[i - 4] ^ t;
    }
}

// The bitsliced CBC decrypt on real data: alone (bsw waves per CU) or beside the T kernel.
// Checked against FIPS-197 C.1 (block 0) and a byte-wise InvCipher + CBC of two lanes' blocks.
template <bool STRIDED>
static void run_cbc(const char* name, bool t, int bsw, const uint32_t* d_dk, int cus, int it_t, int it_b,
                    const uint8_t* sbox, const uint8_t* isbox) {
    streams();
    const int nt = t ? cus * 16 : 0, nb = cus * bsw;
    const size_t nblk = (size_t)nb * 64 * 32;
    std::vector<uint8_t> h_ct(nblk * 16);
    uint32_t x = 0x12345678u;
    for (auto& b : h_ct) {
        x = x * 1664525u + 1013904223u;
        b = (uint8_t)(x >> 24);
    }
    const uint8_t key[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
    const uint8_t c1[16] = {0x69, 0xc4, 0xe0, 0xd8, 0x6a, 0x7b, 0x04, 0x30, 0xd8, 0xcd, 0xb7, 0x80, 0x70, 0xb4, 0xc5, 0x5a};
    for (int i = 0; i < 16; i++) h_ct[i] = c1[i];
    uint32_t rk[44];
    expand128(key, rk, sbox);
    uint32_t *d_rk, *t_out = nullptr, *done, *b_it;
    uint64_t *t_cyc = nullptr, *b_cyc;
    uint4 *d_ct, *d_pt;
    (void)hipMalloc(&d_rk, sizeof(rk));
    (void)hipMemcpy(d_rk, rk, sizeof(rk), hipMemcpyHostToDevice);
    (void)hipMalloc(&d_ct, nblk * 16);
    (void)hipMalloc(&d_pt, nblk * 16);
    (void)hipMemcpy(d_ct, h_ct.data(), nblk * 16, hipMemcpyHostToDevice);
    (void)hipMalloc(&done, 256);  // one 128-byte line per pass
    (void)hipMalloc(&b_it, (size_t)nb * 4);
    (void)hipMalloc(&b_cyc, (size_t)nb * 8);
    if (nt) {
        (void)hipMalloc(&t_out, (size_t)nt * 64 * 16);
        (void)hipMalloc(&t_cyc, (size_t)nt * 8);
    }
    const uint32_t stop = nt ? (uint32_t)nt : 0u;
    const int b_cap = stop ? 100 * it_b : it_b;
    hipEvent_t e0, ea, eb;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&ea);
    (void)hipEventCreate(&eb);
    for (int pass = 0; pass < 2; pass++) {
        (void)hipMemset(done, 0, 256);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, sa);
        (void)hipStreamWaitEvent(sb, e0, 0);
        if (nt) hipLaunchKernelGGL(t_kernel, dim3(cus), dim3(1024), AES_DEC_LDS_BYTES, sa, d_dk, t_out, t_cyc,
                                   pass ? it_t : 2, done + 32 * pass);
        hipLaunchKernelGGL(bcbc_kernel<STRIDED>, dim3(nb), dim3(64), 0, sb, (const uint32_t*)d_rk, (const uint4*)d_ct, d_pt,
                           b_cyc, pass ? b_cap : 1, (const uint32_t*)(done + 32 * pass), stop, b_it);
        (void)hipEventRecord(ea, sa);
        (void)hipEventRecord(eb, sb);
        (void)hipDeviceSynchronize();
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        printf("%s: HIP error %s\n", name, hipGetErrorString(err));
        exit(1);
    }
    float ma = 0, mb = 0;
    (void)hipEventElapsedTime(&ma, e0, ea);
    (void)hipEventElapsedTime(&mb, e0, eb);
    std::vector<uint32_t> its(nb);
    (void)hipMemcpy(its.data(), b_it, (size_t)nb * 4, hipMemcpyDeviceToHost);
    double b_iters = 0;
    for (uint32_t v : its) b_iters += v;
    const double sec_b = (stop ? ma : mb) * 1e-3;
    const double br_t = (double)nt * 64 * it_t * NR, br_b = b_iters * 64 * 32 * NR;
    const double rt = nt ? br_t / (ma * 1e-3) / 1e9 : 0, rb = br_b / sec_b / 1e9;
    printf("%-8s T: %7.3f ms %7.2f G block-rounds/s | CBC-B %2d/CU: %7.3f ms %6.1f it/wave %7.2f G block-rounds/s "
           "(%7.2f GiB/s decrypted, %.0f GB/s HBM) | sum %7.2f G block-rounds/s\n",
           name, nt ? ma : 0.f, rt, bsw, sec_b * 1e3, b_iters / nb, rb, br_b / NR * 16 / sec_b / (1u << 30),
           br_b / NR * 32 / sec_b / 1e9, rt + rb);
    // check two lanes (first and last) against the byte-wise InvCipher + CBC
    std::vector<uint8_t> h_pt(nblk * 16);
    (void)hipMemcpy(h_pt.data(), d_pt, nblk * 16, hipMemcpyDeviceToHost);
    bool ok = true;
    for (size_t lane : {(size_t)0, (size_t)nb * 64 - 1})
        for (size_t j = lane * 32; j < lane * 32 + 32; j++) {
            uint8_t st[16];
            for (int i = 0; i < 16; i++) st[i] = h_ct[j * 16 + i] ^ (uint8_t)(rk[40 + i / 4] >> (8 * (i % 4)));
            for (int r = 9; r >= 1; r--) ref_round(st, rk + 4 * r, isbox);
            ref_last(st, rk, isbox);
            for (int i = 0; i < 16; i++) {
                const uint8_t prev = j ? h_ct[(j - 1) * 16 + i] : 0;
                ok = ok && h_pt[j * 16 + i] == (uint8_t)(st[i] ^ prev);
            }
        }
    bool kat = true;
    for (int i = 0; i < 16; i++) kat = kat && h_pt[i] == (uint8_t)(0x11 * i);
    printf("  check: FIPS-197 C.1 block %s; lanes 0 and %zu == byte-wise InvCipher + CBC: %s\n", kat ? "ok" : "WRONG",
           (size_t)nb * 64 - 1, ok ? "yes" : "NO");
    fflush(stdout);
    if (!ok || !kat) exit(1);
    (void)hipFree(d_rk); (void)hipFree(d_ct); (void)hipFree(d_pt); (void)hipFree(done); (void)hipFree(b_it);
    (void)hipFree(b_cyc);
    if (nt) { (void)hipFree(t_out); (void)hipFree(t_cyc); }
}

int main(int argc, char** argv) {
    const int it_t = argc > 1 ? atoi(argv[1]) : 20000;  // T: blocks per lane (10 rounds each)
    const int it_b = argc > 2 ? atoi(argv[2]) : 400;   // B: iterations per lane (2 rounds x 32 blocks)
    int dev = 0, cus = 0, clk = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    uint32_t dk[4 * (NR + 1)];
    for (int i = 0; i < 4 * (NR + 1); i++) dk[i] = 0x01234567u * (i + 3) ^ (i << 20);
    uint32_t* d_dk;
    (void)hipMalloc(&d_dk, sizeof(dk));
    (void)hipMemcpy(d_dk, dk, sizeof(dk), hipMemcpyHostToDevice);
    constexpr tg::AesTables TB;
    uint8_t isbox[256], sbox[256];
    for (int e = 0; e < 256; e++) {
        isbox[e] = TB.inv_sbox[e];
        sbox[e] = TB.sbox[e];
    }
    printf("CUs %d, peak shader clock %d kHz; T: %d blocks per lane x 10 rounds, 16 waves per CU; "
           "B alone: %d x 2 rounds x 32 blocks per lane\n", cus, clk, it_t, it_b);
    run("T", true, 0, d_dk, cus, it_t, it_b, dk, isbox, false);
    run("B4", false, 4, d_dk, cus, it_t, it_b, dk, isbox, true);
    run("B8", false, 8, d_dk, cus, it_t, it_b, dk, isbox, false);
    run("B12", false, 12, d_dk, cus, it_t, it_b, dk, isbox, false);
    run("T+B4", true, 4, d_dk, cus, it_t, it_b, dk, isbox, true);
    run("T+B8", true, 8, d_dk, cus, it_t, it_b, dk, isbox, false);
    const int it_c = argc > 3 ? atoi(argv[3]) : 40;  // CBC-B alone: passes over the lane's 32 blocks
    run_cbc<false>("CBC-B4", false, 4, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<false>("CBC-B8", false, 8, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<false>("CBC-B12", false, 12, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<false>("T+CBC-B4", true, 4, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<false>("T+CBC-B8", true, 8, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<true>("CBC-S8", false, 8, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<true>("CBC-S12", false, 12, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<true>("T+CBC-S4", true, 4, d_dk, cus, it_t, it_c, sbox, isbox);
    run_cbc<true>("T+CBC-S8", true, 8, d_dk, cus, it_t, it_c, sbox, isbox);
    return 0;
}

// valu_rate_microbench.hip -- issue cost of the VALU instructions the cipher and MAC
// loops are made of (diagnostic tool): per kernel, W waves per SIMD each run 8
// independent chains of one instruction kind; reports SIMD cycles per wave-instruction
// (s_memtime over the loop, 4 SIMDs per CU).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/valu_rate_microbench.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ uint32_t dppx(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}

template <int KIND>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b, uint32_t c) {
    if constexpr (KIND == 0) return a ^ b;                                          // v_xor_b32
    if constexpr (KIND == 1) return dppx<0x39>(a) ^ b;                              // v_xor_b32 dpp quad_perm
    if constexpr (KIND == 2) return __builtin_amdgcn_perm(a, b, c);                 // v_perm_b32
    if constexpr (KIND == 3) return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);     // v_bitop3_b32
    if constexpr (KIND == 4) return a + b + c;                                      // v_add3_u32
    if constexpr (KIND == 5) return __builtin_amdgcn_alignbit(a, b, c);             // v_alignbit_b32
    if constexpr (KIND == 6) return dppx<0x141>(a) ^ b;                             // v_xor_b32 dpp row_half_mirror
    uint32_t r;
    // inline asm: exactly this instruction, nothing the compiler can fold
    if constexpr (KIND == 10) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 11) asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 12) asm volatile("v_lshlrev_b32 %0, 3, %1" : "=v"(r) : "v"(a));
    if constexpr (KIND == 13) asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    if constexpr (KIND == 15) asm volatile("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 16) asm volatile("v_bfe_u32 %0, %1, 8, 8" : "=v"(r) : "v"(a));
    if constexpr (KIND == 17) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(r) : "v"(a));
    if constexpr (KIND == 18) asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    if constexpr (KIND == 19) asm volatile("v_alignbyte_b32 %0, %1, %2, 1" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 20) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 21) asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "v"(c), "v"(a));
    if constexpr (KIND == 22) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    if constexpr (KIND == 23) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    if constexpr (KIND == 24) asm volatile("v_or3_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    if constexpr (KIND == 25) asm volatile("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    if constexpr (KIND == 26) asm volatile("v_lshrrev_b32_e32 %0, 8, %1" : "=v"(r) : "v"(a));
    if constexpr (KIND == 27) asm volatile("v_and_b32_e32 %0, 0xff00, %1" : "=v"(r) : "v"(a));
    if constexpr (KIND == 28) asm volatile("v_xor_b32_e32 %0, s8, %1" : "=v"(r) : "v"(a) : "s8");
    if constexpr (KIND == 29) asm volatile("v_bitop3_b32 %0, %1, s8, %2 bitop3:0xec" : "=v"(r) : "v"(a), "v"(c) : "s8");
    if constexpr (KIND == 30) asm volatile("v_or_b32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 31) asm volatile("v_lshlrev_b32_e32 %0, %1, %2" : "=v"(r) : "v"(c), "v"(a));
    if constexpr (KIND == 32) asm volatile("v_xor_b32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 33) asm volatile("v_and_b32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    // SDWA (VOP1/VOP2 with byte selects): a T-table address built in one op -- byte b of the
    // state word into bits 8..15 of the address register, its other bits (lane copy, table
    // select) preserved from the previous round
    if constexpr (KIND == 34) { r = a; asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(r) : "v"(b)); }
    if constexpr (KIND == 35) asm volatile("v_lshlrev_b32_sdwa %0, 8, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(a));
    if constexpr (KIND == 36) asm volatile("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND == 37) asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    if constexpr (KIND == 38) asm volatile("v_alignbit_b32 %0, %1, %1, 27" : "=v"(r) : "v"(a));
    if constexpr (KIND == 39) asm volatile("v_add_u32_e32 %0, 0x5a827999, %1" : "=v"(r) : "v"(a));
    if constexpr (KIND == 40) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(r) : "v"(a));
    if constexpr (KIND == 41) asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    if constexpr (KIND >= 10) return r;
    return 0;
}

// mixed streams: chains 0..3 run op A, chains 4..7 op B (does a 4-cycle op issue beside
// 2-cycle ops, or do their costs add?)
template <int KIND>
__device__ __forceinline__ uint32_t mixop(int i, uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    if (i < 4) {
        if constexpr (KIND == 60 || KIND == 64) asm volatile("v_alignbit_b32 %0, %1, %1, 27" : "=v"(r) : "v"(a));
        if constexpr (KIND == 61) asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
        if constexpr (KIND == 62) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
        if constexpr (KIND == 63) asm volatile("v_xor_b32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(r) : "v"(a), "v"(b));
    } else {
        if constexpr (KIND == 64) asm volatile("v_alignbit_b32 %0, %1, %1, 27" : "=v"(r) : "v"(a));
        else asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    }
    return r;
}

template <int KIND>
__global__ void __launch_bounds__(1024) rate_kernel(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) {
    uint32_t x[8];
    const uint32_t c = 0x05040302u ^ (seed & 7);
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x * 0x9E3779B9u + i;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        // x[i] from x[i ^ 4]: two dependent steps of 4 independent chains per group of 8,
        // nothing the compiler can fold
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int i = 0; i < 8; i++)
                if constexpr (KIND >= 60) x[i] = mixop<KIND>(i, x[i], x[i ^ 4], c ^ x[(i + 2) & 7]);
                else x[i] = op<KIND>(x[i], x[i ^ 4], (KIND == 3 || KIND == 13 || KIND == 14 || (KIND >= 18 && KIND != 31 && KIND < 34) || KIND == 37) ? x[(i + 2) & 7] : KIND == 31 ? (c & 7) : c);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    // every wave's start and end: the block's span is max(end) - min(start)
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 16 + threadIdx.x / 64)] = t0;
        cyc[2 * (blockIdx.x * 16 + threadIdx.x / 64) + 1] = t1;
    }
}

template <int KIND>
static void run(const char* name, int cus, int waves_per_simd, int iters) {
    const int threads = 4 * 64 * waves_per_simd;
    uint32_t* d_out;
    uint64_t* d_cyc;
    (void)hipMalloc(&d_out, (size_t)cus * threads * 4);
    (void)hipMalloc(&d_cyc, (size_t)cus * 16 * 16);
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(cus), dim3(threads), 0, 0, d_out, d_cyc, 16, 1u);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(cus), dim3(threads), 0, 0, d_out, d_cyc, iters, 1u);
    (void)hipDeviceSynchronize();
    const int waves = threads / 64;
    uint64_t st[32];
    (void)hipMemcpy(st, d_cyc, (size_t)waves * 16, hipMemcpyDeviceToHost);  // block 0
    uint64_t lo = st[0], hi = st[1];
    for (int w = 1; w < waves; w++) {
        lo = st[2 * w] < lo ? st[2 * w] : lo;
        hi = st[2 * w + 1] > hi ? st[2 * w + 1] : hi;
    }
    const uint64_t c = hi - lo;
    const double instrs_per_simd = (double)iters * 64 * waves_per_simd;  // 8 x 8 per iteration per wave
    printf("%-22s waves/SIMD %d: %5.2f cycles per wave-instruction per SIMD\n", name, waves_per_simd,
           (double)c / instrs_per_simd);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 4096;
    for (int w : {2, 4}) {
        run<26>("v_lshrrev_b32 const", cus, w, iters);
        run<27>("v_and_b32 literal", cus, w, iters);
        run<28>("v_xor_b32 sgpr", cus, w, iters);
        run<29>("v_bitop3_b32 sgpr", cus, w, iters);
        run<30>("v_or_b32", cus, w, iters);
        run<31>("v_lshlrev_b32 vgpr", cus, w, iters);
        run<32>("v_xor_b32 dpp (asm)", cus, w, iters);
        run<33>("v_and_b32", cus, w, iters);
        run<10>("v_xor_b32 (asm)", cus, w, iters);
        run<23>("v_bitop3_b32 (asm)", cus, w, iters);
        run<2>("v_perm_b32", cus, w, iters);
        run<34>("v_mov_b32_sdwa preserve", cus, w, iters);
        run<35>("v_lshlrev_b32_sdwa", cus, w, iters);
        run<36>("v_or_b32_sdwa", cus, w, iters);
        run<37>("v_perm_b32 (asm)", cus, w, iters);
        run<38>("v_alignbit_b32 (asm)", cus, w, iters);
        run<39>("v_add_u32 literal", cus, w, iters);
        run<40>("v_mov_b32_sdwa pad", cus, w, iters);
        run<41>("v_pk_add_u16", cus, w, iters);
        run<60>("mix alignbit | xor", cus, w, iters);
        run<61>("mix perm | xor", cus, w, iters);
        run<62>("mix add3 | xor", cus, w, iters);
        run<63>("mix xor_dpp | xor", cus, w, iters);
        run<64>("alignbit (mix ref)", cus, w, iters);
    }
    return 0;
}

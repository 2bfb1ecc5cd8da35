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
    return 0;
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
            for (int i = 0; i < 8; i++) x[i] = op<KIND>(x[i], x[i ^ 4], KIND == 3 ? x[(i + 2) & 7] : c);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char* name, int cus, int waves_per_simd, int iters) {
    const int threads = 4 * 64 * waves_per_simd;
    uint32_t* d_out;
    uint64_t* d_cyc;
    (void)hipMalloc(&d_out, (size_t)cus * threads * 4);
    (void)hipMalloc(&d_cyc, cus * 8);
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(cus), dim3(threads), 0, 0, d_out, d_cyc, 16, 1u);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(cus), dim3(threads), 0, 0, d_out, d_cyc, iters, 1u);
    (void)hipDeviceSynchronize();
    uint64_t c = 0;
    (void)hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
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
    for (int w : {1, 2, 4}) {
        run<0>("v_xor_b32", cus, w, iters);
        run<1>("v_xor_b32 dpp quad", cus, w, iters);
        run<6>("v_xor_b32 dpp row_half", cus, w, iters);
        run<2>("v_perm_b32", cus, w, iters);
        run<3>("v_bitop3_b32", cus, w, iters);
        run<4>("v_add3_u32", cus, w, iters);
        run<5>("v_alignbit_b32", cus, w, iters);
    }
    return 0;
}

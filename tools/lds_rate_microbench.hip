// lds_rate_microbench.hip -- the LDS read rate a CU sustains for the table-lookup shapes the
// AES kernels use, with the VALU work around each read cut to a minimum: is the ~0.75 of the
// 32-lanes-per-cycle ds_read_b32 rate that both the seal's pair round (176 vs 128 cycles per
// round, tools/aes_layout_microbench.hip) and the open's lane decrypt (0.79 vs 0.59 ms,
// tools/aes_dec_microbench.hip) reach a property of the LDS pipe itself?  (Round 5.)
//   b32      8 independent ds_read_b32 per iteration, conflict-free (copy = lane & 31, the
//            product layout), row index from a per-lane LCG (2 VALU per read)
//   b32fix   the same reads at loop-invariant addresses (no address VALU at all)
//   b64      8 ds_read_b64 per iteration, 64 banks (copy = lane & 63, 8-byte entries)
//   b128     4 ds_read_b128 per iteration
// Reports lane-reads (and bytes) per nanosecond per CU, and per shader cycle at the clock
// s_memtime / s_memrealtime report.  Diagnostic tool only.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lds_rate_microbench.hip -o tools/lds_rate_mb.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x2 lds_u64_t;
typedef __attribute__((address_space(3))) u32x4 lds_u128_t;

template <int MODE>
__global__ void __launch_bounds__(1024) rate_kernel(uint32_t* out, uint64_t* t, int iters) {
    for (uint32_t i = threadIdx.x; i < 32768; i += blockDim.x) *(lds_u32_t*)(size_t)(i * 4) = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t acc = 0, x = threadIdx.x * 7919u + 1u;
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        if constexpr (MODE == 0 || MODE == 1) {
            uint32_t v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t e = MODE == 0 ? ((x >> (3 * k)) & 255u) : ((uint32_t)k * 17u + (uint32_t)i) & 255u;
                v[k] = *(const lds_u32_t*)(size_t)(e * 256u + (lane & 31) * 4u + (k & 1) * 128u + (k & 2) * 32768u);
            }
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= v[k];
        } else if constexpr (MODE == 2) {
            u32x2 v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t e = (x >> (3 * k)) & 127u;
                v[k] = *(const lds_u64_t*)(size_t)(e * 512u + (lane & 63) * 8u + (k & 1) * 65536u);
            }
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= v[k].x ^ v[k].y;
        } else {
            u32x4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t e = (x >> (3 * k)) & 63u;
                v[k] = *(const lds_u128_t*)(size_t)(e * 1024u + (lane & 63) * 16u + (k & 1) * 65536u);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
        x = x * 1664525u + 1013904223u;  // addresses independent of the reads: throughput, not latency
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = c1 - c0;
        t[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int MODE>
static void run(const char* name, int cus, int waves, int iters) {
    auto kern = rate_kernel<MODE>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    uint32_t* d_out;
    uint64_t* d_t;
    (void)hipMalloc(&d_out, (size_t)cus * 1024 * 4);
    (void)hipMalloc(&d_t, cus * 16);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * waves), 131072, 0, d_out, d_t, 16);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * waves), 131072, 0, d_out, d_t, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t t[2];
    (void)hipMemcpy(t, d_t, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)t[0] / ((double)t[1] * 10.0);  // s_memrealtime: 100 MHz
    const int reads = MODE == 3 ? 4 : 8, bytes = MODE == 2 ? 8 : MODE == 3 ? 16 : 4;
    const double lane_reads = (double)iters * reads * 64 * waves;  // per CU
    const double per_ns = lane_reads / (ms * 1e6);
    printf("%-7s waves/CU %2d  %8.3f ms  %7.2f lane-reads/ns/CU  %7.1f B/ns/CU  (s_memtime clock %.2f GHz: "
           "%5.1f lane-reads/cycle, %5.1f B/cycle)\n",
           name, waves, ms, per_ns, per_ns * bytes, ghz, per_ns / ghz, per_ns * bytes / ghz);
    fflush(stdout);
    (void)hipFree(d_out);
    (void)hipFree(d_t);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int w : {4, 8, 16}) {
        run<0>("b32", cus, w, iters);
        run<1>("b32fix", cus, w, iters);
        run<2>("b64", cus, w, iters);
        run<3>("b128", cus, w, iters);
    }
    return 0;
}

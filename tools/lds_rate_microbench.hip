// lds_rate_microbench.hip -- how many ds_read_b32 lane-lookups per shader cycle a
// CU sustains for the AES table layouts, and what clock the chip holds meanwhile
// (s_memtime shader cycles vs s_memrealtime 100 MHz ticks).  Diagnostic tool only.
//   mode 0: copy = lane & 31 (lanes l, l+32 share a bank: the tg_device.h layout)
//   mode 1: copy = lane & 63 over 64 dwords per row (every lane its own bank)
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lds_rate_microbench.hip -o tools/lds_rate_mb.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;

template <int MODE>
__global__ void __launch_bounds__(1024) rate_kernel(uint32_t* out, uint64_t* t, int iters) {
    for (uint32_t i = threadIdx.x; i < 32768; i += blockDim.x) *(lds_u32_t*)(size_t)(i * 4) = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t off = MODE == 0 ? (lane & 31) * 4 : lane * 4;
    uint32_t acc = 0, x = threadIdx.x * 7919u;
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t e = (x >> (4 * k)) & 255u;
            v[k] = *(const lds_u32_t*)(size_t)(e * 256u + off + (MODE == 0 ? (k & 1) * 128u : 0u) + (k & 2) * 32768u);
        }
#pragma unroll
        for (int k = 0; k < 8; k++) acc ^= v[k];
        x = x * 1664525u + 1013904223u + (acc & 1u);
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = c1 - c0;
        t[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int MODE>
static void run(int cus, int threads, int iters) {
    auto kern = rate_kernel<MODE>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    uint32_t* out;
    uint64_t* t;
    (void)hipMalloc(&out, (size_t)cus * 1024 * 4);
    (void)hipMalloc(&t, (size_t)cus * 16);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), 131072, 0, out, t, 10);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), 131072, 0, out, t, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t* h = new uint64_t[2 * cus];
    (void)hipMemcpy(h, t, (size_t)cus * 16, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int i = 0; i < cus; i++) { cyc += h[2 * i]; rt += h[2 * i + 1]; }
    cyc /= cus; rt /= cus;
    const double lookups = (double)threads * iters * 8;
    printf("mode %d waves/CU %2d: %.3f ms, %.1f lane-lookups/cycle/CU, clock %.2f GHz (memtime/memrealtime), "
           "%.1f G lookups/s/CU\n", MODE, threads / 64, ms, lookups / cyc, cyc / (rt * 10.0), lookups / (ms * 1e6));
    delete[] h;
    (void)hipFree(out);
    (void)hipFree(t);
}

int main(int argc, char** argv) {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    for (int w : {4, 8, 16}) run<0>(cus, 64 * w, iters);
    for (int w : {4, 8, 16}) run<1>(cus, 64 * w, iters);
    return 0;
}

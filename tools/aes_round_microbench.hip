// aes_round_microbench.hip -- cycles per AES round of the quad layout
// (tg_aesq.h QuadAes) as a function of chains per quad (ILP) and cipher
// waves per CU, with no global-memory traffic.  Diagnostic tool only.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/aes_round_microbench.hip -o /tmp/aesmb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../tlslite_amd/csrc/tg_aesq.h"

using namespace tg;

template <int ILP>
__global__ void __launch_bounds__(1024) round_bench(uint32_t* out, int blocks, uint32_t seed) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    QuadAes aes;
    aes.init();
    uint32_t k[11];
#pragma unroll
    for (int r = 0; r < 11; r++) k[r] = seed * (r + 1) + threadIdx.x;
    uint32_t x[ILP];
#pragma unroll
    for (int i = 0; i < ILP; i++) x[i] = threadIdx.x * 2654435761u + i;
    for (int b = 0; b < blocks; b++) {
#pragma unroll
        for (int i = 0; i < ILP; i++) x[i] ^= k[0];
#pragma unroll
        for (int r = 1; r < 10; r++) {
            uint32_t y[ILP];
#pragma unroll
            for (int i = 0; i < ILP; i++) y[i] = aes.round<0>(x[i], k[r]);
#pragma unroll
            for (int i = 0; i < ILP; i++) x[i] = y[i];
        }
#pragma unroll
        for (int i = 0; i < ILP; i++) x[i] = aes.last(x[i], k[10]);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < ILP; i++) acc ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int ILP>
static void run(int waves, int blocks) {
    auto kern = round_bench<ILP>;
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    int grid = 256;
    uint32_t* out;
    hipMalloc(&out, (size_t)grid * 1024 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), 131072, 0, out, blocks, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), 131072, 0, out, blocks, 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    double rounds = (double)blocks * 10;
    double chains_per_cu = waves * 16.0 * ILP;
    double ns_per_round = ms * 1e6 / rounds;
    // chain-rounds per CU per ns -> equivalent cfg2 time for 256 chains x 10280 rounds
    double cfg2_ms = ms * (256.0 / chains_per_cu) * (10280.0 / rounds);
    printf("ILP=%d waves/CU=%2d chains/CU=%4.0f  %.1f ns/round (%.0f cyc@1.9GHz)  -> cfg2-equivalent %.3f ms\n", ILP,
           waves, chains_per_cu, ns_per_round, ns_per_round * 1.9, cfg2_ms);
    hipFree(out);
}

int main(int argc, char** argv) {
    int blocks = argc > 1 ? atoi(argv[1]) : 400;
    for (int w : {4, 8, 12, 16}) run<1>(w, blocks);
    for (int w : {4, 8, 12, 16}) run<2>(w, blocks);
    for (int w : {4, 8}) run<3>(w, blocks);
    for (int w : {4, 8}) run<4>(w, blocks);
    return 0;
}

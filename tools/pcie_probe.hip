// pcie_probe.hip -- host<->device copy rates on this box (diagnostic tool): pinned
// H2D alone, D2H alone, and both directions at once on two streams (hipMemcpyAsync,
// the engines tlsgpu_host_pipeline_seal uses), for one 1 GiB copy and for 64 MiB pieces.
//   hipcc -O3 --offload-arch=gfx950 tools/pcie_probe.hip -o pcie_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t N = (size_t)1 << 30, PIECE = (size_t)64 << 20;
    void *h1, *h2, *d1, *d2;
    CK(hipHostMalloc(&h1, N, hipHostMallocDefault));
    CK(hipHostMalloc(&h2, N, hipHostMallocDefault));
    CK(hipMalloc(&d1, N));
    CK(hipMalloc(&d2, N));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (size_t piece : {N, PIECE}) {
        for (int mode = 1; mode <= 3; mode++) {
            double best = 1e9;
            for (int rep = 0; rep < 4; rep++) {
                CK(hipDeviceSynchronize());
                const double t0 = now();
                for (size_t o = 0; o < N; o += piece) {
                    if (mode & 1) CK(hipMemcpyAsync((char*)d1 + o, (char*)h1 + o, piece, hipMemcpyHostToDevice, s1));
                    if (mode & 2) CK(hipMemcpyAsync((char*)h2 + o, (char*)d2 + o, piece, hipMemcpyDeviceToHost, s2));
                }
                CK(hipStreamSynchronize(s1));
                CK(hipStreamSynchronize(s2));
                const double dt = now() - t0;
                if (rep) best = dt < best ? dt : best;
            }
            const double bytes = (double)N * (mode == 3 ? 2 : 1);
            printf("piece %5zu MiB  %-9s %6.1f GB/s total\n", piece >> 20,
                   mode == 1 ? "H2D" : mode == 2 ? "D2H" : "H2D+D2H", bytes / best / 1e9);
        }
    }
    return 0;
}

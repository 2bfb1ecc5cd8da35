// pcie_kernel_probe.hip -- can a copy KERNEL move bytes over PCIe faster than the copy engines
// when both directions run at once?  (diagnostic for the host pipelines)
// The host pipelines' D2H copies run at ~47 GB/s beside the H2D ones (56 alone).  Here a
// kernel reads device memory and stores into pinned, device-mapped host memory (a D2H done by
// the GPU's own stores), or loads from host memory into device memory (H2D), with G
// workgroups; rates alone and beside a hipMemcpyAsync of the other direction (1 GiB each way).
//   hipcc -O3 --offload-arch=gfx950 tools/pcie_kernel_probe.hip -o tools/pcie_kernel_probe.bin
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

// NUMA node of the page holding p (move_pages with no target nodes only reports), -1 if unknown
static int numa_node_of(void* p) {
    void* pages[1] = {p};
    int status[1] = {-1};
    if (syscall(SYS_move_pages, 0, 1, pages, nullptr, status, 0) != 0) return -1;
    return status[0];
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid-stride copy of n16 16-byte words; NT: non-temporal stores
template <bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {  // four loads in flight per lane
        const u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        if constexpr (NT) {
            __builtin_nontemporal_store(a, dst + i);
            __builtin_nontemporal_store(b, dst + i + stride);
            __builtin_nontemporal_store(c, dst + i + 2 * stride);
            __builtin_nontemporal_store(d, dst + i + 3 * stride);
        } else {
            dst[i] = a;
            dst[i + stride] = b;
            dst[i + 2 * stride] = c;
            dst[i + 3 * stride] = d;
        }
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

int main(int argc, char** argv) {
    const bool quick = argc > 1 && !strcmp(argv[1], "quick");
    const size_t N = (size_t)1 << 30;
    void *h_in, *h_out, *d_in, *d_out, *hd_in, *hd_out;
    CK(hipHostMalloc(&h_in, N, hipHostMallocDefault));
    CK(hipHostMalloc(&h_out, N, hipHostMallocDefault));
    memset(h_in, 1, N);
    memset(h_out, 2, N);
    printf("process on cpu %d; h_in on NUMA node %d, h_out on node %d\n", sched_getcpu(), numa_node_of(h_in),
           numa_node_of(h_out));
    CK(hipHostGetDevicePointer(&hd_in, h_in, 0));
    CK(hipHostGetDevicePointer(&hd_out, h_out, 0));
    CK(hipMalloc(&d_in, N));
    CK(hipMalloc(&d_out, N));
    CK(hipMemset(d_in, 3, N));
    CK(hipMemset(d_out, 4, N));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    // what: bit 0 = H2D, bit 1 = D2H; kh / kd: the direction done by a kernel (else hipMemcpyAsync)
    struct Mode {
        const char* name;
        int what;
        bool kh, kd, nt;
        int grid;
    };
    Mode modes[] = {
        {"H2D sdma", 1, false, false, false, 0},         {"D2H sdma", 2, false, false, false, 0},
        {"both sdma", 3, false, false, false, 0},        {"D2H kernel g64", 2, false, true, false, 64},
        {"D2H kernel g128", 2, false, true, false, 128}, {"D2H kernel g256", 2, false, true, false, 256},
        {"D2H kernel g256 nt", 2, false, true, true, 256}, {"D2H kernel g512", 2, false, true, false, 512},
        {"H2D kernel g256", 1, true, false, false, 256}, {"H2D kernel g512", 1, true, false, false, 512},
        {"H2D sdma + D2H kernel g128", 3, false, true, false, 128},
        {"H2D sdma + D2H kernel g256", 3, false, true, false, 256},
        {"H2D sdma + D2H kernel g256 nt", 3, false, true, true, 256},
        {"H2D sdma + D2H kernel g512", 3, false, true, false, 512},
        {"H2D kernel g256 + D2H sdma", 3, true, false, false, 256},
        {"H2D kernel g256 + D2H kernel g256", 3, true, true, false, 256},
    };
    for (size_t piece : {N, (size_t)64 << 20}) {
    if (quick && piece == N) continue;
    printf("-- copies of %zu MiB\n", piece >> 20);
    for (const Mode& m : modes) {
        if (quick && strcmp(m.name, "D2H sdma") && strcmp(m.name, "both sdma") && strcmp(m.name, "D2H kernel g256") &&
            strcmp(m.name, "H2D sdma + D2H kernel g256"))
            continue;
        double best = 1e9, bh = 1e9, bd = 1e9;
        for (int rep = 0; rep < 4; rep++) {
            CK(hipDeviceSynchronize());
            hipEvent_t e0, eh, ed;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&eh));
            CK(hipEventCreate(&ed));
            const double t0 = now();
            CK(hipEventRecord(e0, s1));
            CK(hipStreamWaitEvent(s2, e0, 0));
            for (size_t o = 0; o < N; o += piece) {
                const size_t q = o / 16, pn = piece / 16;
                if (m.what & 1) {
                    if (m.kh) hipLaunchKernelGGL(copy_kernel<false>, dim3(m.grid), dim3(256), 0, s1,
                                                 (const u32x4*)hd_in + q, (u32x4*)d_in + q, pn);
                    else CK(hipMemcpyAsync((char*)d_in + o, (char*)h_in + o, piece, hipMemcpyHostToDevice, s1));
                }
                if (m.what & 2) {
                    if (m.kd) {
                        if (m.nt) hipLaunchKernelGGL(copy_kernel<true>, dim3(m.grid), dim3(256), 0, s2,
                                                     (const u32x4*)d_out + q, (u32x4*)hd_out + q, pn);
                        else hipLaunchKernelGGL(copy_kernel<false>, dim3(m.grid), dim3(256), 0, s2,
                                                (const u32x4*)d_out + q, (u32x4*)hd_out + q, pn);
                    } else {
                        CK(hipMemcpyAsync((char*)h_out + o, (char*)d_out + o, piece, hipMemcpyDeviceToHost, s2));
                    }
                }
            }
            CK(hipEventRecord(eh, s1));
            CK(hipEventRecord(ed, s2));
            CK(hipStreamSynchronize(s1));
            CK(hipStreamSynchronize(s2));
            const double dt = now() - t0;
            float mh = 0, md = 0;
            CK(hipEventElapsedTime(&mh, e0, eh));
            CK(hipEventElapsedTime(&md, e0, ed));
            if (rep) {
                best = dt < best ? dt : best;
                bh = mh < bh ? mh : bh;
                bd = md < bd ? md : bd;
            }
            CK(hipEventDestroy(e0));
            CK(hipEventDestroy(eh));
            CK(hipEventDestroy(ed));
        }
        CK(hipGetLastError());
        const double bytes = (double)N * ((m.what & 1) + ((m.what >> 1) & 1));
        printf("%-36s wall %7.2f ms  %6.1f GB/s total", m.name, best * 1e3, bytes / best / 1e9);
        if (m.what & 1) printf("  H2D %6.1f GB/s", N / (bh * 1e-3) / 1e9);
        if (m.what & 2) printf("  D2H %6.1f GB/s", N / (bd * 1e-3) / 1e9);
        printf("\n");
        fflush(stdout);
    }
    }
    // the kernel D2H moved the bytes: host buffer now holds d_out's pattern (4)
    size_t bad = 0;
    for (size_t i = 0; i < N; i += 4099) bad += ((unsigned char*)h_out)[i] != 4;
    printf("kernel D2H content check: %s\n", bad ? "WRONG" : "ok");
    return 0;
}

// traffic_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte
// counts for the access patterns of the seal kernels (diagnostic tool; run each pass as
// `rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./traffic_calib`, then WRITE_SIZE):
//   rd16     16 B per lane, a wave reads 1 KiB contiguous (streaming reference)
//   rdquad   cbc_kernel's loads: 4 lanes per record, 4 B per lane (one 16-B block per quad
//            per instruction), 16 records per wave, records of REC bytes back to back
//   wrquad   cbc_kernel's stores, same pattern
//   rdcoop   mac_kernel's cooperative loads: per instruction a quad reads 64 contiguous
//            bytes of one of its 4 records (lane q: bytes [16q, 16q+16))
//   rdstate / rdstate2 / rdstate64  scattered narrow reads of 2 KiB connection states (one lane
//            per state: a few dwords of one / two 64-B sectors, or one whole sector as dwordx4):
//            payload = 64 B per sector touched, NSTATE states (1 GiB span)
// Each kernel moves exactly BYTES (reads) or BYTES (writes) of payload once.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/traffic_calib.hip -o traffic_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr uint32_t REC = 1440;  // cfg3-like record stride (16-B aligned)
constexpr size_t NREC = 1u << 20;
constexpr size_t BYTES = NREC * REC;

__global__ void __launch_bounds__(256) rd16(const uint4* __restrict__ p, size_t n16, uint32_t* out) {
    uint32_t a = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x12345678u) out[0] = a;
}

// one quad per record, records r = quad id + k * nquads
__global__ void __launch_bounds__(1024) rdquad(const uint8_t* __restrict__ p, uint32_t* out) {
    const uint32_t q = threadIdx.x & 3;
    const size_t nq = (size_t)gridDim.x * 256;
    uint32_t a = 0;
    for (size_t r = (size_t)blockIdx.x * 256 + (threadIdx.x >> 2); r < NREC; r += nq) {
        const uint8_t* P = p + r * REC + 4 * q;
#pragma unroll 8
        for (uint32_t b = 0; b < REC / 16; b++) a = (a << 1 | a >> 31) ^ *(const uint32_t*)(P + 16 * b);
    }
    if (a == 0x12345678u) out[0] = a;
}

__global__ void __launch_bounds__(1024) wrquad(uint8_t* __restrict__ p) {
    const uint32_t q = threadIdx.x & 3;
    const size_t nq = (size_t)gridDim.x * 256;
    for (size_t r = (size_t)blockIdx.x * 256 + (threadIdx.x >> 2); r < NREC; r += nq) {
        uint8_t* P = p + r * REC + 4 * q;
#pragma unroll 8
        for (uint32_t b = 0; b < REC / 16; b++) *(uint32_t*)(P + 16 * b) = (uint32_t)(r * 131 + b);
    }
}

// one lane per record, quads cooperate: per step lane q loads 16 B of each of the quad's 4 records
__global__ void __launch_bounds__(256) rdcoop(const uint8_t* __restrict__ p, uint32_t* out) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= NREC) return;
    const uint32_t q = threadIdx.x & 3;
    const size_t r0 = r - q;
    uint32_t a = 0;
    for (uint32_t c = 0; c < REC / 64; c++)
#pragma unroll
        for (uint32_t L = 0; L < 4; L++) {
            const uint4 v = *(const uint4*)(p + (r0 + L) * REC + 64 * c + 16 * q);
            a ^= v.x + v.y + v.z + v.w + L;
        }
    if (a == 0x12345678u) out[0] = a;
}

// scattered narrow loads (prefix_kernel / cipher-kernel state reads): one lane per 2 KiB
// connection state, a few dwords of its first 64 bytes (one 64-B sector touched per lane);
// payload counted as 64 B per lane
constexpr size_t NSTATE = 1u << 19;
__global__ void __launch_bounds__(256) rdstate(const uint8_t* __restrict__ p, uint32_t* out) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= NSTATE) return;
    const uint32_t* s = (const uint32_t*)(p + r * 2048);
    const uint32_t a = s[0] ^ s[4] ^ s[6] ^ s[9] ^ s[12];
    if (a == 0x12345678u) out[0] = a;
}
// the same, two sectors per lane (bytes 0..63 and 128..191 of the state)
__global__ void __launch_bounds__(256) rdstate2(const uint8_t* __restrict__ p, uint32_t* out) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= NSTATE) return;
    const uint32_t* s = (const uint32_t*)(p + r * 2048);
    const uint32_t a = s[0] ^ s[4] ^ s[33] ^ s[40];
    if (a == 0x12345678u) out[0] = a;
}
// one full 64-B sector per lane as 4 x dwordx4 (the round keys of a state), 2 KiB apart
__global__ void __launch_bounds__(256) rdstate64(const uint8_t* __restrict__ p, uint32_t* out) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= NSTATE) return;
    const uint4* s = (const uint4*)(p + r * 2048 + 256);
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) a ^= s[i].x + s[i].y + s[i].z + s[i].w;
    if (a == 0x12345678u) out[0] = a;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint8_t* buf;
    uint32_t* out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, BYTES);
    (void)hipDeviceSynchronize();
    printf("payload per kernel: %zu bytes (%u-B records x %zu)\n", BYTES, REC, NREC);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(rd16, dim3(cus * 8), dim3(256), 0, 0, (const uint4*)buf, BYTES / 16, out);
        hipLaunchKernelGGL(rdquad, dim3(cus), dim3(1024), 0, 0, buf, out);
        hipLaunchKernelGGL(wrquad, dim3(cus), dim3(1024), 0, 0, buf);
        hipLaunchKernelGGL(rdcoop, dim3((NREC + 255) / 256), dim3(256), 0, 0, buf, out);
        hipLaunchKernelGGL(rdstate, dim3(NSTATE / 256), dim3(256), 0, 0, buf, out);
        hipLaunchKernelGGL(rdstate2, dim3(NSTATE / 256), dim3(256), 0, 0, buf, out);
        hipLaunchKernelGGL(rdstate64, dim3(NSTATE / 256), dim3(256), 0, 0, buf, out);
    }
    (void)hipDeviceSynchronize();
    printf("done\n");
    return 0;
}

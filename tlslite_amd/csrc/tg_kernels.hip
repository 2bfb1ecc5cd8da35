// tg_kernels.hip -- gfx950 kernels of libtlsgpu.so and their launchers:
//   prefix/mac/cbc_kernel, tdes4_kernel   split AES / 3DES seal (tg_aes3.h)
//   rc4_seal_kernel  fused per-record MAC -> RC4 -> header, one lane per connection
//                    chain (tlsrecordlayer.py:538-617, python_rc4.py:25-41)
//   open_*_kernel    AES / 3DES open, block-parallel (tg_open3.h); rc4_open_kernel: RC4 open, lane per chain
//   cipher_kernel    raw stateful CBC / RC4 encrypt+decrypt for the cipher-object
//                    surface (python_aes.py:20-69, python_rc4.py:25-41)
//   derive_kernel    batched _calcPendingStates (tg_derive.h)
//   fill_kernel      deterministic synthetic input (splitmix64 byte stream)
//   host_store_kernel  D2H copy by the GPU's own stores into pinned host memory (host pipelines)
// The library has exactly one kernel per (direction, suite variant): no runtime
// selection between implementations.
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <set>
#include <map>
#include <utility>
#include "tg_device.h"
#include "tg_quad.h"
#include "tg_aes3.h"
#include "tg_open3.h"
#include "tg_frame.h"
#include "tg_derive.h"
#include "tg_launch.h"
#include <hip/hip_ext.h>
#include <string>

namespace tg {

constexpr uint32_t RC4_LDS_BYTES = RC4_LDS_BYTES_PER_WAVE * (SEAL_BLOCK / 64);

// RC4 suites: one lane = one chain (a connection's ordered run of records); the
// keystream is serial per connection (python_rc4.py:30-35), so MAC and cipher run
// in the same lane.
template <int MAC, bool SSL3>
__global__ void __launch_bounds__(SEAL_BLOCK) rc4_seal_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                             const tlsgpu_record* __restrict__ recs,
                                                             const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                                                             ConnState* __restrict__ states,
                                                             int32_t* __restrict__ wire_len, uint32_t nrecords,
                                                             uint64_t pt_cap, uint64_t wire_cap, uint32_t nstates) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    const uint32_t cnt = ch.first >= nrecords ? 0u : min(ch.count, nrecords - ch.first);  // records past nrecords: ignored
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    if (ch.state >= nstates) {  // a state outside the caller's array: refused, nothing read (ABI 6)
        for (uint32_t k = 0; k < cnt; k++) wire_len[ch.first + k] = TLSGPU_EINVAL;
        return;
    }
    ConnState* st = states + ch.state;
    if (st->cipher != (uint32_t)TLSGPU_CIPHER_RC4 || st->mac != (uint32_t)MAC || st->ssl3 != (SSL3 ? 1u : 0u) ||
        st->raw) {
        for (uint32_t k = 0; k < cnt; k++) wire_len[ch.first + k] = TLSGPU_EMISMATCH;
        return;
    }
    Rc4Stream cipher;
    cipher.load(st, lds);
    uint64_t seq = st->seqnum;
    const uint32_t vmaj = st->vmaj, vmin = st->vmin;

    for (uint32_t k = 0; k < cnt; k++) {
        const tlsgpu_record R = recs[ch.first + k];
        const uint32_t n = R.pt_len;
        if (n == 0) {  // empty record: nothing sent, no seqnum consumed (tlsrecordlayer.py:551-556)
            wire_len[ch.first + k] = 0;
            continue;
        }
        const uint32_t body = n + DL;
        if (body > 0xffffu) {
            wire_len[ch.first + k] = TLSGPU_ETOOBIG;
            continue;
        }
        if (!in_arena(R.pt_off, n, pt_cap) || !in_arena(R.wire_off, 5u + body, wire_cap)) {
            wire_len[ch.first + k] = TLSGPU_EINVAL;  // outside the caller's arenas: nothing written, no seqnum
            continue;
        }
        const uint8_t* P = pt + R.pt_off;
        uint8_t* W = wire + R.wire_off;
        uint8_t* B = W + 5;

        M mac;
        mac.begin(st, seq, R.content_type, n);
        const uint32_t nfull = n >> 6;
        for (uint32_t c = 0; c < nfull; c++) {
            uint32_t cur[16];
            load64(P + 64 * c, cur);
            mac.update(cur);
            cipher.enc64(cur);
            store64(B + 64 * c, cur);
        }
        const uint32_t r = n & 63;
        uint32_t tail[16];
        load_partial(P + 64 * nfull, r, tail);
        uint32_t m[8];
        mac.finish(tail, (int)r, n, st, m);
        if (R.flags & TLSGPU_FAULT_BAD_MAC) m[0] = (m[0] & ~0xffu) | ((m[0] + 1u) & 0xffu);
        // tail stream = P[64*nfull ..) | MAC (tlsrecordlayer.py:611-613), staged in a private buffer
        uint32_t tb[32];
#pragma unroll
        for (int q = 0; q < 16; q++) tb[q] = tail[q];
#pragma unroll
        for (int q = 16; q < 32; q++) tb[q] = 0;
        uint8_t* tbb = reinterpret_cast<uint8_t*>(tb);
#pragma unroll
        for (int i = 0; i < DL; i++) tbb[r + i] = (uint8_t)(m[i >> 2] >> (8 * (i & 3)));
        uint8_t* Bt = B + 64 * nfull;
        const uint32_t T = r + DL;
        for (uint32_t p = 0; p < T; p++) Bt[p] = (uint8_t)(tbb[p] ^ cipher.R.ks());
        W[0] = R.content_type;
        W[1] = (uint8_t)vmaj;
        W[2] = (uint8_t)vmin;
        W[3] = (uint8_t)(body >> 8);
        W[4] = (uint8_t)body;
        wire_len[ch.first + k] = (int32_t)(body + 5);
        seq++;
    }
    st->seqnum = seq;
    cipher.save(st);
}

// ---------------------------------------------------------------- raw cipher object
template <int NR>
struct AesCbcDec {
    uint32_t dk[4 * (NR + 1)];
    uint32_t iv[4];
    AesLds L;
    __device__ __forceinline__ void load(const ConnState* st, const void* lds) {
        L.init(lds);
#pragma unroll
        for (int k = 0; k < 4 * (NR + 1); k++) dk[k] = st->dk[k];
#pragma unroll
        for (int k = 0; k < 4; k++) iv[k] = st->iv[k];
    }
    __device__ __forceinline__ void save(ConnState* st) {
#pragma unroll
        for (int k = 0; k < 4; k++) st->iv[k] = iv[k];
    }
    __device__ __forceinline__ void dec_block(uint32_t* d) {
        uint32_t c[4] = {d[0], d[1], d[2], d[3]};
        uint32_t s[4] = {d[0], d[1], d[2], d[3]};
        aes_decrypt<NR>(s, dk, L);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            d[k] = s[k] ^ iv[k];
            iv[k] = c[k];
        }
    }
};

template <int CIPHER, bool DEC>
__global__ void __launch_bounds__(SEAL_BLOCK) cipher_kernel(const tlsgpu_span* __restrict__ spans, uint32_t nspans,
                                                           const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                           ConnState* __restrict__ states) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr bool AES = CIPHER == TLSGPU_CIPHER_AES128 || CIPHER == TLSGPU_CIPHER_AES256 ||
                         CIPHER == TLSGPU_CIPHER_AES192;
    constexpr int NR = CIPHER == TLSGPU_CIPHER_AES256 ? 14 : CIPHER == TLSGPU_CIPHER_AES192 ? 12 : 10;
    if constexpr (AES) aes_lds_fill(lds, DEC);
    else if constexpr (CIPHER == TLSGPU_CIPHER_3DES) des_lds_fill(lds);
    __syncthreads();
    const uint32_t sid = blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= nspans) return;
    const tlsgpu_span sp = spans[sid];
    ConnState* st = states + sp.state;
    if (st->cipher != (uint32_t)CIPHER) return;
    const uint8_t* src = in + sp.off;
    uint8_t* dst = out + sp.off;
    if constexpr (AES && !DEC) {
        AesCbc<NR> c;
        c.load(st, lds);
        for (uint32_t off = 0; off + 16 <= sp.len; off += 16) {
            uint32_t d[4];
            load16(src + off, d);
            c.enc_block(d);
            store16(dst + off, d);
        }
        c.save(st);
    } else if constexpr (AES && DEC) {
        AesCbcDec<NR> c;
        c.load(st, lds);
        for (uint32_t off = 0; off + 16 <= sp.len; off += 16) {
            uint32_t d[4];
            load16(src + off, d);
            c.dec_block(d);
            store16(dst + off, d);
        }
        c.save(st);
    } else if constexpr (CIPHER == TLSGPU_CIPHER_3DES) {
        TdesCbc c;
        c.load(st, lds);
        for (uint32_t off = 0; off + 8 <= sp.len; off += 8) {
            uint32_t d[2];
            load8(src + off, d);
            if (!DEC) c.enc_block(d);
            else c.dec_block(d);
            store8(dst + off, d);
        }
        c.save(st);
    } else {
        Rc4Stream c;
        c.load(st, lds);
        for (uint32_t off = 0; off < sp.len; off++) dst[off] = (uint8_t)(src[off] ^ c.R.ks());
        c.save(st);
    }
}

// ---------------------------------------------------------------- record open (lane)
// _decryptRecord (tlsrecordlayer.py:958-1044) for the RC4 suites: the keystream is serial
// per connection (python_rc4.py:30-35), so one lane per chain decrypts (RC4 state
// carried), recomputes and compares the MAC.  The plaintext (followed by the MAC bytes)
// is written at pt + pt_off; status = plaintext length or an alert code.  With
// TLSGPU_CHAIN_STOP_ON_ALERT the chain stops at its first alert: later records get
// TLSGPU_ALERT_SKIPPED and the state stays as the failing record left it (the reference
// closes the connection there).  The CBC suites open block-parallel (tg_open3.h).
template <int MAC, bool SSL3>
__global__ void __launch_bounds__(SEAL_BLOCK) rc4_open_kernel(const tlsgpu_chain* __restrict__ chains,
                                                             uint32_t nchains,
                                                             const tlsgpu_open_record* __restrict__ recs,
                                                             const uint8_t* __restrict__ wire,
                                                             uint8_t* __restrict__ pt, ConnState* __restrict__ states,
                                                             int32_t* __restrict__ status, uint32_t nrecords,
                                                             uint64_t wire_cap, uint64_t pt_cap, uint32_t nstates) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    const uint32_t cnt = ch.first >= nrecords ? 0u : min(ch.count, nrecords - ch.first);  // records past nrecords: ignored
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    if (ch.state >= nstates) {  // a state outside the caller's array: refused, nothing read (ABI 6)
        for (uint32_t k = 0; k < cnt; k++) status[ch.first + k] = TLSGPU_EINVAL;
        return;
    }
    ConnState* st = states + ch.state;
    if (st->cipher != (uint32_t)TLSGPU_CIPHER_RC4 || st->mac != (uint32_t)MAC || st->ssl3 != (SSL3 ? 1u : 0u) ||
        st->raw) {
        for (uint32_t k = 0; k < cnt; k++) status[ch.first + k] = TLSGPU_EMISMATCH;
        return;
    }
    if (st->closed) {  // closed by an earlier alert (ConnState.closed): nothing opened, state untouched
        for (uint32_t k = 0; k < cnt; k++) status[ch.first + k] = TLSGPU_ALERT_SKIPPED;
        return;
    }
    const bool stop = (ch.flags & TLSGPU_CHAIN_STOP_ON_ALERT) != 0;
    Rc4Stream dc;
    dc.load(st, lds);
    uint64_t seq = st->seqnum;
    for (uint32_t k = 0; k < cnt; k++) {
        const tlsgpu_open_record R = recs[ch.first + k];
        const uint8_t* Cb = wire + R.ct_off;
        uint8_t* Pb = pt + R.pt_off;
        const uint32_t len = R.ct_len;
        if (!in_arena(R.ct_off, len, wire_cap) || !in_arena(R.pt_off, len, pt_cap)) {
            status[ch.first + k] = TLSGPU_EINVAL;  // outside the caller's arenas: not opened, state untouched
            continue;
        }
        bool macGood = true;
        uint32_t n = 0;
        if ((uint32_t)DL > len) {  // :1006-1007
            for (uint32_t i = 0; i < len; i++) Pb[i] = (uint8_t)(Cb[i] ^ dc.R.ks());
            macGood = false;
        } else {
            n = len - DL;
            M mac;
            mac.begin(st, seq, R.content_type, n);
            // whole 64-byte payload chunks: decrypt and MAC from the same registers (the
            // plaintext is not read back), then the last n & 63 payload bytes and the MAC
            // bytes one at a time
            const uint32_t nfull = n >> 6;
            for (uint32_t c = 0; c < nfull; c++) {
                uint32_t cur[16];
                load64(Cb + 64 * c, cur);
                dc.enc64(cur);
                store64(Pb + 64 * c, cur);
                mac.update(cur);
            }
            for (uint32_t i = 64 * nfull; i < len; i++) Pb[i] = (uint8_t)(Cb[i] ^ dc.R.ks());
            uint32_t tail[16];
            load_partial(Pb + 64 * nfull, n & 63, tail);
            uint32_t m[8];
            mac.finish(tail, (int)(n & 63), n, st, m);
            seq++;  // getSeqNumBytes (:1018) runs whenever the MAC is computed
#pragma unroll
            for (int i = 0; i < DL; i++)
                if (Pb[n + i] != (uint8_t)(m[i >> 2] >> (8 * (i & 3)))) macGood = false;
        }
        const int32_t res = macGood ? (int32_t)n : TLSGPU_ALERT_BAD_RECORD_MAC;
        status[ch.first + k] = res;
        if (stop && res < 0) {
            for (uint32_t j = k + 1; j < cnt; j++) status[ch.first + j] = TLSGPU_ALERT_SKIPPED;
            st->closed = 1u;
            break;
        }
    }
    st->seqnum = seq;
    dc.save(st);
}

// ---------------------------------------------------------------- launch plumbing
// The device a launch runs on is its stream's (hipStreamGetDevice), not the calling
// thread's current device: a caller may hold streams of several GPUs.  The null stream
// belongs to the current device.
int stream_device(hipStream_t s) {
    int dev = 0;
    if (s) {
        hipDevice_t d = 0;
        if (hipStreamGetDevice(s, &d) == hipSuccess) return (int)d;
        (void)hipGetLastError();
    }
    (void)hipGetDevice(&dev);
    return dev;
}

// hipFuncSetAttribute is per device: remember which (kernel, device) pairs have it; the
// attribute is set with the stream's device current
static hipError_t set_lds(const void* kern, uint32_t bytes, hipStream_t s) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    const int dev = stream_device(s);
    std::lock_guard<std::mutex> g(mu);
    if (done.count({kern, dev})) return hipSuccess;
    DeviceGuard guard(dev);
    hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) done.insert({kern, dev});
    return e;
}
template <class K>
static hipError_t set_lds(K kern, uint32_t bytes, hipStream_t s) {
    return set_lds(reinterpret_cast<const void*>(kern), bytes, s);
}

// CUs of the stream's device (cached per device)
static uint32_t cu_count(hipStream_t s) {
    static std::atomic<int> ncu[64];
    const int dev = stream_device(s) & 63;
    int n = ncu[dev].load(std::memory_order_relaxed);
    if (!n) {
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        n = n > 0 ? n : 256;
        ncu[dev].store(n, std::memory_order_relaxed);
    }
    return (uint32_t)n;
}

template <int MAC, bool SSL3>
static hipError_t launch_rc4_open(const tlsgpu_chain* chains, uint32_t n, const tlsgpu_open_record* recs,
                                  uint32_t nrecords, const uint8_t* wire, uint8_t* pt, ConnState* states,
                                  int32_t* status, hipStream_t s, const Bounds& b) {
    auto kern = rc4_open_kernel<MAC, SSL3>;
    hipError_t e = set_lds(kern, RC4_LDS_BYTES, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((n + SEAL_BLOCK - 1) / SEAL_BLOCK), dim3(SEAL_BLOCK), RC4_LDS_BYTES, s, chains, n, recs,
                       wire, pt, states, status, nrecords, b.wire_cap, b.pt_cap, b.nstates);
    return hipGetLastError();
}

// ---------------------------------------------------------------- synthetic input
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_kernel(uint8_t* __restrict__ p, size_t bytes, uint64_t seed, uint64_t start) {
    size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (i0 >= bytes) return;
    uint32_t d[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; b++) {
        uint64_t g = start + i0 + b;
        uint32_t v = (uint32_t)(splitmix64(seed + (g >> 3)) >> (8 * (g & 7))) & 0xffu;
        d[b >> 2] |= v << (8 * (b & 3));
    }
    if (i0 + 16 <= bytes) {
        store16(p + i0, d);
    } else {
        for (size_t b = 0; i0 + b < bytes; b++) p[i0 + b] = (uint8_t)(d[b >> 2] >> (8 * (b & 3)));
    }
}

// A device-to-host copy done by the GPU's own stores into pinned, device-mapped host memory
// (tlsgpu_host_pipeline_*: where the copy engine's D2H runs slow).  src and dst
// have the same address mod 16: byte copies up to the first 16-B boundary and after the last,
// the body in 16-B words, four loads in flight per lane (grid-stride).  Vector stores only.
__global__ void __launch_bounds__(256) host_store_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         size_t n) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    size_t head = (16 - ((uintptr_t)src & 15)) & 15;
    head = head < n ? head : n;
    const size_t body = (n - head) >> 4, tail0 = head + (body << 4);
    if (tid < head) dst[tid] = src[tid];
    if (tid < n - tail0) dst[tail0 + tid] = src[tail0 + tid];
    const uint4* __restrict__ s = reinterpret_cast<const uint4*>(src + head);
    uint4* __restrict__ d = reinterpret_cast<uint4*>(dst + head);
    size_t i = tid;
    for (; i + 3 * nth < body; i += 4 * nth) {
        const uint4 a = s[i], b = s[i + nth], c = s[i + 2 * nth], e = s[i + 3 * nth];
        d[i] = a;
        d[i + nth] = b;
        d[i + 2 * nth] = c;
        d[i + 3 * nth] = e;
    }
    for (; i < body; i += nth) d[i] = s[i];
}

hipError_t launch_host_store(const uint8_t* src, uint8_t* dst_dev, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    if (((uintptr_t)src ^ (uintptr_t)dst_dev) & 15) return hipErrorInvalidValue;
    // 128 workgroups: the probe's rate (55 GB/s) from 64 up, and few enough to sit beside the
    // seal / open kernels without taking their CUs (no LDS)
    hipLaunchKernelGGL(host_store_kernel, dim3(128), dim3(256), 0, s, src, dst_dev, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------- seal launchers
size_t seal_workspace_bytes(uint32_t nrecords) { return (size_t)nrecords * (sizeof(RecMeta) + TAIL_SLOT); }

// AES batches with more chains than one generation of 16-wave cipher workgroups: the
// many-chains configuration (the pair kernel with CFG_PAIR_GM-block groups, MAC kernel at MAC_LB_MANY)
static bool many_chains(uint32_t nchains, hipStream_t s) {
    return nchains > (uint32_t)C3_CHAINS * cu_count(s);
}

// The AES cipher phase runs 2 lanes per chain (cbc_pair_kernel) when every CU gets at
// least a full workgroup of chains (C3_CHAINS = 256: cfg2, cfg3), the quad layout
// (cbc_kernel, latency form) with fewer (cfg4's 2-16 chains per CU).
static bool pair_regime(uint32_t nchains, hipStream_t s) {
    return nchains >= (uint32_t)C3_CHAINS * cu_count(s);
}

// phase 1 (stream s1): meta memset + seqnum prefix + per-record MAC / tail / header.
// NR 0 = 3DES (8-byte blocks)
template <int NR, int MAC, bool SSL3>
static hipError_t launch_mac_phase(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                   uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states,
                                   int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s,
                                   const Bounds& sb) {
    constexpr int CID = NR == 10 ? TLSGPU_CIPHER_AES128 : NR == 14 ? TLSGPU_CIPHER_AES256 : TLSGPU_CIPHER_3DES;
    constexpr int BS = NR == 0 ? 8 : 16;
    RecMeta* meta = reinterpret_cast<RecMeta*>(ws);
    uint8_t* tails = ws + (size_t)nrecords * sizeof(RecMeta);
    // the records this launch's chains use (a host-pipeline sub-batch: its own window)
    const uint32_t r1 = sb.rec_hi < nrecords ? sb.rec_hi : nrecords;
    const uint32_t r0 = sb.rec_lo < r1 ? sb.rec_lo : r1;
    if (r1 == r0) return hipSuccess;
    hipError_t e = hipMemsetAsync(meta + r0, 0, (size_t)(r1 - r0) * sizeof(RecMeta), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((prefix_kernel<CID, MAC, SSL3>), dim3((nchains + 255) / 256), dim3(256), 0, s, chains, nchains,
                       recs, states, wire_len, meta, nrecords, epoch, sb.pt_cap, sb.wire_cap, sb.nstates);
    const dim3 grid((r1 - r0 + 255) / 256);
    const bool mac_many = NR != 0 && many_chains(nchains, s);
    // (many chains: two 128-VGPR MAC waves per SIMD fit beside the cipher waves; beside the
    // two 88-VGPR pair waves the 168-VGPR kernel would fit two too -- measured the same on
    // cfg3, profiles/r03/ab_mac.txt)
    if (mac_many)
        hipLaunchKernelGGL((mac_kernel<MAC, SSL3, BS, MAC_LB_MANY, MAC_PF_MANY>), grid, dim3(256), CFG_MAC_MANY_LDS, s,
                           recs, r1, pt, wire, states, wire_len, meta, tails, epoch, r0);
    else
        hipLaunchKernelGGL((mac_kernel<MAC, SSL3, BS>), grid, dim3(256), 0, s, recs, r1, pt, wire, states, wire_len,
                           meta, tails, epoch, r0);
    return hipGetLastError();
}

// phase 2 (stream s2, after phase 1): CBC over [explicit IV | P blocks | tail]
// A cipher-phase kernel launch; with both events given, the events are those of the kernel's own
// dispatch (hipExtLaunchKernelGGL: start and end of the kernel itself, no event packets of their
// own on the stream between kernels -- the bench's sampled kernel times)
template <typename K, typename... A>
static void launch_timed(K kern, dim3 grid, dim3 block, uint32_t shm, hipStream_t s, hipEvent_t t0, hipEvent_t t1,
                         A... args) {
    if (t0 && t1) {
        hipExtLaunchKernelGGL(kern, grid, block, shm, s, t0, t1, 0, args...);
        return;
    }
    if (t0) (void)hipEventRecord(t0, s);  // one event alone: a record of its own on the stream
    hipLaunchKernelGGL(kern, grid, block, shm, s, args...);
    if (t1) (void)hipEventRecord(t1, s);
}

template <int NR>
static hipError_t launch_cbc_phase(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                   uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states,
                                   uint8_t* ws, uint32_t epoch, hipStream_t s, uint32_t nstates,
                                   hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr) {
    const uint32_t ncu = cu_count(s);
    RecMeta* meta = reinterpret_cast<RecMeta*>(ws);
    uint8_t* tails = ws + (size_t)nrecords * sizeof(RecMeta);
    if constexpr (NR == 0) {  // 3DES: 4 lanes per chain
        uint32_t pw = (nchains + ncu - 1) / ncu;
        pw = pw < 1 ? 1 : (pw > (uint32_t)D4_CHAINS ? (uint32_t)D4_CHAINS : pw);
        hipError_t e = set_lds(tdes4_kernel, D4_LDS_BYTES, s);
        if (e != hipSuccess) return e;
        launch_timed(tdes4_kernel, dim3((nchains + pw - 1) / pw), dim3(D4_THREADS), D4_LDS_BYTES, s, t0, t1, chains,
                     nchains, recs, nrecords, pt, wire, states, meta, tails, pw, epoch, nstates);
        return hipGetLastError();
    } else {
        const bool many = many_chains(nchains, s);
        if (pair_regime(nchains, s)) {
            // a CU gets at least a workgroup's worth of chains: 2 lanes per chain
            const uint32_t waves = many ? PAIR_WAVES_MANY : PAIR_WAVES;
            const uint32_t pwg = 32u * waves;
            uint32_t cpw = (nchains + ncu - 1) / ncu;
            cpw = cpw > pwg ? pwg : cpw;
            auto kern = many ? cbc_pair_kernel<NR, PAIR_WAVES_MANY, CFG_PAIR_GM>
                             : cbc_pair_kernel<NR, PAIR_WAVES, CFG_PAIR_G1>;
            hipError_t e = set_lds(kern, AES_LDS_BYTES, s);
            if (e != hipSuccess) return e;
            uint32_t grid = (nchains + cpw - 1) / cpw;
            grid = grid > ncu ? ncu : grid;
            launch_timed(kern, dim3(grid), dim3(64 * waves), AES_LDS_BYTES, s, t0, t1, chains, nchains, recs,
                         nrecords, pt, wire, states, meta, tails, cpw, epoch, nstates);
            return hipGetLastError();
        }
        // fewer chains than the pair regime's (so at most one generation of C3_CHAINS per CU)
        uint32_t cpw = (nchains + ncu - 1) / ncu;
        cpw = cpw < 1 ? 1 : (cpw > (uint32_t)C3_CHAINS ? (uint32_t)C3_CHAINS : cpw);
        // fewer chains than a workgroup's quads: the latency form of the AES round
        auto kern = cpw < (uint32_t)C3_CHAINS ? cbc_kernel<NR, true> : cbc_kernel<NR, false>;
        hipError_t e = set_lds(kern, AES_LDS_BYTES, s);
        if (e != hipSuccess) return e;
        // persistent: at most one workgroup per CU, quads loop over chain generations
        uint32_t grid = (nchains + cpw - 1) / cpw;
        grid = grid > ncu ? ncu : grid;
        launch_timed(kern, dim3(grid), dim3(C3_THREADS), AES_LDS_BYTES, s, t0, t1, chains,
                     nchains, recs, nrecords, pt, wire, states, meta, tails, cpw, epoch, nstates);
        return hipGetLastError();
    }
}

// The cipher-phase kernel launch_cbc_phase / launch_seal picks for a call of nchains
// chains on the current device, as rocprofv3 names it (bench.py's dominant kernel).
std::string seal_cipher_kernel(uint32_t variant, uint32_t nchains) {
    const uint32_t c = variant & 0xff;
    if (c == TLSGPU_CIPHER_RC4) return "rc4_seal_kernel";
    if (c == TLSGPU_CIPHER_3DES) return "tdes4_kernel";
    if (c != TLSGPU_CIPHER_AES128 && c != TLSGPU_CIPHER_AES256) return "";
    const int nr = c == TLSGPU_CIPHER_AES128 ? 10 : 14;
    const uint32_t ncu = cu_count(nullptr);
    const bool many = many_chains(nchains, nullptr);
    char b[64];
    if (pair_regime(nchains, nullptr)) {
        snprintf(b, sizeof b, "cbc_pair_kernel<%d, %d, %d>", nr, many ? PAIR_WAVES_MANY : PAIR_WAVES,
                 many ? CFG_PAIR_GM : CFG_PAIR_G1);
        return b;
    }
    const uint32_t cpw = (nchains + ncu - 1) / ncu;
    snprintf(b, sizeof b, "cbc_kernel<%d, %s>", nr, cpw < (uint32_t)C3_CHAINS ? "true" : "false");
    return b;
}

// The (cipher, MAC, SSL3) variants of the split seal path (AES and 3DES suites)
#define TG_SPLIT_VARIANTS(X)                             \
    X(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, false)   \
    X(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, false)   \
    X(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA256, false) \
    X(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA256, false) \
    X(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, true)    \
    X(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, true)    \
    X(TLSGPU_CIPHER_3DES, 0, TLSGPU_MAC_SHA1, false)      \
    X(TLSGPU_CIPHER_3DES, 0, TLSGPU_MAC_SHA1, true)

// Split seal with the two phases on two streams (pipeline API; s1 == s2 for one stream).
hipError_t launch_seal_phases(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                              const tlsgpu_record* recs, uint32_t nrecords, const uint8_t* pt, uint8_t* wire,
                              ConnState* states, int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s1,
                              hipEvent_t mac_done, hipStream_t s2, hipEvent_t cbc_start, hipEvent_t cbc_stop,
                              bool* known, const Bounds& sb) {
    *known = true;
    hipError_t e = hipSuccess;
#define TG_PH(CID, NR, MAC_ID, SSL3)                                                                            \
    if (variant == TLSGPU_VARIANT(CID, MAC_ID, SSL3)) {                                                          \
        e = launch_mac_phase<NR, MAC_ID, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, ws,   \
                                               epoch, s1, sb);                                                   \
        if (e != hipSuccess) return e;                                                                           \
        if (s2 != s1) {                                                                                          \
            if ((e = hipEventRecord(mac_done, s1)) != hipSuccess) return e;                                      \
            if ((e = hipStreamWaitEvent(s2, mac_done, 0)) != hipSuccess) return e;                               \
        }                                                                                                        \
        return launch_cbc_phase<NR>(chains, nchains, recs, nrecords, pt, wire, states, ws, epoch, s2, sb.nstates, \
                                    cbc_start, cbc_stop);                                                        \
    }
    TG_SPLIT_VARIANTS(TG_PH)
#undef TG_PH
    *known = false;
    return hipSuccess;
}

template <int MAC, bool SSL3>
static hipError_t launch_rc4_seal(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                  uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states,
                                  int32_t* wire_len, hipStream_t s, const Bounds& b) {
    auto kern = rc4_seal_kernel<MAC, SSL3>;
    hipError_t e = set_lds(kern, RC4_LDS_BYTES, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((nchains + SEAL_BLOCK - 1) / SEAL_BLOCK), dim3(SEAL_BLOCK), RC4_LDS_BYTES, s, chains,
                       nchains, recs, pt, wire, states, wire_len, nrecords, b.pt_cap, b.wire_cap, b.nstates);
    return hipGetLastError();
}

bool seal_needs_workspace(uint32_t variant) {
    const uint32_t c = variant & 0xff;
    return c == TLSGPU_CIPHER_AES128 || c == TLSGPU_CIPHER_AES256 || c == TLSGPU_CIPHER_3DES;
}

hipError_t launch_seal(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                       uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states, int32_t* wire_len,
                       uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known, const Bounds& b) {
    if (seal_needs_workspace(variant))
        return launch_seal_phases(variant, chains, nchains, recs, nrecords, pt, wire, states, wire_len, ws, epoch, s,
                                  nullptr, s, nullptr, nullptr, known, b);
    *known = true;
#define TG_RC4_CASE(MAC_ID, SSL3)                       \
    if (variant == TLSGPU_VARIANT(TLSGPU_CIPHER_RC4, MAC_ID, SSL3)) \
        return launch_rc4_seal<MAC_ID, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, s, b);
    TG_RC4_CASE(TLSGPU_MAC_SHA1, false)
    TG_RC4_CASE(TLSGPU_MAC_MD5, false)
    TG_RC4_CASE(TLSGPU_MAC_SHA1, true)
    TG_RC4_CASE(TLSGPU_MAC_MD5, true)
#undef TG_RC4_CASE
    *known = false;
    return hipSuccess;
}

template <int CIPHER, bool DEC>
static hipError_t launch_cipher_t(const tlsgpu_span* spans, uint32_t n, const uint8_t* in, uint8_t* out,
                                  ConnState* states, hipStream_t s) {
    auto kern = cipher_kernel<CIPHER, DEC>;
    constexpr bool AES = CIPHER == TLSGPU_CIPHER_AES128 || CIPHER == TLSGPU_CIPHER_AES256 ||
                         CIPHER == TLSGPU_CIPHER_AES192;
    constexpr uint32_t lds = AES ? (DEC ? AES_DEC_LDS_BYTES : AES_LDS_BYTES)
                                 : CIPHER == TLSGPU_CIPHER_3DES ? DES_LDS_BYTES : RC4_LDS_BYTES;
    hipError_t e = set_lds(kern, lds, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((n + SEAL_BLOCK - 1) / SEAL_BLOCK), dim3(SEAL_BLOCK), lds, s, spans, n, in, out,
                       states);
    return hipGetLastError();
}

hipError_t launch_cipher(int cipher, int dec, const tlsgpu_span* spans, uint32_t n, const uint8_t* in, uint8_t* out,
                         ConnState* states, hipStream_t s, bool* known) {
    *known = true;
#define TG_CIPHER_CASE(ID)                                                                     \
    if (cipher == ID)                                                                          \
        return dec ? launch_cipher_t<ID, true>(spans, n, in, out, states, s)                   \
                   : launch_cipher_t<ID, false>(spans, n, in, out, states, s);
    TG_CIPHER_CASE(TLSGPU_CIPHER_AES128)
    TG_CIPHER_CASE(TLSGPU_CIPHER_AES256)
    TG_CIPHER_CASE(TLSGPU_CIPHER_AES192)
    TG_CIPHER_CASE(TLSGPU_CIPHER_3DES)
    TG_CIPHER_CASE(TLSGPU_CIPHER_RC4)
#undef TG_CIPHER_CASE
    *known = false;
    return hipSuccess;
}

hipError_t launch_derive(const tlsgpu_derive_desc* descs, uint32_t n, ConnState* ws, ConnState* rs,
                         uint8_t* master_out, uint8_t* kb_out, int32_t* status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(derive_kernel, dim3((n + 63) / 64), dim3(64), 0, s, descs, n, ws, rs, master_out, kb_out,
                       status);
    return hipGetLastError();
}

hipError_t launch_fill(uint8_t* p, size_t bytes, uint64_t seed, uint64_t start, hipStream_t s) {
    size_t threads = (bytes + 15) / 16;
    dim3 grid((unsigned)((threads + 255) / 256));
    if (threads == 0) return hipSuccess;
    hipLaunchKernelGGL(fill_kernel, grid, dim3(256), 0, s, p, bytes, seed, start);
    return hipGetLastError();
}

// ---------------------------------------------------------------- open launchers
// per record: the OpenMeta, and the MAC's hash state between block-range parts
size_t open_workspace_bytes(uint32_t nrecords) { return (size_t)nrecords * (sizeof(OpenMeta) + sizeof(OpenMacState)); }

// CBC suites (every AES variant: SHA1 TLS/SSL3, SHA256 TLS 1.2; 3DES-SHA) open block-parallel
static bool open_split_variant(uint32_t v) {
    const uint32_t c = v & 0xff;
    return c == TLSGPU_CIPHER_AES128 || c == TLSGPU_CIPHER_AES256 || c == TLSGPU_CIPHER_3DES;
}
bool open_needs_workspace(uint32_t variant) { return open_split_variant(variant); }

// The second stream of a split open (launch_open_split): one per (device, priority), at a
// priority other than the caller's stream so the two never share a hardware queue (a shared
// queue runs its kernels in submission order: no overlap), with the events
// that order the parts.  Enqueueing holds the mutex: calls from several host threads
// serialise their (microsecond) enqueue, and the events are reused only under it.  Limits
// (tlsgpu.h): split opens issued on different caller streams of one priority share this
// stream, so their decrypt passes run one after another; and a caller stream under HIP graph
// capture pulls it into the capture.  tlsgpu_release_workspaces() destroys them.
constexpr int OPEN_PARTS = 4;
struct OpenAux {
    hipStream_t s2 = nullptr;
    hipEvent_t pre_done = nullptr;
    hipEvent_t dec_done[OPEN_PARTS] = {};
};
static std::mutex open_aux_mu;
static std::map<std::pair<int, int>, OpenAux> open_aux_map;
static hipError_t open_aux(hipStream_t s, OpenAux** out) {
    const int dev = stream_device(s);
    int least = 0, greatest = 0, p = 0;
    DeviceGuard guard(dev);
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    if ((e = hipStreamGetPriority(s, &p)) != hipSuccess) return e;
    const int prio = p == greatest ? least : greatest;
    OpenAux& a = open_aux_map[{dev, prio}];
    if (!a.s2) {
        if ((e = hipStreamCreateWithPriority(&a.s2, hipStreamNonBlocking, prio)) != hipSuccess) return e;
        for (auto& ev : a.dec_done)
            if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
        if ((e = hipEventCreateWithFlags(&a.pre_done, hipEventDisableTiming)) != hipSuccess) return e;
    }
    *out = &a;
    return hipSuccess;
}

// the split open's library streams and events (tlsgpu_release_workspaces): each stream is
// drained first; every entry is dropped even when a call fails (the first error is returned)
hipError_t release_open_aux() {
    std::lock_guard<std::mutex> g(open_aux_mu);
    hipError_t first = hipSuccess;
    auto keep = [&first](hipError_t e) {
        if (e != hipSuccess && first == hipSuccess) first = e;
    };
    for (auto& kv : open_aux_map) {
        DeviceGuard guard(kv.first.first);
        OpenAux& a = kv.second;
        if (a.s2) {
            keep(hipStreamSynchronize(a.s2));
            keep(hipStreamDestroy(a.s2));
        }
        for (auto& ev : a.dec_done)
            if (ev) keep(hipEventDestroy(ev));
        if (a.pre_done) keep(hipEventDestroy(a.pre_done));
    }
    open_aux_map.clear();
    return first;
}

size_t open_aux_count() {
    std::lock_guard<std::mutex> g(open_aux_mu);
    return open_aux_map.size();
}

// How an open is split (tlsgpu_set_open_parts: tests force each form on small batches).
//   chain-range parts: large batches of short chains (cfg3: 1 Mi records of one record per
//     connection) -- OPEN_PARTS ranges of chains, each part's decrypt + padding pass on the
//     second stream, its MAC pass on the caller's stream beside the next part's decrypt.
//   block-range parts (3DES suites): every record's tail blocks (the padding) first, then
//     OPEN_PARTS block ranges of every record on the second stream, the MAC of the payload
//     decrypted so far beside the next range's decrypt, its hash state kept in the
//     workspace; the last MAC pass finishes.  The 3DES decrypt (48 Feistel rounds of 8 SP
//     lookups per 8-byte block) leaves the SIMDs' VALU issue to the MAC beside it: cfg5 open
//     310-314 vs 268-272 GiB/s in one pass (profiles/r05/ab_open.txt).
// (For AES, round 5 measured the block-range parts slower than one pass on cfg2 (741-745 vs 783-789 GiB/s with the round-5 decrypt;
// cfg3 230 vs 374-402): every pass re-enters every record, and the part MACs, latency-bound
// at one wave per SIMD, slowed the decrypt beside them.  Removed; commit 2a0577e has them.
// Round 5 then fused the two: 12 decrypt waves and 4 MAC waves per workgroup, the MAC hashing
// each 64-block stripe of 256 records as soon as the decrypt waves publish it.  Its timeline
// (profiles/r05/trace_open_fused.txt) shows every stripe's decrypt slowed by the full MAC time
// beside it -- the two share the SIMDs' issue, so overlapping them saves nothing: cfg2
// 675-684 vs 781-806 GiB/s.  Removed; commit ce9d3c2 has it.)
enum { OPEN_SPLIT_AUTO = 0, OPEN_SPLIT_CHAINS = 1, OPEN_SPLIT_NONE = 2, OPEN_SPLIT_BLOCKS = 3 };
static std::atomic<int> open_split_mode{OPEN_SPLIT_AUTO};
static std::atomic<long long> open_split_min{-1};
int set_open_parts(int mode, long long min_records) {
    if (mode < OPEN_SPLIT_AUTO || mode > OPEN_SPLIT_BLOCKS) return -1;
    open_split_mode.store(mode, std::memory_order_relaxed);
    open_split_min.store(min_records < 0 ? -1 : min_records, std::memory_order_relaxed);
    return 0;
}

// NR 0 = 3DES (8-byte blocks, open_tdes_kernel).  Passes: prefix (caller's stream), then the
// decrypt / padding / MAC passes (in chain-range parts, or all once on the caller's stream),
// then the stop pass.
template <int NR, int MAC, bool SSL3>
static hipError_t launch_open_split(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_open_record* recs,
                                    uint32_t nrecords, const uint8_t* wire, uint8_t* pt, ConnState* states,
                                    int32_t* status, uint8_t* ws, uint32_t epoch, hipStream_t s, const Bounds& b) {
    constexpr int CID = NR == 10 ? TLSGPU_CIPHER_AES128 : NR == 14 ? TLSGPU_CIPHER_AES256 : TLSGPU_CIPHER_3DES;
    constexpr int BS = NR == 0 ? 8 : 16;
    OpenMeta* meta = reinterpret_cast<OpenMeta*>(ws);
    OpenMacState* ms = reinterpret_cast<OpenMacState*>(ws + (size_t)nrecords * sizeof(OpenMeta));
    hipError_t e = hipMemsetAsync(meta, 0, (size_t)nrecords * sizeof(OpenMeta), s);
    if (e != hipSuccess) return e;
    const dim3 gc((nchains + 255) / 256), gr((nrecords + 255) / 256);
    hipLaunchKernelGGL((open_prefix_kernel<CID, MAC, SSL3>), gc, dim3(256), 0, s, chains, nchains, recs, nrecords,
                       wire, states, status, meta, epoch, b.wire_cap, b.pt_cap, b.nstates);
    constexpr uint32_t WPB = (NR == 0 ? OT_THREADS : O3_THREADS) / 64;  // records per decrypt workgroup step
    const uint32_t ncu = cu_count(s);
    if (NR == 0) {
        if ((e = set_lds(open_tdes_kernel, DES_LDS_BYTES, s)) != hipSuccess) return e;
    } else {
        if ((e = set_lds(open_aes_kernel<NR == 0 ? 10 : NR>, AES_DEC_LDS_BYTES, s)) != hipSuccess) return e;
    }
    // the decrypt (persistent: at most one workgroup per CU) of chains [c0, c1)
    // (3DES: blocks of block-range part `part` of `nparts`, every block when part < 0)
    auto dec = [&](uint32_t c0, uint32_t c1, uint32_t nrec_part, hipStream_t s, int part = -1, int nparts = 0) {
        uint32_t grid = (nrec_part + WPB - 1) / WPB;
        grid = grid > ncu ? ncu : (grid ? grid : 1u);
        if constexpr (NR == 0)
            hipLaunchKernelGGL(open_tdes_kernel, dim3(grid), dim3(OT_THREADS), DES_LDS_BYTES, s, recs, nrecords, wire,
                               pt, states, meta, epoch, c0, c1, part, nparts);
        else
            hipLaunchKernelGGL(open_aes_kernel<NR == 0 ? 10 : NR>, dim3(grid), dim3(O3_THREADS), AES_DEC_LDS_BYTES, s,
                               recs, nrecords, wire, pt, states, meta, epoch, c0, c1);
    };
    auto seq = [&](uint32_t c0, uint32_t c1, hipStream_t s) {
        hipLaunchKernelGGL((open_seq_kernel<MAC, SSL3>), dim3((c1 - c0 + 255) / 256), dim3(256), 0, s, chains, nchains,
                           recs, nrecords, pt, states, status, meta, epoch, c0, c1, b.nstates);
    };
    // At most one wave of records per CU (the receive pipeline's sub-batches): the MAC is
    // latency-bound -- cooperative loads, and one wave per workgroup so the waves spread over
    // as many CUs as there are waves (four 256-lane workgroups put a 1,024-record batch on 4
    // CUs, where the concurrent sub-batches' MAC and framing kernels land too: 1.4 ms in the
    // pipeline against 0.35 ms alone, tools/open_mac_probe.py)
    const bool coop = nrecords <= (uint32_t)CFG_OPEN_MAC_COOP_PER_CU * ncu;
    auto mac = [&](uint32_t c0, uint32_t c1, hipStream_t s, int part = -1, int nparts = 0) {
        if (coop)
            hipLaunchKernelGGL((open_mac_kernel<MAC, SSL3, BS, true>), dim3((nrecords + 63) / 64), dim3(64), 0, s, recs,
                               nrecords, pt, states, status, meta, ms, epoch, c0, c1, part, nparts);
        else
            hipLaunchKernelGGL((open_mac_kernel<MAC, SSL3, BS, false>), gr, dim3(256), 0, s, recs, nrecords, pt,
                               states, status, meta, ms, epoch, c0, c1, part, nparts);
    };
    // Chain-range parts only when each part's MAC pass alone holds two waves per SIMD (one lane
    // per record: with fewer records a part's MAC takes as long as the whole batch's, and four
    // in a row lose -- cfg2: 535-543 vs 733 GiB/s; cfg3, 1 Mi records: 452 vs 402), and only for
    // short chains (<= 4 records per chain on average: a part's padding pass walks each chain's
    // records one dependent load after another -- cfg4 587-591 vs 668).
    const int mode_set = open_split_mode.load(std::memory_order_relaxed);
    const long long min_set = open_split_min.load(std::memory_order_relaxed);
    // Block-range parts (3DES only) when the batch's MAC passes hold at least two waves per CU.
    int mode = OPEN_SPLIT_NONE;
    const uint64_t min_rec = (uint64_t)(min_set < 0 ? 0 : min_set);
    if (mode_set == OPEN_SPLIT_AUTO) {
        if (nchains >= (uint32_t)OPEN_PARTS && nrecords >= (uint64_t)OPEN_PARTS * 512u * ncu &&
            nrecords <= 4ull * nchains)
            mode = OPEN_SPLIT_CHAINS;
        else if (NR == 0 && nrecords >= 128u * ncu)
            mode = OPEN_SPLIT_BLOCKS;
    } else if (mode_set == OPEN_SPLIT_CHAINS) {
        if (nchains >= (uint32_t)OPEN_PARTS && nrecords >= min_rec) mode = OPEN_SPLIT_CHAINS;
    } else if (mode_set == OPEN_SPLIT_BLOCKS) {
        if (NR == 0 && nrecords >= min_rec) mode = OPEN_SPLIT_BLOCKS;
    }
    if (mode == OPEN_SPLIT_NONE) {
        dec(0, nchains, nrecords, s);
        seq(0, nchains, s);
        mac(0u, nchains, s);
    } else if (mode == OPEN_SPLIT_BLOCKS) {
        std::lock_guard<std::mutex> g(open_aux_mu);
        OpenAux* a = nullptr;
        if ((e = open_aux(s, &a)) != hipSuccess) return e;
        if ((e = hipEventRecord(a->pre_done, s)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(a->s2, a->pre_done, 0)) != hipSuccess) return e;
        // tail blocks + padding pass, then block range h of every record beside the MAC of the
        // payload that ranges < h produced; the last MAC pass hashes the rest and compares
        dec(0, nchains, nrecords, a->s2, OPEN_PARTS, OPEN_PARTS);
        seq(0, nchains, a->s2);
        for (int h = 0; h < OPEN_PARTS; h++) {
            dec(0, nchains, nrecords, a->s2, h, OPEN_PARTS);
            if ((e = hipEventRecord(a->dec_done[h], a->s2)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(s, a->dec_done[h], 0)) != hipSuccess) return e;
            mac(0u, nchains, s, h, OPEN_PARTS);
        }
        mac(0u, nchains, s, OPEN_PARTS, OPEN_PARTS);
    } else {
        std::lock_guard<std::mutex> g(open_aux_mu);
        OpenAux* a = nullptr;
        if ((e = open_aux(s, &a)) != hipSuccess) return e;
        // the decrypt + padding passes on the second stream, the MAC passes on the caller's: the
        // second stream is the high-priority one whenever the caller's is not, and the decrypt's
        // workgroups (all of a CU's LDS, 4 waves per SIMD) then get the CUs first as the MAC
        // waves leave (cfg3 469 vs 454 GiB/s with the MAC passes on the second stream)
        if ((e = hipEventRecord(a->pre_done, s)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(a->s2, a->pre_done, 0)) != hipSuccess) return e;
        for (int h = 0; h < OPEN_PARTS; h++) {
            const uint32_t c0 = (uint32_t)((uint64_t)nchains * h / OPEN_PARTS);
            const uint32_t c1 = (uint32_t)((uint64_t)nchains * (h + 1) / OPEN_PARTS);
            dec(c0, c1, nrecords / OPEN_PARTS, a->s2);
            seq(c0, c1, a->s2);
            if ((e = hipEventRecord(a->dec_done[h], a->s2)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(s, a->dec_done[h], 0)) != hipSuccess) return e;
            mac(c0, c1, s);
        }
    }
    hipLaunchKernelGGL(open_stop_kernel, gc, dim3(256), 0, s, chains, nchains, recs, nrecords, wire, states, status,
                       meta, epoch, b.nstates);
    return hipGetLastError();
}

hipError_t launch_open(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                       const tlsgpu_open_record* recs, uint32_t nrecords, const uint8_t* wire, uint8_t* pt,
                       ConnState* states, int32_t* status, uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known,
                       const Bounds& b) {
    *known = true;
#define TG_OPEN3(CID, NR, MAC_ID, SSL3)                                                                         \
    if (variant == TLSGPU_VARIANT(CID, MAC_ID, SSL3))                                                           \
        return launch_open_split<NR, MAC_ID, SSL3>(chains, nchains, recs, nrecords, wire, pt, states, status, ws, \
                                                    epoch, s, b);
    TG_OPEN3(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, false)
    TG_OPEN3(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, false)
    TG_OPEN3(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA256, false)
    TG_OPEN3(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA256, false)
    TG_OPEN3(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, true)
    TG_OPEN3(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, true)
    TG_OPEN3(TLSGPU_CIPHER_3DES, 0, TLSGPU_MAC_SHA1, false)
    TG_OPEN3(TLSGPU_CIPHER_3DES, 0, TLSGPU_MAC_SHA1, true)
#undef TG_OPEN3
#define TG_OPEN_RC4(MAC_ID, SSL3)                                      \
    if (variant == TLSGPU_VARIANT(TLSGPU_CIPHER_RC4, MAC_ID, SSL3)) \
        return launch_rc4_open<MAC_ID, SSL3>(chains, nchains, recs, nrecords, wire, pt, states, status, s, b);
    TG_OPEN_RC4(TLSGPU_MAC_SHA1, false)
    TG_OPEN_RC4(TLSGPU_MAC_MD5, false)
    TG_OPEN_RC4(TLSGPU_MAC_SHA1, true)
    TG_OPEN_RC4(TLSGPU_MAC_MD5, true)
#undef TG_OPEN_RC4
    *known = false;
    return hipSuccess;
}


// ---------------------------------------------------------------- receive framing
// per connection its record count (uint32), then per block of connections its 64-bit sum
size_t frame_workspace_bytes(uint32_t n) {
    return (((size_t)n * 4 + 7) & ~(size_t)7) + (size_t)((n + FRAME_BLOCK - 1) / FRAME_BLOCK) * 8 + 16;
}
hipError_t launch_frame(const uint8_t* stream, uint64_t cap, const tlsgpu_span* conns, uint32_t n,
                        tlsgpu_open_record* recs, uint32_t max_records, tlsgpu_chain* chains, uint32_t chain_flags,
                        uint32_t* consumed, int32_t* status, uint32_t* total, uint8_t* ws, hipStream_t s) {
    const uint32_t nb = (n + FRAME_BLOCK - 1) / FRAME_BLOCK;
    uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
    uint64_t* bsum = reinterpret_cast<uint64_t*>(ws + (((size_t)n * 4 + 7) & ~(size_t)7));
    hipLaunchKernelGGL(frame_count_kernel, dim3(nb), dim3(FRAME_BLOCK), 0, s, stream, cap, conns, n, counts, bsum);
    hipLaunchKernelGGL(frame_scan_kernel, dim3(1), dim3(1024), 0, s, bsum, nb, total, max_records);
    hipLaunchKernelGGL(frame_write_kernel, dim3(nb), dim3(FRAME_BLOCK), 0, s, stream, cap, conns, n, counts, bsum,
                       recs, max_records, chains, chain_flags, consumed, status);
    return hipGetLastError();
}

}  // namespace tg


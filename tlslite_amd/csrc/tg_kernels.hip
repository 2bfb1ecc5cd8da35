// tg_kernels.hip -- gfx950 kernels of libtlsgpu.so:
//   seal_kernel    fused per-record  MAC -> pad -> CBC/RC4 encrypt -> header,
//                  one lane per connection chain (tlsrecordlayer.py:538-617)
//   cipher_kernel  raw stateful CBC / RC4 encrypt+decrypt for the
//                  cipher-object surface (python_aes.py:20-69, python_rc4.py:25-41)
//   fill_kernel    deterministic synthetic input (splitmix64 byte stream)
#include <stdlib.h>
#include <string.h>
#include "tg_device.h"
#include "tg_aesq.h"
#include "tg_aes3.h"
#include "tg_open3.h"
#include "tg_derive.h"
#include "tg_launch.h"

namespace tg {

template <class C>
struct CipherTraits;
template <>
struct CipherTraits<AesCbc<10>> {
    static constexpr int ID = TLSGPU_CIPHER_AES128;
    static constexpr uint32_t LDS = AES_LDS_BYTES;
};
template <>
struct CipherTraits<AesCbc<14>> {
    static constexpr int ID = TLSGPU_CIPHER_AES256;
    static constexpr uint32_t LDS = AES_LDS_BYTES;
};
template <>
struct CipherTraits<TdesCbc> {
    static constexpr int ID = TLSGPU_CIPHER_3DES;
    static constexpr uint32_t LDS = DES_LDS_BYTES;
};
template <>
struct CipherTraits<Rc4Stream> {
    static constexpr int ID = TLSGPU_CIPHER_RC4;
    static constexpr uint32_t LDS = RC4_LDS_BYTES_PER_WAVE * (SEAL_BLOCK / 64);
};

template <class C>
__device__ __forceinline__ void fill_tables(uint32_t* lds) {
    if constexpr (CipherTraits<C>::ID == TLSGPU_CIPHER_AES128 || CipherTraits<C>::ID == TLSGPU_CIPHER_AES256)
        aes_lds_fill(lds, false);
    else if constexpr (CipherTraits<C>::ID == TLSGPU_CIPHER_3DES)
        des_lds_fill(lds);
}

// One lane = one chain (a connection's ordered run of records).
template <class C, int MAC, bool SSL3>
__global__ void __launch_bounds__(SEAL_BLOCK) seal_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                         const tlsgpu_record* __restrict__ recs,
                                                         const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                                                         ConnState* __restrict__ states,
                                                         int32_t* __restrict__ wire_len) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    fill_tables<C>(lds);
    __syncthreads();

    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    ConnState* st = states + ch.state;
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    constexpr int BS = C::BS;

    if (st->cipher != (uint32_t)CipherTraits<C>::ID || st->mac != (uint32_t)MAC || st->ssl3 != (SSL3 ? 1u : 0u) ||
        st->raw) {
        for (uint32_t k = 0; k < ch.count; k++) wire_len[ch.first + k] = TLSGPU_EMISMATCH;
        return;
    }
    C cipher;
    cipher.load(st, lds);
    uint64_t seq = st->seqnum;
    const uint32_t E = (!C::STREAM && st->explicit_iv) ? (uint32_t)BS : 0u;
    const uint32_t vmaj = st->vmaj, vmin = st->vmin;

    for (uint32_t k = 0; k < ch.count; k++) {
        const tlsgpu_record R = recs[ch.first + k];
        const uint32_t n = R.pt_len;
        if (n == 0) {  // empty record: nothing sent, no seqnum consumed (tlsrecordlayer.py:551-556)
            wire_len[ch.first + k] = 0;
            continue;
        }
        uint32_t body;
        if (C::STREAM) {
            body = n + DL;
        } else {
            uint32_t cur = E + n + DL;
            body = cur + (BS - (cur % BS));  // pad = BS-1-(cur%BS), plus the length byte
        }
        if (body > 0xffffu) {
            wire_len[ch.first + k] = TLSGPU_ETOOBIG;
            continue;
        }
        const uint8_t* P = pt + R.pt_off;
        uint8_t* W = wire + R.wire_off;
        uint8_t* B = W + 5;

        M mac;
        mac.begin(st, seq, R.content_type, n);
        if (!C::STREAM && E) {  // TLS>=1.1: fixedIVBlock encrypted with the chained residue
            uint32_t blk[4] = {st->fixed_iv[0], st->fixed_iv[1], st->fixed_iv[2], st->fixed_iv[3]};
            if constexpr (!C::STREAM) {
                cipher.enc_block(blk);
                cipher.store_block(B, blk);
            }
        }
        const uint32_t nfull = n >> 6;
        uint8_t* Bp = B + E;
        for (uint32_t c = 0; c < nfull; c++) {
            uint32_t cur[16];
            load64(P + 64 * c, cur);
            mac.update(cur);
            cipher.enc64(cur);
            store64(Bp + 64 * c, cur);
        }
        const uint32_t r = n & 63;
        uint32_t tail[16];
        load_partial(P + 64 * nfull, r, tail);
        uint32_t m[8];
        mac.finish(tail, (int)r, n, st, m);
        if (R.flags & TLSGPU_FAULT_BAD_MAC) m[0] = (m[0] & ~0xffu) | ((m[0] + 1u) & 0xffu);

        // tail stream = P[64*nfull ..) | MAC | pad, staged in a private buffer
        uint32_t tb[32];
#pragma unroll
        for (int q = 0; q < 16; q++) tb[q] = tail[q];
#pragma unroll
        for (int q = 16; q < 32; q++) tb[q] = 0;
        uint8_t* tbb = reinterpret_cast<uint8_t*>(tb);
#pragma unroll
        for (int i = 0; i < DL; i++) tbb[r + i] = (uint8_t)(m[i >> 2] >> (8 * (i & 3)));
        uint8_t* Bt = Bp + 64 * nfull;
        if constexpr (!C::STREAM) {
            const uint32_t padl = BS - 1 - ((r + DL) % BS);
            for (uint32_t i = 0; i <= padl; i++) tbb[r + DL + i] = (uint8_t)padl;
            if (R.flags & TLSGPU_FAULT_BAD_PADDING) tbb[r + DL] = (uint8_t)(padl + 1);
            const uint32_t T = r + DL + padl + 1;
            for (uint32_t off = 0; off < T; off += BS) {
                uint32_t blk[4];
#pragma unroll
                for (int q = 0; q < BS / 4; q++) blk[q] = tb[(off >> 2) + q];
                cipher.enc_block(blk);
                cipher.store_block(Bt + off, blk);
            }
        } else {
            const uint32_t T = r + DL;
            for (uint32_t p = 0; p < T; p++) Bt[p] = (uint8_t)(tbb[p] ^ cipher.R.ks());
        }
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
            if (!DEC) {
                c.enc_block(d);
            } else {
                uint32_t c0 = d[0], c1 = d[1];
                uint32_t hi = bswap32(d[0]), lo = bswap32(d[1]);
                tdes_block<true>(hi, lo, c.ks, c.L);
                d[0] = bswap32(hi) ^ c.iv[0];
                d[1] = bswap32(lo) ^ c.iv[1];
                c.iv[0] = c0;
                c.iv[1] = c1;
            }
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

// ---------------------------------------------------------------- record open
// _decryptRecord (tlsrecordlayer.py:958-1044): decrypt (CBC residue / RC4
// state carried), strip the TLS>=1.1 explicit IV, check padding, recompute and
// compare the MAC.  One lane per chain; the plaintext (followed by the MAC
// and padding bytes) is written at pt + pt_off.  status = plaintext length or
// an alert code.  Two passes over the record: decrypt+store, then verify by
// re-reading the lane's own stores.
template <int NR>
struct AesDecAdapter {
    static constexpr int BS = 16;
    AesCbcDec<NR> c;
    __device__ __forceinline__ void load(const ConnState* st, const void* lds) { c.load(st, lds); }
    __device__ __forceinline__ void save(ConnState* st) { c.save(st); }
    __device__ __forceinline__ void dec_block(uint32_t* d) { c.dec_block(d); }
};
struct TdesDecAdapter {
    static constexpr int BS = 8;
    TdesCbc c;
    __device__ __forceinline__ void load(const ConnState* st, const void* lds) { c.load(st, lds); }
    __device__ __forceinline__ void save(ConnState* st) { c.save(st); }
    __device__ __forceinline__ void dec_block(uint32_t* d) {
        uint32_t c0 = d[0], c1 = d[1];
        uint32_t hi = bswap32(d[0]), lo = bswap32(d[1]);
        tdes_block<true>(hi, lo, c.ks, c.L);
        d[0] = bswap32(hi) ^ c.iv[0];
        d[1] = bswap32(lo) ^ c.iv[1];
        c.iv[0] = c0;
        c.iv[1] = c1;
    }
};

template <int CIPHER>
struct OpenTraits;
template <> struct OpenTraits<TLSGPU_CIPHER_AES128> { using D = AesDecAdapter<10>; static constexpr uint32_t LDS = AES_DEC_LDS_BYTES; };
template <> struct OpenTraits<TLSGPU_CIPHER_AES256> { using D = AesDecAdapter<14>; static constexpr uint32_t LDS = AES_DEC_LDS_BYTES; };
template <> struct OpenTraits<TLSGPU_CIPHER_3DES> { using D = TdesDecAdapter; static constexpr uint32_t LDS = DES_LDS_BYTES; };
template <> struct OpenTraits<TLSGPU_CIPHER_RC4> { using D = Rc4Stream; static constexpr uint32_t LDS = RC4_LDS_BYTES_PER_WAVE * (SEAL_BLOCK / 64); };

template <int CIPHER, int MAC, bool SSL3>
__global__ void __launch_bounds__(SEAL_BLOCK) open_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                         const tlsgpu_open_record* __restrict__ recs,
                                                         const uint8_t* __restrict__ wire, uint8_t* __restrict__ pt,
                                                         ConnState* __restrict__ states,
                                                         int32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr bool AES = CIPHER == TLSGPU_CIPHER_AES128 || CIPHER == TLSGPU_CIPHER_AES256;
    constexpr bool STREAM = CIPHER == TLSGPU_CIPHER_RC4;
    if constexpr (AES) aes_lds_fill(lds, true);
    else if constexpr (CIPHER == TLSGPU_CIPHER_3DES) des_lds_fill(lds);
    __syncthreads();
    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    ConnState* st = states + ch.state;
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    if (st->cipher != (uint32_t)CIPHER || st->mac != (uint32_t)MAC || st->ssl3 != (SSL3 ? 1u : 0u) || st->raw) {
        for (uint32_t k = 0; k < ch.count; k++) status[ch.first + k] = TLSGPU_EMISMATCH;
        return;
    }
    typename OpenTraits<CIPHER>::D dc;
    dc.load(st, lds);
    uint64_t seq = st->seqnum;
    for (uint32_t k = 0; k < ch.count; k++) {
        const tlsgpu_open_record R = recs[ch.first + k];
        const uint8_t* Cb = wire + R.ct_off;
        uint8_t* Pb = pt + R.pt_off;
        const uint32_t L = R.ct_len;
        uint32_t len, totalPad = 0;
        bool padGood = true;
        if constexpr (!STREAM) {
            constexpr uint32_t BS = OpenTraits<CIPHER>::D::BS;
            const uint32_t E = st->explicit_iv ? BS : 0u;
            if (L % BS) {  // :964-968
                status[ch.first + k] = TLSGPU_ALERT_DECRYPTION_FAILED;
                continue;
            }
            for (uint32_t off = 0; off < L; off += BS) {
                uint32_t d[4];
                if (BS == 16) load16(Cb + off, d); else load8(Cb + off, d);
                dc.dec_block(d);
                if (off >= E) {
                    if (BS == 16) store16(Pb + off - E, d); else store8(Pb + off - E, d);
                }
            }
            len = L > E ? L - E : 0u;  // :970-971 (b[E:] of a shorter b is empty)
            if (len == 0) {  // :973-977
                status[ch.first + k] = TLSGPU_ALERT_DECRYPTION_FAILED;
                continue;
            }
            const uint32_t pl = Pb[len - 1];
            if (pl + 1 > len) {  // :981-983
                padGood = false;
            } else {
                totalPad = pl + 1;
                if (!SSL3) {  // TLS: every padding byte must equal the length (:986-993)
                    for (uint32_t i = len - totalPad; i < len - 1; i++)
                        if (Pb[i] != pl) padGood = false;
                    if (!padGood) totalPad = 0;
                }
            }
        } else {
            for (uint32_t i = 0; i < L; i++) Pb[i] = (uint8_t)(Cb[i] ^ dc.R.ks());
            len = L;
        }
        bool macGood = true;
        const uint32_t endLen = DL + totalPad;
        uint32_t n = 0;
        if (endLen > len) {  // :1006-1007
            macGood = false;
        } else {
            n = len - endLen;
            M mac;
            mac.begin(st, seq, R.content_type, n);
            const uint32_t nfull = n >> 6;
            for (uint32_t c = 0; c < nfull; c++) {
                uint32_t cur[16];
                load64(Pb + 64 * c, cur);
                mac.update(cur);
            }
            uint32_t tail[16];
            load_partial(Pb + 64 * nfull, n & 63, tail);
            uint32_t m[8];
            mac.finish(tail, (int)(n & 63), n, st, m);
            seq++;  // getSeqNumBytes (:1018) runs whenever the MAC is computed
#pragma unroll
            for (int i = 0; i < DL; i++)
                if (Pb[n + i] != (uint8_t)(m[i >> 2] >> (8 * (i & 3)))) macGood = false;
        }
        status[ch.first + k] = (padGood && macGood) ? (int32_t)n : TLSGPU_ALERT_BAD_RECORD_MAC;
    }
    st->seqnum = seq;
    dc.save(st);
}

template <int CIPHER, int MAC, bool SSL3>
static hipError_t launch_open_t(const tlsgpu_chain* chains, uint32_t n, const tlsgpu_open_record* recs,
                                const uint8_t* wire, uint8_t* pt, ConnState* states, int32_t* status, hipStream_t s) {
    auto kern = open_kernel<CIPHER, MAC, SSL3>;
    constexpr uint32_t lds = OpenTraits<CIPHER>::LDS;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    dim3 grid((n + SEAL_BLOCK - 1) / SEAL_BLOCK);
    hipLaunchKernelGGL(kern, grid, dim3(SEAL_BLOCK), lds, s, chains, n, recs, wire, pt, states, status);
    return hipGetLastError();
}

static hipError_t launch_open_lane(uint32_t variant, const tlsgpu_chain* chains, uint32_t n,
                                   const tlsgpu_open_record* recs, const uint8_t* wire, uint8_t* pt,
                                   ConnState* states, int32_t* status, hipStream_t s, bool* known) {
    *known = true;
#define TG_OPEN_CASE(CIPHER_ID, MAC_ID, SSL3)                                                  \
    if (variant == TLSGPU_VARIANT(CIPHER_ID, MAC_ID, SSL3))                                    \
        return launch_open_t<CIPHER_ID, MAC_ID, SSL3>(chains, n, recs, wire, pt, states, status, s);
    TG_OPEN_CASE(TLSGPU_CIPHER_AES128, TLSGPU_MAC_SHA1, false)
    TG_OPEN_CASE(TLSGPU_CIPHER_AES256, TLSGPU_MAC_SHA1, false)
    TG_OPEN_CASE(TLSGPU_CIPHER_AES128, TLSGPU_MAC_SHA256, false)
    TG_OPEN_CASE(TLSGPU_CIPHER_AES256, TLSGPU_MAC_SHA256, false)
    TG_OPEN_CASE(TLSGPU_CIPHER_3DES, TLSGPU_MAC_SHA1, false)
    TG_OPEN_CASE(TLSGPU_CIPHER_RC4, TLSGPU_MAC_SHA1, false)
    TG_OPEN_CASE(TLSGPU_CIPHER_RC4, TLSGPU_MAC_MD5, false)
    TG_OPEN_CASE(TLSGPU_CIPHER_AES128, TLSGPU_MAC_SHA1, true)
    TG_OPEN_CASE(TLSGPU_CIPHER_AES256, TLSGPU_MAC_SHA1, true)
    TG_OPEN_CASE(TLSGPU_CIPHER_3DES, TLSGPU_MAC_SHA1, true)
    TG_OPEN_CASE(TLSGPU_CIPHER_RC4, TLSGPU_MAC_SHA1, true)
    TG_OPEN_CASE(TLSGPU_CIPHER_RC4, TLSGPU_MAC_MD5, true)
#undef TG_OPEN_CASE
    *known = false;
    return hipSuccess;
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

// ---------------------------------------------------------------- launchers
template <class K>
static hipError_t set_lds(K kern, uint32_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

// AES implementation: 0 = split (prefix/mac/cbc, default), 1 = fused quad
// kernel (TLSGPU_SEAL_IMPL=fused), 2 = one lane per chain (=lane).  A/B only.
static int aes_impl() {  // TLSGPU_SEAL_IMPL, read per launch: split (default) / fused / lane
    const char* e = getenv("TLSGPU_SEAL_IMPL");
    return (e && e[0] == 'f') ? 1 : (e && e[0] == 'l') ? 2 : 0;
}
static uint32_t debug_skip_flags() {
    static uint32_t skip = 0xffffffffu;
    if (skip == 0xffffffffu) {  // TLSGPU_DEBUG_SKIP: 1 = no CBC bulk, 2 = no MAC bulk, bits 4-7 wave priorities, bits 12-13 CBC probes (tg_aes3.h); timing experiments only
        const char* e = getenv("TLSGPU_DEBUG_SKIP");
        skip = e ? (uint32_t)atoi(e) : 0u;
    }
    return skip;
}
// A/B switches for the seal kernels' memory paths, read per launch (tests flip them):
// TLSGPU_MAC_LOAD=quad -> mac_kernel<.., QL> (quad-cooperative loads), TLSGPU_CBC_IO=16 ->
// cbc_kernel<NR, IO16> (16-byte I/O).  Defaults (measured faster on cfg2):
// per-lane MAC loads, column-word CBC I/O.
static bool env_is(const char* name, char c0) {
    const char* e = getenv(name);
    return e && e[0] == c0;
}
static int cu_count() {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (ncu <= 0) ncu = 256;
    }
    return ncu;
}

size_t seal_workspace_bytes(uint32_t nrecords) { return (size_t)nrecords * (sizeof(RecMeta) + TAIL_SLOT); }

// phase 1 (stream s1): meta memset + seqnum prefix + per-record MAC / tail / header
template <int NR, int MAC, bool SSL3>
static hipError_t launch_mac_phase(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                   uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states,
                                   int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s) {
    // NR 0 = 3DES (8-byte blocks)
    constexpr int CID = NR == 10 ? TLSGPU_CIPHER_AES128 : NR == 14 ? TLSGPU_CIPHER_AES256 : TLSGPU_CIPHER_3DES;
    constexpr int BS = NR == 0 ? 8 : 16;
    RecMeta* meta = reinterpret_cast<RecMeta*>(ws);
    uint8_t* tails = ws + (size_t)nrecords * sizeof(RecMeta);
    hipError_t e = hipMemsetAsync(meta, 0, (size_t)nrecords * sizeof(RecMeta), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((prefix_kernel<CID, MAC, SSL3>), dim3((nchains + 255) / 256), dim3(256), 0, s, chains, nchains,
                       recs, states, wire_len, meta, nrecords, epoch);
    auto mk = (BS == 16 && env_is("TLSGPU_MAC_LOAD", 'q')) ? mac_kernel<MAC, SSL3, true, BS>
                                                           : mac_kernel<MAC, SSL3, false, BS>;
    hipLaunchKernelGGL(mk, dim3((nrecords + 255) / 256), dim3(256), 0, s, recs, nrecords, pt, wire, states, wire_len,
                       meta, tails, epoch, debug_skip_flags());
    return hipGetLastError();
}

// phase 2 (stream s2, after phase 1): CBC over [explicit IV | P blocks | tail]
template <int NR>
static hipError_t launch_cbc_phase(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                   uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states,
                                   uint8_t* ws, uint32_t epoch, hipStream_t s, int cus = 0) {
    // cus > 0: the stream is CU-masked to that many CUs (pipeline with TLSGPU_PIPE_MAC_CUS)
    const uint32_t ncu = cus > 0 ? (uint32_t)cus : (uint32_t)cu_count();
    RecMeta* meta = reinterpret_cast<RecMeta*>(ws);
    uint8_t* tails = ws + (size_t)nrecords * sizeof(RecMeta);
    if constexpr (NR == 0) {  // 3DES: 8 lanes per chain
        uint32_t pw = (nchains + ncu - 1) / ncu;
        pw = pw < 1 ? 1 : (pw > (uint32_t)D8_CHAINS ? (uint32_t)D8_CHAINS : pw);
        static bool attrd = false;
        if (!attrd) {
            hipError_t e = set_lds(tdes8_kernel, DES_LDS_BYTES);
            if (e != hipSuccess) return e;
            attrd = true;
        }
        hipLaunchKernelGGL(tdes8_kernel, dim3((nchains + pw - 1) / pw), dim3(D8_THREADS), DES_LDS_BYTES, s, chains,
                           nchains, recs, nrecords, pt, wire, states, meta, tails, pw, epoch);
        return hipGetLastError();
    } else {
        // TLSGPU_CBC_ILP (read per launch): 1 = cbc_kernel (16 waves, 1 chain per quad), 2 = cbc2_kernel
        // (8 waves, 2 chains per quad)
        const char* ilp_env = getenv("TLSGPU_CBC_ILP");
        const int ilp = (ilp_env && atoi(ilp_env) == 2) ? 2 : 1;
        // TLSGPU_CBC_LAYOUT (read per launch): "pair" = cbcp_kernel (2 lanes per chain, up to 512
        // chains per CU; A/B only: 5 % slower on cfg2, 8 % on cfg3, same box), otherwise the quad
        // layout cbc_kernel / cbc2_kernel (4 lanes per chain)
        const char* lay_env = getenv("TLSGPU_CBC_LAYOUT");
        // on a CU-masked stream (cus > 0) more than 256 chains per CU need the pair layout (one
        // workgroup generation); on the whole chip extra chains run as further generations
        const bool quad = (!(lay_env && lay_env[0] == 'p') || ilp == 2 || env_is("TLSGPU_CBC_IO", '1')) &&
                          (cus <= 0 || (nchains + ncu - 1) / ncu <= (uint32_t)C3_CHAINS);
        if (!quad) {
            uint32_t pw = (nchains + ncu - 1) / ncu;
            pw = pw < 1 ? 1 : (pw > (uint32_t)CP_CHAINS ? (uint32_t)CP_CHAINS : pw);
            auto kern = cbcp_kernel<NR>;
            static bool attrp = false;
            if (!attrp) {
                hipError_t e = set_lds(kern, AES_LDS_BYTES);
                if (e != hipSuccess) return e;
                attrp = true;
            }
            hipLaunchKernelGGL(kern, dim3((nchains + pw - 1) / pw), dim3(CP_THREADS), AES_LDS_BYTES, s, chains, nchains,
                               recs, nrecords, pt, wire, states, meta, tails, pw, epoch, debug_skip_flags());
            return hipGetLastError();
        }
        uint32_t cpw = (nchains + ncu - 1) / ncu;
        cpw = cpw < 1 ? 1 : (cpw > (uint32_t)C3_CHAINS ? (uint32_t)C3_CHAINS : cpw);
        if (ilp == 2) {
            auto kern = cbc2_kernel<NR>;
            static bool attr2 = false;
            if (!attr2) {
                hipError_t e = set_lds(kern, AES_LDS_BYTES);
                if (e != hipSuccess) return e;
                attr2 = true;
            }
            hipLaunchKernelGGL(kern, dim3((nchains + cpw - 1) / cpw), dim3(C2_THREADS), AES_LDS_BYTES, s, chains, nchains,
                               recs, nrecords, pt, wire, states, meta, tails, cpw, epoch, debug_skip_flags());
            return hipGetLastError();
        }
        const bool io16 = env_is("TLSGPU_CBC_IO", '1');
        auto kern = io16 ? cbc_kernel<NR, true> : cbc_kernel<NR, false>;
        static bool attr[2] = {false, false};
        if (!attr[io16]) {
            hipError_t e = set_lds(kern, AES_LDS_BYTES);
            if (e != hipSuccess) return e;
            attr[io16] = true;
        }
        // persistent: at most one workgroup per CU, quads loop over chain generations
        uint32_t grid = (nchains + cpw - 1) / cpw;
        grid = grid > ncu ? ncu : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(C3_THREADS), AES_LDS_BYTES, s, chains, nchains, recs, nrecords, pt,
                           wire, states, meta, tails, cpw, epoch, debug_skip_flags());
        return hipGetLastError();
    }
}

template <int NR, int MAC, bool SSL3>
static hipError_t launch_seal_split(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                    uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states,
                                    int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s) {
    hipError_t e = launch_mac_phase<NR, MAC, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, ws,
                                                   epoch, s);
    if (e != hipSuccess) return e;
    return launch_cbc_phase<NR>(chains, nchains, recs, nrecords, pt, wire, states, ws, epoch, s);
}

// Split AES seal with the two phases on two streams (pipeline API).
hipError_t launch_seal_phases(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                              const tlsgpu_record* recs, uint32_t nrecords, const uint8_t* pt, uint8_t* wire,
                              ConnState* states, int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s1,
                              hipEvent_t mac_done, hipStream_t s2, hipEvent_t cbc_start, hipEvent_t cbc_stop,
                              bool* known, int cbc_cus) {
    *known = true;
    hipError_t e = hipSuccess;
#define TG_PH(CID, NR, MAC_ID, SSL3)                                                                            \
    if (variant == TLSGPU_VARIANT(CID, MAC_ID, SSL3)) {                                                          \
        e = launch_mac_phase<NR, MAC_ID, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, ws,   \
                                               epoch, s1);                                                       \
        if (e != hipSuccess) return e;                                                                           \
        if ((e = hipEventRecord(mac_done, s1)) != hipSuccess) return e;                                          \
        if ((e = hipStreamWaitEvent(s2, mac_done, 0)) != hipSuccess) return e;                                   \
        if (cbc_start && (e = hipEventRecord(cbc_start, s2)) != hipSuccess) return e;                           \
        e = launch_cbc_phase<NR>(chains, nchains, recs, nrecords, pt, wire, states, ws, epoch, s2, cbc_cus);     \
        if (e == hipSuccess && cbc_stop) e = hipEventRecord(cbc_stop, s2);                                       \
        return e;                                                                                                \
    }
    TG_PH(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, false)
    TG_PH(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, false)
    TG_PH(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA256, false)
    TG_PH(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA256, false)
    TG_PH(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, true)
    TG_PH(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, true)
    TG_PH(TLSGPU_CIPHER_3DES, 0, TLSGPU_MAC_SHA1, false)
    TG_PH(TLSGPU_CIPHER_3DES, 0, TLSGPU_MAC_SHA1, true)
#undef TG_PH
    *known = false;
    return hipSuccess;
}

template <int NR, int MAC, bool SSL3>
static hipError_t launch_seal_aesq(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                   const uint8_t* pt, uint8_t* wire, ConnState* states, int32_t* wire_len,
                                   hipStream_t s) {
    auto kern = seal_aesq_kernel<NR, MAC, SSL3>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = set_lds(kern, Q_LDS_BYTES);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const uint32_t ncu = (uint32_t)cu_count();
    uint32_t cpw = (nchains + ncu - 1) / ncu;
    cpw = cpw < 1 ? 1 : (cpw > (uint32_t)Q_CHAINS ? (uint32_t)Q_CHAINS : cpw);
    dim3 grid((nchains + cpw - 1) / cpw);
    const uint32_t skip = debug_skip_flags();
    hipLaunchKernelGGL(kern, grid, dim3(Q_THREADS), Q_LDS_BYTES, s, chains, nchains, recs, pt, wire, states, wire_len,
                       cpw, skip);
    return hipGetLastError();
}

template <class C, int MAC, bool SSL3>
static hipError_t launch_seal_t(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                                uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states,
                                int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s) {
    if constexpr (CipherTraits<C>::ID == TLSGPU_CIPHER_AES128 || CipherTraits<C>::ID == TLSGPU_CIPHER_AES256) {
        constexpr int NR = CipherTraits<C>::ID == TLSGPU_CIPHER_AES128 ? 10 : 14;
        if (aes_impl() == 0)
            return launch_seal_split<NR, MAC, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, ws,
                                                    epoch, s);
        if (aes_impl() == 1)
            return launch_seal_aesq<NR, MAC, SSL3>(chains, nchains, recs, pt, wire, states, wire_len, s);
    }
    if constexpr (CipherTraits<C>::ID == TLSGPU_CIPHER_3DES) {
        if (aes_impl() == 0)  // split: prefix / MAC / 8-lane 3DES (TLSGPU_SEAL_IMPL=lane: one lane per chain)
            return launch_seal_split<0, MAC, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, ws,
                                                   epoch, s);
    }
    auto kern = seal_kernel<C, MAC, SSL3>;
    constexpr uint32_t lds = CipherTraits<C>::LDS;
    static bool attr = false;
    if (!attr) {
        hipError_t e = set_lds(kern, lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    dim3 grid((nchains + SEAL_BLOCK - 1) / SEAL_BLOCK);
    hipLaunchKernelGGL(kern, grid, dim3(SEAL_BLOCK), lds, s, chains, nchains, recs, pt, wire, states, wire_len);
    return hipGetLastError();
}

bool seal_needs_workspace(uint32_t variant) {
    const uint32_t c = variant & 0xff;
    return aes_impl() == 0 && (c == TLSGPU_CIPHER_AES128 || c == TLSGPU_CIPHER_AES256 || c == TLSGPU_CIPHER_3DES);
}

hipError_t launch_seal(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                       uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states, int32_t* wire_len,
                       uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known) {
    *known = true;
#define TG_SEAL_CASE(CIPHER_ID, CTYPE, MAC_ID, SSL3)                                                      \
    if (variant == TLSGPU_VARIANT(CIPHER_ID, MAC_ID, SSL3))                                               \
        return launch_seal_t<CTYPE, MAC_ID, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, ws, \
                                                  epoch, s);
    // TLS 1.0-1.2 HMAC suites (constants.py:159-201)
    TG_SEAL_CASE(TLSGPU_CIPHER_AES128, AesCbc<10>, TLSGPU_MAC_SHA1, false)
    TG_SEAL_CASE(TLSGPU_CIPHER_AES256, AesCbc<14>, TLSGPU_MAC_SHA1, false)
    TG_SEAL_CASE(TLSGPU_CIPHER_AES128, AesCbc<10>, TLSGPU_MAC_SHA256, false)
    TG_SEAL_CASE(TLSGPU_CIPHER_AES256, AesCbc<14>, TLSGPU_MAC_SHA256, false)
    TG_SEAL_CASE(TLSGPU_CIPHER_3DES, TdesCbc, TLSGPU_MAC_SHA1, false)
    TG_SEAL_CASE(TLSGPU_CIPHER_RC4, Rc4Stream, TLSGPU_MAC_SHA1, false)
    TG_SEAL_CASE(TLSGPU_CIPHER_RC4, Rc4Stream, TLSGPU_MAC_MD5, false)
    // SSL 3.0 MAC_SSL suites (mathtls.py:125-151)
    TG_SEAL_CASE(TLSGPU_CIPHER_AES128, AesCbc<10>, TLSGPU_MAC_SHA1, true)
    TG_SEAL_CASE(TLSGPU_CIPHER_AES256, AesCbc<14>, TLSGPU_MAC_SHA1, true)
    TG_SEAL_CASE(TLSGPU_CIPHER_3DES, TdesCbc, TLSGPU_MAC_SHA1, true)
    TG_SEAL_CASE(TLSGPU_CIPHER_RC4, Rc4Stream, TLSGPU_MAC_SHA1, true)
    TG_SEAL_CASE(TLSGPU_CIPHER_RC4, Rc4Stream, TLSGPU_MAC_MD5, true)
#undef TG_SEAL_CASE
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
                                 : CIPHER == TLSGPU_CIPHER_3DES ? DES_LDS_BYTES
                                                                : RC4_LDS_BYTES_PER_WAVE * (SEAL_BLOCK / 64);
    static bool attr = false;
    if (!attr) {
        hipError_t e = set_lds(kern, lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    dim3 grid((n + SEAL_BLOCK - 1) / SEAL_BLOCK);
    hipLaunchKernelGGL(kern, grid, dim3(SEAL_BLOCK), lds, s, spans, n, in, out, states);
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


// ---------------------------------------------------------------- block-parallel AES open
size_t open_workspace_bytes(uint32_t nrecords) { return (size_t)nrecords * sizeof(OpenMeta); }

static bool open_split_variant(uint32_t v) {
    const uint32_t c = v & 0xff, m = (v >> 8) & 0xff, ssl3 = (v >> 16) & 1;
    const bool aes = c == TLSGPU_CIPHER_AES128 || c == TLSGPU_CIPHER_AES256;
    return aes && (m == TLSGPU_MAC_SHA1 || (m == TLSGPU_MAC_SHA256 && !ssl3)) && !(getenv("TLSGPU_OPEN_IMPL") &&
                                                                                   !strcmp(getenv("TLSGPU_OPEN_IMPL"), "lane"));
}
bool open_needs_workspace(uint32_t variant) { return open_split_variant(variant); }

template <int NR, int MAC, bool SSL3>
static hipError_t launch_open_split(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_open_record* recs,
                                    uint32_t nrecords, const uint8_t* wire, uint8_t* pt, ConnState* states,
                                    int32_t* status, uint8_t* ws, uint32_t epoch, hipStream_t s) {
    constexpr int CID = NR == 10 ? TLSGPU_CIPHER_AES128 : TLSGPU_CIPHER_AES256;
    OpenMeta* meta = reinterpret_cast<OpenMeta*>(ws);
    hipError_t e = hipMemsetAsync(meta, 0, (size_t)nrecords * sizeof(OpenMeta), s);
    if (e != hipSuccess) return e;
    const dim3 gc((nchains + 255) / 256), gr((nrecords + 255) / 256);
    hipLaunchKernelGGL((open_prefix_kernel<CID, MAC, SSL3>), gc, dim3(256), 0, s, chains, nchains, recs, nrecords,
                       wire, states, status, meta, epoch);
    auto dec = open_dec_kernel<NR>;
    static bool attr = false;
    if (!attr) {
        if ((e = set_lds(dec, AES_DEC_LDS_BYTES)) != hipSuccess) return e;
        attr = true;
    }
    uint32_t grid = (nrecords + (O3_THREADS / 64) - 1) / (O3_THREADS / 64);
    grid = grid > (uint32_t)cu_count() ? (uint32_t)cu_count() : (grid ? grid : 1u);
    hipLaunchKernelGGL(dec, dim3(grid), dim3(O3_THREADS), AES_DEC_LDS_BYTES, s, recs, nrecords, wire, pt, states, meta,
                       epoch);
    hipLaunchKernelGGL((open_seq_kernel<MAC, SSL3>), gc, dim3(256), 0, s, chains, nchains, recs, nrecords, pt, states,
                       status, meta, epoch);
    hipLaunchKernelGGL((open_mac_kernel<MAC, SSL3>), gr, dim3(256), 0, s, recs, nrecords, pt, states, status, meta,
                       epoch);
    return hipGetLastError();
}

hipError_t launch_open(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                       const tlsgpu_open_record* recs, uint32_t nrecords, const uint8_t* wire, uint8_t* pt,
                       ConnState* states, int32_t* status, uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known) {
    if (open_split_variant(variant)) {
        *known = true;
#define TG_OPEN3(CID, NR, MAC_ID, SSL3)                                                                         \
        if (variant == TLSGPU_VARIANT(CID, MAC_ID, SSL3))                                                       \
            return launch_open_split<NR, MAC_ID, SSL3>(chains, nchains, recs, nrecords, wire, pt, states, status, \
                                                        ws, epoch, s);
        TG_OPEN3(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, false)
        TG_OPEN3(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, false)
        TG_OPEN3(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA256, false)
        TG_OPEN3(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA256, false)
        TG_OPEN3(TLSGPU_CIPHER_AES128, 10, TLSGPU_MAC_SHA1, true)
        TG_OPEN3(TLSGPU_CIPHER_AES256, 14, TLSGPU_MAC_SHA1, true)
#undef TG_OPEN3
    }
    return launch_open_lane(variant, chains, nchains, recs, wire, pt, states, status, s, known);
}

}  // namespace tg

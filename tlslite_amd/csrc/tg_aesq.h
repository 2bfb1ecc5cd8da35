// tg_aesq.h -- the AES record-seal kernel laid out for a CDNA4 CU.
//
// One 768-thread workgroup per CU owns 256 connection chains:
//   waves 0..7   "cipher waves": 4 lanes per chain PAIR.  Lane q holds AES
//                state column q of two independent chains (ILP 2: the two
//                CBC chains interleave so one chain's LDS lookups are in
//                flight while the other's XORs issue).  A round per chain is
//                4 conflict-free LDS T-table lookups + one plain and three
//                DPP quad_perm XORs per lane: the ShiftRows/MixColumns
//                exchange between the 4 columns rides in the DPP operand.
//   waves 8..11  "MAC waves": 1 lane per chain, HMAC / MAC_SSL over the record
//                (the serial hash chain runs beside the serial CBC chain), then
//                the CBC tail (last P bytes | MAC | padding) is staged in a
//                64-byte LDS slot, plus the 5-byte record header.
// Per record: [cipher: explicit IV + full P blocks | MAC: MAC, tail, header]
//             -> barrier -> [cipher: tail blocks] -> barrier.
//
// LDS: [0, 128K) the 4 T-tables x 32 lane copies (layout of aes_lds_fill:
//      T0/T1 rows in the low 64K, T2/T3 in the high 64K; the address is one
//      v_perm of the state word), [128K, 144K) 256 tail slots, then scalars.
#pragma once
#include "tg_device.h"

namespace tg {

constexpr int Q_CHAINS = 256;     // chains per workgroup
constexpr int Q_AES_WAVES = 8;    // 16 quads x 2 chains each
constexpr int Q_MAC_WAVES = 4;    // 64 chains each
constexpr int Q_THREADS = 64 * (Q_AES_WAVES + Q_MAC_WAVES);
constexpr uint32_t Q_TAB_BYTES = AES_LDS_BYTES;  // 128 KiB
constexpr uint32_t Q_SLOT_BYTES = 64;
constexpr uint32_t Q_LDS_BYTES = Q_TAB_BYTES + Q_CHAINS * Q_SLOT_BYTES + 16;

typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) uint8_t lds_u8_t;

__device__ __forceinline__ uint32_t lds_read32(uint32_t addr) { return *(const lds_u32_t*)(size_t)addr; }
__device__ __forceinline__ void lds_write8(uint32_t addr, uint32_t v) { *(lds_u8_t*)(size_t)addr = (uint8_t)v; }
__device__ __forceinline__ void lds_write32(uint32_t addr, uint32_t v) { *(lds_u32_t*)(size_t)addr = v; }

// v_xor_b32_dpp-able quad permutation (update_dpp with old=0 lets the DPP
// combiner fold the move into the consuming XOR)
template <int CTRL>
__device__ __forceinline__ uint32_t quad_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

struct QuadAes {
    uint32_t lo, hi;  // lane-copy offset words (table pair select in byte 2)
    __device__ __forceinline__ void init() {
        lo = (__lane_id() & 31) * 4;
        hi = lo | 0x10000u;
    }
    template <int T, int B>  // T_t[byte B of s]
    __device__ __forceinline__ uint32_t look(uint32_t s) const {
        constexpr uint32_t sel = 0x0c000000u | (2u << 16) | ((4u + B) << 8) | 0u;
        return lds_read32(perm(s, T >= 2 ? hi : lo, sel) + (T & 1) * 128);
    }
    // Column q of the next state = T0[b0(q)] ^ T1[b1(q+1)] ^ T2[b2(q+2)] ^ T3[b3(q+3)] ^ k[q], with
    // the lookup of byte b done by lane q+b.  XOR tree: dpp2(t2) ^ dpp3(t3) = dpp2(t2 ^ dpp1(t3)),
    // and the round key rides in that inner term: k2 is the key column of lane q+2 (round_keys()),
    // so once the T0/T1 lookups return only two dependent DPP XORs remain (a chain needs four).
    // The T2/T3 lookups are issued first: they feed the inner term.
    template <int R>
    __device__ __forceinline__ uint32_t round(uint32_t x, uint32_t k2) const {
        const uint32_t t2 = look<2, 2>(x);
        const uint32_t t3 = look<3, 3>(x);
        const uint32_t t0 = look<0, 0>(x);
        const uint32_t t1 = look<1, 1>(x);
        const uint32_t u = (t2 ^ k2) ^ quad_dpp<0x39>(t3);
        const uint32_t z = t0 ^ quad_dpp<0x39>(t1);
        return z ^ quad_dpp<0x4E>(u);
    }
    // per-lane round keys in the layout round()/last() expect: k[0] = whitening column q,
    // k[r >= 1] = column (q+2)&3 of round key r
    template <int NR>
    static __device__ __forceinline__ void round_keys(const uint32_t* ek, uint32_t q, uint32_t* k) {
        k[0] = ek[q];
#pragma unroll
        for (int r = 1; r <= NR; r++) k[r] = ek[4 * r + ((q + 2) & 3)];
    }
    __device__ __forceinline__ uint32_t last(uint32_t x, uint32_t k) const {
        // S-box byte r sits at byte r of table (r+2)&3
        const uint32_t s2 = look<0, 2>(x) & 0xff0000u;
        const uint32_t s3 = look<1, 3>(x) & 0xff000000u;
        const uint32_t s0 = look<2, 0>(x) & 0xffu;
        const uint32_t s1 = look<3, 1>(x) & 0xff00u;
        const uint32_t u = (s2 ^ k) ^ quad_dpp<0x39>(s3);
        const uint32_t z = s0 ^ quad_dpp<0x39>(s1);
        return z ^ quad_dpp<0x4E>(u);
    }
    // one block of one chain
    template <int NR>
    __device__ __forceinline__ uint32_t encrypt1(uint32_t a, const uint32_t* ka) const {
        a ^= ka[0];
#pragma unroll
        for (int r = 1; r < NR; r++) a = round<0>(a, ka[r]);
        return last(a, ka[NR]);
    }
    // one block whose input is already whitened (x = block ^ k[0])
    template <int NR>
    __device__ __forceinline__ uint32_t encrypt_w(uint32_t a, const uint32_t* ka) const {
#pragma unroll
        for (int r = 1; r < NR; r++) a = round<0>(a, ka[r]);
        return last(a, ka[NR]);
    }
    // two independent blocks (chains a and b) interleaved round by round
    template <int NR>
    __device__ __forceinline__ void encrypt2(uint32_t& a, uint32_t& b, const uint32_t* ka, const uint32_t* kb) const {
        a ^= ka[0];
        b ^= kb[0];
#pragma unroll
        for (int r = 1; r < NR; r++) {
            uint32_t na = round<0>(a, ka[r]);
            uint32_t nb = round<0>(b, kb[r]);
            a = na;
            b = nb;
        }
        uint32_t la = last(a, ka[NR]);
        uint32_t lb = last(b, kb[NR]);
        a = la;
        b = lb;
    }
};

__device__ __forceinline__ uint32_t ld32(const uint8_t* p, bool al) {
    if (al) return *(const uint32_t*)p;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ void st32(uint8_t* p, uint32_t v, bool al) {
    if (al) {
        *(uint32_t*)p = v;
    } else {
        p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
    }
}

// Per-chain record bookkeeping of a cipher lane.
struct QChain {
    bool go;
    uint32_t n, nb, E;
    const uint8_t* P;
    uint8_t* B;
    bool al;
};

template <int NR, int MAC, bool SSL3>
__global__ void __launch_bounds__(Q_THREADS, 3)
seal_aesq_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
                 const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire, ConnState* __restrict__ states,
                 int32_t* __restrict__ wire_len, uint32_t cpw, uint32_t debug_skip) {
    // cpw = chains per workgroup (<= 256): small batches are spread over all
    // CUs instead of packing 256 chains into a handful of workgroups
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    constexpr uint32_t CIPHER_ID = NR == 10 ? TLSGPU_CIPHER_AES128 : TLSGPU_CIPHER_AES256;
    constexpr uint32_t SLOTS = Q_TAB_BYTES;
    constexpr uint32_t MISC = Q_TAB_BYTES + Q_CHAINS * Q_SLOT_BYTES;

    aes_lds_fill(nullptr, false);
    if (threadIdx.x == 0) lds_write32(MISC, 0);
    __syncthreads();

    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool is_aes = wave < Q_AES_WAVES;
    const uint32_t q = lane & 3;
    const uint32_t base = blockIdx.x * cpw;
    const uint32_t half = (cpw + 1) >> 1;  // quad j carries chains j and j + half

    if (!is_aes) {
        // ================================================= MAC lanes
        const uint32_t local = (wave - Q_AES_WAVES) * 64 + lane;
        const uint32_t cid = base + local;
        tlsgpu_chain ch = {0, 0, 0, 0};
        ConnState* st = nullptr;
        bool ok = false;
        if (local < cpw && cid < nchains) {
            ch = chains[cid];
            st = states + ch.state;
            ok = st->cipher == CIPHER_ID && st->mac == (uint32_t)MAC && st->ssl3 == (SSL3 ? 1u : 0u) && !st->raw;
            __hip_atomic_fetch_max((lds_u32_t*)(size_t)MISC, ch.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (!ok)
                for (uint32_t k = 0; k < ch.count; k++) wire_len[ch.first + k] = TLSGPU_EMISMATCH;
        }
        __syncthreads();
        const uint32_t maxcount = lds_read32(MISC);
        const uint32_t slot = SLOTS + local * Q_SLOT_BYTES;
        uint64_t seq = ok ? st->seqnum : 0;
        const uint32_t E = ok && st->explicit_iv ? 16u : 0u;
        for (uint32_t k = 0; k < maxcount; k++) {
            if (ok && k < ch.count) {
                const tlsgpu_record R = recs[ch.first + k];
                const uint32_t n = R.pt_len;
                const uint32_t cur0 = E + n + DL;
                const uint32_t body = cur0 + (16 - (cur0 & 15));
                if (n == 0 || body > 0xffffu) {
                    wire_len[ch.first + k] = n == 0 ? 0 : TLSGPU_ETOOBIG;
                } else {
                    const uint8_t* P = pt + R.pt_off;
                    uint8_t* W = wire + R.wire_off;
                    M mac;
                    mac.begin(st, seq, R.content_type, n);
                    const uint32_t nfull = (debug_skip & 2) ? 0u : (n >> 6);
                    // double-buffered 64-byte chunks: the next load is in flight during a compression
                    uint32_t nxt[16];
                    if (nfull) load64(P, nxt);
                    for (uint32_t c = 0; c < nfull; c++) {
                        uint32_t cur[16];
#pragma unroll
                        for (int j = 0; j < 16; j++) cur[j] = nxt[j];
                        if (c + 1 < nfull) load64(P + 64 * (c + 1), nxt);
                        mac.update(cur);
                    }
                    const uint32_t nf = n >> 6;
                    const uint32_t r64 = n & 63;
                    uint32_t tail[16];
                    load_partial(P + 64 * nf, r64, tail);
                    uint32_t m[8];
                    mac.finish(tail, (int)r64, n, st, m);
                    if (R.flags & TLSGPU_FAULT_BAD_MAC) m[0] = (m[0] & ~0xffu) | ((m[0] + 1u) & 0xffu);
                    // CBC tail slot: P[16*nb ..) | MAC | pad  (tlsrecordlayer.py:597-606)
                    const uint32_t r16 = n & 15;
                    const uint8_t* Pt = P + (n - r16);
                    for (uint32_t i = 0; i < r16; i++) lds_write8(slot + i, Pt[i]);
#pragma unroll
                    for (int i = 0; i < DL; i++) lds_write8(slot + r16 + i, m[i >> 2] >> (8 * (i & 3)));
                    const uint32_t padl = 15 - ((r16 + DL) & 15);
                    for (uint32_t i = 0; i <= padl; i++) lds_write8(slot + r16 + DL + i, padl);
                    if (R.flags & TLSGPU_FAULT_BAD_PADDING) lds_write8(slot + r16 + DL, padl + 1);
                    W[0] = R.content_type;  // RecordHeader3 (messages.py:36-42)
                    W[1] = st->vmaj;
                    W[2] = st->vmin;
                    W[3] = (uint8_t)(body >> 8);
                    W[4] = (uint8_t)body;
                    wire_len[ch.first + k] = (int32_t)(body + 5);
                    seq++;
                }
            }
            __syncthreads();  // tail slots ready
            __syncthreads();  // tail slots consumed
        }
        if (ok) st->seqnum = seq;
        return;
    }

    // ===================================================== cipher lanes
    // The cipher waves are the long pole (latency-bound CBC chains): let them
    // win issue arbitration; the MAC waves fill the remaining slots.
    __builtin_amdgcn_s_setprio(2);
    const uint32_t quad = wave * 16 + (lane >> 2);  // 0..127
    const uint32_t lA = quad, lB = quad + half;     // local chain ids
    tlsgpu_chain cA = {0, 0, 0, 0}, cB = {0, 0, 0, 0};
    ConnState *sA = nullptr, *sB = nullptr;
    bool okA = false, okB = false;
    auto chk = [&](ConnState* s) {
        return s->cipher == CIPHER_ID && s->mac == (uint32_t)MAC && s->ssl3 == (SSL3 ? 1u : 0u) && !s->raw;
    };
    if (lA < half && base + lA < nchains) { cA = chains[base + lA]; sA = states + cA.state; okA = chk(sA); }
    if (lB < cpw && base + lB < nchains) { cB = chains[base + lB]; sB = states + cB.state; okB = chk(sB); }
    __syncthreads();
    const uint32_t maxcount = lds_read32(MISC);
    QuadAes aes;
    aes.init();
    uint32_t kA[NR + 1], kB[NR + 1];
    uint32_t ivA = 0, ivB = 0;
#pragma unroll
    for (int r = 0; r <= NR; r++) {
        kA[r] = okA ? sA->ek[r == 0 ? q : 4 * r + ((q + 2) & 3)] : 0u;
        kB[r] = okB ? sB->ek[r == 0 ? q : 4 * r + ((q + 2) & 3)] : 0u;
    }
    if (okA) ivA = sA->iv[q];
    if (okB) ivB = sB->iv[q];
    const uint32_t EA = okA && sA->explicit_iv ? 16u : 0u;
    const uint32_t EB = okB && sB->explicit_iv ? 16u : 0u;

    for (uint32_t k = 0; k < maxcount; k++) {
        QChain A, Bc;
        auto setup = [&](QChain& C, bool ok, const tlsgpu_chain& ch, uint32_t E) {
            C.go = false;
            C.n = 0; C.nb = 0; C.E = E; C.P = pt; C.B = wire; C.al = true;
            if (ok && k < ch.count) {
                const tlsgpu_record R = recs[ch.first + k];
                const uint32_t cur0 = E + R.pt_len + DL;
                const uint32_t body = cur0 + (16 - (cur0 & 15));
                C.n = R.pt_len;
                C.go = C.n != 0 && body <= 0xffffu;
                C.P = pt + R.pt_off;
                C.B = wire + R.wire_off + 5;
                C.al = (((uintptr_t)C.P | (uintptr_t)C.B) & 3) == 0;
                C.nb = (debug_skip & 1) ? 0u : (C.n >> 4);
            }
        };
        setup(A, okA, cA, EA);
        setup(Bc, okB, cB, EB);
        // ---------------- phase A: explicit IV block + full plaintext blocks
        if (A.go || Bc.go) {
            if (A.E | Bc.E) {
                uint32_t xa = A.E ? (sA->fixed_iv[q] ^ ivA) : 0u;
                uint32_t xb = Bc.E ? (sB->fixed_iv[q] ^ ivB) : 0u;
                aes.encrypt2<NR>(xa, xb, kA, kB);
                if (A.go && A.E) { ivA = xa; st32(A.B + 4 * q, xa, A.al); }
                if (Bc.go && Bc.E) { ivB = xb; st32(Bc.B + 4 * q, xb, Bc.al); }
            }
            const uint32_t nbA = A.go ? A.nb : 0u, nbB = Bc.go ? Bc.nb : 0u;
            const uint32_t nbm = nbA > nbB ? nbA : nbB;
            const uint8_t* PA = A.P + 4 * q;
            const uint8_t* PB = Bc.P + 4 * q;
            uint8_t* OA = A.B + A.E + 4 * q;
            uint8_t* OB = Bc.B + Bc.E + 4 * q;
            // plaintext column words fetched 8 blocks ahead
            uint32_t fa[8], fb[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                fa[j] = (uint32_t)j < nbA ? ld32(PA + 16 * j, A.al) : 0u;
                fb[j] = (uint32_t)j < nbB ? ld32(PB + 16 * j, Bc.al) : 0u;
            }
            for (uint32_t b0 = 0; b0 < nbm; b0 += 8) {
                uint32_t ca[8], cb[8];
#pragma unroll
                for (int j = 0; j < 8; j++) { ca[j] = fa[j]; cb[j] = fb[j]; }
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t b = b0 + 8 + j;
                    fa[j] = b < nbA ? ld32(PA + 16 * b, A.al) : 0u;
                    fb[j] = b < nbB ? ld32(PB + 16 * b, Bc.al) : 0u;
                }
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t b = b0 + j;
                    uint32_t xa = ca[j] ^ ivA, xb = cb[j] ^ ivB;
                    aes.encrypt2<NR>(xa, xb, kA, kB);
                    if (b < nbA) { ivA = xa; st32(OA + 16 * b, xa, A.al); }
                    if (b < nbB) { ivB = xb; st32(OB + 16 * b, xb, Bc.al); }
                }
            }
        }
        __syncthreads();  // tail slots ready
        // ---------------- phase B: tail blocks from the LDS slots
        if (A.go || Bc.go) {
            auto tl = [&](const QChain& C) {
                const uint32_t r16 = C.n & 15;
                return C.go ? r16 + DL + 16 - ((r16 + DL) & 15) : 0u;
            };
            const uint32_t TA = tl(A), TB = tl(Bc);
            const uint32_t Tm = TA > TB ? TA : TB;
            const uint32_t slA = SLOTS + lA * Q_SLOT_BYTES + 4 * q, slB = SLOTS + lB * Q_SLOT_BYTES + 4 * q;
            uint8_t* OA = A.B + A.E + (A.n & ~15u) + 4 * q;
            uint8_t* OB = Bc.B + Bc.E + (Bc.n & ~15u) + 4 * q;
            for (uint32_t off = 0; off < Tm; off += 16) {
                uint32_t xa = lds_read32(slA + off) ^ ivA, xb = lds_read32(slB + off) ^ ivB;
                aes.encrypt2<NR>(xa, xb, kA, kB);
                if (off < TA) { ivA = xa; st32(OA + off, xa, A.al); }
                if (off < TB) { ivB = xb; st32(OB + off, xb, Bc.al); }
            }
        }
        __syncthreads();  // tail slots consumed
    }
    if (okA) sA->iv[q] = ivA;
    if (okB) sB->iv[q] = ivB;
}

}  // namespace tg

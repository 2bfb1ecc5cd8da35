// tg_aes3.h -- three-kernel AES record seal (the default AES path).
//
//   prefix_kernel  one lane per chain: validates the state, assigns each
//                  record its seqnum (empty / oversized records consume none,
//                  tlsrecordlayer.py:551-556), advances state->seqnum and
//                  publishes {seq, state, status, epoch} per record.
//   mac_kernel     one lane per RECORD: HMAC / MAC_SSL over the record, the
//                  CBC tail (last P bytes | MAC | padding, <= 63 B) into a
//                  64-byte workspace slot, the 5-byte header, wire_len.  All
//                  records are independent here, also those of one connection.
//   cbc_kernel     16 waves x 16 quads: 4 lanes per chain (AES state column per
//                  lane, DPP quad exchange), one chain per quad (ILP 1) -- the
//                  configuration tools/aes_round_microbench.hip measured best
//                  for 256 chains per CU.  No barriers: each quad streams its
//                  chain: explicit IV, full P blocks, then the tail slot.
//
// Workspace per record: 16 B meta + 64 B tail slot.  Kernels run in stream
// order (prefix -> mac -> cbc).
#pragma once
#include "tg_aesq.h"

namespace tg {

// wave priority from a runtime value (s_setprio takes an immediate)
__device__ __forceinline__ void set_prio(uint32_t p) {
    switch (p) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}
// debug_skip bits 4-5 / 6-7: (priority + 1) of the CBC / MAC waves, 0 = built-in default
__device__ __forceinline__ uint32_t prio_of(uint32_t debug_skip, int shift, uint32_t dflt) {
    const uint32_t v = (debug_skip >> shift) & 3u;
    return v ? v - 1 : dflt;
}

struct RecMeta {
    uint64_t seq;
    uint32_t state;
    uint32_t epoch;     // launch id: entries of other launches are ignored
    uint32_t status;    // 1 = seal, 0 = skip (empty / error)
    uint32_t tail_len;  // bytes of CBC tail (multiple of 16)
    uint32_t pad[2];
};
static_assert(sizeof(RecMeta) == 32, "RecMeta");
constexpr uint32_t TAIL_SLOT = 64;
constexpr int C3_THREADS = 1024;  // 16 cipher waves
constexpr int C3_CHAINS = 256;

template <int CIPHER_ID, int MAC, bool SSL3>
__global__ void __launch_bounds__(256) prefix_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                    const tlsgpu_record* __restrict__ recs,
                                                    ConnState* __restrict__ states, int32_t* __restrict__ wire_len,
                                                    RecMeta* __restrict__ meta, uint32_t nrecords, uint32_t epoch) {
    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    ConnState* st = states + ch.state;
    const bool ok = st->cipher == (uint32_t)CIPHER_ID && st->mac == (uint32_t)MAC &&
                    st->ssl3 == (SSL3 ? 1u : 0u) && !st->raw;
    constexpr int DL = Hash<MAC>::DLEN;
    uint64_t seq = st->seqnum;
    const uint32_t E = st->explicit_iv ? 16u : 0u;
    for (uint32_t k = 0; k < ch.count; k++) {
        const uint32_t r = ch.first + k;
        if (r >= nrecords) break;
        RecMeta m;
        m.state = ch.state;
        m.epoch = epoch;
        m.seq = seq;
        m.status = 0;
        m.tail_len = 0;
        m.pad[0] = m.pad[1] = 0;
        if (!ok) {
            wire_len[r] = TLSGPU_EMISMATCH;
        } else {
            const uint32_t n = recs[r].pt_len;
            const uint32_t cur = E + n + DL;
            const uint32_t body = cur + (16 - (cur & 15));
            if (n == 0) {
                wire_len[r] = 0;
            } else if (body > 0xffffu) {
                wire_len[r] = TLSGPU_ETOOBIG;
            } else {
                const uint32_t r16 = n & 15;
                m.status = 1;
                m.tail_len = r16 + DL + 16 - ((r16 + DL) & 15);
                seq++;
            }
        }
        meta[r] = m;
    }
    if (ok) st->seqnum = seq;
}

template <int MAC, bool SSL3>
__global__ void __launch_bounds__(256) mac_kernel(const tlsgpu_record* __restrict__ recs, uint32_t nrecords,
                                                 const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                                                 const ConnState* __restrict__ states, int32_t* __restrict__ wire_len,
                                                 const RecMeta* __restrict__ meta, uint8_t* __restrict__ tails,
                                                 uint32_t epoch, uint32_t debug_skip) {
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrecords) return;
    const RecMeta mt = meta[r];
    if (mt.epoch != epoch || mt.status != 1) return;
    set_prio(prio_of(debug_skip, 6, 0));
    const ConnState* st = states + mt.state;
    const tlsgpu_record R = recs[r];
    const uint32_t n = R.pt_len;
    const uint32_t E = st->explicit_iv ? 16u : 0u;
    const uint32_t cur0 = E + n + DL;
    const uint32_t body = cur0 + (16 - (cur0 & 15));
    const uint8_t* P = pt + R.pt_off;
    uint8_t* W = wire + R.wire_off;
    M mac;
    mac.begin(st, mt.seq, R.content_type, n);
    const uint32_t nfull = (debug_skip & 2) ? 0u : (n >> 6);
    uint32_t nxt[16];
    if (nfull) load64(P, nxt);
    for (uint32_t c = 0; c < nfull; c++) {
        uint32_t cur[16];
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] = nxt[j];
        if (c + 1 < nfull) load64(P + 64 * (c + 1), nxt);
        mac.update(cur);
    }
    const uint32_t nf = n >> 6, r64 = n & 63;
    uint32_t tail[16];
    load_partial(P + 64 * nf, r64, tail);
    uint32_t m[8];
    mac.finish(tail, (int)r64, n, st, m);
    if (R.flags & TLSGPU_FAULT_BAD_MAC) m[0] = (m[0] & ~0xffu) | ((m[0] + 1u) & 0xffu);
    // CBC tail: P[16*nb ..) | MAC | pad  (tlsrecordlayer.py:597-606), built as dwords
    uint8_t* slot = tails + (size_t)r * TAIL_SLOT;
    const uint32_t r16 = n & 15;
    const uint8_t* Pt = P + (n - r16);
    const uint32_t padl = 15 - ((r16 + DL) & 15);
    const uint32_t T = r16 + DL + padl + 1;
    uint32_t out[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t pos = 4 * q + b;
            uint32_t byte;
            if (pos < r16) byte = Pt[pos];
            else if (pos < r16 + DL) {
                const uint32_t i = pos - r16;
                // i is runtime: select the MAC dword, then the byte
                uint32_t w = 0;
#pragma unroll
                for (int j = 0; j < DL / 4; j++) w = (i >> 2) == (uint32_t)j ? m[j] : w;
                byte = (w >> (8 * (i & 3))) & 0xffu;
            } else {
                byte = padl;
                if (pos == r16 + DL && (R.flags & TLSGPU_FAULT_BAD_PADDING)) byte = padl + 1;
            }
            v |= (pos < T ? byte : 0u) << (8 * b);
        }
        out[q] = v;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) *(uint4*)(slot + 16 * q) = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
    W[0] = R.content_type;  // RecordHeader3 (messages.py:36-42)
    W[1] = st->vmaj;
    W[2] = st->vmin;
    W[3] = (uint8_t)(body >> 8);
    W[4] = (uint8_t)body;
    wire_len[r] = (int32_t)(body + 5);
}

template <int NR>
__global__ void __launch_bounds__(C3_THREADS, 1)
cbc_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
           uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
           ConnState* __restrict__ states, const RecMeta* __restrict__ meta, const uint8_t* __restrict__ tails,
           uint32_t cpw, uint32_t epoch, uint32_t debug_skip) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t local = (threadIdx.x >> 6) * 16 + (lane >> 2);
    const uint32_t q = lane & 3;
    const uint32_t cid = blockIdx.x * cpw + local;
    if (local >= cpw || cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    ConnState* st = states + ch.state;
    // the prefix kernel validated the state: any record it marked status 1 belongs to a matching state
    set_prio(prio_of(debug_skip, 4, 1));
    QuadAes aes;
    aes.init();
    uint32_t k[NR + 1];
    uint32_t iv = st->iv[q];
    const uint32_t fiv = st->fixed_iv[q];
    const uint32_t E = st->explicit_iv ? 16u : 0u;
    bool any = false;
    QuadAes::round_keys<NR>(st->ek, q, k);
    for (uint32_t j = 0; j < ch.count; j++) {
        const uint32_t r = ch.first + j;
        if (r >= nrecords) break;
        const RecMeta mt = meta[r];
        if (mt.epoch != epoch || mt.status != 1) continue;
        any = true;
        const tlsgpu_record R = recs[r];
        const uint32_t n = R.pt_len;
        const uint8_t* P = pt + R.pt_off + 4 * q;
        uint8_t* B = wire + R.wire_off + 5;
        const bool al = (((uintptr_t)(pt + R.pt_off) | (uintptr_t)B) & 3) == 0;
        if (E) {
            iv = aes.encrypt1<NR>(fiv ^ iv, k);
            st32(B + 4 * q, iv, al);
        }
        uint8_t* O = B + E + 4 * q;
        const uint32_t nb = (debug_skip & 1) ? 0u : (n >> 4);
        // whitening: block ^ previous ciphertext ^ k[0] as one 3-input v_bitop3
        uint32_t f[8];
#pragma unroll
        for (int i = 0; i < 8; i++) f[i] = (uint32_t)i < nb ? ld32(P + 16 * i, al) : 0u;
        for (uint32_t b0 = 0; b0 < nb; b0 += 8) {
            uint32_t c[8];
#pragma unroll
            for (int i = 0; i < 8; i++) c[i] = f[i];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint32_t b = b0 + 8 + i;
                f[i] = b < nb ? ld32(P + 16 * b, al) : 0u;
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (b0 + i < nb) {
                    iv = aes.encrypt_w<NR>(__builtin_amdgcn_bitop3_b32(c[i], iv, k[0], 0x96), k);
                    st32(O + 16 * (b0 + i), iv, al);
                }
            }
        }
        // tail blocks from the MAC kernel's slot
        const uint32_t r16 = n & 15;
        const uint8_t* slot = tails + (size_t)r * TAIL_SLOT + 4 * q;
        uint8_t* Ot = B + E + (n - r16) + 4 * q;
        const uint32_t T = mt.tail_len;
        for (uint32_t off = 0; off < T; off += 16) {
            iv = aes.encrypt1<NR>(*(const uint32_t*)(slot + off) ^ iv, k);
            st32(Ot + off, iv, al);
        }
    }
    if (any) st->iv[q] = iv;
}

}  // namespace tg

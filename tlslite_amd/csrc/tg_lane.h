// tg_lane.h -- lseal_kernel: the AES record seal with one lane per chain, for batches
// of many connections (cfg3: 1 Mi one-record connections = 4,096 chains per CU).
//
// The split path (tg_aes3.h) gives a chain a quad and runs the MAC of every record in a
// separate kernel: right when a CU has few chains (cfg2: 256), because a quad's dependent
// AES round is 4x shorter than a lane's.  With thousands of chains per CU the cipher is
// no longer short of chains in flight, and the split path's costs dominate: the quad
// layout's DPP XOR tree (1.75 VALU cycles per chain-round against the lane layout's
// ~1.1), a second plaintext read by the MAC kernel, the per-record workspace traffic, and
// only one MAC wave per SIMD beside the cipher waves.  Here a lane does the whole
// `_sendMsg` seal block of its chain's records (tlsrecordlayer.py:538-617): per 64-byte
// plaintext chunk one MAC compression (mathtls.py:116-151, RecMac) and four CBC blocks
// (python_aes.py:20-45, rijndael.py:278-319) from the same registers -- the plaintext is
// read once, the SHA VALU work and the AES LDS lookups of a chunk are independent and
// interleave in the wave's instruction stream.  The explicit IV (:594-595), the padding
// (:597-606) and the header (messages.py:36-42) are built in the lane.
//
// LDS: the 128 KiB T-tables of tg_quad.h (32 lane copies, conflict-free b32 reads);
// each lane reads its own copy.  Persistent: one workgroup per CU, lanes loop over chains.
#pragma once
#include "tg_aes3.h"

namespace tg {

#ifndef TG_AB_LS_WAVES
#define TG_AB_LS_WAVES 8
#endif
constexpr int LS_THREADS = 64 * TG_AB_LS_WAVES;

// One AES block, lane layout: s = block ^ round key 0 (whitened by the caller) as four LE
// column words; the lane does all 16 T-table lookups of a round (QuadAes's address forms).
template <int NR>
__device__ __forceinline__ void lane_aes_w(const QuadAes& A, uint32_t s[4], const uint32_t* rk) {
    uint32_t s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = bx3(bx3(A.look<0, 0>(s0), A.look<1, 1>(s1), A.look<2, 2>(s2)), A.look<3, 3>(s3), rk[4 * r]);
        const uint32_t t1 = bx3(bx3(A.look<0, 0>(s1), A.look<1, 1>(s2), A.look<2, 2>(s3)), A.look<3, 3>(s0), rk[4 * r + 1]);
        const uint32_t t2 = bx3(bx3(A.look<0, 0>(s2), A.look<1, 1>(s3), A.look<2, 2>(s0)), A.look<3, 3>(s1), rk[4 * r + 2]);
        const uint32_t t3 = bx3(bx3(A.look<0, 0>(s3), A.look<1, 1>(s0), A.look<2, 2>(s1)), A.look<3, 3>(s2), rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // final round: S-box byte b sits at byte b of table (b+2)&3
    const uint32_t* k = rk + 4 * NR;
    s[0] = ((A.look<2, 0>(s0) & 0xffu) | (A.look<3, 1>(s1) & 0xff00u) | (A.look<0, 2>(s2) & 0xff0000u) |
            (A.look<1, 3>(s3) & 0xff000000u)) ^ k[0];
    s[1] = ((A.look<2, 0>(s1) & 0xffu) | (A.look<3, 1>(s2) & 0xff00u) | (A.look<0, 2>(s3) & 0xff0000u) |
            (A.look<1, 3>(s0) & 0xff000000u)) ^ k[1];
    s[2] = ((A.look<2, 0>(s2) & 0xffu) | (A.look<3, 1>(s3) & 0xff00u) | (A.look<0, 2>(s0) & 0xff0000u) |
            (A.look<1, 3>(s1) & 0xff000000u)) ^ k[2];
    s[3] = ((A.look<2, 0>(s3) & 0xffu) | (A.look<3, 1>(s0) & 0xff00u) | (A.look<0, 2>(s1) & 0xff0000u) |
            (A.look<1, 3>(s2) & 0xff000000u)) ^ k[3];
}

// CBC step: iv = E(d ^ iv) (the whitening key folded into the same 3-input XOR)
template <int NR>
__device__ __forceinline__ void lane_cbc(const QuadAes& A, const uint32_t d[4], uint32_t iv[4], const uint32_t* rk) {
    uint32_t s[4];
#pragma unroll
    for (int j = 0; j < 4; j++) s[j] = bx3(d[j], iv[j], rk[j]);
    lane_aes_w<NR>(A, s, rk);
#pragma unroll
    for (int j = 0; j < 4; j++) iv[j] = s[j];
}

// One AES round in two halves, so independent work can sit between the LDS lookups and
// their use: look() issues the 16 T-table reads of state x, mix() combines them with the
// round key (LAST: the final round's S-box bytes, no MixColumns).
template <bool LAST>
__device__ __forceinline__ void lane_look(const QuadAes& A, const uint32_t x[4], uint32_t t[16]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if constexpr (!LAST) {
            t[4 * j + 0] = A.look<0, 0>(x[j]);
            t[4 * j + 1] = A.look<1, 1>(x[(j + 1) & 3]);
            t[4 * j + 2] = A.look<2, 2>(x[(j + 2) & 3]);
            t[4 * j + 3] = A.look<3, 3>(x[(j + 3) & 3]);
        } else {
            t[4 * j + 0] = A.look<2, 0>(x[j]);
            t[4 * j + 1] = A.look<3, 1>(x[(j + 1) & 3]);
            t[4 * j + 2] = A.look<0, 2>(x[(j + 2) & 3]);
            t[4 * j + 3] = A.look<1, 3>(x[(j + 3) & 3]);
        }
    }
}
template <bool LAST>
__device__ __forceinline__ void lane_mix(const uint32_t t[16], const uint32_t* k, uint32_t x[4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if constexpr (!LAST)
            x[j] = bx3(bx3(t[4 * j], t[4 * j + 1], t[4 * j + 2]), t[4 * j + 3], k[j]);
        else
            x[j] = ((t[4 * j] & 0xffu) | (t[4 * j + 1] & 0xff00u) | (t[4 * j + 2] & 0xff0000u) |
                    (t[4 * j + 3] & 0xff000000u)) ^ k[j];
    }
}

template <bool AL>
__device__ __forceinline__ void ls_load64(const uint8_t* p, uint32_t d[16]) {
#if defined(TG_AB_LS_NOMEM) || defined(TG_AB_LS_NOLOAD)  // timing only: bulk chunks synthesised in registers
    if constexpr (AL) {
#pragma unroll
        for (int q = 0; q < 16; q++) d[q] = (uint32_t)(uintptr_t)p ^ (0x9e3779b9u * (q + 1));
        return;
    }
#endif
    if constexpr (AL) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 v = ((const uint4*)p)[q];
            d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
        }
    } else {
        load64(p, d);
    }
}
template <bool AL>
__device__ __forceinline__ void ls_store16(uint8_t* p, const uint32_t d[4]) {
#if defined(TG_AB_LS_NOMEM) || defined(TG_AB_LS_NOSTORE)  // timing only: no bulk ciphertext stores
    if constexpr (AL) return;
#endif
    if constexpr (AL) *(uint4*)p = make_uint4(d[0], d[1], d[2], d[3]);
    else store16(p, d);
}

// round step G of a chunk (compile-time recursion: every index below is a constant, so
// the hash state, the message window and the round keys stay in named VGPRs)
template <int NR, bool AL, class H, int G>
__device__ __forceinline__ void ls_step(const QuadAes& A, const uint32_t cur[16], uint32_t iv[4], const uint32_t* rk,
                                        uint32_t x[4], uint32_t s[8], uint32_t w[16], uint32_t out[16]) {
    constexpr int NG = 4 * NR, SR = H::ROUNDS, B = G / NR, R = G % NR;
    constexpr int H0 = G * SR / NG, H1 = (G + 1) * SR / NG;
    static_assert(H1 - H0 <= 2, "at most two hash rounds per AES round step");
    if constexpr (R == 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) x[j] = bx3(cur[4 * B + j], iv[j], rk[j]);
    }
    uint32_t t[16];
    lane_look<R == NR - 1>(A, x, t);
    if constexpr (H0 < H1) H::round(H0, s, w);
    if constexpr (H0 + 1 < H1) H::round(H0 + 1, s, w);
    lane_mix<R == NR - 1>(t, rk + 4 * (R + 1), x);
    if constexpr (R == NR - 1) {
#pragma unroll
        for (int j = 0; j < 4; j++) iv[j] = out[4 * B + j] = x[j];
    }
    if constexpr (G + 1 < NG) ls_step<NR, AL, H, G + 1>(A, cur, iv, rk, x, s, w, out);
}

// One 64-byte chunk: its MAC compression and its four CBC blocks, interleaved by hand.
// The 4 x NR AES round steps are serial (CBC) and each waits on 16 LDS reads; the hash
// rounds are serial too but independent of the AES, so ROUNDS / (4 NR) of them sit
// between every round's lookups and their use (left to itself the compiler scheduled
// the hash and the AES as two separate sequences).  The ciphertext goes to out[].
template <int NR, bool AL, class M>
__device__ __forceinline__ void ls_chunk(const QuadAes& A, M& mac, const uint32_t cur[16], uint32_t iv[4],
                                         const uint32_t* rk, uint32_t out[16]) {
    using H = typename M::H;
    uint32_t w[16];
    mac.block_words(cur, w);
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = mac.h[i];
    uint32_t x[4];
    ls_step<NR, AL, H, 0>(A, cur, iv, rk, x, s, w, out);
#pragma unroll
    for (int i = 0; i < H::NS; i++) mac.h[i] += s[i];
#pragma unroll
    for (int i = 0; i < 4; i++) mac.prev[i] = cur[12 + i];
}

// MAC + CBC over the nfull 64-byte chunks of P (next chunk prefetched, index clamped).
// Ciphertext leaves in whole 64-byte-aligned sectors: with thousands of records in flight
// per XCD the L2 evicts partly written lines, and 16-byte-aligned 64-byte chunk stores
// straddle two sectors (cfg3: WRITE_SIZE 3x the wire bytes, the bulk stores 0.37 ms of
// a 2.9 ms kernel).  m = the blocks of the first sector that precede O; sector k >= 1 is
// the previous chunk's last m blocks and this chunk's first 4 - m, assembled with
// m-selects; the first sector's own blocks and the last chunk's last m blocks are stored
// per block.
template <int NR, bool AL, class M>
__device__ __forceinline__ void ls_bulk(const QuadAes& A, M& mac, uint32_t iv[4], const uint32_t* rk,
                                        const uint8_t* P, uint8_t* O, uint32_t nfull) {
    if (nfull == 0) return;
    const uint32_t m = AL ? ((uint32_t)(uintptr_t)O >> 4) & 3u : 0u;
    uint32_t prv[12] = {};  // the previous chunk's blocks 1..3
    uint32_t nxt[16];
    ls_load64<AL>(P, nxt);
    for (uint32_t c = 0; c < nfull; c++) {
        uint32_t cur[16];
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] = nxt[j];
        const uint32_t cn = c + 1 < nfull ? c + 1 : c;
        ls_load64<AL>(P + 64 * cn, nxt);
        uint32_t out[16];
        ls_chunk<NR, AL>(A, mac, cur, iv, rk, out);
        if constexpr (!AL) {
#pragma unroll
            for (int b = 0; b < 4; b++) ls_store16<AL>(O + 64 * c + 16 * b, out + 4 * b);
        } else if (c == 0) {
#pragma unroll
            for (int b = 0; b < 4; b++)
                if ((uint32_t)b + m < 4u) ls_store16<AL>(O + 16 * b, out + 4 * b);
        } else {
            // sector block i = E[4 - m + i] of E = [prv blocks 1..3 at E[1..3] | out blocks at E[4..7]]
            uint32_t sec[16];
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    auto E = [&](int k) { return k >= 4 ? out[4 * (k - 4) + q] : prv[4 * (k - 1) + q]; };
                    const uint32_t v3 = E(1 + i), v2 = E(2 + i), v1 = E(3 + i), v0 = E(4 + i);
                    sec[4 * i + q] = m == 0 ? v0 : m == 1 ? v1 : m == 2 ? v2 : v3;
                }
            uint8_t* S = O + 64 * c - 16 * m;
#pragma unroll
            for (int b = 0; b < 4; b++) ls_store16<AL>(S + 16 * b, sec + 4 * b);
        }
#pragma unroll
        for (int j = 0; j < 12; j++) prv[j] = out[4 + j];
    }
    if constexpr (AL) {  // the last chunk's last m blocks
        uint8_t* L = O + 64 * (nfull - 1);
#pragma unroll
        for (int b = 1; b < 4; b++)
            if ((uint32_t)b + m >= 4u) ls_store16<AL>(L + 16 * b, prv + 4 * (b - 1));
    }
}

template <int NR, int MAC, bool SSL3>
__global__ void __launch_bounds__(LS_THREADS, 1)
lseal_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
             uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
             ConnState* __restrict__ states, int32_t* __restrict__ wire_len) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    constexpr uint32_t CID = NR == 10 ? TLSGPU_CIPHER_AES128 : TLSGPU_CIPHER_AES256;
    __builtin_amdgcn_s_setprio(1);
    QuadAes A;
    A.init();
    for (uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x; cid < nchains; cid += gridDim.x * blockDim.x) {
        const tlsgpu_chain ch = chains[cid];
        ConnState* st = states + ch.state;
        if (st->cipher != CID || st->mac != (uint32_t)MAC || st->ssl3 != (SSL3 ? 1u : 0u) || st->raw) {
            for (uint32_t k = 0; k < ch.count && ch.first + k < nrecords; k++) wire_len[ch.first + k] = TLSGPU_EMISMATCH;
            continue;
        }
        uint32_t rk[4 * (NR + 1)];
#pragma unroll
        for (int k = 0; k < 4 * (NR + 1); k++) rk[k] = st->ek[k];
        uint32_t iv[4] = {st->iv[0], st->iv[1], st->iv[2], st->iv[3]};
        uint64_t seq = st->seqnum;
        const uint32_t E = st->explicit_iv ? 16u : 0u;
        for (uint32_t k = 0; k < ch.count; k++) {
            const uint32_t r = ch.first + k;
            if (r >= nrecords) break;
            const tlsgpu_record R = recs[r];
            const uint32_t n = R.pt_len;
            const uint32_t cur0 = E + n + DL;
            const uint32_t body = cur0 + (16u - (cur0 & 15u));
            if (n == 0) {  // nothing sent, no seqnum consumed (tlsrecordlayer.py:551-556)
                wire_len[r] = 0;
                continue;
            }
            if (body > 0xffffu) {
                wire_len[r] = TLSGPU_ETOOBIG;
                continue;
            }
            const uint8_t* P = pt + R.pt_off;
            uint8_t* W = wire + R.wire_off;
            uint8_t* B = W + 5;
            if (E) {  // E(fixedIVBlock ^ residue) (tlsrecordlayer.py:594-595)
                const uint32_t f[4] = {st->fixed_iv[0], st->fixed_iv[1], st->fixed_iv[2], st->fixed_iv[3]};
                lane_cbc<NR>(A, f, iv, rk);
                store16(B, iv);
            }
            uint8_t* O = B + E;
            M mac;
            mac.begin(st, seq, R.content_type, n);
            const uint32_t nfull = n >> 6;
            if ((((uintptr_t)P | (uintptr_t)O) & 15) == 0) ls_bulk<NR, true>(A, mac, iv, rk, P, O, nfull);
            else ls_bulk<NR, false>(A, mac, iv, rk, P, O, nfull);
            // the last n & 63 plaintext bytes: MAC finish, their full blocks, then
            // P[16 nb ..) | MAC | padding (tlsrecordlayer.py:597-606)
            const uint32_t rem = n & 63;
            const uint8_t* Pr = P + 64 * nfull;
            uint8_t* Or = O + 64 * nfull;
            uint32_t tail[16];
            load_partial(Pr, rem, tail);
            uint32_t m[8];
            mac.finish(tail, (int)rem, n, st, m);
            if (R.flags & TLSGPU_FAULT_BAD_MAC) m[0] = (m[0] & ~0xffu) | ((m[0] + 1u) & 0xffu);
            const uint32_t rb = rem >> 4;
#pragma unroll
            for (int b = 0; b < 3; b++) {
                if ((uint32_t)b < rb) {
                    lane_cbc<NR>(A, tail + 4 * b, iv, rk);
                    store16(Or + 16 * b, iv);
                }
            }
            const uint32_t r16 = rem & 15;
            const uint8_t* Pt = Pr + 16 * rb;
            uint8_t* Ot = Or + 16 * rb;
            const uint32_t padl = 15u - ((r16 + DL) & 15u);
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
            for (int b = 0; b < 4; b++) {
                if ((uint32_t)(16 * b) < T) {
                    lane_cbc<NR>(A, out + 4 * b, iv, rk);
                    store16(Ot + 16 * b, iv);
                }
            }
            W[0] = R.content_type;  // RecordHeader3 (messages.py:36-42)
            W[1] = st->vmaj;
            W[2] = st->vmin;
            W[3] = (uint8_t)(body >> 8);
            W[4] = (uint8_t)body;
            wire_len[r] = (int32_t)(body + 5);
            seq++;
        }
        st->seqnum = seq;
#pragma unroll
        for (int j = 0; j < 4; j++) st->iv[j] = iv[j];
    }
}

}  // namespace tg

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
    constexpr uint32_t BS = CIPHER_ID == TLSGPU_CIPHER_3DES ? 8u : 16u;
    uint64_t seq = st->seqnum;
    const uint32_t E = st->explicit_iv ? BS : 0u;
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
            const uint32_t body = cur + (BS - (cur & (BS - 1)));
            if (n == 0) {
                wire_len[r] = 0;
            } else if (body > 0xffffu) {
                wire_len[r] = TLSGPU_ETOOBIG;
            } else {
                const uint32_t rb = n & (BS - 1);
                m.status = 1;
                m.tail_len = rb + DL + BS - ((rb + DL) & (BS - 1));
                seq++;
            }
        }
        meta[r] = m;
    }
    if (ok) st->seqnum = seq;
}

// value of register v in lane L of the calling lane's quad
template <int L>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
    return quad_dpp<L * 0x55>(v);
}
template <int K>
__device__ __forceinline__ uint32_t sel4(const uint32_t x[4], uint32_t q) {  // x[(q + K) & 3]
    const uint32_t i = (q + K) & 3u;
    return i == 0 ? x[0] : i == 1 ? x[1] : i == 2 ? x[2] : x[3];
}
// quad_perm control: lane q reads lane (q + K) & 3
template <int K>
constexpr int quad_rot_ctrl() {
    return ((0 + K) & 3) | (((1 + K) & 3) << 2) | (((2 + K) & 3) << 4) | (((3 + K) & 3) << 6);
}
// 4x4 transpose across a quad: on entry lane q holds row q in x[0..3], on exit lane q
// holds column q (x[i] = entry row i, element q).  Step K: every lane offers its element
// (q - K) & 3 and reads lane (q + K) & 3, which offered exactly element q.
__device__ __forceinline__ void quad_transpose(uint32_t x[4], uint32_t q) {
    const uint32_t u0 = sel4<0>(x, q);
    const uint32_t u1 = quad_dpp<quad_rot_ctrl<1>()>(sel4<3>(x, q));
    const uint32_t u2 = quad_dpp<quad_rot_ctrl<2>()>(sel4<2>(x, q));
    const uint32_t u3 = quad_dpp<quad_rot_ctrl<3>()>(sel4<1>(x, q));
    // u_K belongs at index (q + K) & 3
    const uint32_t u[4] = {u0, u1, u2, u3};
    x[0] = sel4<0>(u, (4u - q) & 3u);
    x[1] = sel4<0>(u, (5u - q) & 3u);
    x[2] = sel4<0>(u, (6u - q) & 3u);
    x[3] = sel4<0>(u, (7u - q) & 3u);
}

// 64-byte chunk load: 4 x dwordx4 when 16-byte aligned, else the generic path
template <bool AL16>
__device__ __forceinline__ void load64t(const uint8_t* p, uint32_t d[16]) {
    if constexpr (AL16) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 v = ((const uint4*)p)[q];
            d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
        }
    } else {
        load64(p, d);
    }
}

// MAC over nfull 64-byte chunks with the next chunk prefetched; the prefetch index is
// clamped instead of guarded so the loop body has no branch on the load
template <bool AL16, class M>
__device__ __forceinline__ void mac_bulk(M& mac, const uint8_t* P, uint32_t nfull) {
    if (nfull == 0) return;
    uint32_t nxt[16];
    load64t<AL16>(P, nxt);
    for (uint32_t c = 0; c < nfull; c++) {
        uint32_t cur[16];
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] = nxt[j];
        const uint32_t cn = c + 1 < nfull ? c + 1 : c;
        load64t<AL16>(P + 64 * cn, nxt);
        mac.update(cur);
    }
}

// MAC over nfull 64-byte chunks of the quad's four records (equal nfull, 16-byte aligned
// plaintext), loaded cooperatively: per load instruction lane q fetches bytes [16q, 16q+16)
// of record L's chunk, so a quad reads a record's 64 contiguous bytes with one instruction
// (a wave: 16 records x 64 B) instead of 64 scattered 16-byte pieces, which is what let the
// MAC phase's plaintext stream slow the concurrent CBC phase.  Four quad transposes per
// chunk hand every lane its own record's 16 words.
template <class M>
__device__ __forceinline__ void mac_bulk_quad(M& mac, const uint8_t* P, uint32_t nfull, uint32_t q) {
    if (nfull == 0) return;
    const uint32_t lo = (uint32_t)(uintptr_t)P, hi = (uint32_t)((uintptr_t)P >> 32);
    const uint8_t* PL[4];
    PL[0] = (const uint8_t*)(((uint64_t)quad_bcast<0>(hi) << 32) | quad_bcast<0>(lo)) + 16 * q;
    PL[1] = (const uint8_t*)(((uint64_t)quad_bcast<1>(hi) << 32) | quad_bcast<1>(lo)) + 16 * q;
    PL[2] = (const uint8_t*)(((uint64_t)quad_bcast<2>(hi) << 32) | quad_bcast<2>(lo)) + 16 * q;
    PL[3] = (const uint8_t*)(((uint64_t)quad_bcast<3>(hi) << 32) | quad_bcast<3>(lo)) + 16 * q;
    uint4 nxt[4];
#pragma unroll
    for (int L = 0; L < 4; L++) nxt[L] = *(const uint4*)PL[L];
    for (uint32_t c = 0; c < nfull; c++) {
        uint4 cur[4];
#pragma unroll
        for (int L = 0; L < 4; L++) cur[L] = nxt[L];
        const uint32_t cn = c + 1 < nfull ? c + 1 : c;
#pragma unroll
        for (int L = 0; L < 4; L++) nxt[L] = *(const uint4*)(PL[L] + 64 * cn);
        // lane q row L = record L bytes [16q, 16q+16); after the transpose lane q holds
        // record q's sub-block s (x[s]) of component j: its word 4s + j
        uint32_t d[16];
        uint32_t x[4];
        x[0] = cur[0].x; x[1] = cur[1].x; x[2] = cur[2].x; x[3] = cur[3].x;
        quad_transpose(x, q);
        d[0] = x[0]; d[4] = x[1]; d[8] = x[2]; d[12] = x[3];
        x[0] = cur[0].y; x[1] = cur[1].y; x[2] = cur[2].y; x[3] = cur[3].y;
        quad_transpose(x, q);
        d[1] = x[0]; d[5] = x[1]; d[9] = x[2]; d[13] = x[3];
        x[0] = cur[0].z; x[1] = cur[1].z; x[2] = cur[2].z; x[3] = cur[3].z;
        quad_transpose(x, q);
        d[2] = x[0]; d[6] = x[1]; d[10] = x[2]; d[14] = x[3];
        x[0] = cur[0].w; x[1] = cur[1].w; x[2] = cur[2].w; x[3] = cur[3].w;
        quad_transpose(x, q);
        d[3] = x[0]; d[7] = x[1]; d[11] = x[2]; d[15] = x[3];
        mac.update(d);
    }
}

// QL: quad-cooperative plaintext loads (mac_bulk_quad) where a quad allows them; a
// separate instantiation so the default kernel keeps its small register footprint
// (a MAC wave must fit beside four cbc_kernel waves on a SIMD: 4 x 96 + 128 <= 512 VGPRs)
template <int MAC, bool SSL3, bool QL = false, int BS = 16>
__global__ void __launch_bounds__(256) mac_kernel(const tlsgpu_record* __restrict__ recs, uint32_t nrecords,
                                                 const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                                                 const ConnState* __restrict__ states, int32_t* __restrict__ wire_len,
                                                 const RecMeta* __restrict__ meta, uint8_t* __restrict__ tails,
                                                 uint32_t epoch, uint32_t debug_skip) {
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    // no early exit before the bulk: the lanes of a quad exchange loaded data (DPP)
    RecMeta mt = {};
    bool act = r < nrecords;
    if (act) {
        mt = meta[r];
        act = mt.epoch == epoch && mt.status == 1;
    }
    set_prio(prio_of(debug_skip, 6, 0));
    const ConnState* st = states;
    tlsgpu_record R = {};
    const uint8_t* P = pt;
    M mac;
    if (act) {
        st = states + mt.state;
        R = recs[r];
        P = pt + R.pt_off;
        mac.begin(st, mt.seq, R.content_type, R.pt_len);
    }
    const uint32_t n = R.pt_len;
    const uint32_t nfull = (!act || (debug_skip & 2)) ? 0u : (n >> 6);
    const bool al16 = ((uintptr_t)P & 15) == 0;
    // quad-cooperative loads when the quad's four records are all sealed, 16-byte aligned
    // and of equal chunk count
    bool quad = false;
    if constexpr (QL) {
        const uint32_t key = (act && al16) ? nfull : 0xffffffffu;
        quad = key != 0xffffffffu && quad_bcast<0>(key) == key && quad_bcast<1>(key) == key &&
               quad_bcast<2>(key) == key && quad_bcast<3>(key) == key;
        if (quad) mac_bulk_quad(mac, P, nfull, threadIdx.x & 3u);
    }
    if (!quad && act) {
        if (al16) mac_bulk<true>(mac, P, nfull);
        else mac_bulk<false>(mac, P, nfull);
    }
    if (!act) return;
    const uint32_t E = st->explicit_iv ? (uint32_t)BS : 0u;
    const uint32_t cur0 = E + n + DL;
    const uint32_t body = cur0 + (BS - (cur0 & (BS - 1)));
    uint8_t* W = wire + R.wire_off;
    const uint32_t nf = n >> 6, r64 = n & 63;
    uint32_t tail[16];
    load_partial(P + 64 * nf, r64, tail);
    uint32_t m[8];
    mac.finish(tail, (int)r64, n, st, m);
    if (R.flags & TLSGPU_FAULT_BAD_MAC) m[0] = (m[0] & ~0xffu) | ((m[0] + 1u) & 0xffu);
    // CBC tail: P[BS*nb ..) | MAC | pad  (tlsrecordlayer.py:597-606), built as dwords
    uint8_t* slot = tails + (size_t)r * TAIL_SLOT;
    const uint32_t r16 = n & (BS - 1);
    const uint8_t* Pt = P + (n - r16);
    const uint32_t padl = (BS - 1) - ((r16 + DL) & (BS - 1));
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


template <bool AL>
__device__ __forceinline__ uint32_t ld32t(const uint8_t* p) {
    if constexpr (AL) return *(const uint32_t*)p;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
template <bool AL>
__device__ __forceinline__ void st32t(uint8_t* p, uint32_t v) {
    if constexpr (AL) {
        *(uint32_t*)p = v;
    } else {
        p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
    }
}

// CBC over nb full plaintext blocks of one chain (P / O include the lane's column offset).
// Groups of 8 blocks with the next group's columns prefetched; the group loop has no
// branches and the prefetch index is clamped to the last block (never out of the record),
// so the compiler's vmcnt waits cover only the loads a block actually consumes -- a
// conditional load per block made it wait for the whole prefetch (vmcnt(0)) every group.
// PROBE (timing experiments only): 1 = no plaintext loads, 2 = no ciphertext stores.
template <int NR, bool AL, int PROBE = 0>
__device__ __forceinline__ uint32_t cbc_bulk(const QuadAes& aes, const uint32_t* k, uint32_t iv,
                                             const uint8_t* P, uint8_t* O, uint32_t nb) {
    if (nb == 0) return iv;
    const uint32_t last = nb - 1;
    uint32_t f[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        f[i] = PROBE == 1 ? (uint32_t)i : ld32t<AL>(P + 16 * ((uint32_t)i < last ? (uint32_t)i : last));
    uint32_t b0 = 0;
    for (; b0 + 8 <= nb; b0 += 8) {
        uint32_t c[8];
#pragma unroll
        for (int i = 0; i < 8; i++) c[i] = f[i];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t b = b0 + 8 + i;
            f[i] = PROBE == 1 ? b ^ c[i] : ld32t<AL>(P + 16 * (b < last ? b : last));
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            iv = aes.encrypt_w<NR>(__builtin_amdgcn_bitop3_b32(c[i], iv, k[0], 0x96), k);
            if (PROBE != 2) st32t<AL>(O + 16 * (b0 + i), iv);
        }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        if (b0 + i < nb) {
            iv = aes.encrypt_w<NR>(__builtin_amdgcn_bitop3_b32(f[i], iv, k[0], 0x96), k);
            st32t<AL>(O + 16 * (b0 + i), iv);
        }
    }
    return iv;
}

// CBC over ng groups of 4 blocks with 16-byte I/O: lane q loads and stores block 4g+q whole
// (one dwordx4 per lane, 64 contiguous bytes per quad and instruction -- a quarter of the
// VMEM instructions of the column-word path, and full 64-byte segments), and two quad
// transposes per group convert between that and the column-per-lane AES state.  The
// prefetch runs D groups ahead with the index clamped to the last group.  P, O: the
// record's first full block, both 16-byte aligned.
template <int NR, int D = 4>
__device__ __forceinline__ uint32_t cbc_bulk16(const QuadAes& aes, const uint32_t* k, uint32_t iv,
                                               const uint8_t* P, uint8_t* O, uint32_t ng, uint32_t q) {
    if (ng == 0) return iv;
    const uint32_t last = ng - 1;
    const uint8_t* Pq = P + 16 * q;
    uint8_t* Oq = O + 16 * q;
    uint4 f[D];
#pragma unroll
    for (int i = 0; i < D; i++) f[i] = *(const uint4*)(Pq + 64 * ((uint32_t)i < last ? (uint32_t)i : last));
    for (uint32_t g = 0; g < ng; g++) {
        uint32_t x[4] = {f[0].x, f[0].y, f[0].z, f[0].w};
#pragma unroll
        for (int i = 0; i + 1 < D; i++) f[i] = f[i + 1];
        const uint32_t gn = g + D < last ? g + D : last;
        f[D - 1] = *(const uint4*)(Pq + 64 * gn);
        quad_transpose(x, q);  // lane q: column q of blocks 4g .. 4g+3
#pragma unroll
        for (int i = 0; i < 4; i++) {
            iv = aes.encrypt_w<NR>(__builtin_amdgcn_bitop3_b32(x[i], iv, k[0], 0x96), k);
            x[i] = iv;
        }
        quad_transpose(x, q);  // lane q: block 4g+q
        *(uint4*)(Oq + 64 * g) = make_uint4(x[0], x[1], x[2], x[3]);
    }
    return iv;
}

// IO16: 16-byte plaintext/ciphertext I/O (cbc_bulk16) for 16-byte aligned records; a
// separate instantiation (it needs ~95 VGPRs against ~44, see mac_kernel)
template <int NR, bool IO16 = false>
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
    if (local >= cpw) return;
    // the prefix kernel validated the state: any record it marked status 1 belongs to a matching state
    set_prio(prio_of(debug_skip, 4, 1));
    QuadAes aes;
    aes.init();
    // persistent over chain generations: with more chains than CUs x cpw (cfg3: 4,096 chains per
    // CU) a quad takes chain cid + gridDim.x * cpw next -- tables filled once per CU, no
    // workgroup drain / relaunch between generations (cfg3 cipher phase 2.96 -> 2.26 ms)
    for (uint32_t cid = blockIdx.x * cpw + local; cid < nchains; cid += gridDim.x * cpw) {
    const tlsgpu_chain ch = chains[cid];
    ConnState* st = states + ch.state;
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
        if (debug_skip & 0x1000u)  // timing probe: bulk without plaintext loads (wrong ciphertext)
            iv = cbc_bulk<NR, true, 1>(aes, k, iv, P, O, nb);
        else if (debug_skip & 0x2000u)  // timing probe: bulk without ciphertext stores
            iv = cbc_bulk<NR, true, 2>(aes, k, iv, P, O, nb);
        else if (IO16 && ((((uintptr_t)(pt + R.pt_off)) | (uintptr_t)(B + E)) & 15) == 0) {
            // 16-byte I/O for the 4-block groups, column words for the last nb % 4 blocks
            const uint32_t ng = nb >> 2;
            iv = cbc_bulk16<NR>(aes, k, iv, pt + R.pt_off, B + E, ng, q);
            iv = cbc_bulk<NR, true>(aes, k, iv, P + 64 * ng, O + 64 * ng, nb & 3);
        } else
            iv = al ? cbc_bulk<NR, true>(aes, k, iv, P, O, nb) : cbc_bulk<NR, false>(aes, k, iv, P, O, nb);
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
}

// ---------------------------------------------------------------------------
// cbc2_kernel: 8 waves x 16 quads, TWO chains per quad (ILP 2): the bulk blocks
// of the two chains' current records are encrypted interleaved round by round;
// explicit-IV and tail blocks (a few per record) run one chain at a time.  Same
// results as cbc_kernel; chosen when a CU holds more chains than one wave's
// issue slots can keep in flight (TLSGPU_CBC_ILP selects explicitly).
struct CbcCur {
    const tlsgpu_chain* ch;
    uint32_t first, count, j;  // chain records, next record index
    uint32_t r, n, nb, b, T, E;
    const uint8_t* P;
    uint8_t* O;
    uint8_t* Ot;
    const uint8_t* slot;
    bool al, active, done, any;
    uint32_t iv, fiv;
};

template <int NR>
struct Cbc2 {
    const tlsgpu_record* recs;
    const RecMeta* meta;
    const uint8_t* pt;
    uint8_t* wire;
    const uint8_t* tails;
    uint32_t nrecords, epoch, q, skip_bulk;
    QuadAes aes;

    // tail blocks of the current record, then inactive
    __device__ __forceinline__ void finish(CbcCur& c, const uint32_t* k) const {
        for (uint32_t off = 0; off < c.T; off += 16) {
            c.iv = aes.encrypt1<NR>(*(const uint32_t*)(c.slot + off) ^ c.iv, k);
            st32(c.Ot + off, c.iv, c.al);
        }
        c.active = false;
    }
    // move to the next sealable record: explicit-IV block, bulk cursor; records
    // without bulk blocks are finished on the spot
    __device__ __forceinline__ void advance(CbcCur& c, const uint32_t* k) const {
        while (!c.active && !c.done) {
            if (c.j >= c.count || c.first + c.j >= nrecords) {
                c.done = true;
                break;
            }
            const uint32_t r = c.first + c.j++;
            const RecMeta mt = meta[r];
            if (mt.epoch != epoch || mt.status != 1) continue;
            c.any = true;
            const tlsgpu_record R = recs[r];
            c.r = r;
            c.n = R.pt_len;
            uint8_t* B = wire + R.wire_off + 5;
            c.al = (((uintptr_t)(pt + R.pt_off) | (uintptr_t)B) & 3) == 0;
            if (c.E) {
                c.iv = aes.encrypt1<NR>(c.fiv ^ c.iv, k);
                st32(B + 4 * q, c.iv, c.al);
            }
            c.P = pt + R.pt_off + 4 * q;
            c.O = B + c.E + 4 * q;
            c.nb = skip_bulk ? 0u : (c.n >> 4);
            c.b = 0;
            const uint32_t r16 = c.n & 15;
            c.slot = tails + (size_t)r * TAIL_SLOT + 4 * q;
            c.Ot = B + c.E + (c.n - r16) + 4 * q;
            c.T = mt.tail_len;
            c.active = true;
            if (c.nb == 0) finish(c, k);
        }
    }
    // m bulk blocks of one chain (prefetch 8 ahead)
    __device__ __forceinline__ void bulk1(CbcCur& c, uint32_t m, const uint32_t* k) const {
        const uint8_t* P = c.P + 16 * c.b;
        uint8_t* O = c.O + 16 * c.b;
        uint32_t f[8];
#pragma unroll
        for (int i = 0; i < 8; i++) f[i] = (uint32_t)i < m ? ld32(P + 16 * i, c.al) : 0u;
        for (uint32_t b0 = 0; b0 < m; b0 += 8) {
            uint32_t x[8];
#pragma unroll
            for (int i = 0; i < 8; i++) x[i] = f[i];
#pragma unroll
            for (int i = 0; i < 8; i++) f[i] = b0 + 8 + i < m ? ld32(P + 16 * (b0 + 8 + i), c.al) : 0u;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (b0 + i < m) {
                    c.iv = aes.encrypt_w<NR>(__builtin_amdgcn_bitop3_b32(x[i], c.iv, k[0], 0x96), k);
                    st32(O + 16 * (b0 + i), c.iv, c.al);
                }
            }
        }
        c.b += m;
    }
    // m bulk blocks of both chains, interleaved (prefetch 4 ahead each)
    __device__ __forceinline__ void bulk2(CbcCur& a, const uint32_t* ka, CbcCur& b, const uint32_t* kb,
                                          uint32_t m) const {
        const uint8_t* Pa = a.P + 16 * a.b;
        const uint8_t* Pb = b.P + 16 * b.b;
        uint8_t* Oa = a.O + 16 * a.b;
        uint8_t* Ob = b.O + 16 * b.b;
        uint32_t fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            fa[i] = (uint32_t)i < m ? ld32(Pa + 16 * i, a.al) : 0u;
            fb[i] = (uint32_t)i < m ? ld32(Pb + 16 * i, b.al) : 0u;
        }
        for (uint32_t b0 = 0; b0 < m; b0 += 4) {
            uint32_t xa[4], xb[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                xa[i] = fa[i];
                xb[i] = fb[i];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const bool v = b0 + 4 + i < m;
                fa[i] = v ? ld32(Pa + 16 * (b0 + 4 + i), a.al) : 0u;
                fb[i] = v ? ld32(Pb + 16 * (b0 + 4 + i), b.al) : 0u;
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (b0 + i < m) {
                    uint32_t ya = __builtin_amdgcn_bitop3_b32(xa[i], a.iv, ka[0], 0x96);
                    uint32_t yb = __builtin_amdgcn_bitop3_b32(xb[i], b.iv, kb[0], 0x96);
#pragma unroll
                    for (int rr = 1; rr < NR; rr++) {
                        const uint32_t na = aes.round<0>(ya, ka[rr]);
                        const uint32_t nb2 = aes.round<0>(yb, kb[rr]);
                        ya = na;
                        yb = nb2;
                    }
                    a.iv = aes.last(ya, ka[NR]);
                    b.iv = aes.last(yb, kb[NR]);
                    st32(Oa + 16 * (b0 + i), a.iv, a.al);
                    st32(Ob + 16 * (b0 + i), b.iv, b.al);
                }
            }
        }
        a.b += m;
        b.b += m;
    }
};

constexpr int C2_THREADS = 512;  // 8 waves x 16 quads x 2 chains = 256 chains

template <int NR>
__global__ void __launch_bounds__(C2_THREADS, 1)
cbc2_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
            uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
            ConnState* __restrict__ states, const RecMeta* __restrict__ meta, const uint8_t* __restrict__ tails,
            uint32_t cpw, uint32_t epoch, uint32_t debug_skip) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t local = (threadIdx.x >> 6) * 16 + (lane >> 2);  // 0..127
    const uint32_t q = lane & 3;
    const uint32_t half = (cpw + 1) / 2;
    const uint32_t la = local, lb = local + half;
    const bool hasA = la < half && blockIdx.x * cpw + la < nchains;
    const bool hasB = lb < cpw && blockIdx.x * cpw + lb < nchains;
    if (!hasA) return;
    set_prio(prio_of(debug_skip, 4, 1));
    Cbc2<NR> E2;
    E2.recs = recs;
    E2.meta = meta;
    E2.pt = pt;
    E2.wire = wire;
    E2.tails = tails;
    E2.nrecords = nrecords;
    E2.epoch = epoch;
    E2.q = q;
    E2.skip_bulk = debug_skip & 1;
    E2.aes.init();
    CbcCur A, B;
    uint32_t ka[NR + 1], kb[NR + 1];
    ConnState* sa = states + chains[blockIdx.x * cpw + la].state;
    ConnState* sb = nullptr;
    {
        const tlsgpu_chain c = chains[blockIdx.x * cpw + la];
        A.first = c.first; A.count = c.count; A.j = 0;
        A.E = sa->explicit_iv ? 16u : 0u; A.iv = sa->iv[q]; A.fiv = sa->fixed_iv[q];
        A.active = false; A.done = false; A.any = false;
        QuadAes::round_keys<NR>(sa->ek, q, ka);
    }
    if (hasB) {
        const tlsgpu_chain c = chains[blockIdx.x * cpw + lb];
        sb = states + c.state;
        B.first = c.first; B.count = c.count; B.j = 0;
        B.E = sb->explicit_iv ? 16u : 0u; B.iv = sb->iv[q]; B.fiv = sb->fixed_iv[q];
        B.active = false; B.done = false; B.any = false;
        QuadAes::round_keys<NR>(sb->ek, q, kb);
    } else {
        B.done = true; B.active = false; B.any = false;
#pragma unroll
        for (int r = 0; r <= NR; r++) kb[r] = 0;
        B.iv = 0;
    }
    E2.advance(A, ka);
    E2.advance(B, kb);
    while (A.active || B.active) {
        if (A.active && B.active) {
            const uint32_t ra = A.nb - A.b, rb = B.nb - B.b;
            E2.bulk2(A, ka, B, kb, ra < rb ? ra : rb);
        } else if (A.active) {
            E2.bulk1(A, A.nb - A.b, ka);
        } else {
            E2.bulk1(B, B.nb - B.b, kb);
        }
        if (A.active && A.b == A.nb) {
            E2.finish(A, ka);
            E2.advance(A, ka);
        }
        if (B.active && B.b == B.nb) {
            E2.finish(B, kb);
            E2.advance(B, kb);
        }
    }
    if (A.any) sa->iv[q] = A.iv;
    if (hasB && B.any) sb->iv[q] = B.iv;
}

// ---------------------------------------------------------------------------
// cbcp_kernel: 16 waves x 32 lane PAIRS, 2 lanes per chain, up to 512 chains per
// workgroup.  Lane h holds AES state columns 2h and 2h+1: a round is 8 conflict-free
// T-table lookups per lane; each lane XORs, for each of its columns, the two terms it
// owns, and the two terms its partner needs (with the partner's round-key column
// folded in) cross over in ONE DPP swap per column (tools/aes_layout_microbench.hip:
// 84.9 ns/round at 256 chains per CU against 89.5 for the quad layout, 87 % of the
// LDS lookup floor at 512 chains per CU).  Plaintext / ciphertext move as 8-byte
// column pairs.  Same results as cbc_kernel.
constexpr int CP_THREADS = 1024;
constexpr int CP_CHAINS = 512;

__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {  // lane h <- lane h^1
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);
}

struct PairAes : QuadAes {
    // column j of the next state = T0[b0(s_j)] ^ T1[b1(s_j+1)] ^ T2[b2(s_j+2)] ^ T3[b3(s_j+3)] ^ k_j;
    // pk = the partner's key columns (round_keys_pair)
    __device__ __forceinline__ void round(uint32_t& a, uint32_t& b, uint32_t ka, uint32_t kb) const {
        const uint32_t a2 = look<2, 2>(a), b3 = look<3, 3>(b), a1 = look<1, 1>(a), b2 = look<2, 2>(b);
        const uint32_t a0 = look<0, 0>(a), b1 = look<1, 1>(b), b0 = look<0, 0>(b), a3 = look<3, 3>(a);
        const uint32_t sA = __builtin_amdgcn_bitop3_b32(a2, b3, ka, 0x96);
        const uint32_t sB = __builtin_amdgcn_bitop3_b32(a1, b2, kb, 0x96);
        a = (a0 ^ b1) ^ pair_swap(sA);
        b = (b0 ^ a3) ^ pair_swap(sB);
    }
    // final round: S-box byte B of s sits at byte B of table (B+2)&3
    __device__ __forceinline__ void last(uint32_t& a, uint32_t& b, uint32_t ka, uint32_t kb) const {
        const uint32_t ta0 = look<2, 0>(a), tb1 = look<3, 1>(b), ta2 = look<0, 2>(a), tb3 = look<1, 3>(b);
        const uint32_t tb0 = look<2, 0>(b), ta3 = look<1, 3>(a), ta1 = look<3, 1>(a), tb2 = look<0, 2>(b);
        const uint32_t oA = perm(tb1, ta0, 0x0c0c0500u);
        const uint32_t sA = perm(tb3, ta2, 0x07020c0cu) ^ ka;
        const uint32_t oB = perm(ta3, tb0, 0x070c0c00u);
        const uint32_t sB = perm(tb2, ta1, 0x0c06010cu) ^ kb;
        a = oA ^ pair_swap(sA);
        b = oB ^ pair_swap(sB);
    }
    // kw = own whitening columns; k[2r], k[2r+1] (r >= 1) = the partner's columns of round key r
    template <int NR>
    static __device__ __forceinline__ void round_keys(const uint32_t* ek, uint32_t h, uint32_t* k) {
        const uint32_t ca = 2 * h, pa = 2 - ca;
        k[0] = ek[ca];
        k[1] = ek[ca + 1];
#pragma unroll
        for (int r = 1; r <= NR; r++) {
            k[2 * r] = ek[4 * r + pa];
            k[2 * r + 1] = ek[4 * r + pa + 1];
        }
    }
    // one block whose input is already whitened
    template <int NR>
    __device__ __forceinline__ void encrypt_w(uint32_t& a, uint32_t& b, const uint32_t* k) const {
#pragma unroll
        for (int r = 1; r < NR; r++) round(a, b, k[2 * r], k[2 * r + 1]);
        last(a, b, k[2 * NR], k[2 * NR + 1]);
    }
};

template <bool AL>
__device__ __forceinline__ uint2 ld64t(const uint8_t* p) {
    if constexpr (AL) return *(const uint2*)p;
    return make_uint2(ld32t<false>(p), ld32t<false>(p + 4));
}
template <bool AL>
__device__ __forceinline__ void st64t(uint8_t* p, uint32_t a, uint32_t b) {
    if constexpr (AL) {
        *(uint2*)p = make_uint2(a, b);
    } else {
        st32t<false>(p, a);
        st32t<false>(p + 4, b);
    }
}

// CBC over nb full blocks (P / O include the lane's 8-byte column-pair offset); groups of
// 8 blocks with the next group prefetched, index clamped to the last block (cbc_bulk).
template <int NR, bool AL>
__device__ __forceinline__ void cbcp_bulk(const PairAes& aes, const uint32_t* k, uint32_t& ia, uint32_t& ib,
                                          const uint8_t* P, uint8_t* O, uint32_t nb) {
    if (nb == 0) return;
    const uint32_t last = nb - 1;
    uint2 f[8];
#pragma unroll
    for (int i = 0; i < 8; i++) f[i] = ld64t<AL>(P + 16 * ((uint32_t)i < last ? (uint32_t)i : last));
    uint32_t b0 = 0;
    for (; b0 + 8 <= nb; b0 += 8) {
        uint2 c[8];
#pragma unroll
        for (int i = 0; i < 8; i++) c[i] = f[i];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t b = b0 + 8 + i;
            f[i] = ld64t<AL>(P + 16 * (b < last ? b : last));
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            ia = __builtin_amdgcn_bitop3_b32(c[i].x, ia, k[0], 0x96);
            ib = __builtin_amdgcn_bitop3_b32(c[i].y, ib, k[1], 0x96);
            aes.encrypt_w<NR>(ia, ib, k);
            st64t<AL>(O + 16 * (b0 + i), ia, ib);
        }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        if (b0 + i < nb) {
            ia = __builtin_amdgcn_bitop3_b32(f[i].x, ia, k[0], 0x96);
            ib = __builtin_amdgcn_bitop3_b32(f[i].y, ib, k[1], 0x96);
            aes.encrypt_w<NR>(ia, ib, k);
            st64t<AL>(O + 16 * (b0 + i), ia, ib);
        }
    }
}

template <int NR>
__global__ void __launch_bounds__(CP_THREADS, 1)
cbcp_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
            uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
            ConnState* __restrict__ states, const RecMeta* __restrict__ meta, const uint8_t* __restrict__ tails,
            uint32_t cpw, uint32_t epoch, uint32_t debug_skip) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t local = (threadIdx.x >> 6) * 32 + (lane >> 1);
    const uint32_t h = lane & 1;
    const uint32_t cid = blockIdx.x * cpw + local;
    if (local >= cpw || cid >= nchains) return;  // both lanes of a pair leave together
    const tlsgpu_chain ch = chains[cid];
    ConnState* st = states + ch.state;
    set_prio(prio_of(debug_skip, 4, 1));
    PairAes aes;
    aes.init();
    uint32_t k[2 * (NR + 1)];
    PairAes::round_keys<NR>(st->ek, h, k);
    uint32_t ia = st->iv[2 * h], ib = st->iv[2 * h + 1];
    const uint32_t fa = st->fixed_iv[2 * h], fb = st->fixed_iv[2 * h + 1];
    const uint32_t E = st->explicit_iv ? 16u : 0u;
    bool any = false;
    for (uint32_t j = 0; j < ch.count; j++) {
        const uint32_t r = ch.first + j;
        if (r >= nrecords) break;
        const RecMeta mt = meta[r];
        if (mt.epoch != epoch || mt.status != 1) continue;
        any = true;
        const tlsgpu_record R = recs[r];
        const uint32_t n = R.pt_len;
        const uint8_t* P = pt + R.pt_off + 8 * h;
        uint8_t* B = wire + R.wire_off + 5;
        const bool al8 = (((uintptr_t)(pt + R.pt_off) | (uintptr_t)B) & 7) == 0;
        const bool al4 = (((uintptr_t)(pt + R.pt_off) | (uintptr_t)B) & 3) == 0;
        if (E) {  // E_K(fixedIVBlock ^ residue) (tlsrecordlayer.py:594-595)
            ia = fa ^ ia ^ k[0];
            ib = fb ^ ib ^ k[1];
            aes.encrypt_w<NR>(ia, ib, k);
            st32(B + 8 * h, ia, al4);
            st32(B + 8 * h + 4, ib, al4);
        }
        uint8_t* O = B + E + 8 * h;
        const uint32_t nb = (debug_skip & 1) ? 0u : (n >> 4);
        if (al8)
            cbcp_bulk<NR, true>(aes, k, ia, ib, P, O, nb);
        else
            cbcp_bulk<NR, false>(aes, k, ia, ib, P, O, nb);
        // tail blocks from the MAC kernel's slot
        const uint32_t r16 = n & 15;
        const uint8_t* slot = tails + (size_t)r * TAIL_SLOT + 8 * h;
        uint8_t* Ot = B + E + (n - r16) + 8 * h;
        const uint32_t T = mt.tail_len;
        for (uint32_t off = 0; off < T; off += 16) {
            const uint2 t = *(const uint2*)(slot + off);
            ia = t.x ^ ia ^ k[0];
            ib = t.y ^ ib ^ k[1];
            aes.encrypt_w<NR>(ia, ib, k);
            st32(Ot + off, ia, al4);
            st32(Ot + off + 4, ib, al4);
        }
    }
    if (any) {
        st->iv[2 * h] = ia;
        st->iv[2 * h + 1] = ib;
    }
}

// ---------------------------------------------------------------------------
// tdes8_kernel: 3DES-EDE-CBC (openssl_tripledes.py:23, FIPS 46-3) with 8 lanes per
// chain.  Lane j of a chain's 8-lane group evaluates ONE of the eight SP-box terms of
// the Feistel function (a rotate, a key XOR, a 6-bit extract and one conflict-free LDS
// lookup) and three DPP XOR steps (quad [1,0,3,2], quad [2,3,0,1], half-row mirror) sum
// the eight terms in every lane of the group, so a round's critical path is one
// lookup + three XORs instead of one lane issuing all eight lookups and their XOR chain.
// The (l, r) halves are replicated in the group's lanes; lanes 0/1 store the two
// ciphertext words.  128 chains per 1024-thread workgroup.  The MAC, the tail slot and
// the header come from prefix_kernel / mac_kernel<.., 8> as for AES.
constexpr int D8_THREADS = 1024;
constexpr int D8_CHAINS = D8_THREADS / 8;

struct Des8 {
    uint32_t base, sa;
    bool odd;
    __device__ __forceinline__ void init() {
        const uint32_t lane = __lane_id(), j = lane & 7;
        // SP table of each lane: j < 4 take bytes 0..3 of w = r ^ k_even (tables 7,5,3,1),
        // j >= 4 bytes 0..3 of v = rotr4(r) ^ k_odd = rotr4(r ^ rotl4(k_odd)) (tables 6,4,2,0)
        // -- des_rounds()
        const uint32_t K = j < 4 ? 7 - 2 * j : 6 - 2 * (j - 4);
        base = (lane & 31) * 4 + K * 8192;
        odd = j >= 4;
        // rotate so that the lane's 6 index bits (bit (j>=4 ? 4 : 0) + 8*(j&3) of t) land at bits 7..12
        sa = ((odd ? 4u : 0u) + 8 * (j & 3) + 25u) & 31u;
    }
    // this lane's key word for the SP lookup (odd words pre-rotated, see init)
    __device__ __forceinline__ uint32_t key(uint32_t even, uint32_t oddw) const {
        return odd ? ((oddw << 4) | (oddw >> 28)) : even;
    }
    // Feistel f of t = r ^ key, summed over the 8 lanes of the group
    __device__ __forceinline__ uint32_t f(uint32_t t) const {
        const uint32_t u = __builtin_amdgcn_alignbit(t, t, sa);
        uint32_t v = lds_read32((u & 0x1f80u) | base);
        v ^= quad_dpp<0xB1>(v);
        v ^= quad_dpp<0x4E>(v);
        v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);  // row_half_mirror
        return v;
    }
    // block as two big-endian words; kw[16p + i] = this lane's key word of pass p, round i.
    // The next round's t = r' ^ k = l ^ f ^ k is one 3-input XOR off the critical path's f.
    __device__ __forceinline__ void block(uint32_t& hi, uint32_t& lo, const uint32_t* kw) const {
        uint32_t l = hi, r = lo;
        des_ip(l, r);
        uint32_t t = r ^ kw[0];
#pragma unroll
        for (int g = 0; g < 48; g++) {
            const uint32_t fv = f(t);
            const uint32_t rn = l ^ fv;
            if (g % 16 != 15) {
                if (g + 1 < 48) t = __builtin_amdgcn_bitop3_b32(l, fv, kw[g + 1], 0x96);
                l = r;
                r = rn;
            } else {  // end of a DES pass: (l, r) = (R16, L16) feeds the next pass
                l = rn;
                if (g + 1 < 48) t = r ^ kw[g + 1];
            }
        }
        des_fp(l, r);
        hi = l;
        lo = r;
    }
    // CBC on LE words (TdesCbc::enc_block): c = E(p ^ iv), iv = c
    __device__ __forceinline__ void cbc(uint32_t d0, uint32_t d1, uint32_t& iv0, uint32_t& iv1,
                                        const uint32_t* kw) const {
        uint32_t hi = bswap32(d0 ^ iv0), lo = bswap32(d1 ^ iv1);
        block(hi, lo, kw);
        iv0 = bswap32(hi);
        iv1 = bswap32(lo);
    }
};

__global__ void __launch_bounds__(D8_THREADS, 1)
tdes8_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
             uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
             ConnState* __restrict__ states, const RecMeta* __restrict__ meta, const uint8_t* __restrict__ tails,
             uint32_t cpw, uint32_t epoch) {
    // SP tables at LDS offset 0 (the kernel's only LDS), read back by absolute address (Des8::f)
    extern __shared__ __attribute__((aligned(16))) uint32_t d8_lds[];
    des_lds_fill(d8_lds);
    __syncthreads();
    const uint32_t j = threadIdx.x & 7;
    const uint32_t local = threadIdx.x >> 3;
    const uint32_t cid = blockIdx.x * cpw + local;
    if (local >= cpw || cid >= nchains) return;  // the 8 lanes of a chain leave together
    const tlsgpu_chain ch = chains[cid];
    ConnState* st = states + ch.state;
    Des8 D;
    D.init();
    uint32_t kw[48];
#pragma unroll
    for (int p = 0; p < 3; p++)
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int k = p == 1 ? 15 - i : i;  // EDE: the middle pass decrypts (keys backwards)
            kw[16 * p + i] = D.key(st->des[p][2 * k], st->des[p][2 * k + 1]);
        }
    uint32_t iv0 = st->iv[0], iv1 = st->iv[1];
    const uint32_t f0 = st->fixed_iv[0], f1 = st->fixed_iv[1];
    const uint32_t E = st->explicit_iv ? 8u : 0u;
    bool any = false;
    for (uint32_t q = 0; q < ch.count; q++) {
        const uint32_t r = ch.first + q;
        if (r >= nrecords) break;
        const RecMeta mt = meta[r];
        if (mt.epoch != epoch || mt.status != 1) continue;
        any = true;
        const tlsgpu_record R = recs[r];
        const uint32_t n = R.pt_len;
        const uint8_t* P = pt + R.pt_off;
        uint8_t* B = wire + R.wire_off + 5;
        const bool al = (((uintptr_t)P | (uintptr_t)B) & 3) == 0;
        if (E) {  // E_K(fixedIVBlock ^ residue) (tlsrecordlayer.py:594-595)
            D.cbc(f0, f1, iv0, iv1, kw);
            if (j < 2) st32(B + 4 * j, j ? iv1 : iv0, al);
        }
        uint8_t* O = B + E;
        const uint32_t nb = n >> 3;
        uint32_t n0 = ld32(P, al), n1 = ld32(P + 4, al);
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t d0 = n0, d1 = n1;
            const uint32_t bn = b + 1 < nb ? b + 1 : b;  // prefetch, clamped to the last block
            n0 = ld32(P + 8 * bn, al);
            n1 = ld32(P + 8 * bn + 4, al);
            D.cbc(d0, d1, iv0, iv1, kw);
            if (j < 2) st32(O + 8 * b + 4 * j, j ? iv1 : iv0, al);
        }
        // tail blocks from the MAC kernel's slot
        const uint8_t* slot = tails + (size_t)r * TAIL_SLOT;
        uint8_t* Ot = O + 8 * nb;
        const uint32_t T = mt.tail_len;
        for (uint32_t off = 0; off < T; off += 8) {
            D.cbc(*(const uint32_t*)(slot + off), *(const uint32_t*)(slot + off + 4), iv0, iv1, kw);
            if (j < 2) st32(Ot + off + 4 * j, j ? iv1 : iv0, al);
        }
    }
    if (any && j < 2) st->iv[j] = j ? iv1 : iv0;
}

}  // namespace tg

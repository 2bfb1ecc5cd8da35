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
//                  lane, DPP quad exchange), one chain per quad -- the layout
//                  tools/aes_layout_microbench.hip measured best for 256 chains
//                  per CU.  No barriers: each quad streams its chain: explicit
//                  IV, full P blocks, then the tail slot.
//   tdes4_kernel   the 3DES cipher phase (4 lanes per chain).
//
// Workspace per record: 32 B meta + 64 B tail slot.  Kernels run in stream
// order (prefix -> mac -> cbc).  Wave priorities are fixed: the cipher waves
// (latency-bound CBC chains) at 1, the MAC waves (issue-bound) at 0, so when
// the pipeline runs the MAC phase of batch k+1 beside the cipher phase of
// batch k the cipher waves win issue arbitration.
#pragma once
#include "tg_quad.h"
#include <tg_config.h>

namespace tg {

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
constexpr int C3_THREADS = 64 * CFG_CBC_WAVES;  // 16 cipher waves
constexpr int C3_CHAINS = 16 * CFG_CBC_WAVES;
// Many-chains regime (more chains than one generation of 16-wave workgroups, cfg3): the MAC
// kernel at <= 128 VGPRs with a one-chunk prefetch.  Beside the pair cipher kernel (8 waves
// per CU, 89 VGPRs: 2 x 96 allocated per SIMD) two MAC waves per SIMD fit with either MAC
// form; the two-chunk ring at launch bound 3 (148 VGPRs) measured 1.5 % slower on cfg3 in
// round 4 (profiles/r04/ab/ab_cfg3_r04.txt).
constexpr int MAC_LB_MANY = CFG_MAC_LB_MANY, MAC_PF_MANY = CFG_MAC_PF_MANY;

template <int CIPHER_ID, int MAC, bool SSL3>
__global__ void __launch_bounds__(256) prefix_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                    const tlsgpu_record* __restrict__ recs,
                                                    ConnState* __restrict__ states, int32_t* __restrict__ wire_len,
                                                    RecMeta* __restrict__ meta, uint32_t nrecords, uint32_t epoch,
                                                    uint64_t pt_cap, uint64_t wire_cap, uint32_t nstates) {
    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    // a state index outside the caller's array: every record of the chain is refused and no
    // state is read (ABI 6)
    const bool sok = ch.state < nstates;
    ConnState* st = states + (sok ? ch.state : 0u);
    // the state's first 32 bytes in two 16-byte loads (one line request), tested without
    // short-circuit branches: field-by-field loads behind each comparison cost a dependent
    // memory latency apiece (cfg3: 1 Mi chains)
    uint4 h0 = make_uint4(0, 0, 0, 0), h1 = make_uint4(0, 0, 0, 0);
    if (sok) {
        h0 = *(const uint4*)st;                          // cipher, mac, vmaj..maclen, ssl3
        h1 = *(const uint4*)((const uint8_t*)st + 16);   // seqnum (lo, hi), explicit_iv, raw
    }
    static_assert(__builtin_offsetof(ConnState, mac) == 4 && __builtin_offsetof(ConnState, ssl3) == 12 &&
                      __builtin_offsetof(ConnState, seqnum) == 16 && __builtin_offsetof(ConnState, explicit_iv) == 24 &&
                      __builtin_offsetof(ConnState, raw) == 28,
                  "state header layout");
    const bool ok = sok & (h0.x == (uint32_t)CIPHER_ID) & (h0.y == (uint32_t)MAC) & (h0.w == (SSL3 ? 1u : 0u)) &
                    (h1.w == 0u);
    constexpr int DL = Hash<MAC>::DLEN;
    constexpr uint32_t BS = CIPHER_ID == TLSGPU_CIPHER_3DES ? 8u : 16u;
    uint64_t seq = (uint64_t)h1.x | ((uint64_t)h1.y << 32);
    const uint32_t E = h1.z ? BS : 0u;
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
            wire_len[r] = sok ? TLSGPU_EMISMATCH : TLSGPU_EINVAL;
        } else {
            const tlsgpu_record R = recs[r];
            const uint32_t n = R.pt_len;
            const uint32_t cur = E + n + DL;
            const uint32_t body = cur + (BS - (cur & (BS - 1)));
            if (n == 0) {
                wire_len[r] = 0;
            } else if (body > 0xffffu) {
                wire_len[r] = TLSGPU_ETOOBIG;
            } else if (!in_arena(R.pt_off, n, pt_cap) || !in_arena(R.wire_off, 5u + body, wire_cap)) {
                wire_len[r] = TLSGPU_EINVAL;  // the record would read / write outside the caller's arenas
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

// Tuning constants: tg_config.h (experiment builds replace it, tools/build_ab.sh).  Variants
// measured slower and not kept -- non-temporal loads / stores, v_perm byte-1 addresses,
// v_cndmask transposes, flat loads, the quad cipher layout in the throughput regimes, 12
// cipher waves with a 128-VGPR MAC kernel, the one-kernel seal (last in
// commit c22dfb8, tlslite_amd/csrc/tg_fused.h) -- are in DESIGN.md and profiles/r0{2,3,4}/.

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

// MAC over nfull 64-byte chunks at any byte alignment (round 6): the lane loads the whole
// 16-byte words its chunks overlap -- four per chunk, the window's first word carried over from
// the previous chunk -- and funnel-shifts its chunk out of them: v_alignbyte by the byte offset
// within a dword, then a dword select by the offset's dword index.  The generic load16 path
// had taken 64 byte loads per chunk, and a receive stream's records sit at any offset (bodies
// follow 5-byte headers): the receive pipeline's open MAC took 1.4 ms for 256 compressions.
// Reads stay inside the record body: the last window ends < 16 bytes past the last full
// chunk, which the MAC (>= 16 bytes) follows.
template <class M>
__device__ __forceinline__ void mac_bulk_unaligned(M& mac, const uint8_t* P, uint32_t nfull) {
    if (nfull == 0) return;
    const uintptr_t a = (uintptr_t)P;
    const uint4* B = (const uint4*)(a & ~(uintptr_t)15);
    const uint32_t sb = (uint32_t)(a & 3), q = (uint32_t)(a >> 2) & 3u;
    uint4 w0 = B[0];
    uint4 nx[4];
#pragma unroll
    for (int i = 0; i < 4; i++) nx[i] = B[1 + i];
    for (uint32_t c = 0; c < nfull; c++) {
        uint32_t W[20];
        W[0] = w0.x; W[1] = w0.y; W[2] = w0.z; W[3] = w0.w;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            W[4 + 4 * i] = nx[i].x; W[5 + 4 * i] = nx[i].y; W[6 + 4 * i] = nx[i].z; W[7 + 4 * i] = nx[i].w;
        }
        w0 = nx[3];
        const uint32_t cn = c + 1 < nfull ? c + 1 : c;  // clamped: no branch on the load
#pragma unroll
        for (int i = 0; i < 4; i++) nx[i] = B[4 * cn + 1 + i];
        uint32_t x[19];
#pragma unroll
        for (int k = 0; k < 19; k++) x[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], sb);
        uint32_t d[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t lo = (q & 1u) ? x[k + 1] : x[k];
            const uint32_t hi = (q & 1u) ? x[k + 3] : x[k + 2];
            d[k] = (q & 2u) ? hi : lo;
        }
        mac.update(d);
    }
}

// MAC over nfull 64-byte chunks with the next chunk prefetched; the prefetch index is
// clamped instead of guarded so the loop body has no branch on the load
template <bool AL16, class M>
__device__ __forceinline__ void mac_bulk(M& mac, const uint8_t* P, uint32_t nfull) {
    if constexpr (!AL16) {
        mac_bulk_unaligned(mac, P, nfull);
        return;
    }
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

constexpr int MAC_PF = CFG_MAC_PF;  // chunks prefetched ahead by the cooperative MAC loop

// 16-byte load through a global-address-space pointer: the quad's record pointers are
// rebuilt from DPP-exchanged integers, which the compiler would otherwise turn into
// flat_load (address space unknown)
__device__ __forceinline__ uint4 ldg16(const uint8_t* p) {
#if !defined(__HIP_DEVICE_COMPILE__)
    return *(const uint4*)p;
#else
    typedef __attribute__((address_space(1))) const uint32_t g_u32;
    const g_u32* g = (const g_u32*)(size_t)p;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)g;
    return make_uint4(v.x, v.y, v.z, v.w);
#endif
}

// value of v in lane L of the calling lane's quad
template <int L>
__device__ __forceinline__ uint32_t quad_lane(uint32_t v) {
    return quad_dpp<L * 0x55>(v);
}

// One butterfly stage of a 4x4 transpose across a quad (partner lane q ^ 1 for CTRL 0xB1,
// q ^ 2 for 0x4E): of the register pair (a, b) the lane keeps the element whose index
// bit equals its own bit `hi` and trades the other with the partner -- it sends exactly
// the element it overwrites.  3 VALU per pair (the DPP rides in the selects).
// the selects as v_bitop3 (m ? x : y, 2 cycles with all-VGPR operands) on a per-lane
// all-ones / all-zeros mask instead of v_cndmask on a lane mask in SGPRs (4 cycles)
template <int CTRL>
__device__ __forceinline__ void quad_bfly(uint32_t& a, uint32_t& b, uint32_t m) {
    const uint32_t r = quad_dpp<CTRL>(__builtin_amdgcn_bitop3_b32(m, a, b, 0xCA));
    const uint32_t na = __builtin_amdgcn_bitop3_b32(m, r, a, 0xCA);
    b = __builtin_amdgcn_bitop3_b32(m, b, r, 0xCA);
    a = na;
}
// lane p holds x[L] = M[L][p]  ->  lane q holds x[s] = M[q][s]   (4 DPP + 8 selects)
__device__ __forceinline__ void quad_transpose4(uint32_t x[4], uint32_t q) {
    const uint32_t m0 = 0u - (q & 1u), m1 = 0u - ((q >> 1) & 1u);
    quad_bfly<0xB1>(x[0], x[1], m0);
    quad_bfly<0xB1>(x[2], x[3], m0);
    quad_bfly<0x4E>(x[0], x[2], m1);
    quad_bfly<0x4E>(x[1], x[3], m1);
}

// Quad-cooperative chunk load: lane q fetches bytes [16q, 16q+16) of each quad member L's
// 64-byte chunk at src (member L's own pointer, exchanged over DPP) into nx[L].  Every lane of
// the quad must execute it; src must point at 64 readable bytes, 16-byte aligned.
__device__ __forceinline__ void coop_load(const uint8_t* src, uint32_t q, uint4 nx[4]) {
    const uint32_t lo = (uint32_t)(uintptr_t)src, hi = (uint32_t)((uintptr_t)src >> 32);
#define TG_QL(L) nx[L] = ldg16((const uint8_t*)(((uint64_t)quad_lane<L>(hi) << 32) | quad_lane<L>(lo)) + 16 * q);
    TG_QL(0) TG_QL(1) TG_QL(2) TG_QL(3)
#undef TG_QL
}
// The lane's own chunk words out of a coop_load ring slot: four 4x4 quad transposes
// (component t of lane p's piece of record L = record L's word 4p + t)
__device__ __forceinline__ void coop_transpose(const uint4 nx[4], uint32_t q, uint32_t d[16]) {
    uint32_t x[4];
    x[0] = nx[0].x; x[1] = nx[1].x; x[2] = nx[2].x; x[3] = nx[3].x;
    quad_transpose4(x, q);
    d[0] = x[0]; d[4] = x[1]; d[8] = x[2]; d[12] = x[3];
    x[0] = nx[0].y; x[1] = nx[1].y; x[2] = nx[2].y; x[3] = nx[3].y;
    quad_transpose4(x, q);
    d[1] = x[0]; d[5] = x[1]; d[9] = x[2]; d[13] = x[3];
    x[0] = nx[0].z; x[1] = nx[1].z; x[2] = nx[2].z; x[3] = nx[3].z;
    quad_transpose4(x, q);
    d[2] = x[0]; d[6] = x[1]; d[10] = x[2]; d[14] = x[3];
    x[0] = nx[0].w; x[1] = nx[1].w; x[2] = nx[2].w; x[3] = nx[3].w;
    quad_transpose4(x, q);
    d[3] = x[0]; d[7] = x[1]; d[11] = x[2]; d[15] = x[3];
}

// MAC over the 64-byte chunks of the quad's four records, loaded cooperatively: per load
// instruction lane q fetches bytes [16q, 16q+16) of record L's chunk, so a quad reads a
// record's 64 contiguous bytes with one instruction -- a wave touches 16 segments per load
// instead of 64 (the per-lane pattern's 64-segment loads crowd the CU's memory pipeline,
// which the concurrently running cipher phase shares).  Four 4x4 transposes (48 VALU per
// chunk, ~8 % of a SHA-1 block) hand every lane its own record's 16 words.  The quad walks
// its longest record; a lane compresses only its own chunks and loads never leave a
// record (chunk index clamped to the record's last one).  Needs nfull >= 1 in every lane.
template <int PF, class M>
__device__ __forceinline__ void mac_bulk_coop(M& mac, const uint8_t* P, uint32_t nfull, uint32_t q) {
    uint32_t nmax = max(nfull, quad_dpp<0xB1>(nfull));
    nmax = max(nmax, quad_dpp<0x4E>(nmax));
    const uint32_t lo = (uint32_t)(uintptr_t)P, hi = (uint32_t)((uintptr_t)P >> 32);
    const uint8_t* PL[4];
    uint32_t NL[4];
#define TG_QL(L)                                                                                       \
    PL[L] = (const uint8_t*)(((uint64_t)quad_lane<L>(hi) << 32) | quad_lane<L>(lo)) + 16 * q;            \
    NL[L] = quad_lane<L>(nfull) - 1;
    TG_QL(0) TG_QL(1) TG_QL(2) TG_QL(3)
#undef TG_QL
    // prefetch ring of PF chunks: under the cipher phase's HBM traffic a load takes longer
    // than one chunk's compression
    uint4 nxt[PF][4];
#pragma unroll
    for (int d = 0; d < PF; d++)
#pragma unroll
        for (int L = 0; L < 4; L++) {
            nxt[d][L] = ldg16(PL[L] + 64 * min((uint32_t)d, NL[L]));
        }
    // The loop is unrolled by PF with ring slot k fixed per unrolled step: slot k's chunk is
    // transposed out first and its registers reloaded straight away, so no register copies
    // rotate the ring (they were 32 v_mov per chunk, ~4 % of the MAC phase's issue cycles).
    for (uint32_t c0 = 0; c0 < nmax; c0 += PF) {
#pragma unroll
        for (int k = 0; k < PF; k++) {
            const uint32_t c = c0 + k;
            if (c >= nmax) break;
            uint32_t d[16];
            coop_transpose(nxt[k], q, d);
            // the ring is reloaded as a whole after its last slot is transposed: a record's
            // consecutive 64-B chunks (whole 128-B lines) are requested back to back rather than
            // one compression apart (cfg2 901-902 -> 916-918 GiB/s with PF = 2)
            if (k == PF - 1) {
#pragma unroll
                for (int kk = 0; kk < PF; kk++)
#pragma unroll
                    for (int L = 0; L < 4; L++) nxt[kk][L] = ldg16(PL[L] + 64 * min(c0 + kk + PF, NL[L]));
            }
            if (c < nfull) mac.update(d);
        }
    }
}

// Register budget: a MAC wave must fit beside four cbc_kernel waves on a SIMD
// (4 x 80 + 168 <= 512 VGPRs) for the pipeline to overlap the two phases: the launch
// bound's 3 waves per SIMD caps it at 168.
template <int MAC, bool SSL3, int BS = 16, int LB = CFG_MAC_LB, int PF = MAC_PF>
__global__ void __launch_bounds__(256, LB) mac_kernel(const tlsgpu_record* __restrict__ recs, uint32_t nrecords,
                                                 const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                                                 const ConnState* __restrict__ states, int32_t* __restrict__ wire_len,
                                                 const RecMeta* __restrict__ meta, uint8_t* __restrict__ tails,
                                                 uint32_t epoch, uint32_t r0) {
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    const uint32_t r = r0 + blockIdx.x * blockDim.x + threadIdx.x;  // records [r0, nrecords)
    // no early exit before the bulk: the lanes of a quad exchange loaded data (DPP)
    RecMeta mt = {};
    bool act = r < nrecords;
    if (act) {
        mt = meta[r];
        act = mt.epoch == epoch && mt.status == 1;
    }
    __builtin_amdgcn_s_setprio(CFG_MAC_PRIO);
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
    const uint32_t nfull = act ? n >> 6 : 0u;
    const bool al16 = ((uintptr_t)P & 15) == 0;
    // quad-cooperative loads when the quad's four records are sealed, 16-byte aligned and
    // at least one chunk long (a quad-uniform decision)
    uint32_t coop = (act && al16 && nfull) ? 1u : 0u;
    coop &= quad_dpp<0xB1>(coop);
    coop &= quad_dpp<0x4E>(coop);
    if (coop) {
        mac_bulk_coop<PF>(mac, P, nfull, threadIdx.x & 3u);
    } else if (act) {
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

// 8 blocks of CBC: take the prefetched column words f (blocks b0..b0+7), refill f with
// blocks b0+8..b0+15, then encrypt and store the 8 blocks.  CLAMP: the refill index is
// clamped to the last block (the record's final groups); otherwise the 8 loads are one
// base address + immediate offsets (fewer VGPRs and no per-block address arithmetic).
template <int NR, bool LAT, bool AL, bool CLAMP>
__device__ __forceinline__ uint32_t cbc_group8(const QuadAes& aes, const uint32_t* k, uint32_t iv,
                                               const uint8_t* P, uint8_t* O, uint32_t b0, uint32_t last,
                                               uint32_t f[8]) {
    uint32_t c[8];
#pragma unroll
    for (int i = 0; i < 8; i++) c[i] = f[i];
    if constexpr (CLAMP) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t b = b0 + 8 + i;
            f[i] = ld32t<AL>(P + 16 * (b < last ? b : last));
        }
    } else {
        const uint8_t* Pn = P + 16 * (b0 + 8);
#pragma unroll
        for (int i = 0; i < 8; i++) f[i] = ld32t<AL>(Pn + 16 * i);
    }
    uint8_t* Ob = O + 16 * b0;
    // the group's ciphertext is kept and stored at the group's end (round 5, as the pair
    // kernel's pcbc_group): a chain's eight 16-B pieces of a line reach the L2 together and
    // merge, instead of one piece per block ~4 us apart, which let partial lines be written
    // back early and again later (cfg4 PMC: 32.5 GB written for 17.2 GB of wire)
    uint32_t o[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        iv = aes.encrypt_w<NR, LAT>(__builtin_amdgcn_bitop3_b32(c[i], iv, k[0], 0x96), k);
        o[i] = iv;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) st32t<AL>(Ob + 16 * i, o[i]);
    return iv;
}

// CBC over nb full plaintext blocks of one chain (P / O include the lane's column offset):
// groups of 8 blocks with the next group's columns prefetched.  The first group is peeled
// off the loop: then every path into the loop header ends in the same memory-op pattern
// (8 loads, 8 stores), and the vmcnt wait the compiler puts at the header only covers the
// previous group's loads.  With the loop entered straight from the 8 prologue loads, the
// merged header wait was vmcnt(1) -- every 8 blocks the wave waited for the previous
// group's stores, which stalls the chain when HBM is loaded (the MAC phase's stream).
template <int NR, bool LAT, bool AL>
__device__ __forceinline__ uint32_t cbc_bulk(const QuadAes& aes, const uint32_t* k, uint32_t iv,
                                             const uint8_t* P, uint8_t* O, uint32_t nb) {
    if (nb == 0) return iv;
    // Records of at least 16 blocks first run the head blocks up to the output's next 128-B
    // boundary, so every group stores whole lines (round 5, as pcbc_bulk); the head's loads
    // are issued with the first group's.
    uint32_t head = 0;
    if (nb >= 16) {
        // the chain's block address, the same in the quad's four lanes (O carries the lane's
        // column offset 4q; the output need not be 16-byte aligned)
        const uint32_t ob = (uint32_t)(uintptr_t)O - 4u * (__lane_id() & 3u);
        head = ((128u - (ob & 127u)) & 127u) >> 4;
    }
    uint32_t hp[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        if ((uint32_t)i < head) hp[i] = ld32t<AL>(P + 16 * i);
    P += 16 * head;
    nb -= head;
    const uint32_t last = nb - 1;  // nb >= 16 - 7 here when head > 0
    uint32_t f[8];
#pragma unroll
    for (int i = 0; i < 8; i++) f[i] = ld32t<AL>(P + 16 * ((uint32_t)i < last ? (uint32_t)i : last));
#pragma unroll
    for (int i = 0; i < 8; i++)
        if ((uint32_t)i < head) {
            iv = aes.encrypt_w<NR, LAT>(__builtin_amdgcn_bitop3_b32(hp[i], iv, k[0], 0x96), k);
            st32t<AL>(O + 16 * i, iv);
        }
    O += 16 * head;
    uint32_t b0 = 0;
    if (nb >= 16) {
        // groups whose refill (blocks b0+8..b0+15) lies inside the record
        iv = cbc_group8<NR, LAT, AL, false>(aes, k, iv, P, O, 0, last, f);
        for (b0 = 8; b0 + 16 <= nb; b0 += 8) iv = cbc_group8<NR, LAT, AL, false>(aes, k, iv, P, O, b0, last, f);
    }
    if (b0 + 8 <= nb) {  // the last full group: refill clamped
        iv = cbc_group8<NR, LAT, AL, true>(aes, k, iv, P, O, b0, last, f);
        b0 += 8;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        if (b0 + i < nb) {
            iv = aes.encrypt_w<NR, LAT>(__builtin_amdgcn_bitop3_b32(f[i], iv, k[0], 0x96), k);
            st32t<AL>(O + 16 * (b0 + i), iv);
        }
    }
    return iv;
}

// LAT: the few-chains (latency) form of the round, QuadAes::round; the launcher picks it
// when a CU gets fewer chains than it has quads (cfg4), the throughput form otherwise
template <int NR, bool LAT, int WAVES = CFG_CBC_WAVES>
__global__ void __launch_bounds__(64 * WAVES, 1)
cbc_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
           uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
           ConnState* __restrict__ states, const RecMeta* __restrict__ meta, const uint8_t* __restrict__ tails,
           uint32_t cpw, uint32_t epoch, uint32_t nstates) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t local = (threadIdx.x >> 6) * 16 + (lane >> 2);
    const uint32_t q = lane & 3;
    // Few chains (cpw < 16, cfg4-like): the idle quads of the first wave mirror its live
    // quads -- same chain, same records, so they compute and store the same bytes to the
    // same addresses and write back the same state.  A full wave runs the dependent round
    // faster than a mostly masked one (cfg4 cipher phase 130 -> 115 cycles per round at 512
    // chains, the clock unchanged at 2.39 GHz).
    // Mirroring is only sound when every quad runs exactly one chain (one generation, in
    // lockstep with its mirror inside the wave): a mirror must never start a chain its
    // original is not running at the same time, or the two would race on st->iv and the
    // wire.  The launcher only picks this kernel form with cpw < C3_CHAINS chains per CU,
    // i.e. grid * cpw >= nchains; the guard keeps it so for any other caller.
    if (local >= cpw && (threadIdx.x >> 6) == 0 && (uint64_t)gridDim.x * cpw >= nchains) local %= cpw;
    if (local >= cpw) return;
    // the prefix kernel validated the state: any record it marked status 1 belongs to a matching state
    __builtin_amdgcn_s_setprio(CFG_CBC_PRIO);
    QuadAes aes;
    aes.init();
    // persistent over chain generations: with more chains than CUs x cpw (cfg3: 4,096 chains per
    // CU) a quad takes chain cid + gridDim.x * cpw next -- tables filled once per CU, no
    // workgroup drain / relaunch between generations (cfg3 cipher phase 2.96 -> 2.26 ms)
    for (uint32_t cid = blockIdx.x * cpw + local; cid < nchains; cid += gridDim.x * cpw) {
    const tlsgpu_chain ch = chains[cid];
    if (ch.state >= nstates) continue;  // refused by the prefix kernel (ABI 6): no state read
    ConnState* st = states + ch.state;
    uint32_t k[NR + 1];
    uint32_t iv = st->iv[q];
    const uint32_t fiv = st->fixed_iv[q];
    const uint32_t E = st->explicit_iv ? 16u : 0u;
    bool any = false;
    QuadAes::round_keys<NR, LAT>(st->ek, q, k);
    for (uint32_t j = 0; j < ch.count; j++) {
        const uint32_t r = ch.first + j;
        if (r >= nrecords) break;
        // the record descriptor is loaded with the meta entry, not behind its test (one memory
        // latency fewer at each record's start)
        const tlsgpu_record R = recs[r];
        const RecMeta mt = meta[r];
        asm volatile("" ::"v"(R.pt_off), "v"(R.wire_off), "v"(R.pt_len));
        if (mt.epoch != epoch || mt.status != 1) continue;
        any = true;
        const uint32_t n = R.pt_len;
        const uint8_t* P = pt + R.pt_off + 4 * q;
        uint8_t* B = wire + R.wire_off + 5;
        const bool al = (((uintptr_t)(pt + R.pt_off) | (uintptr_t)B) & 3) == 0;
        if (E) {
            iv = aes.encrypt1<NR, LAT>(fiv ^ iv, k);
            st32(B + 4 * q, iv, al);
        }
        uint8_t* O = B + E + 4 * q;
        const uint32_t nb = n >> 4;
        iv = al ? cbc_bulk<NR, LAT, true>(aes, k, iv, P, O, nb) : cbc_bulk<NR, LAT, false>(aes, k, iv, P, O, nb);
        // tail blocks from the MAC kernel's slot
        const uint32_t r16 = n & 15;
        const uint8_t* slot = tails + (size_t)r * TAIL_SLOT + 4 * q;
        uint8_t* Ot = B + E + (n - r16) + 4 * q;
        const uint32_t T = mt.tail_len;
        for (uint32_t off = 0; off < T; off += 16) {
            iv = aes.encrypt1<NR, LAT>(*(const uint32_t*)(slot + off) ^ iv, k);
            st32(Ot + off, iv, al);
        }
    }
    if (any) st->iv[q] = iv;
    }
}

// ---------------------------------------------------------------------------
// cbc_pair_kernel: the cipher phase with 2 lanes per chain (PairAes, tg_quad.h) for the
// throughput regimes (a CU gets at least a workgroup's worth of chains).  Lane h holds
// state columns 2h, 2h+1 and moves 8 bytes per block (one dwordx2 load and store).
// Same stream of work per chain as cbc_kernel: explicit IV, full P blocks in groups of
// 8 with the next group prefetched, the MAC kernel's tail slot.
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

// c = E(p ^ prev): (va, vb) is the chain's residue in, the ciphertext out
template <int NR>
__device__ __forceinline__ void pair_block(const PairAes& aes, const uint32_t* kw, const uint32_t* ka,
                                           const uint32_t* kb, uint32_t& va, uint32_t& vb, uint32_t pa, uint32_t pb) {
    uint32_t a = __builtin_amdgcn_bitop3_b32(pa, va, kw[0], 0x96);
    uint32_t b = __builtin_amdgcn_bitop3_b32(pb, vb, kw[1], 0x96);
    aes.encrypt_w<NR>(a, b, ka, kb);
    va = a;
    vb = b;
}

// Pair-kernel configurations (same-box A/Bs, profiles/r03/ab_pair_r03*.txt):
//   one generation (a CU gets exactly one workgroup of chains, cfg2): 8 waves, 8-block
//   prefetch groups (103 VGPRs; one 168-VGPR MAC wave per SIMD beside the two cipher
//   waves): cfg2 824 -> 855 GiB/s.  4-block groups (87 VGPRs) let a second MAC wave in,
//   which slows the cipher phase -- the step's critical path -- more than it helps (794).
//   many chains (cfg3): 8 waves, 4-block groups (95 VGPRs for AES-256) + two 128-VGPR MAC
//   waves per SIMD (the MAC phase is that regime's critical path): cfg3 523 -> 540 GiB/s.
constexpr int PAIR_WAVES = 8;
constexpr int PAIR_WAVES_MANY = CFG_PAIR_WAVES_MANY;  // waves per CU in the many-chains regime

// Issue-priority turns of the pair kernel's waves (round 5).  Two cipher waves share a SIMD
// (8 waves per CU: w and w + 4), and the SIMD's issue arbiter favours the older one at equal
// priority: it ran ahead, its partner lagged (per-wave loop time 157 vs 181 cycles per round
// in tools/aes_layout_microbench.hip's trace mode), and the CU's last rounds ran on the
// laggards alone.  Taking turns at the higher priority, one G-block group each, keeps the
// waves of a CU together (168-177 cycles per round): the cfg2-shaped loop 0.911 -> 0.882 ms
// alone, 0.943 -> 0.864 ms beside a SHA-1 co-runner (profiles/r05/trace_mb.txt).  Both turns
// stay above the MAC waves' priority (CFG_MAC_PRIO).
struct PrioTurn {
    uint32_t turn;  // group count + the wave's SIMD-pair parity
    __device__ __forceinline__ void init() { turn = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8) & 1u; }
    template <int G, int BASE = CFG_CBC_PRIO>
    __device__ __forceinline__ void tick() {
        // one-generation layout (cfg2, 8-block groups): 500 + 500-step cfg2 966 -> 983 GiB/s,
        // unchanged at 20 + 5; the many-chains form (cfg3, 4-block groups) measured 552 -> 548
        // (profiles/r05/ab_seal.txt), so it keeps the fixed priority
        if constexpr (G >= 8) {
            // wave-uniform (an SGPR, so the branch is a scalar one): inside a chain's group loop
            // the lanes of chains of different lengths would count differently, and a per-lane
            // condition issues both s_setprio arms
            turn = __builtin_amdgcn_readfirstlane(turn + 1u);
            if (turn & 1u) __builtin_amdgcn_s_setprio(BASE + 1);
            else __builtin_amdgcn_s_setprio(BASE);
        }
    }
};

template <int NR, int G, bool AL, bool CLAMP>
__device__ __forceinline__ void pcbc_group(const PairAes& aes, const uint32_t* kw, const uint32_t* ka,
                                           const uint32_t* kb, uint32_t& va, uint32_t& vb, const uint8_t* P,
                                           uint8_t* O, uint32_t b0, uint32_t last, uint2 f[G], PrioTurn& turns) {
    constexpr int PAIR_G = G;
    turns.tick<G>();
    uint2 c[PAIR_G];
#pragma unroll
    for (int i = 0; i < PAIR_G; i++) c[i] = f[i];
    if constexpr (CLAMP) {
#pragma unroll
        for (int i = 0; i < PAIR_G; i++) {
            const uint32_t b = b0 + PAIR_G + i;
            f[i] = ld64t<AL>(P + 16 * (b < last ? b : last));
        }
    } else {
        const uint8_t* Pn = P + 16 * (b0 + PAIR_G);
#pragma unroll
        for (int i = 0; i < PAIR_G; i++) f[i] = ld64t<AL>(Pn + 16 * i);
    }
    uint8_t* Ob = O + 16 * b0;
    // the group's ciphertext is kept in registers and stored at the group's end: the chain's
    // stores reach the L2 together and merge into whole lines (with aligned groups, pcbc_bulk)
    uint2 o[PAIR_G];
#pragma unroll
    for (int i = 0; i < PAIR_G; i++) {
        pair_block<NR>(aes, kw, ka, kb, va, vb, c[i].x, c[i].y);
        o[i] = make_uint2(va, vb);
    }
#pragma unroll
    for (int i = 0; i < PAIR_G; i++) st64t<AL>(Ob + 16 * i, o[i].x, o[i].y);
}

constexpr uint32_t PAIR_ALIGN_MIN = 16;  // blocks: records this long align their groups

template <int NR, int GI, bool AL>
__device__ __forceinline__ void pcbc_bulk(const PairAes& aes, const uint32_t* kw, const uint32_t* ka,
                                          const uint32_t* kb, uint32_t& va, uint32_t& vb, const uint8_t* P,
                                          uint8_t* O, uint32_t nb, PrioTurn& turns) {
    if (nb == 0) return;
    constexpr uint32_t G = GI;
    // Records of at least PAIR_ALIGN_MIN blocks first run the head blocks up to the output's
    // next (16 G)-byte boundary, so every group stores whole lines (G = 8) / sectors (G = 4).
    // The head's loads and the first group's are issued together: one exposed load latency per
    // record, as without the head (with the head's loads first, cfg3's 89-block records lost
    // more than the alignment gained).  Same-box A/B against one store per block as it
    // completed: cfg2 850-854 -> 908-911, cfg3 536-537 -> 551-553 GiB/s (profiles/r03/ab_pair.txt).
    uint32_t head = 0;
    if (nb >= PAIR_ALIGN_MIN) {
        constexpr uint32_t A = 16 * G;
        // the chain's block address, the same in both lanes of the pair (O carries the lane's
        // 8-byte column offset; an 8-byte-aligned output need not be 16-byte aligned: with the
        // offset masked off instead, the lanes of a pair could pick different heads)
        const uint32_t ob = (uint32_t)(uintptr_t)O - 8u * (__lane_id() & 1u);
        head = ((A - (ob & (A - 1))) & (A - 1)) >> 4;
        head = head < nb ? head : nb;
    }
    uint2 hp[G];
#pragma unroll
    for (int i = 0; i < (int)G; i++)
        if ((uint32_t)i < head) hp[i] = ld64t<AL>(P + 16 * i);
    const uint8_t* Pg = P + 16 * head;
    uint8_t* Og = O + 16 * head;
    const uint32_t ng = nb - head;
    const uint32_t last = ng ? ng - 1 : 0;
    uint2 f[G];
    if (ng) {
#pragma unroll
        for (int i = 0; i < (int)G; i++) f[i] = ld64t<AL>(Pg + 16 * ((uint32_t)i < last ? (uint32_t)i : last));
    }
#pragma unroll
    for (int i = 0; i < (int)G; i++)
        if ((uint32_t)i < head) {
            pair_block<NR>(aes, kw, ka, kb, va, vb, hp[i].x, hp[i].y);
            st64t<AL>(O + 16 * i, va, vb);
        }
    if (ng == 0) return;
    uint32_t b0 = 0;
    if (ng >= 2 * G) {  // first group peeled, as cbc_bulk
        pcbc_group<NR, GI, AL, false>(aes, kw, ka, kb, va, vb, Pg, Og, 0, last, f, turns);
        for (b0 = G; b0 + 2 * G <= ng; b0 += G)
            pcbc_group<NR, GI, AL, false>(aes, kw, ka, kb, va, vb, Pg, Og, b0, last, f, turns);
    }
    if (b0 + G <= ng) {
        pcbc_group<NR, GI, AL, true>(aes, kw, ka, kb, va, vb, Pg, Og, b0, last, f, turns);
        b0 += G;
    }
#pragma unroll
    for (int i = 0; i < (int)G; i++) {
        if (b0 + i < ng) {
            pair_block<NR>(aes, kw, ka, kb, va, vb, f[i].x, f[i].y);
            st64t<AL>(Og + 16 * (b0 + i), va, vb);
        }
    }
}

template <int NR, int WAVES, int G>
__global__ void __launch_bounds__(64 * WAVES, 1)
cbc_pair_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
                uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                ConnState* __restrict__ states, const RecMeta* __restrict__ meta, const uint8_t* __restrict__ tails,
                uint32_t cpw, uint32_t epoch, uint32_t nstates) {
    aes_lds_fill(nullptr, false);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t local = (threadIdx.x >> 6) * 32 + (lane >> 1);
    const uint32_t h = lane & 1;
    if (local >= cpw) return;  // both lanes of a pair leave together
    __builtin_amdgcn_s_setprio(CFG_CBC_PRIO);
    PairAes aes;
    aes.init();
    PrioTurn turns;
    turns.init();
    // persistent over chain generations (as cbc_kernel)
    for (uint32_t cid = blockIdx.x * cpw + local; cid < nchains; cid += gridDim.x * cpw) {
        const tlsgpu_chain ch = chains[cid];
        if (ch.state >= nstates) continue;  // refused by the prefix kernel (ABI 6): no state read
        ConnState* st = states + ch.state;
        uint32_t kw[2], ka[NR + 1], kb[NR + 1];
        PairAes::round_keys<NR>(st->ek, h, kw, ka, kb);
        uint32_t va = st->iv[2 * h], vb = st->iv[2 * h + 1];
        const uint32_t fa = st->fixed_iv[2 * h], fb = st->fixed_iv[2 * h + 1];
        const uint32_t E = st->explicit_iv ? 16u : 0u;
        bool any = false;
        for (uint32_t j = 0; j < ch.count; j++) {
            const uint32_t r = ch.first + j;
            if (r >= nrecords) break;
            // the record descriptor is loaded with the meta entry, not behind its test (one memory
            // latency fewer at each record's start)
            const tlsgpu_record R = recs[r];
            const RecMeta mt = meta[r];
            asm volatile("" ::"v"(R.pt_off), "v"(R.wire_off), "v"(R.pt_len));
            if (mt.epoch != epoch || mt.status != 1) continue;
            any = true;
            const uint32_t n = R.pt_len;
            const uint8_t* P = pt + R.pt_off + 8 * h;
            uint8_t* B = wire + R.wire_off + 5;
            const bool al = (((uintptr_t)(pt + R.pt_off) | (uintptr_t)B) & 7) == 0;
            if (E) {  // E_K(fixedIVBlock ^ residue) (tlsrecordlayer.py:594-595)
                pair_block<NR>(aes, kw, ka, kb, va, vb, fa, fb);
                if (al) st64t<true>(B + 8 * h, va, vb);
                else st64t<false>(B + 8 * h, va, vb);
            }
            uint8_t* O = B + E + 8 * h;
            const uint32_t nb = n >> 4;
            if (al) pcbc_bulk<NR, G, true>(aes, kw, ka, kb, va, vb, P, O, nb, turns);
            else pcbc_bulk<NR, G, false>(aes, kw, ka, kb, va, vb, P, O, nb, turns);
            // tail blocks from the MAC kernel's slot (8-byte aligned)
            const uint32_t r16 = n & 15;
            const uint8_t* slot = tails + (size_t)r * TAIL_SLOT + 8 * h;
            uint8_t* Ot = B + E + (n - r16) + 8 * h;
            const uint32_t T = mt.tail_len;
            for (uint32_t off = 0; off < T; off += 16) {
                const uint2 p = *(const uint2*)(slot + off);
                pair_block<NR>(aes, kw, ka, kb, va, vb, p.x, p.y);
                if (al) st64t<true>(Ot + off, va, vb);
                else st64t<false>(Ot + off, va, vb);
            }
        }
        if (any) {
            st->iv[2 * h] = va;
            st->iv[2 * h + 1] = vb;
        }
    }
}

// ---------------------------------------------------------------------------
// tdes4_kernel: 3DES-EDE-CBC (openssl_tripledes.py:23, FIPS 46-3) with 4 lanes per
// chain.  The Feistel function is eight SP-box lookups, four indexed by the bytes of
// w = r ^ k_even (tables 7,5,3,1) and four by the bytes of v = rotr4(r) ^ k_odd =
// rotr4(r ^ rotl4(k_odd)) (tables 6,4,2,0) -- des_rounds().  Lane j of a chain's quad
// covers byte j of both: ONE lookup in a combined table (Des4C below) returns the XOR of
// its even and odd SP terms, and two DPP XOR steps (quad [1,0,3,2], quad [2,3,0,1]) sum
// the four lanes' terms in every lane of the quad.  A round's critical path: one LDS read
// -> two DPP XORs -> rotate f into the lane's frame -> one v_bitop3 (the key and table-base
// part of the next address is formed before f returns).  (4 lanes per chain with
// two lookups each measured 6.24 vs 7.25 ms against 8 lanes with one, round 2,
// tools/des_layout_microbench.hip.)  (l, r) are replicated in the quad; lanes 0/1 store
// the two ciphertext words.  Up to 128 chains per 512-thread workgroup.  The MAC, the tail
// slot and the header come from prefix_kernel / mac_kernel<.., 8> as for AES.
constexpr int D4_THREADS = 512;
constexpr int D4_CHAINS = D4_THREADS / 4;

// tdes4_kernel's tables (round 3, "combined"): lane j's even index (bits 8j..8j+5 of r ^ k_even) and odd index
// (bits 8j+4..8j+9 of r ^ rotl4(k_odd)) both lie in the 10-bit window x = bits 8j..8j+9 of
// t = r ^ Kc_j, where Kc_j takes k_even's bits on 8j..8j+5 and rotl4(k_odd)'s on 8j+6..8j+9.
// The two window bits both indices share (8j+4, 8j+5) see different key bits; their
// difference d (2 key bits per lane and round) selects one of four tables:
//   C_j[d][x] = SP[7-2j][x & 63] ^ SP[6-2j][((x >> 4) & 63) ^ d]
// so a lane does ONE lookup per round (address: v_alignbit + v_bitop3 with the round's
// per-lane base j*4 + d*16K), and the eight-term f is that lookup + the two DPP XOR steps.
// 4 lanes x 4 d x 1024 x 4 B = 64 KiB, one copy (the 10-bit windows are random: bank
// conflicts, PMC 0.7 of the LDS cycles; the kernel is latency-bound and a conflict adds a
// few cycles to one read).  Replaces round 2's
// two lookups per lane (32-copy SP tables; round 3's byte-row tables for the even half):
// cfg5 164.2 -> 193.9 GiB/s, tdes4 6.08 -> 5.15 ms (same-box A/B, profiles/r03/ab_des.txt).
// Layout: lane j's index bits sit in the address's bank bits (dword j + 4x + 4096d), so only
// lanes of one j can collide: a half-wave's 8 lanes of each j share 8 banks instead of all 32
// lanes sharing 32 (cfg5 5.147 -> 5.105 ms; a second copy in bank bit 4, 128 KiB: 5.86 ms;
// profiles/r03/ab_des.txt).
constexpr uint32_t D4_LDS_BYTES = 65536u;
__device__ __forceinline__ void des_lds_fill_comb(uint32_t* lds) {
    for (uint32_t idx = threadIdx.x; idx < D4_LDS_BYTES / 4; idx += blockDim.x) {
        const uint32_t j = idx & 3, x = (idx >> 2) & 1023, d = idx >> 12;
        lds[idx] = c_des.sp[7 - 2 * j][x & 63] ^ c_des.sp[6 - 2 * j][((x >> 4) & 63) ^ d];
    }
}
struct Des4C {
    uint32_t s, m;
    __device__ __forceinline__ void init() {
        const uint32_t j = __lane_id() & 3;
        s = (8 * j + 28) & 31;  // rotr by 8j - 4: window bit 8j -> address bit 4
        m = vconst(0x3ff0u);
    }
    // round constants of lane j from the round's even and (unrotated) odd key words
    static __device__ __forceinline__ void key(uint32_t ke, uint32_t ko, uint32_t j, uint32_t& kc, uint32_t& kb) {
        const uint32_t ko4 = (ko << 4) | (ko >> 28);
        const uint32_t sh = 8 * j, so = (8 * j + 6) & 31;
        const uint32_t me = 63u << sh, mo = (15u << so) | (15u >> (32 - so));  // rotl(15, so)
        kc = (ke & me) | (ko4 & mo);
        kb = j * 4u + (((ke ^ ko4) >> (sh + 4)) & 3u) * 16384u;
    }
    // one round constant per lane and round: the round's address bits outside the window (its
    // table base) and the key bits inside it, in the lane's rotated frame
    static __device__ __forceinline__ uint32_t key2(uint32_t ke, uint32_t ko, uint32_t j) {
        uint32_t kc, kb;
        key(ke, ko, j, kc, kb);
        const uint32_t s = (8 * j + 28) & 31;
        return (((kc >> s) | (kc << (32 - s))) & 0x3ff0u) | kb;
    }
    // 48 rounds in the lane's rotated frame (L, R) = (rotr(l, s), rotr(r, s)): the next
    // round's address is x ^ (rotr(f, s) & m) with x = (L & m) ^ B2 formed before f returns,
    // so after the last DPP XOR only the rotate of f and one v_bitop3 precede the next read
    // (against a 3-input key XOR, the rotate and the mask before: cfg5 5.11 -> 5.00 ms)
    __device__ __forceinline__ void block(uint32_t& hi, uint32_t& lo, const uint32_t* b2) const {
        uint32_t l = hi, r = lo;
        des_ip(l, r);
        uint32_t L = __builtin_amdgcn_alignbit(l, l, s), R = __builtin_amdgcn_alignbit(r, r, s);
        uint32_t addr = __builtin_amdgcn_bitop3_b32(R, m, b2[0], 0x6A);  // (R & m) ^ b2
#pragma unroll
        for (int g = 0; g < 48; g++) {
            uint32_t v = lds_read32(addr);
            v ^= quad_dpp<0xB1>(v);
            v ^= quad_dpp<0x4E>(v);
            const uint32_t y = __builtin_amdgcn_alignbit(v, v, s);
            const uint32_t rn = L ^ y;
            if (g % 16 != 15) {
                if (g + 1 < 48)
                    addr = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(L, m, b2[g + 1], 0x6A), y, m,
                                                       0x78);  // x ^ (y & m)
                L = R;
                R = rn;
            } else {  // end of a DES pass: (l, r) = (R16, L16) feeds the next pass
                L = rn;
                if (g + 1 < 48) addr = __builtin_amdgcn_bitop3_b32(R, m, b2[g + 1], 0x6A);
            }
        }
        l = __builtin_amdgcn_alignbit(L, L, 32 - s);
        r = __builtin_amdgcn_alignbit(R, R, 32 - s);
        des_fp(l, r);
        hi = l;
        lo = r;
    }
    __device__ __forceinline__ void cbc(uint32_t d0, uint32_t d1, uint32_t& iv0, uint32_t& iv1,
                                        const uint32_t* b2) const {
        uint32_t hi = bswap32(d0 ^ iv0), lo = bswap32(d1 ^ iv1);
        block(hi, lo, b2);
        iv0 = bswap32(hi);
        iv1 = bswap32(lo);
    }
};

__global__ void __launch_bounds__(D4_THREADS, 1)
tdes4_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
             uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
             ConnState* __restrict__ states, const RecMeta* __restrict__ meta, const uint8_t* __restrict__ tails,
             uint32_t cpw, uint32_t epoch, uint32_t nstates) {
    // combined tables at LDS offset 0 (the kernel's only LDS), read back by absolute address (Des4C::f)
    extern __shared__ __attribute__((aligned(16))) uint32_t d4_lds[];
    des_lds_fill_comb(d4_lds);
    __syncthreads();
    const uint32_t j = threadIdx.x & 3;
    const uint32_t local = threadIdx.x >> 2;
    const uint32_t cid = blockIdx.x * cpw + local;
    if (local >= cpw || cid >= nchains) return;  // the 4 lanes of a chain leave together
    const tlsgpu_chain ch = chains[cid];
    if (ch.state >= nstates) return;  // refused by the prefix kernel (ABI 6): no state read
    ConnState* st = states + ch.state;
    Des4C D;
    D.init();
    // the two waves of a SIMD take turns at the higher issue priority, one 8-block group each
    // (as cbc_pair_kernel: 8 waves per CU, w and w + 4 on one SIMD)
    PrioTurn turns;
    turns.init();
    uint32_t b2[48];  // per round: the lane's key / table-base word (Des4C::key2)
#pragma unroll
    for (int p = 0; p < 3; p++)
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int k = p == 1 ? 15 - i : i;  // EDE: the middle pass decrypts (keys backwards)
            b2[16 * p + i] = Des4C::key2(st->des[p][2 * k], st->des[p][2 * k + 1], j);
        }
    uint32_t iv0 = st->iv[0], iv1 = st->iv[1];
    const uint32_t f0 = st->fixed_iv[0], f1 = st->fixed_iv[1];
    const uint32_t E = st->explicit_iv ? 8u : 0u;
    bool any = false;
    for (uint32_t q = 0; q < ch.count; q++) {
        const uint32_t r = ch.first + q;
        if (r >= nrecords) break;
        // the record descriptor is loaded with the meta entry, not behind its test (one memory
        // latency fewer at each record's start)
        const tlsgpu_record R = recs[r];
        const RecMeta mt = meta[r];
        asm volatile("" ::"v"(R.pt_off), "v"(R.wire_off), "v"(R.pt_len));
        if (mt.epoch != epoch || mt.status != 1) continue;
        any = true;
        const uint32_t n = R.pt_len;
        const uint8_t* P = pt + R.pt_off;
        uint8_t* B = wire + R.wire_off + 5;
        const bool al = (((uintptr_t)P | (uintptr_t)B) & 3) == 0;
        if (E) {  // E_K(fixedIVBlock ^ residue) (tlsrecordlayer.py:594-595)
            D.cbc(f0, f1, iv0, iv1, b2);
            if (j < 2) st32(B + 4 * j, j ? iv1 : iv0, al);
        }
        uint8_t* O = B + E;
        const uint32_t nb = n >> 3;
        uint32_t n0 = ld32(P, al), n1 = ld32(P + 4, al);
        uint32_t b = 0;
        // head blocks up to the output's next 64-B sector, so every group stores whole sectors
        uint32_t head = ((64u - ((uint32_t)(uintptr_t)O & 63u)) & 63u) >> 3;
        head = head < nb ? head : nb;
        for (; b < head; b++) {
            const uint32_t d0 = n0, d1 = n1;
            const uint32_t bn = b + 1 < nb ? b + 1 : b;  // prefetch, clamped to the last block
            n0 = ld32(P + 8 * bn, al);
            n1 = ld32(P + 8 * bn + 4, al);
            D.cbc(d0, d1, iv0, iv1, b2);
            if (j < 2) st32(O + 8 * b + 4 * j, j ? iv1 : iv0, al);
        }
        // groups of 8 blocks: every lane of the quad holds each block's two ciphertext words;
        // lane j keeps blocks 2j, 2j+1 of the group and stores their 16 bytes at the group's end
        // (one 64-B piece per chain per group instead of 8 B per block as it completed: the
        // L2 merges whole sectors; cfg5 199.8 -> 210.5 GiB/s, tdes4 5.00 -> 4.74 ms)
        for (; b + 8 <= nb; b += 8) {
            turns.tick<8, 0>();  // 1 / 0: the RC4 kernel beside it (cfg5) runs at 0
            uint32_t k0 = 0, k1 = 0, k2 = 0, k3 = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint32_t d0 = n0, d1 = n1;
                const uint32_t bn = b + i + 1 < nb ? b + i + 1 : b + i;  // prefetch, clamped to the last block
                n0 = ld32(P + 8 * bn, al);
                n1 = ld32(P + 8 * bn + 4, al);
                D.cbc(d0, d1, iv0, iv1, b2);
                if (i & 1) {
                    k2 = j == (uint32_t)(i >> 1) ? iv0 : k2;
                    k3 = j == (uint32_t)(i >> 1) ? iv1 : k3;
                } else {
                    k0 = j == (uint32_t)(i >> 1) ? iv0 : k0;
                    k1 = j == (uint32_t)(i >> 1) ? iv1 : k1;
                }
            }
            uint8_t* Og = O + 8 * (b + 2 * j);
            st32(Og, k0, al);
            st32(Og + 4, k1, al);
            st32(Og + 8, k2, al);
            st32(Og + 12, k3, al);
        }
        for (; b < nb; b++) {
            const uint32_t d0 = n0, d1 = n1;
            const uint32_t bn = b + 1 < nb ? b + 1 : b;  // prefetch, clamped to the last block
            n0 = ld32(P + 8 * bn, al);
            n1 = ld32(P + 8 * bn + 4, al);
            D.cbc(d0, d1, iv0, iv1, b2);
            if (j < 2) st32(O + 8 * b + 4 * j, j ? iv1 : iv0, al);
        }
        // tail blocks from the MAC kernel's slot
        const uint8_t* slot = tails + (size_t)r * TAIL_SLOT;
        uint8_t* Ot = O + 8 * nb;
        const uint32_t T = mt.tail_len;
        for (uint32_t off = 0; off < T; off += 8) {
            D.cbc(*(const uint32_t*)(slot + off), *(const uint32_t*)(slot + off + 4), iv0, iv1, b2);
            if (j < 2) st32(Ot + off + 4 * j, j ? iv1 : iv0, al);
        }
    }
    if (any && j < 2) st->iv[j] = j ? iv1 : iv0;
}

}  // namespace tg

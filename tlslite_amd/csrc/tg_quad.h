// tg_quad.h -- the AES round laid out for a CDNA4 quad of lanes.
//
// 4 lanes per AES block ("quad"): lane q holds state column q.  A round is 4
// conflict-free LDS T-table lookups per lane (one v_perm_b32 builds each
// address from the state word and a per-lane bank-copy offset) combined by an
// XOR tree across the quad whose lane exchanges ride in the DPP operand of
// v_xor_b32 (rijndael.py:304-310 restated for the quad).
//
// LDS: [0, 128K) the 4 T-tables x 32 lane copies in the layout of aes_lds_fill
// (T0/T1 rows in the low 64K, T2/T3 in the high 64K).
#pragma once
#include "tg_device.h"

namespace tg {

typedef __attribute__((address_space(3))) uint32_t lds_u32_t;

__device__ __forceinline__ uint32_t lds_read32(uint32_t addr) { return *(const lds_u32_t*)(size_t)addr; }

// v_xor_b32_dpp-able quad permutation.  bound_ctrl set: every lane of a quad_perm reads
// an in-range lane, so the "old" operand is never used and the compiler needs no zeroed
// destination register for an unfolded v_mov_b32_dpp (it kept 16 of them live in the
// cipher loop, plus a v_mov each, when the final round's masks blocked the fold).
template <int CTRL>
__device__ __forceinline__ uint32_t quad_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}

// A VGPR holding a constant: gfx950 issues v_bitop3_b32 and the plain VOP2 logic ops in 2
// cycles per wave64 only when every operand is a VGPR (or an inline / literal constant);
// an SGPR operand, a DPP modifier, v_perm_b32, v_alignbit_b32, v_add3_u32 or v_lshlrev_b32
// take 4 (tools/valu_rate_microbench.hip, 4 waves per SIMD).
__device__ __forceinline__ uint32_t vconst(uint32_t c) {
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "i"(c));
    return v;
}

struct QuadAes {
    uint32_t lo, hi;  // lane-copy offset words (table pair select in byte 2)
    uint32_t m8;      // 0xff00 in a VGPR (byte-1 address mask)
    __device__ __forceinline__ void init() {
        lo = (__lane_id() & 31) * 4;
        hi = lo | 0x10000u;
        m8 = vconst(0xff00u);
    }
    template <int T, int B>  // T_t[byte B of s]
    __device__ __forceinline__ uint32_t look(uint32_t s) const {
        if constexpr (B == 1) {
            // byte 1 already sits at the row-index bits: (s & 0xff00) | base, one 2-cycle
            // v_bitop3 instead of a 4-cycle v_perm
            return lds_read32(__builtin_amdgcn_bitop3_b32(s, m8, T >= 2 ? hi : lo, 0xEA) + (T & 1) * 128);
        }
        constexpr uint32_t sel = 0x0c000000u | (2u << 16) | ((4u + B) << 8) | 0u;
        return lds_read32(perm(s, T >= 2 ? hi : lo, sel) + (T & 1) * 128);
    }
    // Column q of the next state = T0[b0(q)] ^ T1[b1(q+1)] ^ T2[b2(q+2)] ^ T3[b3(q+3)] ^ k[q], with
    // the lookup of byte b done by lane q+b.  XOR tree: dpp2(t2) ^ dpp3(t3) = dpp2(t2 ^ dpp1(t3)),
    // and the round key rides in that inner term: k2 is the key column of lane q+2 (round_keys()),
    // so once the T0/T1 lookups return only two dependent DPP XORs remain (a chain needs four).
    // The T2/T3 lookups are issued first: they feed the inner term.
    //
    // LAT (the few-chains regime, a lone wave per SIMD, cfg4): w = dpp2(u) is moved while the
    // T0/T1 lookups are still in flight (the scheduling barrier keeps it there; a DPP reading
    // a VGPR written just before needs two wait states, which a fused v_xor_b32_dpp would put
    // on the critical path: cfg4 129.6 -> 125.9 ms in round 2), and the round key goes into the
    // LAST instruction instead, a 3-input XOR of z, w = dpp2(t2 ^ dpp1(t3)) and the lane's
    // own key column: the T2/T3 half (issued first) is xor_dpp -> mov_dpp, hidden under
    // the T0/T1 lookups, and only z = t0 ^ dpp1(t1) and the final v_bitop3 follow the last
    // lookup.  Same 4 VALU as the throughput form (whose separate key XOR it drops).  For a
    // lone wave (tools/aes_round_latency.hip, profiles/r03/round_latency_*.log) a dependent
    // VALU step costs ~9 cycles, a DPP one ~12, an LDS lookup ~51: the round is ~106 cycles
    // (cfg4/512 123.1 -> 122.3 ms).  Issuing the four address ops before the four reads
    // (sched_group_barrier) made it 110.5 (128.2 ms): the reads interleaved with their
    // addresses go out sooner.
    template <bool LAT>
    __device__ __forceinline__ uint32_t round(uint32_t x, uint32_t k) const {
        const uint32_t t2 = look<2, 2>(x);
        const uint32_t t3 = look<3, 3>(x);
        const uint32_t t0 = look<0, 0>(x);
        const uint32_t t1 = look<1, 1>(x);
        if constexpr (!LAT) {  // k = key column q+2 (round_keys<NR, false>)
            const uint32_t u = (t2 ^ k) ^ quad_dpp<0x39>(t3);
            const uint32_t z = t0 ^ quad_dpp<0x39>(t1);
            return z ^ quad_dpp<0x4E>(u);
        } else {  // k = key column q (round_keys<NR, true>)
            const uint32_t w = quad_dpp<0x4E>(t2 ^ quad_dpp<0x39>(t3));
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t z = t0 ^ quad_dpp<0x39>(t1);
            return __builtin_amdgcn_bitop3_b32(z, w, k, 0x96);
        }
    }
    // per-lane round keys in the layout round()/last() expect: k[0] = whitening column q,
    // k[r >= 1] = column (q+2)&3 of round key r (throughput form) / column q (LAT)
    template <int NR, bool LAT = false>
    static __device__ __forceinline__ void round_keys(const uint32_t* ek, uint32_t q, uint32_t* k) {
        k[0] = ek[q];
#pragma unroll
        for (int r = 1; r <= NR; r++) k[r] = ek[4 * r + (LAT ? q : ((q + 2) & 3))];
    }
    template <bool LAT>
    __device__ __forceinline__ uint32_t last(uint32_t x, uint32_t k) const {
        // S-box byte r sits at byte r of table (r+2)&3
        const uint32_t s2 = look<0, 2>(x) & 0xff0000u;
        const uint32_t s3 = look<1, 3>(x) & 0xff000000u;
        const uint32_t s0 = look<2, 0>(x) & 0xffu;
        const uint32_t s1 = look<3, 1>(x) & 0xff00u;
        if constexpr (!LAT) {
            const uint32_t u = (s2 ^ k) ^ quad_dpp<0x39>(s3);
            const uint32_t z = s0 ^ quad_dpp<0x39>(s1);
            return z ^ quad_dpp<0x4E>(u);
        } else {
            const uint32_t w = quad_dpp<0x4E>(s2 ^ quad_dpp<0x39>(s3));
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t z = s0 ^ quad_dpp<0x39>(s1);
            return __builtin_amdgcn_bitop3_b32(z, w, k, 0x96);
        }
    }
    // one block of one chain
    template <int NR, bool LAT>
    __device__ __forceinline__ uint32_t encrypt1(uint32_t a, const uint32_t* ka) const {
        a ^= ka[0];
#pragma unroll
        for (int r = 1; r < NR; r++) a = round<LAT>(a, ka[r]);
        return last<LAT>(a, ka[NR]);
    }
    // one block whose input is already whitened (x = block ^ k[0])
    template <int NR, bool LAT>
    __device__ __forceinline__ uint32_t encrypt_w(uint32_t a, const uint32_t* ka) const {
#pragma unroll
        for (int r = 1; r < NR; r++) a = round<LAT>(a, ka[r]);
        return last<LAT>(a, ka[NR]);
    }
};

// The AES round for 2 lanes per block ("pair"): lane h holds state columns a = 2h and
// b = 2h+1.  Column j of the next state = T0[b0(s_j)] ^ T1[b1(s_j+1)] ^ T2[b2(s_j+2)] ^
// T3[b3(s_j+3)] ^ k_j (rijndael.py:304-310): of the 16 lookups the lane does the 8 that
// read its own two columns; 4 of them belong to its own output columns, the other 4
// (with the partner's key columns folded in) are sent to the partner -- one DPP swap
// per column.  Per 32 blocks (a wave) a round is 8 lookups + 12 VALU (6 v_perm, 2 DPP)
// against 16 lookups + 32 VALU (12 v_perm, 12 DPP) for two quad waves: 20 % fewer VALU
// cycles per block-round, so the MAC phase running beside the cipher phase gets more issue
// slots (tools/aes_layout_microbench.hip "pair1").
struct PairAes : QuadAes {
    // quad_perm [1,0,3,2]: the partner lane (bound_ctrl: no "old" register)
    static __device__ __forceinline__ uint32_t swap(uint32_t v) { return quad_dpp<0xB1>(v); }
    __device__ __forceinline__ void round(uint32_t& a, uint32_t& b, uint32_t ka, uint32_t kb) const {
        const uint32_t a2 = look<2, 2>(a), b3 = look<3, 3>(b), a1 = look<1, 1>(a), b2 = look<2, 2>(b);
        const uint32_t a0 = look<0, 0>(a), b1 = look<1, 1>(b), b0 = look<0, 0>(b), a3 = look<3, 3>(a);
        // (the compiler builds all eight addresses, then issues the eight reads; forcing each
        // read right after its address op measured 11 % slower, cfg2 864 vs 973 GiB/s, round 4:
        // profiles/r04/ab/ab_pair_r04.txt)
        const uint32_t sa = __builtin_amdgcn_bitop3_b32(a2, b3, ka, 0x96);  // partner's column 2h+2
        const uint32_t sb = __builtin_amdgcn_bitop3_b32(a1, b2, kb, 0x96);  // partner's column 2h+3
        // (the partner's terms moved by v_mov_dpp ahead of the last lookups and one 3-input XOR
        // per column after them -- a shorter dependent path, the same VALU count -- measured
        // 3.5 % slower on cfg2, profiles/r03/ab_pair.txt: kept as v_xor + v_xor_dpp)
        a = (a0 ^ b1) ^ swap(sa);
        b = (b0 ^ a3) ^ swap(sb);
    }
    // final round: S-box byte B of s sits at byte B of table (B+2)&3
    __device__ __forceinline__ void last(uint32_t& a, uint32_t& b, uint32_t ka, uint32_t kb) const {
        const uint32_t ta0 = look<2, 0>(a), tb1 = look<3, 1>(b), ta2 = look<0, 2>(a), tb3 = look<1, 3>(b);
        const uint32_t tb0 = look<2, 0>(b), ta3 = look<1, 3>(a), ta1 = look<3, 1>(a), tb2 = look<0, 2>(b);
        const uint32_t oa = perm(tb1, ta0, 0x0c0c0500u);
        const uint32_t sa = perm(tb3, ta2, 0x07020c0cu) ^ ka;
        const uint32_t ob = perm(ta3, tb0, 0x070c0c00u);
        const uint32_t sb = perm(tb2, ta1, 0x0c06010cu) ^ kb;
        a = oa ^ swap(sa);
        b = ob ^ swap(sb);
    }
    // round keys: kw[0..1] = whitening columns 2h, 2h+1; ka/kb[r >= 1] = the partner's
    // columns 2(1-h), 2(1-h)+1 of round key r (folded into the terms sent to it)
    template <int NR>
    static __device__ __forceinline__ void round_keys(const uint32_t* ek, uint32_t h, uint32_t* kw, uint32_t* ka,
                                                      uint32_t* kb) {
        kw[0] = ek[2 * h];
        kw[1] = ek[2 * h + 1];
        const uint32_t pa = 2 * (1 - h);
#pragma unroll
        for (int r = 1; r <= NR; r++) {
            ka[r] = ek[4 * r + pa];
            kb[r] = ek[4 * r + pa + 1];
        }
    }
    // one block whose two columns are already whitened
    template <int NR>
    __device__ __forceinline__ void encrypt_w(uint32_t& a, uint32_t& b, const uint32_t* ka, const uint32_t* kb) const {
#pragma unroll
        for (int r = 1; r < NR; r++) round(a, b, ka[r], kb[r]);
        last(a, b, ka[NR], kb[NR]);
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

}  // namespace tg

// tg_open3.h -- block-parallel record open for the CBC suites (AES and 3DES).
//
// _decryptRecord (tlsrecordlayer.py:958-1044) per record is: CBC-decrypt the
// body, drop the explicit IV, check the padding, compute the MAC with the next
// seqnum, compare.  Only the seqnum and the CBC residue are serial per
// connection, and CBC *decryption* is parallel over blocks (P_i = D(C_i) ^ C_{i-1},
// every C known up front), so the open path is five launches:
//
//   open_prefix_kernel  one lane per chain: length checks (:964-977), the
//                       predecessor ciphertext block of every record's first
//                       block, the connection's new residue.
//   open_aes_kernel /   the decrypt with one lane per block (16 / 8 bytes), 64
//   open_tdes_kernel    blocks of one record per wave step -- every block of every
//                       record in parallel (round 2; round 1's 4-lanes-per-block
//                       open_dec_kernel measured slower and was removed in round 3).
//   open_seq_kernel     one lane per chain: padding check (:979-993) on the
//                       decrypted tail, which decides whether the MAC is
//                       computed and so whether a seqnum is consumed (:1018).
//   open_mac_kernel     one lane per record: MAC over the plaintext, compare
//                       (:1006-1039), status.
//   open_stop_kernel    one lane per chain, TLSGPU_CHAIN_STOP_ON_ALERT chains:
//                       records after the first alert become TLSGPU_ALERT_SKIPPED,
//                       the state is rolled back to what the failing record left
//                       and marked closed (the reference closes the connection at
//                       the alert, :1039-1042); a state closed before the pass has
//                       every record of its chain skipped.
//
// Workspace per record: one 48-byte OpenMeta and one 48-byte OpenMacState.
//
// A large open runs in parts (launch_open_split), the decrypt (and padding) pass of part h+1
// on the library's second stream beside the MAC pass of part h on the caller's stream: by
// chain range for batches of short chains (each kernel after the prefix takes the part's
// chain range [c_lo, c_hi) and skips records of other chains, OpenMeta.chain), by block range
// for 3DES batches (every record's tail first, then block ranges of every record; the MAC
// passes carry the hash state in OpenMacState).
#pragma once
#include "tg_aes3.h"

namespace tg {

struct OpenMeta {
    uint32_t pred[4];  // ciphertext block before this record's first block (CBC residue)
    uint64_t seq;      // seqnum before this record (the MAC's seqnum when OM_VERIFY)
    uint32_t state;
    uint32_t epoch;
    uint32_t flags;  // OM_*
    uint32_t len;    // plaintext length after explicit-IV removal
    uint32_t n;      // payload length (len - MAC - padding)
    uint32_t chain;  // the record's chain (the part filter of a split open, launch_open_split)
};
static_assert(sizeof(OpenMeta) == 48, "OpenMeta");
constexpr uint32_t OM_DEC = 1, OM_VERIFY = 2, OM_PADOK = 4;
constexpr int O3_THREADS = 1024;

// The hash state of a record's MAC between the passes of an open in block-range parts
// (launch_open_split, 3DES suites): RecMac's h[] and its window tail prev[].
struct OpenMacState {
    uint32_t h[8];
    uint32_t prev[4];
};
static_assert(sizeof(OpenMacState) == 48, "OpenMacState");

// Ciphertext blocks [lo, hi) of a record of nb blocks that pass `part` of an open in
// `nparts` block-range parts decrypts:
//   part < 0        every block (an open in one pass, or in chain-range parts);
//   part == nparts  the tail: the last 256 / BS + 1 blocks, which hold every padding byte
//                   (tlsrecordlayer.py:979-993: up to 255 + 1 bytes), decrypted first so
//                   that the padding pass -- and with it the MAC's length field -- is
//                   known before the first MAC part;
//   part h          the h-th of nparts 64-block-aligned pieces of the blocks before the tail.
template <uint32_t BS>
__device__ __forceinline__ void open_part_blocks(uint32_t nb, int part, int nparts, uint32_t& lo, uint32_t& hi) {
    constexpr uint32_t TB = 256u / BS + 1u;
    if (part < 0) {
        lo = 0;
        hi = nb;
        return;
    }
    const uint32_t tail = nb > TB ? nb - TB : 0u;
    if (part >= nparts) {
        lo = tail;
        hi = nb;
        return;
    }
    const uint32_t chunks = (tail + 63u) >> 6;
    lo = min(tail, 64u * (chunks * (uint32_t)part / (uint32_t)nparts));
    hi = min(tail, 64u * (chunks * (uint32_t)(part + 1) / (uint32_t)nparts));
}

// LDS addressing of the equivalent-inverse-cipher tables (FIPS-197 5.3.5,
// rijndael.py:321-362): the Td tables in the encryption tables' layout (aes_lds_fill with
// dec = true) plus the 32-copy inverse S-box for the last round (lane_aes_dec).
struct QuadAesDec {
    QuadAes t;     // same LDS addressing as the encryption tables (decrypt fill)
    uint32_t isw;  // inverse S-box address word: byte 0 = copy * 8, byte 2 = 0x04 (see isb)
    __device__ __forceinline__ void init() {
        t.init();
        isw = ((__lane_id() & 31) * 8u) | 0x40000u;  // lane-dependent: a VGPR
    }
    // InvS[byte B of x], replicated in all four bytes (aes_lds_fill): the entry of byte value
    // e, copy c sits at 0x20000 + e * 128 + c * 4 = (perm(x -> byte 1, isw) >> 1) -- one v_perm
    // and one 2-cycle shift per lookup (round 4: bfe + shift-or + a shift of the result)
    template <int B>
    __device__ __forceinline__ uint32_t isb(uint32_t x) const {
        constexpr uint32_t sel = 0x0c000000u | (2u << 16) | ((4u + B) << 8) | 0u;
        return lds_read32(perm(x, isw, sel) >> 1);
    }
    // bytes 0..3 of the output column from four replicated lookups (two v_perm), key XOR-ed
    __device__ __forceinline__ static uint32_t col(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t k) {
        return __builtin_amdgcn_bitop3_b32(perm(r1, r0, 0x0c0c0500u), perm(r3, r2, 0x07020c0cu), k, 0x96);
    }
};

template <int CIPHER_ID, int MAC, bool SSL3>
__global__ void __launch_bounds__(256) open_prefix_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                         const tlsgpu_open_record* __restrict__ recs, uint32_t nrecords,
                                                         const uint8_t* __restrict__ wire,
                                                         ConnState* __restrict__ states, int32_t* __restrict__ status,
                                                         OpenMeta* __restrict__ meta, uint32_t epoch,
                                                         uint64_t wire_cap, uint64_t pt_cap, uint32_t nstates) {
    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    // a state index outside the caller's array: every record refused, no state read (ABI 6)
    const bool sok = ch.state < nstates;
    ConnState* st = states + (sok ? ch.state : 0u);
    // state header without short-circuit branches (one memory latency, as prefix_kernel)
    uint4 h0 = make_uint4(0, 0, 0, 0), h1 = make_uint4(0, 0, 0, 0);
    uint32_t res[4] = {0, 0, 0, 0};
    constexpr uint32_t BS = CIPHER_ID == TLSGPU_CIPHER_3DES ? 8u : 16u;
    if (sok) {
        h0 = *(const uint4*)st;                         // cipher, mac, vmaj..maclen, ssl3
        h1 = *(const uint4*)((const uint8_t*)st + 16);  // seqnum (lo, hi), explicit_iv, raw
        res[0] = st->iv[0];
        res[1] = st->iv[1];
        res[2] = BS == 16 ? st->iv[2] : 0u;
        res[3] = BS == 16 ? st->iv[3] : 0u;
    }
    const bool ok = sok & (h0.x == (uint32_t)CIPHER_ID) & (h0.y == (uint32_t)MAC) & (h0.w == (SSL3 ? 1u : 0u)) &
                    (h1.w == 0u);
    // a state closed by an earlier alert (ConnState.closed): every record skipped, nothing
    // opened, the state untouched
    const bool closed = ok && st->closed != 0u;
    const uint32_t E = h1.z ? BS : 0u;
    for (uint32_t k = 0; k < ch.count; k++) {
        const uint32_t r = ch.first + k;
        if (r >= nrecords) break;
        OpenMeta m;
#pragma unroll
        for (int i = 0; i < 4; i++) m.pred[i] = res[i];
        m.seq = 0;
        m.state = ch.state;
        m.epoch = epoch;
        m.flags = 0;
        m.len = 0;
        m.n = 0;
        m.chain = cid;
        if (!ok || closed) {
            status[r] = !sok ? TLSGPU_EINVAL : closed ? TLSGPU_ALERT_SKIPPED : TLSGPU_EMISMATCH;
            m.epoch = closed ? 0u : m.epoch;  // no later pass of this launch looks at a closed chain's records
        } else {
            const tlsgpu_open_record R = recs[r];
            const uint32_t L = R.ct_len;
            if (!in_arena(R.ct_off, L, wire_cap) || !in_arena(R.pt_off, L > E ? L - E : 0u, pt_cap)) {
                // outside the caller's arenas: not opened, nothing written, residue and seqnum as
                // if the record were not in the batch
                status[r] = TLSGPU_EINVAL;
                m.epoch = 0;  // no later pass of this launch looks at it (open_seq_kernel: no seqnum)
            } else if (L & (BS - 1)) {  // :964-968 -- not decrypted, residue unchanged
                status[r] = TLSGPU_ALERT_DECRYPTION_FAILED;
            } else {
                if (L) {  // decrypt() keeps the last block
                    if constexpr (BS == 16) load16(wire + R.ct_off + L - 16, res);
                    else load8(wire + R.ct_off + L - 8, res);
                }
                if (L <= E) {                                  // :970-977 nothing left after the IV
                    status[r] = TLSGPU_ALERT_DECRYPTION_FAILED;
                } else {
                    m.flags = OM_DEC;
                    m.len = L - E;
                }
            }
        }
        meta[r] = m;
    }
    if (ok && !closed) {
#pragma unroll
        for (int i = 0; i < (int)BS / 4; i++) st->iv[i] = res[i];
    }
}

// AES decrypt with one lane per block (equivalent inverse cipher, aes_decrypt's column
// order, FIPS-197 5.3.5): the lane does all 16 Td lookups of a round, so the quad's DPP
// XOR tree is gone (the decrypt is throughput-bound: every block of every record is
// independent), and a wave's 64 lanes read and write 1 KiB of contiguous ciphertext /
// plaintext per instruction.  A wave walks one record 64 blocks at a time: the record's
// round keys are wave-uniform scalar loads.
template <int NR>
__device__ __forceinline__ void lane_aes_dec(const QuadAesDec& D, uint32_t s[4], const uint32_t* dk) {
    const QuadAes& A = D.t;
    uint32_t s0 = s[0] ^ dk[0], s1 = s[1] ^ dk[1], s2 = s[2] ^ dk[2], s3 = s[3] ^ dk[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t* k = dk + 4 * r;
        const uint32_t t0 = bx3(bx3(A.look<0, 0>(s0), A.look<1, 1>(s3), A.look<2, 2>(s2)), A.look<3, 3>(s1), k[0]);
        const uint32_t t1 = bx3(bx3(A.look<0, 0>(s1), A.look<1, 1>(s0), A.look<2, 2>(s3)), A.look<3, 3>(s2), k[1]);
        const uint32_t t2 = bx3(bx3(A.look<0, 0>(s2), A.look<1, 1>(s1), A.look<2, 2>(s0)), A.look<3, 3>(s3), k[2]);
        const uint32_t t3 = bx3(bx3(A.look<0, 0>(s3), A.look<1, 1>(s2), A.look<2, 2>(s1)), A.look<3, 3>(s0), k[3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint32_t* k = dk + 4 * NR;
    s[0] = QuadAesDec::col(D.isb<0>(s0), D.isb<1>(s3), D.isb<2>(s2), D.isb<3>(s1), k[0]);
    s[1] = QuadAesDec::col(D.isb<0>(s1), D.isb<1>(s0), D.isb<2>(s3), D.isb<3>(s2), k[1]);
    s[2] = QuadAesDec::col(D.isb<0>(s2), D.isb<1>(s1), D.isb<2>(s0), D.isb<3>(s3), k[2]);
    s[3] = QuadAesDec::col(D.isb<0>(s3), D.isb<1>(s2), D.isb<2>(s1), D.isb<3>(s0), k[3]);
}

// The records a decrypt wave handles: r0 + i * nwaves for i < 64 (the wave's next 64,
// in order), those of this launch's part (chains [c_lo, c_hi)) that decrypt.  One lane
// checks one record's meta, so records of other parts cost no dependent load each.
__device__ __forceinline__ uint64_t open_dec_batch(const OpenMeta* meta, uint32_t nrecords, uint32_t r0,
                                                   uint32_t nwaves, uint32_t epoch, uint32_t c_lo, uint32_t c_hi) {
    const uint32_t rl = r0 + (threadIdx.x & 63) * nwaves;
    bool mine = false;
    if (rl < nrecords) {
        const OpenMeta& m = meta[rl];
        mine = m.epoch == epoch && (m.flags & OM_DEC) && m.chain - c_lo < c_hi - c_lo;
    }
    return __ballot(mine);
}

// Word v of lane l as an unsigned value: __builtin_amdgcn_readlane returns int, and a plain
// (uint64_t) cast of it sign-extends -- round 5's 64-bit offsets rebuilt that way turned every
// low word >= 2^31 into 0xffffffff'xxxxxxxx, the illegal address of cfg4's open (arenas > 2 GiB)
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t lane_u64(uint32_t v, int lo) {
    return (uint64_t)lane_u32(v, lo) | ((uint64_t)lane_u32(v, lo + 1) << 32);
}

// Lane l of wave-wide value v from lane l - 1 (DPP wave_shr:1, one VALU); lane 0 gets `first`
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t first) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xf, 0xf, false);
}

// Issue-priority rotation of the decrypt waves (round 5): 16 waves per CU, 4 per SIMD (w,
// w + 4, w + 8, w + 12), and at equal priority the SIMD's arbiter favours the oldest, so the
// waves' fixed shares of the work finished far apart (per-wave loop time min / avg / max
// 0.69 / 1 / 1.33 in tools/aes_dec_microbench.hip) and the CU's last stretch ran on a few
// waves.  Each wave takes the top priority every fourth chunk: max / avg 1.07, the
// cfg2-shaped decrypt loop 0.767 -> 0.691 ms (profiles/r05/dec_mb.txt).
struct PrioRot4 {
    uint32_t turn;
    __device__ __forceinline__ void init() { turn = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8) & 3u; }
    __device__ __forceinline__ void tick() {
        const uint32_t p = ++turn & 3u;
        if (p == 0) __builtin_amdgcn_s_setprio(3);
        else if (p == 1) __builtin_amdgcn_s_setprio(2);
        else if (p == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    }
};

// The records a decrypt wave opens, one after another (open_dec_batch's batches of 64
// candidates, those of this launch's part), with the NEXT record's descriptor and round keys
// loaded while the current one is decrypted (round 5): lane i holds word i of the next
// record's OpenMeta (0..11) and tlsgpu_open_record (12..17) in `vm`, word i of its state's
// equivalent-inverse round keys (0..4 NR + 3) and the explicit-IV flag (lane 63) in `vk`;
// at the switch they become wave-uniform (v_readlane).  Before, each record began with three
// dependent scalar loads (meta -> state -> round keys, ~1 us each) in front of its first
// chunk, 17 chunks of work apart on cfg2 and 5 passes apart in block-range parts.
struct OpenDecStream {
    const OpenMeta* meta;
    uint32_t nrecords, nwaves, epoch, c_lo, c_hi;
    uint32_t r0;
    uint64_t mask;
    __device__ __forceinline__ uint32_t next() {  // the next record of the wave, or ~0u
        while (!mask) {
            r0 += 64 * nwaves;
            if (r0 >= nrecords) return ~0u;
            mask = open_dec_batch(meta, nrecords, r0, nwaves, epoch, c_lo, c_hi);
        }
        const uint32_t r = r0 + (uint32_t)__builtin_ctzll(mask) * nwaves;
        mask &= mask - 1;
        return r;
    }
};
__device__ __forceinline__ uint32_t open_fetch_desc(const OpenMeta* meta, const tlsgpu_open_record* recs, uint32_t r) {
    const uint32_t lane = __lane_id();
    if (r == ~0u) return 0u;
    if (lane < 12) return ((const uint32_t*)(meta + r))[lane];
    if (lane < 18) return ((const uint32_t*)(recs + r))[lane - 12];
    return 0u;
}
template <int NR>
__device__ __forceinline__ uint32_t open_fetch_keys(const ConnState* states, uint32_t vm, uint32_t r) {
    const uint32_t lane = __lane_id();
    if (r == ~0u) return 0u;
    const ConnState* st = states + lane_u32(vm, 6);  // OpenMeta.state
    if (lane < 4 * (NR + 1)) return st->dk[lane];
    if (lane == 63) return st->explicit_iv;
    return 0u;
}

// A wave walks one record 64 blocks (one 1 KiB chunk) at a time.  Round 5: the next chunk's ciphertext is loaded before the current
// one is decrypted (its HBM latency hides under the chunk's ten rounds instead of stalling the
// wave at every chunk), and a lane's predecessor block C_{b-1} is its left neighbour's
// ciphertext, moved over by DPP (wave_shr:1) -- only lane 0 takes it from the previous
// chunk's lane 63 (readlane) or the record's first predecessor (OpenMeta.pred), instead of
// every lane loading the block again.
template <int NR>
__global__ void __launch_bounds__(O3_THREADS, 1)
open_aes_kernel(const tlsgpu_open_record* __restrict__ recs, uint32_t nrecords, const uint8_t* __restrict__ wire,
                uint8_t* __restrict__ pt, const ConnState* __restrict__ states, const OpenMeta* __restrict__ meta,
                uint32_t epoch, uint32_t c_lo, uint32_t c_hi) {
    aes_lds_fill(nullptr, true);
    __syncthreads();
    QuadAesDec D;
    D.init();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    OpenDecStream rs;
    rs.meta = meta;
    rs.nrecords = nrecords;
    rs.nwaves = gridDim.x * (O3_THREADS / 64);
    rs.epoch = epoch;
    rs.c_lo = c_lo;
    rs.c_hi = c_hi;
    rs.r0 = blockIdx.x * (O3_THREADS / 64) + wv;
    rs.mask = rs.r0 < nrecords ? open_dec_batch(meta, nrecords, rs.r0, rs.nwaves, epoch, c_lo, c_hi) : 0ull;
    uint32_t r = rs.next();
    uint32_t vm = open_fetch_desc(meta, recs, r);
    uint32_t vk = open_fetch_keys<NR>(states, vm, r);
    PrioRot4 rot;
    rot.init();
    while (r != ~0u) {
        // this record's descriptor and keys, wave-uniform
        uint32_t dk[4 * (NR + 1)];
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++) dk[i] = lane_u32(vk, i);
        const uint32_t E = lane_u32(vk, 63) ? 16u : 0u;
        uint32_t carry[4];
#pragma unroll
        for (int i = 0; i < 4; i++) carry[i] = lane_u32(vm, i);  // OpenMeta.pred
        const uint64_t ct_off = lane_u64(vm, 12);  // tlsgpu_open_record.ct_off
        const uint64_t pt_off = lane_u64(vm, 14);  // tlsgpu_open_record.pt_off
        const uint32_t ct_len = lane_u32(vm, 16);
        // the next record's descriptor now; its keys after this record's first chunk
        const uint32_t rn = rs.next();
        vm = open_fetch_desc(meta, recs, rn);
        bool keys_pending = true;
        const uint32_t nb = ct_len >> 4;
        const uint8_t* C = wire + ct_off;
        uint8_t* P = pt + pt_off;
        const uint32_t hi = nb;
        {
            uint32_t c[4] = {0, 0, 0, 0};
            if (lane < hi) load16(C + 16 * lane, c);
            for (uint32_t base = 0; base < hi; base += 64) {
                const uint32_t b = base + lane;
                rot.tick();
                uint32_t cn[4] = {0, 0, 0, 0};
                if (b + 64 < hi) load16(C + 16 * (b + 64), cn);  // the next chunk, in flight meanwhile
                uint32_t p[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    p[i] = wave_shr1(c[i], carry[i]);
                    carry[i] = lane_u32(c[i], 63);  // the next chunk's lane-0 predecessor
                }
                if (b < hi) {
                    uint32_t d[4] = {c[0], c[1], c[2], c[3]};
                    lane_aes_dec<NR>(D, d, dk);
#pragma unroll
                    for (int i = 0; i < 4; i++) d[i] ^= p[i];
                    if (16 * b >= E) store16(P + 16 * b - E, d);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) c[i] = cn[i];
                if (keys_pending) {
                    vk = open_fetch_keys<NR>(states, vm, rn);
                    keys_pending = false;
                }
            }
        }
        if (keys_pending) vk = open_fetch_keys<NR>(states, vm, rn);
        r = rn;
    }
}

// 3DES suites (openssl_tripledes.py:40-47: P_i = D(C_i) ^ C_{i-1}): every 8-byte block of
// every record decrypted in parallel, one lane per block (all eight SP lookups of a round in
// the lane, no cross-lane step: the block count, not a round's latency, is what there is
// to exploit here).  A wave walks a record 64 blocks at a time; the record -- and so the
// connection's 96 subkey words -- is uniform over the wave, so the subkeys are scalar
// loads.  LDS: the 64 KiB SP tables, 32 lane copies (conflict-free).
constexpr int OT_THREADS = 1024;

// DES on one lane, rotated halves as des_rounds() (tg_device.h), SP tables at LDS byte
// (K * 64 + x) * 128 + copy * 4 (des_lds_fill).  w = r ^ k_even and t = r ^ rotl4(k_odd):
// box 7-2j takes bits [8j, 8j+6) of w, box 6-2j bits [8j+4, 8j+10) of t, each moved to
// bits 7..12 by one shift (one rotate for the window that wraps) and masked with the
// lane-copy offset OR-ed in by one all-VGPR v_bitop3; the table offset rides in the
// ds_read offset field.
struct DesLane {
    uint32_t lo, m;
    __device__ __forceinline__ void init() {
        lo = (__lane_id() & 31) * 4;
        m = vconst(0x1f80u);
    }
    __device__ __forceinline__ uint32_t sp(uint32_t u, uint32_t k) const {
        return lds_read32(__builtin_amdgcn_bitop3_b32(u, m, lo, 0xEA) + k * 8192u);
    }
    __device__ __forceinline__ uint32_t f(uint32_t w, uint32_t t) const {
        const uint32_t x1 = bx3(sp(w << 7, 7), sp(w >> 1, 5), sp(w >> 9, 3));
        const uint32_t x2 = bx3(sp(w >> 17, 1), sp(t << 3, 6), sp(t >> 5, 4));
        const uint32_t x3 = sp(t >> 13, 2) ^ sp(__builtin_amdgcn_alignbit(t, t, 21), 0);
        return bx3(x1, x2, x3);
    }
    // 16 rounds with subkey words ks[2k] (even) / ks[2k+1] (odd), k walked backwards when DEC;
    // leaves (l, r) = (R16, L16) like des_rounds
    template <bool DEC>
    __device__ __forceinline__ void rounds(uint32_t& l, uint32_t& r, const uint32_t* ks) const {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int k = DEC ? 15 - i : i;
            const uint32_t ko = ks[2 * k + 1];
            const uint32_t t = l ^ f(r ^ ks[2 * k], r ^ ((ko << 4) | (ko >> 28)));
            l = r;
            r = t;
        }
        const uint32_t t = l;
        l = r;
        r = t;
    }
    // 3DES-EDE decrypt of one block given as two big-endian words (tdes_block<true>)
    __device__ __forceinline__ void decrypt(uint32_t& hi, uint32_t& lo_w, const uint32_t* ks) const {
        uint32_t l = hi, r = lo_w;
        des_ip(l, r);
        rounds<true>(l, r, ks + 64);
        rounds<false>(l, r, ks + 32);
        rounds<true>(l, r, ks);
        des_fp(l, r);
        hi = l;
        lo_w = r;
    }
};
__global__ void __launch_bounds__(OT_THREADS, 1)
open_tdes_kernel(const tlsgpu_open_record* __restrict__ recs, uint32_t nrecords, const uint8_t* __restrict__ wire,
                 uint8_t* __restrict__ pt, const ConnState* __restrict__ states, const OpenMeta* __restrict__ meta,
                 uint32_t epoch, uint32_t c_lo, uint32_t c_hi, int part, int nparts) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ot_lds[];
    des_lds_fill(ot_lds);  // the kernel's only LDS: the tables start at LDS byte 0
    __syncthreads();
    DesLane L;
    L.init();
    // (no priority rotation here, unlike open_aes_kernel: on cfg5 it measured neutral, 268-271
    // vs 270-272 GiB/s, profiles/r05/ab_open.txt)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * (OT_THREADS / 64);
    for (uint32_t r0 = blockIdx.x * (OT_THREADS / 64) + wv; r0 < nrecords; r0 += 64 * nwaves)
    for (uint64_t mask = open_dec_batch(meta, nrecords, r0, nwaves, epoch, c_lo, c_hi); mask; mask &= mask - 1) {
        const uint32_t r = r0 + (uint32_t)__builtin_ctzll(mask) * nwaves;
        const OpenMeta& mt = meta[r];
        const ConnState* st = states + mt.state;
        const uint32_t* ks = &st->des[0][0];
        const tlsgpu_open_record R = recs[r];
        const uint32_t E = st->explicit_iv ? 8u : 0u;
        const uint32_t nb = R.ct_len >> 3;
        const uint8_t* C = wire + R.ct_off;
        uint8_t* P = pt + R.pt_off;
        // next chunk prefetched, predecessor from the left neighbour (as open_aes_kernel); the
        // blocks of this pass (open_part_blocks)
        uint32_t lo, hi;
        open_part_blocks<8>(nb, part, nparts, lo, hi);
        if (lo >= hi) continue;
        uint32_t carry[2] = {mt.pred[0], mt.pred[1]};
        if (lo) load8(C + 8 * (lo - 1), carry);  // wave-uniform: the block before this pass's first
        uint32_t c[2] = {0, 0};
        if (lo + lane < hi) load8(C + 8 * (lo + lane), c);
        for (uint32_t base = lo; base < hi; base += 64) {
            const uint32_t b = base + lane;
            uint32_t cn[2] = {0, 0};
            if (b + 64 < hi) load8(C + 8 * (b + 64), cn);
            uint32_t p[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                p[i] = wave_shr1(c[i], carry[i]);
                carry[i] = lane_u32(c[i], 63);
            }
            if (b < hi) {
                uint32_t whi = bswap32(c[0]), wlo = bswap32(c[1]);
                L.decrypt(whi, wlo, ks);
                uint32_t d[2] = {bswap32(whi) ^ p[0], bswap32(wlo) ^ p[1]};
                if (8 * b >= E) store8(P + 8 * b - E, d);
            }
            c[0] = cn[0];
            c[1] = cn[1];
        }
    }
}

template <int MAC, bool SSL3>
__global__ void __launch_bounds__(256) open_seq_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                      const tlsgpu_open_record* __restrict__ recs, uint32_t nrecords,
                                                      const uint8_t* __restrict__ pt, ConnState* __restrict__ states,
                                                      int32_t* __restrict__ status, OpenMeta* __restrict__ meta,
                                                      uint32_t epoch, uint32_t c_lo, uint32_t c_hi, uint32_t nstates) {
    constexpr uint32_t DL = Hash<MAC>::DLEN;
    const uint32_t cid = c_lo + blockIdx.x * blockDim.x + threadIdx.x;  // chains [c_lo, c_hi) of nchains
    if (cid >= c_hi || cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    if (ch.state >= nstates) return;  // refused by open_prefix_kernel (ABI 6): no state read
    ConnState* st = states + ch.state;
    if (st->closed) return;  // closed by an earlier alert: skipped (open_prefix_kernel), state untouched
    uint64_t seq = st->seqnum;
    bool any = false;
    for (uint32_t k = 0; k < ch.count; k++) {
        const uint32_t r = ch.first + k;
        if (r >= nrecords) break;
        OpenMeta& m = meta[r];
        if (m.epoch != epoch) continue;
        any = true;
        m.seq = seq;
        if (!(m.flags & OM_DEC)) continue;
        const uint8_t* P = pt + recs[r].pt_off;
        const uint32_t len = m.len;
        const uint32_t pl = P[len - 1];
        bool padGood = true;
        uint32_t totalPad = 0;
        if (pl + 1 > len) {  // :981-983
            padGood = false;
        } else {
            totalPad = pl + 1;
            if (!SSL3) {  // TLS: every padding byte equals the length (:986-993)
                for (uint32_t i = len - totalPad; i < len - 1; i++)
                    if (P[i] != pl) padGood = false;
                if (!padGood) totalPad = 0;
            }
        }
        const uint32_t endLen = DL + totalPad;
        if (endLen > len) {  // :1006-1007 -- no MAC computed, no seqnum consumed
            status[r] = TLSGPU_ALERT_BAD_RECORD_MAC;
            m.flags = 0;
        } else {
            m.n = len - endLen;
            seq++;  // getSeqNumBytes (:1018)
            m.flags = OM_DEC | OM_VERIFY | (padGood ? OM_PADOK : 0u);
        }
    }
    if (any) st->seqnum = seq;
}

// MAC over the plaintext, one lane per record, per-lane 64-B chunk loads with the next chunk
// prefetched (mac_bulk).  (The seal's quad-cooperative loads measured 1-2 % slower here,
// round 4: cfg2 718 vs 733, cfg3 397 vs 402 GiB/s -- with one lane per 16 KiB record the
// open's MAC is latency-bound, and the transposes sit on that path;
// profiles/r04/ab/ab_open_r04.txt.)
// part < 0: the whole MAC in one pass.  Block-range parts (3DES): pass h < nparts hashes
// the payload chunks whose blocks the decrypt parts 0..h (and the tail) have produced and
// keeps the hash state in the workspace (OpenMacState); pass nparts hashes the rest,
// finishes and compares.
template <int BS>
__device__ __forceinline__ uint32_t open_chunks_ready(uint32_t nb, uint32_t E, uint32_t nfull, int part, int nparts) {
    uint32_t lo, hi;
    open_part_blocks<BS>(nb, part, nparts, lo, hi);
    const uint32_t bytes = BS * hi > E ? BS * hi - E : 0u;  // payload bytes decrypted from its start
    return min(nfull, bytes >> 6);
}

// COOP (round 6): a batch of at most one record per lane of one wave per CU (the receive
// pipeline's 64 MiB sub-batches of 16 KiB records: 4,096 lanes on 256 CUs) is latency-bound,
// and with per-lane 64-B loads one chunk ahead every compression waited for its load (1.3 ms
// for 256 compressions against the seal MAC's 0.34 ms); there the quad-cooperative loads with
// the seal's two-chunk ring (mac_bulk_coop) feed the lanes.  Large batches keep the per-lane
// loads (round 4: the cooperative form measured 1-2 % slower on cfg2 / cfg3).
template <int MAC, bool SSL3, int BS, bool COOP>
__global__ void __launch_bounds__(256) open_mac_kernel(const tlsgpu_open_record* __restrict__ recs, uint32_t nrecords,
                                                      const uint8_t* __restrict__ pt,
                                                      const ConnState* __restrict__ states,
                                                      int32_t* __restrict__ status,
                                                      const OpenMeta* __restrict__ meta, OpenMacState* __restrict__ ms,
                                                      uint32_t epoch, uint32_t c_lo, uint32_t c_hi, int part,
                                                      int nparts) {
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    // the chain first: records of other parts may be in their padding pass right now
    bool act = r < nrecords && meta[r].chain - c_lo < c_hi - c_lo;
    OpenMeta mt = {};
    if (act) {
        mt = meta[r];
        act = mt.epoch == epoch && (mt.flags & OM_VERIFY);
    }
    if constexpr (!COOP) {
        if (!act) return;
    }
    // no early exit before the bulk in the cooperative form: the quad exchanges loaded data (DPP)
    const ConnState* st = states;
    tlsgpu_open_record R = {};
    const uint8_t* P = pt;
    uint32_t n = 0, nfull = 0, c0 = 0, c1 = 0;
    M mac;
    if (act) {
        st = states + mt.state;
        R = recs[r];
        P = pt + R.pt_off;
        n = mt.n;
        nfull = n >> 6;
        c1 = nfull;
        if (part >= 0) {
            const uint32_t E = st->explicit_iv ? (uint32_t)BS : 0u;
            const uint32_t nb = R.ct_len / BS;
            c0 = part == 0 ? 0u : open_chunks_ready<BS>(nb, E, nfull, part - 1, nparts);
            c1 = part == nparts ? nfull : open_chunks_ready<BS>(nb, E, nfull, part, nparts);
        }
        if (c0 == 0) {
            mac.begin(st, mt.seq, R.content_type, n);
        } else {
            const OpenMacState& q = ms[r];
#pragma unroll
            for (int k = 0; k < 8; k++) mac.h[k] = q.h[k];
#pragma unroll
            for (int k = 0; k < 4; k++) mac.prev[k] = q.prev[k];
        }
    }
    const uint8_t* Pc = P + 64 * c0;
    const bool al16 = ((uintptr_t)P & 15) == 0;
    if constexpr (COOP) {
        uint32_t coop = (act && al16 && c1 > c0) ? 1u : 0u;
        coop &= quad_dpp<0xB1>(coop);
        coop &= quad_dpp<0x4E>(coop);
        if (coop) {
            mac_bulk_coop<MAC_PF>(mac, Pc, c1 - c0, threadIdx.x & 3u);
        } else if (act) {
            if (al16) mac_bulk<true>(mac, Pc, c1 - c0);
            else mac_bulk<false>(mac, Pc, c1 - c0);
        }
        if (!act) return;
    } else {
        if (al16) mac_bulk<true>(mac, Pc, c1 - c0);
        else mac_bulk<false>(mac, Pc, c1 - c0);
    }
    if (part >= 0 && part < nparts) {  // more parts follow: keep the hash state
        OpenMacState& q = ms[r];
#pragma unroll
        for (int k = 0; k < 8; k++) q.h[k] = mac.h[k];
#pragma unroll
        for (int k = 0; k < 4; k++) q.prev[k] = mac.prev[k];
        return;
    }
    uint32_t tail[16];
    load_partial(P + 64 * nfull, n & 63, tail);
    uint32_t m[8];
    mac.finish(tail, (int)(n & 63), n, st, m);
    bool macGood = true;
#pragma unroll
    for (int i = 0; i < DL; i++)
        if (P[n + i] != (uint8_t)(m[i >> 2] >> (8 * (i & 3)))) macGood = false;
    status[r] = ((mt.flags & OM_PADOK) && macGood) ? (int32_t)n : TLSGPU_ALERT_BAD_RECORD_MAC;
}

__global__ void __launch_bounds__(256) open_stop_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                                       const tlsgpu_open_record* __restrict__ recs, uint32_t nrecords,
                                                       const uint8_t* __restrict__ wire, ConnState* __restrict__ states,
                                                       int32_t* __restrict__ status,
                                                       const OpenMeta* __restrict__ meta, uint32_t epoch,
                                                       uint32_t nstates) {
    const uint32_t cid = blockIdx.x * blockDim.x + threadIdx.x;
    if (cid >= nchains) return;
    const tlsgpu_chain ch = chains[cid];
    if (ch.state >= nstates) return;  // refused by open_prefix_kernel (ABI 6)
    ConnState* st = states + ch.state;
    if (st->closed) {
        // closed by an earlier call (open_prefix_kernel skipped the chain's records already):
        // every record of the chain is skipped; the state stays as the closing alert left it.
        for (uint32_t k = 0; k < ch.count && ch.first + k < nrecords; k++) status[ch.first + k] = TLSGPU_ALERT_SKIPPED;
        return;
    }
    if (!(ch.flags & TLSGPU_CHAIN_STOP_ON_ALERT)) return;
    for (uint32_t k = 0; k < ch.count; k++) {
        const uint32_t r = ch.first + k;
        if (r >= nrecords) return;
        const int32_t s = status[r];
        if (s != TLSGPU_ALERT_BAD_RECORD_MAC && s != TLSGPU_ALERT_DECRYPTION_FAILED) continue;
        const OpenMeta& m = meta[r];
        if (m.epoch != epoch) return;
        st->closed = 1u;  // the reference closes the connection at the alert (:524-529, :1039-1042)
        for (uint32_t j = k + 1; j < ch.count && ch.first + j < nrecords; j++) status[ch.first + j] = TLSGPU_ALERT_SKIPPED;
        // state as record r left it: its seqnum was consumed iff its MAC was computed, and its
        // last ciphertext block is the residue iff it was decrypted (a block multiple).  Written
        // even when r is the chain's last record (the state then already holds it).
        st->seqnum = m.seq + ((m.flags & OM_VERIFY) ? 1u : 0u);
        const tlsgpu_open_record R = recs[r];
        uint32_t res[4] = {m.pred[0], m.pred[1], m.pred[2], m.pred[3]};
        if (st->cipher == (uint32_t)TLSGPU_CIPHER_3DES) {
            if (R.ct_len && !(R.ct_len & 7u)) load8(wire + R.ct_off + R.ct_len - 8, res);
            st->iv[0] = res[0];
            st->iv[1] = res[1];
        } else {
            if (R.ct_len && !(R.ct_len & 15u)) load16(wire + R.ct_off + R.ct_len - 16, res);
#pragma unroll
            for (int i = 0; i < 4; i++) st->iv[i] = res[i];
        }
        return;
    }
}

}  // namespace tg

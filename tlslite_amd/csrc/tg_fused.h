// tg_fused.h -- the AES record seal in ONE kernel for the throughput regimes (a CU gets
// at least 256 chains: cfg2, cfg3), reading every plaintext byte from HBM once.
//
// The split path (tg_aes3.h: prefix_kernel -> mac_kernel -> cbc_pair_kernel) reads the
// plaintext twice: once for the MAC phase, once for the cipher phase, a batch apart in the
// pipeline (cfg2: 3.34 GB per call for 2.15 GB of algorithmic traffic).  Here one
// workgroup per CU holds both roles for the same 256 chain slots:
//
//   waves 0-7   cipher: the pair layout of cbc_pair_kernel (2 lanes per chain, slot =
//               32 * wave + lane / 2), explicit IV, full P blocks in line-aligned groups,
//               then the CBC tail (P[16 nb ..) | MAC | padding) from the slot's LDS tail.
//   waves 8-11  MAC: one lane per slot, the work of prefix_kernel + mac_kernel for the
//               slot's records in order -- validation, seqnum, HMAC / MAC_SSL over
//               seq | type | ver | len | P (tlsrecordlayer.py:567-586), the tail with its
//               padding (:597-606) into the slot's LDS tail, the 5-byte header and wire_len.
//
// The MAC lane of a slot reads a 64-B chunk only after the slot's cipher lanes have ISSUED
// the loads of the blocks it covers (LDS counter `loaded`, published once per group), so
// its read finds the line in the L2 (or in flight) instead of HBM.  The cipher lanes wait
// for the MAC only at a record's tail (`ready`); the MAC lane writes the next record's tail
// only after the cipher has consumed the previous one (`done`).  The cipher issues its
// loads a group ahead of its encryption, so the MAC normally finishes a record before the
// cipher reaches its tail.
//
// Deadlock freedom: a cipher pair waits only on its own slot's MAC lane, and that lane can
// always finish the record the cipher waits on (the cipher has issued all its loads and
// consumed the previous tail).  The MAC waves run their lanes as independent state
// machines in one wave-uniform loop (a lane that cannot proceed is masked for the
// iteration, never spins while its wave-mates' work waits behind it), so no MAC lane is
// held by another slot's cipher.  Waits are bounded (watchdog): a wait that outlives it ends
// with wire_len = TLSGPU_EHIP for the record instead of a hung GPU.
//
// Both roles walk the same sequence of chains per slot (chain blockIdx.x * cpw + slot, then
// + gridDim.x * cpw: persistent over generations, as cbc_pair_kernel), and count the slot's
// records and plaintext bytes cumulatively, so their counters agree without a handshake.
// Record status (seal / empty / too big / past the wire arena / state mismatch) is decided
// by both from the descriptor and the state header with the same code (seal_record_status).
#pragma once
#include "tg_aes3.h"

namespace tg {

constexpr int FZ_CIPHER_WAVES = 8;
constexpr int FZ_MAC_WAVES = 4;
constexpr int FZ_SLOTS = 32 * FZ_CIPHER_WAVES;  // 256 chain slots per workgroup
constexpr int FZ_THREADS = 64 * (FZ_CIPHER_WAVES + FZ_MAC_WAVES);
// LDS after the T-tables (byte addresses; the kernel's dynamic LDS starts at 0)
constexpr uint32_t FZ_LOADED = AES_LDS_BYTES;        // u32 per slot: plaintext bytes of the slot's stream whose loads the cipher issued
constexpr uint32_t FZ_DONE = FZ_LOADED + 4 * FZ_SLOTS;  // u32 per slot: records of the slot's stream the cipher finished
constexpr uint32_t FZ_READY = FZ_DONE + 4 * FZ_SLOTS;   // u32 per slot: records the MAC lane finished (tail in the slot)
constexpr uint32_t FZ_TLEN = FZ_READY + 4 * FZ_SLOTS;   // u32 per slot: tail bytes of the record in the slot
constexpr uint32_t FZ_TAIL = FZ_TLEN + 4 * FZ_SLOTS;    // 64 B per slot: P[16 nb ..) | MAC | padding
constexpr uint32_t FZ_LDS_BYTES = FZ_TAIL + TAIL_SLOT * FZ_SLOTS;
static_assert(FZ_LDS_BYTES <= 160 * 1024, "gfx950 LDS per workgroup");
// watchdog: iterations of a wait (each with an s_sleep) before it gives up (~0.5 s)
constexpr uint32_t FZ_WATCHDOG = 1u << 22;
// A/B switches (tools/build_ab.sh): TG_AB_FZ_MAC_PRIO  the MAC waves' priority (default: the
// split path's MAC priority); TG_AB_FZ_NOGATE  MAC loads not gated on the cipher's progress;
// TG_AB_FZ_NOMAC  timing only (wrong MACs): the MAC lanes hand over their tails without
// computing them, i.e. the cipher waves' time inside this kernel
#ifndef TG_AB_FZ_MAC_PRIO
#define TG_AB_FZ_MAC_PRIO TG_AB_MAC_PRIO
#endif

__device__ __forceinline__ uint32_t fz_ld(uint32_t addr) {
    return __hip_atomic_load((lds_u32_t*)(size_t)addr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void fz_st(uint32_t addr, uint32_t v) {
    __hip_atomic_store((lds_u32_t*)(size_t)addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// a >= b on counters that may wrap
__device__ __forceinline__ bool fz_ge(uint32_t a, uint32_t b) { return (int32_t)(a - b) >= 0; }

// The state header test of prefix_kernel: the state belongs to this launch's variant.
template <int CIPHER_ID, int MAC, bool SSL3>
__device__ __forceinline__ bool fz_state_ok(const ConnState* st, uint4& h1) {
    const uint4 h0 = *(const uint4*)st;
    h1 = *(const uint4*)((const uint8_t*)st + 16);
    return (h0.x == (uint32_t)CIPHER_ID) & (h0.y == (uint32_t)MAC) & (h0.w == (SSL3 ? 1u : 0u)) & (h1.w == 0u);
}

// What prefix_kernel decides for a record: 1 = seal, else the wire_len to report (0 empty,
// TLSGPU_ETOOBIG, TLSGPU_EINVAL past the wire arena, TLSGPU_EMISMATCH wrong state).
template <int DL, uint32_t BS>
__device__ __forceinline__ int32_t seal_record_status(bool ok, uint32_t n, uint32_t E, uint64_t wire_off,
                                                      uint64_t wire_cap, uint32_t& body) {
    const uint32_t cur = E + n + DL;
    body = cur + (BS - (cur & (BS - 1)));
    if (!ok) return TLSGPU_EMISMATCH;
    if (n == 0) return 0;
    if (body > 0xffffu) return TLSGPU_ETOOBIG;
    if (wire_off + 5u + body > wire_cap) return TLSGPU_EINVAL;
    return 1;
}

// the cipher lanes' progress hook (pcbc_bulk): blocks issued -> the slot's `loaded` counter
struct FzPub {
    uint32_t addr, base, on;
    __device__ __forceinline__ void operator()(uint32_t blocks) const {
        if (on) fz_st(addr, base + 16u * blocks);
    }
};

template <int NR, int MAC, bool SSL3, int G>
__device__ __forceinline__ void fz_cipher(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                          const tlsgpu_record* __restrict__ recs, uint32_t nrecords,
                                          const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                                          ConnState* __restrict__ states, int32_t* __restrict__ wire_len,
                                          uint32_t cpw, uint64_t wire_cap) {
    constexpr int CID = NR == 10 ? TLSGPU_CIPHER_AES128 : TLSGPU_CIPHER_AES256;
    constexpr int DL = Hash<MAC>::DLEN;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t slot = (threadIdx.x >> 6) * 32 + (lane >> 1);
    const uint32_t h = lane & 1;
    if (slot >= cpw) return;  // both lanes of a pair leave together
    __builtin_amdgcn_s_setprio(TG_AB_CBC_PRIO);
    PairAes aes;
    aes.init();
    const uint32_t a_loaded = FZ_LOADED + 4 * slot, a_done = FZ_DONE + 4 * slot, a_ready = FZ_READY + 4 * slot;
    uint32_t base = 0, k = 0;  // the slot's cumulative plaintext bytes / records
    for (uint32_t cid = blockIdx.x * cpw + slot; cid < nchains; cid += gridDim.x * cpw) {
        const tlsgpu_chain ch = chains[cid];
        ConnState* st = states + ch.state;
        uint4 h1;
        const bool ok = fz_state_ok<CID, MAC, SSL3>(st, h1);
        uint32_t kw[2], ka[NR + 1], kb[NR + 1];
        PairAes::round_keys<NR>(st->ek, h, kw, ka, kb);
        uint32_t va = st->iv[2 * h], vb = st->iv[2 * h + 1];
        const uint32_t fa = st->fixed_iv[2 * h], fb = st->fixed_iv[2 * h + 1];
        const uint32_t E = h1.z ? 16u : 0u;
        bool any = false;
        for (uint32_t j = 0; j < ch.count; j++) {
            const uint32_t r = ch.first + j;
            if (r >= nrecords) break;
            const tlsgpu_record R = recs[r];
            const uint32_t n = R.pt_len;
            uint32_t body;
            const int32_t stt = seal_record_status<DL, 16u>(ok, n, E, R.wire_off, wire_cap, body);
            if (stt != 1) {  // nothing to encrypt: the MAC lane reports wire_len
                if (h == 0) {
                    fz_st(a_loaded, base + n);
                    fz_st(a_done, k + 1);
                }
                base += n;
                k++;
                continue;
            }
            any = true;
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
            const FzPub pub{a_loaded, base, h == 0 ? 1u : 0u};
            if (al) pcbc_bulk<NR, G, true>(aes, kw, ka, kb, va, vb, P, O, nb, pub);
            else pcbc_bulk<NR, G, false>(aes, kw, ka, kb, va, vb, P, O, nb, pub);
            if (h == 0) fz_st(a_loaded, base + n);  // the whole record (the MAC lane loads the partial block)
            // the tail from the MAC lane: wait until it has finished record k
            uint32_t spins = 0;
            while (!fz_ge(fz_ld(a_ready), k + 1)) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > FZ_WATCHDOG) break;
            }
            if (spins > FZ_WATCHDOG) {  // never expected: report and move on instead of hanging
                if (h == 0) wire_len[r] = TLSGPU_EHIP;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const uint32_t T = fz_ld(FZ_TLEN + 4 * slot);
            const uint32_t r16 = n & 15;
            uint8_t* Ot = B + E + (n - r16) + 8 * h;
            const uint32_t tail = FZ_TAIL + TAIL_SLOT * slot + 8 * h;
            for (uint32_t off = 0; off < T; off += 16) {
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 p = *(const __attribute__((address_space(3))) u32x2*)(size_t)(tail + off);
                pair_block<NR>(aes, kw, ka, kb, va, vb, p.x, p.y);
                if (al) st64t<true>(Ot + off, va, vb);
                else st64t<false>(Ot + off, va, vb);
            }
            // the tail slot is free again once both lanes have read it: the pair's lanes
            // are in one wave and read it in the same instruction above
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (h == 0) fz_st(a_done, k + 1);
            base += n;
            k++;
        }
        if (any) {
            st->iv[2 * h] = va;
            st->iv[2 * h + 1] = vb;
        }
    }
}

// MAC lane phases
enum : uint32_t { FZ_NEXT_CHAIN = 0, FZ_NEXT_REC = 1, FZ_BULK = 2, FZ_FIN = 3, FZ_IDLE = 4 };

template <int NR, int MAC, bool SSL3>
__device__ __forceinline__ void fz_mac(const tlsgpu_chain* __restrict__ chains, uint32_t nchains,
                                       const tlsgpu_record* __restrict__ recs, uint32_t nrecords,
                                       const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                                       ConnState* __restrict__ states, int32_t* __restrict__ wire_len, uint32_t cpw,
                                       uint64_t wire_cap) {
    constexpr int CID = NR == 10 ? TLSGPU_CIPHER_AES128 : TLSGPU_CIPHER_AES256;
    using M = RecMac<MAC, SSL3>;
    constexpr int DL = M::DL;
    constexpr uint32_t BS = 16;
    __builtin_amdgcn_s_setprio(TG_AB_FZ_MAC_PRIO);
    const uint32_t slot = ((threadIdx.x >> 6) - FZ_CIPHER_WAVES) * 64 + (threadIdx.x & 63);
    const uint32_t a_loaded = FZ_LOADED + 4 * slot, a_done = FZ_DONE + 4 * slot, a_ready = FZ_READY + 4 * slot;
    uint32_t cid = blockIdx.x * cpw + slot;
    uint32_t phase = (slot < cpw && cid < nchains) ? FZ_NEXT_CHAIN : FZ_IDLE;
    uint32_t base = 0, k = 0;  // the slot's cumulative plaintext bytes / records (as the cipher lanes count)
    uint32_t ch_first = 0, ch_count = 0;  // the current chain's records
    ConnState* st = states;
    bool ok = false;
    uint64_t seq = 0;
    uint32_t E = 0, j = 0, n = 0, nfull = 0, c = 0, ln = 0;
    const uint8_t* P = pt;
    M mac;
    // the BULK phase's ring of two quad-cooperative chunk loads (mac_bulk_coop's pattern: lane
    // q of a quad holds bytes [16q, 16q+16) of each quad member's chunk, one dwordx4 per
    // member, so a load instruction covers 16 whole 64-B pieces)
    uint4 ring0[4], ring1[4];
#pragma unroll
    for (int i = 0; i < 4; i++) ring0[i] = ring1[i] = make_uint4(0, 0, 0, 0);
    bool v0 = false, v1 = false;  // the slot holds this lane's next chunk (slot 0 before slot 1)
    bool coop = true;             // the record's plaintext is 16-byte aligned (else per-lane loads)
    const uint32_t q = threadIdx.x & 3u;
    uint32_t idle_iters = 0;
    // chunk x may be read once the cipher lanes have issued the loads of its bytes (so the
    // read finds the lines in the L2), or TG_AB_FZ_LEAD bytes before
#ifndef TG_AB_FZ_LEAD
#define TG_AB_FZ_LEAD 0
#endif
#ifdef TG_AB_FZ_NOGATE
#define TG_FZ_ALLOWED(x) true
#else
#define TG_FZ_ALLOWED(x) fz_ge(fz_ld(a_loaded) + TG_AB_FZ_LEAD, base + 64u * ((x) + 1))
#endif
    while (__any(phase != FZ_IDLE)) {
        bool progress = false;
        if (__any(phase == FZ_NEXT_CHAIN || phase == FZ_NEXT_REC)) {
            if (phase == FZ_NEXT_CHAIN) {  // start the slot's next chain (prefix_kernel's header test)
                const tlsgpu_chain ch = chains[cid];
                ch_first = ch.first;
                ch_count = ch.count;
                st = states + ch.state;
                uint4 h1;
                ok = fz_state_ok<CID, MAC, SSL3>(st, h1);
                seq = (uint64_t)h1.x | ((uint64_t)h1.y << 32);
                E = h1.z ? BS : 0u;
                j = 0;
                phase = FZ_NEXT_REC;
                progress = true;
            }
            if (phase == FZ_NEXT_REC) {
                const uint32_t r = ch_first + j;
                if (j >= ch_count || r >= nrecords) {  // chain finished
                    if (ok) st->seqnum = seq;
                    cid += gridDim.x * cpw;
                    phase = cid < nchains ? FZ_NEXT_CHAIN : FZ_IDLE;
                } else {
                    const tlsgpu_record R = recs[r];
                    n = R.pt_len;
                    uint32_t body;
                    const int32_t stt = seal_record_status<DL, BS>(ok, n, E, R.wire_off, wire_cap, body);
                    if (stt != 1) {
                        wire_len[r] = stt;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        fz_st(a_ready, k + 1);
                        base += n;
                        k++;
                        j++;
                    } else {
                        P = pt + R.pt_off;
                        coop = ((uintptr_t)P & 15) == 0;
                        mac.begin(st, seq, R.content_type, n);
                        nfull = n >> 6;
                        c = ln = 0;
                        phase = FZ_BULK;
#ifdef TG_AB_FZ_NOMAC
                        c = ln = nfull;
                        phase = FZ_FIN;
#endif
                    }
                }
                progress = true;
            }
        }
        // slot 0 then slot 1: compress the slot's chunk, refill the slot with chunk ln (the
        // other slot's compression hides the load); loads and compressions alternate between
        // the slots in the same order, so chunks are compressed in load order
#define TG_FZ_RING_STEP(rs, vs)                                                                          \
        {                                                                                                \
            if (__any(vs)) {                                                                             \
                uint32_t d[16];                                                                          \
                coop_transpose(rs, q, d);                                                                \
                if (vs) {                                                                                \
                    mac.update(d);                                                                       \
                    c++;                                                                                 \
                    progress = true;                                                                     \
                }                                                                                        \
            }                                                                                            \
            const bool ld = phase == FZ_BULK && coop && ln < nfull && TG_FZ_ALLOWED(ln);                \
            vs = ld;                                                                                     \
            if (__any(ld)) {                                                                             \
                coop_load(ld ? P + 64 * ln : (const uint8_t*)st, q, rs);                                 \
                progress = true;                                                                         \
            }                                                                                            \
            if (ld) ln++;                                                                                \
        }
        TG_FZ_RING_STEP(ring0, v0)
        TG_FZ_RING_STEP(ring1, v1)
#undef TG_FZ_RING_STEP
        if (phase == FZ_BULK && !coop && c < nfull && TG_FZ_ALLOWED(c)) {  // unaligned plaintext: per-lane loads
            uint32_t d[16];
            load64(P + 64 * c, d);
            mac.update(d);
            c++;
            ln++;
            progress = true;
        }
        if (phase == FZ_BULK && c == nfull) phase = FZ_FIN;  // every chunk compressed: the ring is empty
        if (phase == FZ_FIN && fz_ge(fz_ld(a_done), k)) {  // the previous record's tail is consumed
            const uint32_t r = ch_first + j;
            const tlsgpu_record R = recs[r];  // reloaded here rather than kept through the bulk
            const uint32_t r64 = n & 63;
            uint32_t tl[16];
            load_partial(P + 64 * nfull, r64, tl);
            uint32_t m[8];
            mac.finish(tl, (int)r64, n, st, m);
            if (R.flags & TLSGPU_FAULT_BAD_MAC) m[0] = (m[0] & ~0xffu) | ((m[0] + 1u) & 0xffu);
            // CBC tail: P[16 nb ..) | MAC | pad  (tlsrecordlayer.py:597-606), as in mac_kernel
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
                        uint32_t w = 0;
#pragma unroll
                        for (int jj = 0; jj < DL / 4; jj++) w = (i >> 2) == (uint32_t)jj ? m[jj] : w;
                        byte = (w >> (8 * (i & 3))) & 0xffu;
                    } else {
                        byte = padl;
                        if (pos == r16 + DL && (R.flags & TLSGPU_FAULT_BAD_PADDING)) byte = padl + 1;
                    }
                    v |= (pos < T ? byte : 0u) << (8 * b);
                }
                out[q] = v;
            }
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const uint32_t tail = FZ_TAIL + TAIL_SLOT * slot;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                u32x4 v;
                v.x = out[4 * q]; v.y = out[4 * q + 1]; v.z = out[4 * q + 2]; v.w = out[4 * q + 3];
                *(__attribute__((address_space(3))) u32x4*)(size_t)(tail + 16 * q) = v;
            }
            fz_st(FZ_TLEN + 4 * slot, T);
            uint8_t* W = wire + R.wire_off;  // RecordHeader3 (messages.py:36-42)
            const uint32_t cur0 = E + n + DL;
            const uint32_t body = cur0 + (BS - (cur0 & (BS - 1)));
            W[0] = R.content_type;
            W[1] = st->vmaj;
            W[2] = st->vmin;
            W[3] = (uint8_t)(body >> 8);
            W[4] = (uint8_t)body;
            wire_len[r] = (int32_t)(body + 5);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            fz_st(a_ready, k + 1);
            seq++;
            base += n;
            k++;
            j++;
            phase = FZ_NEXT_REC;
            progress = true;
        }
        // nothing moved this round: sleep a little (the cipher lanes are behind); give up
        // after the watchdog bound rather than hang
        if (!__any(progress)) {
            __builtin_amdgcn_s_sleep(2);
            if (++idle_iters > FZ_WATCHDOG) {
                if (phase == FZ_BULK || phase == FZ_FIN) wire_len[ch_first + j] = TLSGPU_EHIP;
                break;
            }
        } else {
            idle_iters = 0;
        }
    }
}

#undef TG_FZ_ALLOWED

// One workgroup per CU (persistent over chain generations), 12 waves: 8 cipher + 4 MAC.
template <int NR, int MAC, bool SSL3, int G>
__global__ void __launch_bounds__(FZ_THREADS, 1)
seal_fused_kernel(const tlsgpu_chain* __restrict__ chains, uint32_t nchains, const tlsgpu_record* __restrict__ recs,
                  uint32_t nrecords, const uint8_t* __restrict__ pt, uint8_t* __restrict__ wire,
                  ConnState* __restrict__ states, int32_t* __restrict__ wire_len, uint32_t cpw, uint64_t wire_cap) {
    aes_lds_fill(nullptr, false);
    for (uint32_t i = threadIdx.x; i < 4 * FZ_SLOTS; i += blockDim.x) fz_st(FZ_LOADED + 4 * i, 0u);
    __syncthreads();
    if ((threadIdx.x >> 6) < FZ_CIPHER_WAVES)
        fz_cipher<NR, MAC, SSL3, G>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, cpw, wire_cap);
    else
        fz_mac<NR, MAC, SSL3>(chains, nchains, recs, nrecords, pt, wire, states, wire_len, cpw, wire_cap);
}

}  // namespace tg

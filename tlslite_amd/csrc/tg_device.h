// tg_device.h -- gfx950 device building blocks: LDS-resident cipher tables,
// AES/3DES/RC4 cores, alignment-aware global loads/stores, and the per-record
// MAC pipeline.  Included by the kernel translation units only.
#pragma once
#include "tg_common.h"
#include "tg_hash.h"

namespace tg {

// ---------------------------------------------------------------- constant tables
__constant__ AesTables c_aes = AesTables();
__constant__ DesSP c_des = DesSP();

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// ---------------------------------------------------------------- global access
// Fast paths for 16/8/4-byte aligned addresses; otherwise byte access.
__device__ __forceinline__ void load16(const uint8_t* p, uint32_t d[4]) {
    uintptr_t a = (uintptr_t)p;
    if ((a & 15) == 0) {
        uint4 v = *(const uint4*)p;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    } else if ((a & 3) == 0) {
        const uint32_t* q = (const uint32_t*)p;
        d[0] = q[0]; d[1] = q[1]; d[2] = q[2]; d[3] = q[3];
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
            d[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
                   ((uint32_t)p[4 * k + 3] << 24);
    }
}
__device__ __forceinline__ void store16(uint8_t* p, const uint32_t d[4]) {
    uintptr_t a = (uintptr_t)p;
    if ((a & 15) == 0) {
        *(uint4*)p = make_uint4(d[0], d[1], d[2], d[3]);
    } else if ((a & 7) == 0) {
        ((uint2*)p)[0] = make_uint2(d[0], d[1]);
        ((uint2*)p)[1] = make_uint2(d[2], d[3]);
    } else if ((a & 3) == 0) {
        uint32_t* q = (uint32_t*)p;
        q[0] = d[0]; q[1] = d[1]; q[2] = d[2]; q[3] = d[3];
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) p[k] = (uint8_t)(d[k >> 2] >> (8 * (k & 3)));
    }
}
__device__ __forceinline__ void load8(const uint8_t* p, uint32_t d[2]) {
    uintptr_t a = (uintptr_t)p;
    if ((a & 7) == 0) {
        uint2 v = *(const uint2*)p;
        d[0] = v.x; d[1] = v.y;
    } else if ((a & 3) == 0) {
        d[0] = ((const uint32_t*)p)[0]; d[1] = ((const uint32_t*)p)[1];
    } else {
#pragma unroll
        for (int k = 0; k < 2; k++)
            d[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
                   ((uint32_t)p[4 * k + 3] << 24);
    }
}
__device__ __forceinline__ void store8(uint8_t* p, const uint32_t d[2]) {
    uintptr_t a = (uintptr_t)p;
    if ((a & 7) == 0) {
        *(uint2*)p = make_uint2(d[0], d[1]);
    } else if ((a & 3) == 0) {
        ((uint32_t*)p)[0] = d[0]; ((uint32_t*)p)[1] = d[1];
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++) p[k] = (uint8_t)(d[k >> 2] >> (8 * (k & 3)));
    }
}
__device__ __forceinline__ void load64(const uint8_t* p, uint32_t d[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++) load16(p + 16 * q, d + 4 * q);
}
__device__ __forceinline__ void store64(uint8_t* p, const uint32_t d[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++) store16(p + 16 * q, d + 4 * q);
}
// first r (< 64) bytes of a chunk; bytes beyond r are zero
__device__ __forceinline__ void load_partial(const uint8_t* p, uint32_t r, uint32_t d[16]) {
    bool al = ((uintptr_t)p & 3) == 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint32_t v = 0;
        if (4 * k + 4 <= (int)r && al) {
            v = ((const uint32_t*)p)[k];
        } else {
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (4 * k + b < (int)r) v |= (uint32_t)p[4 * k + b] << (8 * b);
        }
        d[k] = v;
    }
}

// ---------------------------------------------------------------- AES (LDS T-tables)
// 4 T-tables x 32 lane-copies, 128 KiB.  Entry e of table t for lane copy c
// lives at byte  (t&1)*128 + (t>>1)*65536 + e*256 + c*4, so every lane of a
// 32-lane half-wave reads its own bank: conflict-free ds_read_b32 whatever
// the indices.  The address is built by ONE v_perm_b32 from the state word
// (index byte -> address byte 1) and a per-lane offset word (c*4 in byte 0,
// table-pair select in byte 2); the +128 goes into the ds_read offset field.
constexpr uint32_t AES_LDS_BYTES = 131072;
constexpr uint32_t AES_DEC_LDS_BYTES = 131072 + 32768;  // + inverse S-box (32 copies)

// lds == nullptr: the caller addresses dynamic LDS from byte 0 (no extern symbol)
__device__ __forceinline__ void aes_lds_fill(uint32_t* lds, bool dec) {
    typedef __attribute__((address_space(3))) uint32_t l3_t;
    for (uint32_t idx = threadIdx.x; idx < 32768; idx += blockDim.x) {
        uint32_t t = idx >> 13, e = (idx >> 5) & 255, c = idx & 31;
        uint32_t v = dec ? c_aes.td0[e] : c_aes.te0[e];
        v = (v << (8 * t)) | (t ? (v >> (32 - 8 * t)) : 0u);
        uint32_t byte = (t & 1) * 128 + (t >> 1) * 65536 + e * 256 + c * 4;
        if (lds) lds[byte >> 2] = v;
        else *(l3_t*)(size_t)byte = v;
    }
    if (dec) {
        for (uint32_t idx = threadIdx.x; idx < 8192; idx += blockDim.x) {
            uint32_t e = idx >> 5, c = idx & 31;
            uint32_t byte = 131072 + e * 128 + c * 4;
            // the byte in all four byte lanes: the open path's last round picks each output
            // byte straight out of its lookup with v_perm (tg_open3.h lane_aes_dec)
            const uint32_t v = (uint32_t)c_aes.inv_sbox[e] * 0x01010101u;
            if (lds) lds[byte >> 2] = v;
            else *(l3_t*)(size_t)byte = v;
        }
    }
}

struct AesLds {
    const uint8_t* base;
    uint32_t lo, hi;  // per-lane offset words
    __device__ __forceinline__ void init(const void* lds) {
        base = (const uint8_t*)lds;
        lo = (lane_id() & 31) * 4;
        hi = lo | 0x10000u;
    }
    // T_t[byte b of s]
    template <int T, int B>
    __device__ __forceinline__ uint32_t look(uint32_t s) const {
        constexpr uint32_t sel = 0x0c000000u | (2u << 16) | ((4u + B) << 8) | 0u;
        uint32_t addr = perm(s, T >= 2 ? hi : lo, sel);
        return *(const uint32_t*)(base + addr + (T & 1) * 128);
    }
    // inverse S-box of byte b of s (decrypt tables only)
    template <int B>
    __device__ __forceinline__ uint32_t isb(uint32_t s) const {
        uint32_t idx = (s >> (8 * B)) & 0xff;
        return *(const uint32_t*)(base + 131072 + idx * 128 + lo) & 0xffu;  // entries replicate the byte
    }
};

template <int NR>
__device__ __forceinline__ void aes_encrypt(uint32_t s[4], const uint32_t* rk, const AesLds& L) {
    uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t t0 = L.look<0, 0>(s0) ^ L.look<1, 1>(s1) ^ L.look<2, 2>(s2) ^ L.look<3, 3>(s3) ^ rk[4 * r];
        uint32_t t1 = L.look<0, 0>(s1) ^ L.look<1, 1>(s2) ^ L.look<2, 2>(s3) ^ L.look<3, 3>(s0) ^ rk[4 * r + 1];
        uint32_t t2 = L.look<0, 0>(s2) ^ L.look<1, 1>(s3) ^ L.look<2, 2>(s0) ^ L.look<3, 3>(s1) ^ rk[4 * r + 2];
        uint32_t t3 = L.look<0, 0>(s3) ^ L.look<1, 1>(s0) ^ L.look<2, 2>(s1) ^ L.look<3, 3>(s2) ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // final round: S-box byte r sits at byte r of table (r+2)&3
    uint32_t u0 = (L.look<2, 0>(s0) & 0xffu) | (L.look<3, 1>(s1) & 0xff00u) | (L.look<0, 2>(s2) & 0xff0000u) |
                  (L.look<1, 3>(s3) & 0xff000000u);
    uint32_t u1 = (L.look<2, 0>(s1) & 0xffu) | (L.look<3, 1>(s2) & 0xff00u) | (L.look<0, 2>(s3) & 0xff0000u) |
                  (L.look<1, 3>(s0) & 0xff000000u);
    uint32_t u2 = (L.look<2, 0>(s2) & 0xffu) | (L.look<3, 1>(s3) & 0xff00u) | (L.look<0, 2>(s0) & 0xff0000u) |
                  (L.look<1, 3>(s1) & 0xff000000u);
    uint32_t u3 = (L.look<2, 0>(s3) & 0xffu) | (L.look<3, 1>(s0) & 0xff00u) | (L.look<0, 2>(s1) & 0xff0000u) |
                  (L.look<1, 3>(s2) & 0xff000000u);
    s[0] = u0 ^ rk[4 * NR]; s[1] = u1 ^ rk[4 * NR + 1]; s[2] = u2 ^ rk[4 * NR + 2]; s[3] = u3 ^ rk[4 * NR + 3];
}

// equivalent inverse cipher (FIPS-197 §5.3.5); InvShiftRows reads column c-k for row k
template <int NR>
__device__ __forceinline__ void aes_decrypt(uint32_t s[4], const uint32_t* dk, const AesLds& L) {
    uint32_t s0 = s[0] ^ dk[0], s1 = s[1] ^ dk[1], s2 = s[2] ^ dk[2], s3 = s[3] ^ dk[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t t0 = L.look<0, 0>(s0) ^ L.look<1, 1>(s3) ^ L.look<2, 2>(s2) ^ L.look<3, 3>(s1) ^ dk[4 * r];
        uint32_t t1 = L.look<0, 0>(s1) ^ L.look<1, 1>(s0) ^ L.look<2, 2>(s3) ^ L.look<3, 3>(s2) ^ dk[4 * r + 1];
        uint32_t t2 = L.look<0, 0>(s2) ^ L.look<1, 1>(s1) ^ L.look<2, 2>(s0) ^ L.look<3, 3>(s3) ^ dk[4 * r + 2];
        uint32_t t3 = L.look<0, 0>(s3) ^ L.look<1, 1>(s2) ^ L.look<2, 2>(s1) ^ L.look<3, 3>(s0) ^ dk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    uint32_t u0 = L.isb<0>(s0) | (L.isb<1>(s3) << 8) | (L.isb<2>(s2) << 16) | (L.isb<3>(s1) << 24);
    uint32_t u1 = L.isb<0>(s1) | (L.isb<1>(s0) << 8) | (L.isb<2>(s3) << 16) | (L.isb<3>(s2) << 24);
    uint32_t u2 = L.isb<0>(s2) | (L.isb<1>(s1) << 8) | (L.isb<2>(s0) << 16) | (L.isb<3>(s3) << 24);
    uint32_t u3 = L.isb<0>(s3) | (L.isb<1>(s2) << 8) | (L.isb<2>(s1) << 16) | (L.isb<3>(s0) << 24);
    s[0] = u0 ^ dk[4 * NR]; s[1] = u1 ^ dk[4 * NR + 1]; s[2] = u2 ^ dk[4 * NR + 2]; s[3] = u3 ^ dk[4 * NR + 3];
}

// ---------------------------------------------------------------- 3DES (LDS SP-tables)
// 8 SP tables x 64 entries x 32 lane copies = 64 KiB; entry (k, x) for lane
// copy c at byte ((k*64 + x) << 7) + c*4 (conflict-free like the AES tables).
constexpr uint32_t DES_LDS_BYTES = 65536;

__device__ __forceinline__ void des_lds_fill(uint32_t* lds) {
    for (uint32_t idx = threadIdx.x; idx < 16384; idx += blockDim.x) {
        uint32_t kx = idx >> 5, c = idx & 31;
        lds[(kx << 5) + c] = c_des.sp[kx >> 6][kx & 63];
    }
}

struct DesLds {
    const uint8_t* base;
    uint32_t lo;
    __device__ __forceinline__ void init(const void* lds) {
        base = (const uint8_t*)lds;
        lo = (lane_id() & 31) * 4;
    }
    template <int K>
    __device__ __forceinline__ uint32_t sp(uint32_t six) const {
        return *(const uint32_t*)(base + ((six & 63u) << 7) + lo + K * 8192);
    }
};

// 16 DES rounds on rotated halves (l, r); ks = 16 x {even, odd}; DEC walks keys backwards
template <bool DEC>
__device__ __forceinline__ void des_rounds(uint32_t& l, uint32_t& r, const uint32_t* ks, const DesLds& L) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
        int k = DEC ? 15 - i : i;
        uint32_t w = r ^ ks[2 * k];
        uint32_t v = ((r >> 4) | (r << 28)) ^ ks[2 * k + 1];
        uint32_t f = L.sp<7>(w) ^ L.sp<5>(w >> 8) ^ L.sp<3>(w >> 16) ^ L.sp<1>(w >> 24) ^ L.sp<6>(v) ^
                     L.sp<4>(v >> 8) ^ L.sp<2>(v >> 16) ^ L.sp<0>(v >> 24);
        uint32_t t = l ^ f;
        l = r;
        r = t;
    }
    // leave (l, r) = (R16, L16): the preoutput order
    uint32_t t = l; l = r; r = t;
}

// FIPS 46 IP / IP^-1 as swap-move networks.  des_ip leaves both halves
// rotated left by one (the SP-table domain); des_fp takes rotated halves of
// the preoutput R16||L16 and returns the output block (both big-endian words).
__device__ __forceinline__ void des_ip(uint32_t& l, uint32_t& r) {
    uint32_t w;
    w = ((l >> 4) ^ r) & 0x0f0f0f0fu; r ^= w; l ^= w << 4;
    w = ((l >> 16) ^ r) & 0x0000ffffu; r ^= w; l ^= w << 16;
    w = ((r >> 2) ^ l) & 0x33333333u; l ^= w; r ^= w << 2;
    w = ((r >> 8) ^ l) & 0x00ff00ffu; l ^= w; r ^= w << 8;
    r = (r << 1) | (r >> 31);
    w = (l ^ r) & 0xaaaaaaaau; l ^= w; r ^= w;
    l = (l << 1) | (l >> 31);
}
__device__ __forceinline__ void des_fp(uint32_t& l, uint32_t& r) {
    uint32_t w;
    l = (l >> 1) | (l << 31);
    w = (l ^ r) & 0xaaaaaaaau; l ^= w; r ^= w;
    r = (r >> 1) | (r << 31);
    w = ((r >> 8) ^ l) & 0x00ff00ffu; l ^= w; r ^= w << 8;
    w = ((r >> 2) ^ l) & 0x33333333u; l ^= w; r ^= w << 2;
    w = ((l >> 16) ^ r) & 0x0000ffffu; r ^= w; l ^= w << 16;
    w = ((l >> 4) ^ r) & 0x0f0f0f0fu; r ^= w; l ^= w << 4;
}

// block in/out as two big-endian words; EDE: E_K3(D_K2(E_K1(x))).  Between
// the three DES passes FP and IP cancel and des_rounds already leaves the
// halves as (R16, L16) = the next pass's (L0, R0).
template <bool DEC>
__device__ __forceinline__ void tdes_block(uint32_t& hi, uint32_t& lo, const uint32_t* ks, const DesLds& L) {
    uint32_t l = hi, r = lo;
    des_ip(l, r);
    if (!DEC) {
        des_rounds<false>(l, r, ks, L);
        des_rounds<true>(l, r, ks + 32, L);
        des_rounds<false>(l, r, ks + 64, L);
    } else {
        des_rounds<true>(l, r, ks + 64, L);
        des_rounds<false>(l, r, ks + 32, L);
        des_rounds<true>(l, r, ks, L);
    }
    des_fp(l, r);
    hi = l;
    lo = r;
}

// ---------------------------------------------------------------- RC4 (per-lane S in LDS)
// byte S[x] of lane l at LDS byte x*64 + l (16 KiB per wave)
struct Rc4Lds {
    uint8_t* base;
    uint32_t i, j;
    __device__ __forceinline__ void init(void* lds) {
        base = (uint8_t*)lds + (threadIdx.x >> 6) * 16384 + lane_id();
    }
    __device__ __forceinline__ uint32_t ks() {
        i = (i + 1) & 255;
        uint32_t si = base[i << 6];
        j = (j + si) & 255;
        uint32_t sj = base[j << 6];
        base[i << 6] = (uint8_t)sj;
        base[j << 6] = (uint8_t)si;
        return base[((si + sj) & 255) << 6];
    }
    __device__ __forceinline__ void load(const ConnState* st) {
        const uint32_t* S = (const uint32_t*)st->rc4_S;
        for (int q = 0; q < 64; q++) {
            uint32_t v = S[q];
#pragma unroll
            for (int b = 0; b < 4; b++) base[(4 * q + b) << 6] = (uint8_t)(v >> (8 * b));
        }
        i = st->rc4_i;
        j = st->rc4_j;
    }
    __device__ __forceinline__ void save(ConnState* st) {
        uint32_t* S = (uint32_t*)st->rc4_S;
        for (int q = 0; q < 64; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) v |= (uint32_t)base[(4 * q + b) << 6] << (8 * b);
            S[q] = v;
        }
        st->rc4_i = i;
        st->rc4_j = j;
    }
};
constexpr uint32_t RC4_LDS_BYTES_PER_WAVE = 16384;

// ---------------------------------------------------------------- cipher adapters
// Uniform interface over the stream of bytes  [explicit IV] | P | MAC | pad :
//   enc_block(d)  encrypt one cipher block (CBC) in place  (block ciphers)
//   enc64(d)      encrypt 64 stream bytes (4 AES / 8 DES blocks / 64 RC4 bytes)
template <int NR>
struct AesCbc {
    static constexpr int BS = 16;
    static constexpr bool STREAM = false;
    uint32_t rk[4 * (NR + 1)];
    uint32_t iv[4];
    AesLds L;
    __device__ __forceinline__ void load(const ConnState* st, const void* lds) {
        L.init(lds);
#pragma unroll
        for (int k = 0; k < 4 * (NR + 1); k++) rk[k] = st->ek[k];
#pragma unroll
        for (int k = 0; k < 4; k++) iv[k] = st->iv[k];
    }
    __device__ __forceinline__ void save(ConnState* st) {
#pragma unroll
        for (int k = 0; k < 4; k++) st->iv[k] = iv[k];
    }
    __device__ __forceinline__ void enc_block(uint32_t* d) {
        uint32_t s[4] = {d[0] ^ iv[0], d[1] ^ iv[1], d[2] ^ iv[2], d[3] ^ iv[3]};
        aes_encrypt<NR>(s, rk, L);
#pragma unroll
        for (int k = 0; k < 4; k++) iv[k] = d[k] = s[k];
    }
    __device__ __forceinline__ void enc64(uint32_t d[16]) {
#pragma unroll
        for (int b = 0; b < 4; b++) enc_block(d + 4 * b);
    }
    __device__ __forceinline__ void load_block(const uint8_t* p, uint32_t* d) { load16(p, d); }
    __device__ __forceinline__ void store_block(uint8_t* p, const uint32_t* d) { store16(p, d); }
};

struct TdesCbc {
    static constexpr int BS = 8;
    static constexpr bool STREAM = false;
    uint32_t ks[96];
    uint32_t iv[2];
    DesLds L;
    __device__ __forceinline__ void load(const ConnState* st, const void* lds) {
        L.init(lds);
        const uint32_t* k = &st->des[0][0];
#pragma unroll
        for (int q = 0; q < 96; q++) ks[q] = k[q];
        iv[0] = st->iv[0]; iv[1] = st->iv[1];
    }
    __device__ __forceinline__ void save(ConnState* st) { st->iv[0] = iv[0]; st->iv[1] = iv[1]; }
    __device__ __forceinline__ void enc_block(uint32_t* d) {
        uint32_t hi = bswap32(d[0] ^ iv[0]), lo = bswap32(d[1] ^ iv[1]);
        tdes_block<false>(hi, lo, ks, L);
        iv[0] = d[0] = bswap32(hi);
        iv[1] = d[1] = bswap32(lo);
    }
    // CBC decrypt (openssl_tripledes.py:40-47): p = D(c) ^ iv, iv = c
    __device__ __forceinline__ void dec_block(uint32_t* d) {
        const uint32_t c0 = d[0], c1 = d[1];
        uint32_t hi = bswap32(c0), lo = bswap32(c1);
        tdes_block<true>(hi, lo, ks, L);
        d[0] = bswap32(hi) ^ iv[0];
        d[1] = bswap32(lo) ^ iv[1];
        iv[0] = c0;
        iv[1] = c1;
    }
    __device__ __forceinline__ void enc64(uint32_t d[16]) {
#pragma unroll
        for (int b = 0; b < 8; b++) enc_block(d + 2 * b);
    }
    __device__ __forceinline__ void load_block(const uint8_t* p, uint32_t* d) { load8(p, d); }
    __device__ __forceinline__ void store_block(uint8_t* p, const uint32_t* d) { store8(p, d); }
};

struct Rc4Stream {
    static constexpr int BS = 1;
    static constexpr bool STREAM = true;
    Rc4Lds R;
    __device__ __forceinline__ void load(const ConnState* st, void* lds) {
        R.init(lds);
        R.load(st);
    }
    __device__ __forceinline__ void save(ConnState* st) { R.save(st); }
    __device__ __forceinline__ void enc64(uint32_t d[16]) {
#pragma unroll 4
        for (int k = 0; k < 16; k++) {
            uint32_t a = R.ks(), b = R.ks(), c = R.ks(), e = R.ks();
            d[k] ^= a | (b << 8) | (c << 16) | (e << 24);
        }
    }
};

// ---------------------------------------------------------------- record MAC
// Streaming MAC over  prefix | P  where the prefix (HMAC ipad block / MAC_SSL
// key||pad1, then seq|type|[ver]|len) is fixed-length per variant, so P sits
// at a compile-time offset A inside its first hash block.  Each 64-byte P
// chunk completes exactly one hash block whose 16 words are funnelled out of
// (last 4 dwords of the previous chunk, this chunk) with one v_perm each.
template <int MAC, bool SSL3>
struct RecMac {
    using H = Hash<MAC>;
    static constexpr int A = SSL3 ? (MAC == TLSGPU_MAC_SHA1 ? 7 : 11) : 13;
    static constexpr int PREFIX = SSL3 ? (MAC == TLSGPU_MAC_SHA1 ? 71 : 75) : 77;
    static constexpr int I0 = (64 - A) >> 2;  // first window dword (window = prev[0..15] | cur[0..15])
    static constexpr int SH = (64 - A) & 3;   // byte offset inside it
    static constexpr int DL = H::DLEN;
    uint32_t h[8];
    uint32_t prev[4];  // window dwords 12..15 of the previous chunk

    // message word from window bytes [q, q+4) where q = 4*(I0+k) + SH
    template <int K>
    __device__ __forceinline__ static uint32_t word(uint32_t wlo, uint32_t whi) {
        if (H::BE) {
            constexpr uint32_t sel = ((uint32_t)SH << 24) | ((uint32_t)(SH + 1) << 16) | ((uint32_t)(SH + 2) << 8) | (uint32_t)(SH + 3);
            return perm(whi, wlo, sel);
        } else {
            return __builtin_amdgcn_alignbyte(whi, wlo, SH);
        }
    }
    // window dword accessor: idx 12..15 -> prev, 16..31 -> cur
    __device__ __forceinline__ void block_words(const uint32_t cur[16], uint32_t w[16]) const {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            int i = I0 + k;
            uint32_t lo = i < 16 ? prev[i - 12] : cur[i - 16];
            uint32_t hi = (i + 1) < 16 ? prev[i + 1 - 12] : cur[i + 1 - 16];
            w[k] = word<0>(lo, hi);
        }
    }

    __device__ __forceinline__ void begin(const ConnState* st, uint64_t seq, uint32_t ctype, uint32_t n) {
        uint8_t hb[13];
        int hl = 0;
        if (SSL3 && MAC == TLSGPU_MAC_SHA1) {
            // first block: key(20) | 0x36 x 40 | seq[0..4)  (mathtls.py:135-140, tlsrecordlayer.py:573-575)
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 5; k++) w[k] = st->mac_key[k];
#pragma unroll
            for (int k = 5; k < 15; k++) w[k] = 0x36363636u;
            w[15] = (uint32_t)(seq >> 32);
            H::init(h);
            H::compress(h, w);
#pragma unroll
            for (int b = 4; b < 8; b++) hb[hl++] = (uint8_t)(seq >> (56 - 8 * b));
        } else {
#pragma unroll
            for (int k = 0; k < H::NS; k++) h[k] = st->mac_in[k];
#pragma unroll
            for (int b = 0; b < 8; b++) hb[hl++] = (uint8_t)(seq >> (56 - 8 * b));
        }
        hb[hl++] = (uint8_t)ctype;
        if (!SSL3) {
            hb[hl++] = st->vmaj;
            hb[hl++] = st->vmin;
        }
        hb[hl++] = (uint8_t)(n >> 8);
        hb[hl++] = (uint8_t)n;
        prev[0] = prev[1] = prev[2] = prev[3] = 0;
#pragma unroll
        for (int j = 0; j < A; j++) {
            int pos = 64 - A + j - 48;
            prev[pos >> 2] |= (uint32_t)hb[j] << (8 * (pos & 3));
        }
    }

    __device__ __forceinline__ void update(const uint32_t cur[16]) {
        uint32_t w[16];
        block_words(cur, w);
        H::compress(h, w);
        prev[0] = cur[12]; prev[1] = cur[13]; prev[2] = cur[14]; prev[3] = cur[15];
    }

    // keep the first v bytes of word w (message order), put 0x80 after them
    __device__ __forceinline__ static uint32_t pad_word(uint32_t w, int v) {
        if (v >= 4) return w;
        if (v < 0) return 0u;
        if (H::BE) {
            uint32_t keep = v == 0 ? 0u : (0xffffffffu << (32 - 8 * v));
            return (w & keep) | (0x80u << (24 - 8 * v));
        } else {
            uint32_t keep = (1u << (8 * v)) - 1u;
            return (w & keep) | (0x80u << (8 * v));
        }
    }

    // cur holds the r (< 64) trailing P bytes, zero beyond; n = total P length.
    // Produces the MAC as stream-order LE dwords in mac[0..DL/4).
    __device__ __forceinline__ void finish(const uint32_t cur[16], int r, uint32_t n, const ConnState* st,
                                           uint32_t mac[8]) {
        const int valid = A + r;
        const uint64_t bits = (uint64_t)(PREFIX + n) * 8u;
        const uint32_t bhi = (uint32_t)(bits >> 32), blo = (uint32_t)bits;
        uint32_t w[16];
        block_words(cur, w);
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = pad_word(w[k], valid - 4 * k);
        const bool two = valid + 9 > 64;
        if (!two) {
            if (H::BE) { w[14] = bhi; w[15] = blo; }
            else { w[14] = blo; w[15] = bhi; }
        }
        H::compress(h, w);
        if (two) {
            uint32_t z[16];
            uint32_t p2[4] = {cur[12], cur[13], cur[14], cur[15]};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                int i = I0 + k;  // window = cur | zeros
                uint32_t lo = i < 16 ? p2[i - 12] : 0u;
                uint32_t hi = (i + 1) < 16 ? p2[i + 1 - 12] : 0u;
                z[k] = pad_word(word<0>(lo, hi), valid - 64 - 4 * k);
            }
            if (H::BE) { z[14] = bhi; z[15] = blo; }
            else { z[14] = blo; z[15] = bhi; }
            H::compress(h, z);
        }
        // outer hash
        uint32_t o[8];
        uint32_t x[16];
#pragma unroll
        for (int k = 0; k < 16; k++) x[k] = 0;
        if (SSL3 && MAC == TLSGPU_MAC_SHA1) {
            // key(20) | 0x5c x 40 | inner(20)   (mathtls.py:138-150)
#pragma unroll
            for (int k = 0; k < 5; k++) x[k] = st->mac_key[k];
#pragma unroll
            for (int k = 5; k < 15; k++) x[k] = 0x5c5c5c5cu;
            x[15] = h[0];
            H::init(o);
            H::compress(o, x);
            uint32_t y[16];
#pragma unroll
            for (int k = 0; k < 16; k++) y[k] = 0;
            y[0] = h[1]; y[1] = h[2]; y[2] = h[3]; y[3] = h[4];
            y[4] = 0x80000000u;
            y[15] = 80u * 8u;
            H::compress(o, y);
        } else {
#pragma unroll
            for (int k = 0; k < H::NS; k++) o[k] = st->mac_out[k];
#pragma unroll
            for (int k = 0; k < H::NS; k++) x[k] = h[k];
            if (H::BE) {
                x[DL / 4] = 0x80000000u;
                x[15] = (64u + DL) * 8u;
            } else {
                x[DL / 4] = 0x80u;
                x[14] = (64u + DL) * 8u;
            }
            H::compress(o, x);
        }
#pragma unroll
        for (int k = 0; k < DL / 4; k++) mac[k] = H::BE ? bswap32(o[k]) : o[k];
    }
};

}  // namespace tg

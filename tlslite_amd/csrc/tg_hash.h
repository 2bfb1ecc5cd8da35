// tg_hash.h -- SHA-1 / SHA-256 / MD5 compression functions (FIPS 180-4,
// RFC 1321) for both host (HMAC midstate setup) and gfx950 device code.
// The message schedule is kept in a rolling 16-word window so that, fully
// unrolled, the whole compression lives in VGPRs.
#pragma once
#include "tg_common.h"

#define TG_HD __host__ __device__ __forceinline__

namespace tg {

TG_HD uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
TG_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// 3-input boolean functions: one v_bitop3_b32 on gfx950 (truth table indexed
// by a<<2 | b<<1 | c), plain C on the host.
#ifdef __HIP_DEVICE_COMPILE__
#define TG_BOP3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
TG_HD uint32_t bx3(uint32_t a, uint32_t b, uint32_t c) { return TG_BOP3(a, b, c, 0x96); }        // a^b^c
TG_HD uint32_t bch(uint32_t a, uint32_t b, uint32_t c) { return TG_BOP3(a, b, c, 0xCA); }        // a?b:c
TG_HD uint32_t bmaj(uint32_t a, uint32_t b, uint32_t c) { return TG_BOP3(a, b, c, 0xE8); }       // majority
TG_HD uint32_t bmd5i(uint32_t b, uint32_t c, uint32_t d) { return TG_BOP3(b, c, d, 0x39); }      // c^(b|~d)
#else
TG_HD uint32_t bx3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
TG_HD uint32_t bch(uint32_t a, uint32_t b, uint32_t c) { return (a & b) | (~a & c); }
TG_HD uint32_t bmaj(uint32_t a, uint32_t b, uint32_t c) { return (a & b) | (a & c) | (b & c); }
TG_HD uint32_t bmd5i(uint32_t b, uint32_t c, uint32_t d) { return c ^ (b | ~d); }
#endif

template <int MAC>
struct Hash;

template <>
struct Hash<TLSGPU_MAC_SHA1> {
    static constexpr int NS = 5, DLEN = 20;
    static constexpr bool BE = true;
    TG_HD static void init(uint32_t h[8]) {
        for (int i = 0; i < 5; i++) h[i] = SHA1_IV[i];
    }
    static constexpr int ROUNDS = 80;
    // round t on the working variables s = {a, b, c, d, e} (fully unrolled callers: the
    // array shifts are register renames)
    TG_HD static void round(int t, uint32_t s[8], uint32_t w[16]) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl32(bx3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) {
            f = bch(s[1], s[2], s[3]);
            k = 0x5A827999u;
        } else if (t < 40) {
            f = bx3(s[1], s[2], s[3]);
            k = 0x6ED9EBA1u;
        } else if (t < 60) {
            f = bmaj(s[1], s[2], s[3]);
            k = 0x8F1BBCDCu;
        } else {
            f = bx3(s[1], s[2], s[3]);
            k = 0xCA62C1D6u;
        }
        // two v_add3_u32 (4-cycle) -- four 2-cycle v_add_u32 measured 1-2 % slower on
        // cfg2 / cfg3 (profiles/r03/ab_mac.txt)
        const uint32_t tmp = rotl32(s[0], 5) + f + s[4] + k + wt;
        s[4] = s[3];
        s[3] = s[2];
        s[2] = rotl32(s[1], 30);
        s[1] = s[0];
        s[0] = tmp;
    }
    TG_HD static void compress(uint32_t h[8], uint32_t w[16]) {
        uint32_t s[8] = {h[0], h[1], h[2], h[3], h[4], 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 80; t++) round(t, s, w);
        h[0] += s[0]; h[1] += s[1]; h[2] += s[2]; h[3] += s[3]; h[4] += s[4];
    }
};

struct Sha256K {
    static constexpr uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
};

template <>
struct Hash<TLSGPU_MAC_SHA256> {
    static constexpr int NS = 8, DLEN = 32;
    static constexpr bool BE = true;
    TG_HD static void init(uint32_t h[8]) {
        for (int i = 0; i < 8; i++) h[i] = SHA256_IV[i];
    }
    static constexpr int ROUNDS = 64;
    // round t on the working variables s = {a, b, c, d, e, f, g, h}
    TG_HD static void round(int t, uint32_t s[8], uint32_t w[16]) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
            uint32_t s0 = bx3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
            uint32_t s1 = bx3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
            wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
            w[t & 15] = wt;
        }
        const uint32_t S1 = bx3(rotr32(s[4], 6), rotr32(s[4], 11), rotr32(s[4], 25));
        const uint32_t ch = bch(s[4], s[5], s[6]);
        const uint32_t t1 = s[7] + S1 + ch + Sha256K::K[t] + wt;
        const uint32_t S0 = bx3(rotr32(s[0], 2), rotr32(s[0], 13), rotr32(s[0], 22));
        const uint32_t mj = bmaj(s[0], s[1], s[2]);
        s[7] = s[6]; s[6] = s[5]; s[5] = s[4]; s[4] = s[3] + t1;
        s[3] = s[2]; s[2] = s[1]; s[1] = s[0]; s[0] = t1 + S0 + mj;
    }
    TG_HD static void compress(uint32_t h[8], uint32_t w[16]) {
        uint32_t s[8] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]};
#pragma unroll
        for (int t = 0; t < 64; t++) round(t, s, w);
#pragma unroll
        for (int i = 0; i < 8; i++) h[i] += s[i];
    }
};

struct Md5K {
    static constexpr uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static constexpr uint8_t R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                      5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                      4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                      6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
};

template <>
struct Hash<TLSGPU_MAC_MD5> {
    static constexpr int NS = 4, DLEN = 16;
    static constexpr bool BE = false;
    TG_HD static void init(uint32_t h[8]) {
        for (int i = 0; i < 4; i++) h[i] = MD5_IV[i];
    }
    TG_HD static void compress(uint32_t h[8], uint32_t w[16]) {
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#pragma unroll
        for (int i = 0; i < 64; i++) {
            uint32_t f;
            int g;
            if (i < 16) {
                f = bch(b, c, d);
                g = i;
            } else if (i < 32) {
                f = bch(d, b, c);
                g = (5 * i + 1) & 15;
            } else if (i < 48) {
                f = bx3(b, c, d);
                g = (3 * i + 5) & 15;
            } else {
                f = bmd5i(b, c, d);
                g = (7 * i) & 15;
            }
            uint32_t x = a + f + Md5K::K[i] + w[g];
            a = d;
            d = c;
            c = b;
            b = b + rotl32(x, Md5K::R[i]);
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d;
    }
};

}  // namespace tg

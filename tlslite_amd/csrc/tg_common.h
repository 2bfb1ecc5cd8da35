// tg_common.h -- internal definitions shared by the host code and the gfx950
// kernels of libtlsgpu.so.  Tables are generated at compile time (constexpr)
// from their defining arithmetic, not pasted: AES S-box from GF(2^8)
// inversion + affine map (FIPS-197 §5.1.1), T-tables from MixColumns; DES
// S-boxes and permutations are the FIPS 46-3 constants.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/tlsgpu.h"

namespace tg {

// [off, off + len) lies inside an arena of cap bytes (no wrap-around): the per-record range
// check of the seal / open kernels against the caller's arena sizes (ABI 6)
__host__ __device__ inline bool in_arena(uint64_t off, uint64_t len, uint64_t cap) {
    return len <= cap && off <= cap - len;
}

// ---------------------------------------------------------------- state
// Device-resident connection state (one per connection / chain).  All byte
// strings that feed the cipher are packed as little-endian dwords in stream
// order (byte i of the string in bits 8*(i%4) of word i/4).
struct ConnState {
    uint32_t cipher;       // TLSGPU_CIPHER_*
    uint32_t mac;          // TLSGPU_MAC_* (0 for a raw cipher context)
    uint8_t vmaj, vmin, bs, maclen;
    uint32_t ssl3;         // 1 when version == (3,0): MAC_SSL instead of HMAC
    uint64_t seqnum;       // _ConnectionState.seqnum (tlsrecordlayer.py:31-37)
    uint32_t explicit_iv;  // 1 when version >= (3,2) and block cipher (tlsrecordlayer.py:594-595)
    uint32_t raw;          // 1 for cipher-object contexts (no MAC / framing)
    uint32_t iv[4];        // CBC residue = self.IV (python_aes.py:44)
    uint32_t fixed_iv[4];  // fixedIVBlock (tlsrecordlayer.py:1146-1149)
    uint32_t mac_in[8];    // HMAC: H-state after (K^ipad); SSL3-MD5: after K||pad1
    uint32_t mac_out[8];   // HMAC: H-state after (K^opad); SSL3-MD5: after K||pad2
    uint32_t mac_key[8];   // SSL3-SHA1 MAC key, big-endian words (20 bytes used)
    uint32_t mac_key_len;
    uint32_t rc4_i, rc4_j;
    uint32_t pad0[21];     // ek starts on a 128-B line: HBM reads are 128-B requests even for
                           // scattered narrow loads (tools/traffic_calib.hip), and the 240 B of
                           // AES-256 round keys then take 2 lines instead of 3
    uint32_t ek[60];       // AES encryption round keys, LE column words
    uint32_t dk[60];       // AES equivalent-inverse-cipher round keys, LE column words
    uint32_t des[3][32];   // 3DES: per key, 16 rounds x {even-box word, odd-box word}
    uint8_t rc4_S[256];    // Python_RC4.S (python_rc4.py:21)
    uint32_t closed;       // open direction: 1 once a TLSGPU_CHAIN_STOP_ON_ALERT chain of this state hit
                           // an alert -- the reference closes the connection there (tlsrecordlayer.py:
                           // 524-529, 1039-1042); every later open of the state reports
                           // TLSGPU_ALERT_SKIPPED and leaves it unchanged (round 5)
    uint8_t reserved[TLSGPU_CONN_STATE_BYTES - 1380];
};
// Line map (128 B, the HBM request size): line 0 = everything prefix_kernel reads, the
// chain's CBC residue and fixedIVBlock ([0,64)) and the HMAC midstates ([64,128), mac_kernel);
// lines 2-3 = the AES round keys ([256,496)).  A cipher-kernel chain reads 3 lines.
static_assert(__builtin_offsetof(ConnState, iv) == 32 && __builtin_offsetof(ConnState, fixed_iv) == 48,
              "prefix/cipher fields in the first sector");
static_assert(__builtin_offsetof(ConnState, mac_in) == 64, "HMAC midstates in the second sector");
static_assert(__builtin_offsetof(ConnState, ek) == 256, "round keys line-aligned");
static_assert(__builtin_offsetof(ConnState, closed) == 1376, "closed mark after the RC4 state");
// the ABI blob (tlsgpu_conn_state) and the device struct must have the same stride
static_assert(sizeof(ConnState) == TLSGPU_CONN_STATE_BYTES, "ConnState must be exactly 2048 bytes");

// ---------------------------------------------------------------- AES tables
constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) p ^= a;
        bool hi = a & 0x80;
        a = (uint8_t)(a << 1);
        if (hi) a ^= 0x1b;
        b >>= 1;
    }
    return p;
}
constexpr uint8_t gf_inv(uint8_t x) {
    // x^254 by square-and-multiply (0 -> 0)
    uint8_t r = 1, b = x;
    int e = 254;
    while (e) {
        if (e & 1) r = gf_mul(r, b);
        b = gf_mul(b, b);
        e >>= 1;
    }
    return x ? r : 0;
}
constexpr uint8_t rotl8(uint8_t x, int n) { return (uint8_t)((x << n) | (x >> (8 - n))); }
constexpr uint8_t aes_sbox(uint8_t x) {
    uint8_t b = gf_inv(x);
    return (uint8_t)(b ^ rotl8(b, 1) ^ rotl8(b, 2) ^ rotl8(b, 3) ^ rotl8(b, 4) ^ 0x63);
}

struct AesTables {
    uint8_t sbox[256];
    uint8_t inv_sbox[256];
    uint32_t te0[256];  // LE: bytes (2s, s, s, 3s)  -- MixColumns column for input row 0
    uint32_t td0[256];  // LE: bytes (14i, 9i, 13i, 11i) of i = InvS(x)
    uint32_t im0[256];  // LE: bytes (14x, 9x, 13x, 11x) -- InvMixColumns of a key byte
    constexpr AesTables() : sbox(), inv_sbox(), te0(), td0(), im0() {
        for (int x = 0; x < 256; x++) {
            uint8_t s = aes_sbox((uint8_t)x);
            sbox[x] = s;
            inv_sbox[s] = (uint8_t)x;
        }
        for (int x = 0; x < 256; x++) {
            uint8_t s = sbox[x], i = inv_sbox[x];
            te0[x] = (uint32_t)gf_mul(s, 2) | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)gf_mul(s, 3) << 24);
            td0[x] = (uint32_t)gf_mul(i, 14) | ((uint32_t)gf_mul(i, 9) << 8) | ((uint32_t)gf_mul(i, 13) << 16) |
                     ((uint32_t)gf_mul(i, 11) << 24);
            uint8_t b = (uint8_t)x;
            im0[x] = (uint32_t)gf_mul(b, 14) | ((uint32_t)gf_mul(b, 9) << 8) | ((uint32_t)gf_mul(b, 13) << 16) |
                     ((uint32_t)gf_mul(b, 11) << 24);
        }
    }
};

// ---------------------------------------------------------------- DES tables
// FIPS 46-3: S-boxes, P, PC-1, PC-2, shift schedule (1-indexed, MSB first).
struct DesConst {
    static constexpr uint8_t S[8][64] = {
        {14,4,13,1,2,15,11,8,3,10,6,12,5,9,0,7, 0,15,7,4,14,2,13,1,10,6,12,11,9,5,3,8, 4,1,14,8,13,6,2,11,15,12,9,7,3,10,5,0, 15,12,8,2,4,9,1,7,5,11,3,14,10,0,6,13},
        {15,1,8,14,6,11,3,4,9,7,2,13,12,0,5,10, 3,13,4,7,15,2,8,14,12,0,1,10,6,9,11,5, 0,14,7,11,10,4,13,1,5,8,12,6,9,3,2,15, 13,8,10,1,3,15,4,2,11,6,7,12,0,5,14,9},
        {10,0,9,14,6,3,15,5,1,13,12,7,11,4,2,8, 13,7,0,9,3,4,6,10,2,8,5,14,12,11,15,1, 13,6,4,9,8,15,3,0,11,1,2,12,5,10,14,7, 1,10,13,0,6,9,8,7,4,15,14,3,11,5,2,12},
        {7,13,14,3,0,6,9,10,1,2,8,5,11,12,4,15, 13,8,11,5,6,15,0,3,4,7,2,12,1,10,14,9, 10,6,9,0,12,11,7,13,15,1,3,14,5,2,8,4, 3,15,0,6,10,1,13,8,9,4,5,11,12,7,2,14},
        {2,12,4,1,7,10,11,6,8,5,3,15,13,0,14,9, 14,11,2,12,4,7,13,1,5,0,15,10,3,9,8,6, 4,2,1,11,10,13,7,8,15,9,12,5,6,3,0,14, 11,8,12,7,1,14,2,13,6,15,0,9,10,4,5,3},
        {12,1,10,15,9,2,6,8,0,13,3,4,14,7,5,11, 10,15,4,2,7,12,9,5,6,1,13,14,0,11,3,8, 9,14,15,5,2,8,12,3,7,0,4,10,1,13,11,6, 4,3,2,12,9,5,15,10,11,14,1,7,6,0,8,13},
        {4,11,2,14,15,0,8,13,3,12,9,7,5,10,6,1, 13,0,11,7,4,9,1,10,14,3,5,12,2,15,8,6, 1,4,11,13,12,3,7,14,10,15,6,8,0,5,9,2, 6,11,13,8,1,4,10,7,9,5,0,15,14,2,3,12},
        {13,2,8,4,6,15,11,1,10,9,3,14,5,0,12,7, 1,15,13,8,10,3,7,4,12,5,6,11,0,14,9,2, 7,11,4,1,9,12,14,2,0,6,10,13,15,3,5,8, 2,1,14,7,4,10,8,13,15,12,9,0,3,5,6,11}};
    static constexpr uint8_t P[32] = {16,7,20,21,29,12,28,17,1,15,23,26,5,18,31,10,2,8,24,14,32,27,3,9,19,13,30,6,22,11,4,25};
    static constexpr uint8_t IP[64] = {58,50,42,34,26,18,10,2,60,52,44,36,28,20,12,4,62,54,46,38,30,22,14,6,64,56,48,40,32,24,16,8,
                                       57,49,41,33,25,17,9,1,59,51,43,35,27,19,11,3,61,53,45,37,29,21,13,5,63,55,47,39,31,23,15,7};
    static constexpr uint8_t FP[64] = {40,8,48,16,56,24,64,32,39,7,47,15,55,23,63,31,38,6,46,14,54,22,62,30,37,5,45,13,53,21,61,29,
                                       36,4,44,12,52,20,60,28,35,3,43,11,51,19,59,27,34,2,42,10,50,18,58,26,33,1,41,9,49,17,57,25};
    static constexpr uint8_t PC1[56] = {57,49,41,33,25,17,9,1,58,50,42,34,26,18,10,2,59,51,43,35,27,19,11,3,60,52,44,36,
                                        63,55,47,39,31,23,15,7,62,54,46,38,30,22,14,6,61,53,45,37,29,21,13,5,28,20,12,4};
    static constexpr uint8_t PC2[48] = {14,17,11,24,1,5,3,28,15,6,21,10,23,19,12,4,26,8,16,7,27,20,13,2,
                                        41,52,31,37,47,55,30,40,51,45,33,48,44,49,39,56,34,53,46,42,50,36,29,32};
    static constexpr uint8_t SHIFTS[16] = {1,1,2,2,2,2,2,2,1,2,2,2,2,2,2,1};
};

// SP tables in the rotated domain used by the kernels: R' = rotl(R, 1) makes
// every E-expansion 6-bit group contiguous: group k (1..8) = rotr(R', 32-4k) & 63.
// SPk[x] = rotl(P(S_k(x) << 4*(8-k)), 1).
struct DesSP {
    uint32_t sp[8][64];
    constexpr DesSP() : sp() {
        for (int k = 0; k < 8; k++)
            for (int x = 0; x < 64; x++) {
                int row = ((x >> 4) & 2) | (x & 1), col = (x >> 1) & 15;
                uint32_t pre = (uint32_t)DesConst::S[k][row * 16 + col] << (4 * (7 - k));
                uint32_t post = 0;
                for (int i = 0; i < 32; i++) {
                    uint32_t bit = (pre >> (32 - DesConst::P[i])) & 1;
                    post |= bit << (31 - i);
                }
                sp[k][x] = (post << 1) | (post >> 31);
            }
    }
};

// ---------------------------------------------------------------- hash IVs
constexpr uint32_t SHA1_IV[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
constexpr uint32_t SHA256_IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
constexpr uint32_t MD5_IV[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};

}  // namespace tg

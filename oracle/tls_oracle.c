/*
 * tls_oracle.c -- CPU restatement of tlslite's per-record symmetric seal/open
 * path.  TEST INFRASTRUCTURE ONLY: this file is the parity checker and the
 * `cpu_baseline` leg of bench.py.  Nothing under tlslite_amd/ links, loads or
 * calls it; the product path is the HIP library in tlslite_amd/csrc/.
 *
 * Every function cites the reference behaviour it restates
 * (paths relative to /root/reference, trevp/tlslite 0.4.9):
 *
 *   record seal  ........ tlslite/tlsrecordlayer.py:538-616  (_sendMsg)
 *   record open  ........ tlslite/tlsrecordlayer.py:958-1044 (_decryptRecord)
 *   seqnum .............. tlslite/tlsrecordlayer.py:27-37    (_ConnectionState)
 *   AES (T-table rounds). tlslite/utils/rijndael.py:206-362, python_aes.py:20-69
 *   RC4 ................. tlslite/utils/python_rc4.py:12-41
 *   HMAC ................ tlslite/mathtls.py:116-117 -> CPython hmac (RFC 2104)
 *   SSL3 MAC ............ tlslite/mathtls.py:125-151 (MAC_SSL)
 *   SHA-1/SHA-256/MD5 ... CPython hashlib (OpenSSL 3.0.2) -- FIPS 180-4 / RFC 1321
 *   3DES-EDE-CBC ........ tlslite/utils/openssl_tripledes.py:23 -> OpenSSL
 *                         EVP_des_ede3_cbc (FIPS 46-3); no tlslite pure-Python 3DES
 *
 * Pinned by tests/golden/records.json (generated from the reference by
 * tests/golden/make_golden.py) and by FIPS-197 / RFC 2202 / RFC 4231 / FIPS 46
 * known-answer tests in tests/test_oracle.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "tls_oracle.h"

/* ======================================================================= AES
 * rijndael.py builds S/Si and T1..T4 (enc) / T5..T8 (dec) at import
 * (rijndael.py:55-185) from GF(2^8) arithmetic; we do the same at first use.
 * Words are big-endian (rijndael.py:290-297).                               */
static uint8_t S[256], Si[256];
static uint32_t T1[256], T2[256], T3[256], T4[256];
static uint32_t T5[256], T6[256], T7[256], T8[256];
static uint32_t U1[256], U2[256], U3[256], U4[256];
static pthread_once_t aes_once = PTHREAD_ONCE_INIT;

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

static void aes_tables(void) {
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) for (int y = 1; y < 256; y++) if (gmul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; i++) { r = (uint8_t)((r << 1) | (r >> 7)); s ^= r; }
        s ^= 0x63;
        S[x] = s;
        Si[s] = (uint8_t)x;
    }
    for (int x = 0; x < 256; x++) {
        uint8_t s = S[x], si = Si[x];
        uint32_t t = ((uint32_t)gmul(s, 2) << 24) | ((uint32_t)s << 16) | ((uint32_t)s << 8) | gmul(s, 3);
        T1[x] = t; T2[x] = (t >> 8) | (t << 24); T3[x] = (t >> 16) | (t << 16); T4[x] = (t >> 24) | (t << 8);
        uint32_t u = ((uint32_t)gmul(si, 14) << 24) | ((uint32_t)gmul(si, 9) << 16) |
                     ((uint32_t)gmul(si, 13) << 8) | gmul(si, 11);
        T5[x] = u; T6[x] = (u >> 8) | (u << 24); T7[x] = (u >> 16) | (u << 16); T8[x] = (u >> 24) | (u << 8);
        uint32_t v = ((uint32_t)gmul((uint8_t)x, 14) << 24) | ((uint32_t)gmul((uint8_t)x, 9) << 16) |
                     ((uint32_t)gmul((uint8_t)x, 13) << 8) | gmul((uint8_t)x, 11);
        U1[x] = v; U2[x] = (v >> 8) | (v << 24); U3[x] = (v >> 16) | (v << 16); U4[x] = (v >> 24) | (v << 8);
    }
}

/* key schedule, rijndael.py:206-276 (Ke forward, Kd = reversed + InvMixColumn) */
static void aes_setkey(ora_aes *k, const uint8_t *key, int klen) {
    pthread_once(&aes_once, aes_tables);
    int nk = klen / 4, rounds = nk + 6, total = 4 * (rounds + 1);
    uint32_t w[60];
    for (int i = 0; i < nk; i++)
        w[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) | ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = w[i - 1];
        if (i % nk == 0) {
            t = ((uint32_t)S[(t >> 16) & 0xff] << 24) | ((uint32_t)S[(t >> 8) & 0xff] << 16) |
                ((uint32_t)S[t & 0xff] << 8) | S[t >> 24];
            t ^= (uint32_t)rcon << 24;
            rcon = gmul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = ((uint32_t)S[t >> 24] << 24) | ((uint32_t)S[(t >> 16) & 0xff] << 16) |
                ((uint32_t)S[(t >> 8) & 0xff] << 8) | S[t & 0xff];
        }
        w[i] = w[i - nk] ^ t;
    }
    k->rounds = rounds;
    memcpy(k->ke, w, sizeof(uint32_t) * total);
    for (int r = 0; r <= rounds; r++)
        for (int j = 0; j < 4; j++) {
            uint32_t t = w[4 * (rounds - r) + j];
            if (r > 0 && r < rounds)
                t = U1[t >> 24] ^ U2[(t >> 16) & 0xff] ^ U3[(t >> 8) & 0xff] ^ U4[t & 0xff];
            k->kd[4 * r + j] = t;
        }
}

static inline uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
static inline void put_be32(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v; }
static inline uint32_t le32(const uint8_t *p) { return p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static inline void put_le32(uint8_t *p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24); }

/* rijndael.encrypt, rijndael.py:278-319 */
static void aes_enc_block(const ora_aes *k, const uint8_t in[16], uint8_t out[16]) {
    const uint32_t *K = k->ke;
    uint32_t t0 = be32(in) ^ K[0], t1 = be32(in + 4) ^ K[1], t2 = be32(in + 8) ^ K[2], t3 = be32(in + 12) ^ K[3];
    for (int r = 1; r < k->rounds; r++) {
        K += 4;
        uint32_t a0 = T1[t0 >> 24] ^ T2[(t1 >> 16) & 0xff] ^ T3[(t2 >> 8) & 0xff] ^ T4[t3 & 0xff] ^ K[0];
        uint32_t a1 = T1[t1 >> 24] ^ T2[(t2 >> 16) & 0xff] ^ T3[(t3 >> 8) & 0xff] ^ T4[t0 & 0xff] ^ K[1];
        uint32_t a2 = T1[t2 >> 24] ^ T2[(t3 >> 16) & 0xff] ^ T3[(t0 >> 8) & 0xff] ^ T4[t1 & 0xff] ^ K[2];
        uint32_t a3 = T1[t3 >> 24] ^ T2[(t0 >> 16) & 0xff] ^ T3[(t1 >> 8) & 0xff] ^ T4[t2 & 0xff] ^ K[3];
        t0 = a0; t1 = a1; t2 = a2; t3 = a3;
    }
    K += 4;
    uint32_t t[4] = {t0, t1, t2, t3};
    for (int c = 0; c < 4; c++) {
        uint32_t v = ((uint32_t)S[t[c] >> 24] << 24) | ((uint32_t)S[(t[(c + 1) & 3] >> 16) & 0xff] << 16) |
                     ((uint32_t)S[(t[(c + 2) & 3] >> 8) & 0xff] << 8) | S[t[(c + 3) & 3] & 0xff];
        put_be32(out + 4 * c, v ^ K[c]);
    }
}

/* rijndael.decrypt, rijndael.py:321-362 */
static void aes_dec_block(const ora_aes *k, const uint8_t in[16], uint8_t out[16]) {
    const uint32_t *K = k->kd;
    uint32_t t0 = be32(in) ^ K[0], t1 = be32(in + 4) ^ K[1], t2 = be32(in + 8) ^ K[2], t3 = be32(in + 12) ^ K[3];
    for (int r = 1; r < k->rounds; r++) {
        K += 4;
        uint32_t a0 = T5[t0 >> 24] ^ T6[(t3 >> 16) & 0xff] ^ T7[(t2 >> 8) & 0xff] ^ T8[t1 & 0xff] ^ K[0];
        uint32_t a1 = T5[t1 >> 24] ^ T6[(t0 >> 16) & 0xff] ^ T7[(t3 >> 8) & 0xff] ^ T8[t2 & 0xff] ^ K[1];
        uint32_t a2 = T5[t2 >> 24] ^ T6[(t1 >> 16) & 0xff] ^ T7[(t0 >> 8) & 0xff] ^ T8[t3 & 0xff] ^ K[2];
        uint32_t a3 = T5[t3 >> 24] ^ T6[(t2 >> 16) & 0xff] ^ T7[(t1 >> 8) & 0xff] ^ T8[t0 & 0xff] ^ K[3];
        t0 = a0; t1 = a1; t2 = a2; t3 = a3;
    }
    K += 4;
    uint32_t t[4] = {t0, t1, t2, t3};
    for (int c = 0; c < 4; c++) {
        uint32_t v = ((uint32_t)Si[t[c] >> 24] << 24) | ((uint32_t)Si[(t[(c + 3) & 3] >> 16) & 0xff] << 16) |
                     ((uint32_t)Si[(t[(c + 2) & 3] >> 8) & 0xff] << 8) | Si[t[(c + 1) & 3] & 0xff];
        put_be32(out + 4 * c, v ^ K[c]);
    }
}

/* ======================================================================= DES
 * FIPS 46-3 tables; bit 1 = MSB of the 64-bit block.                        */
static const uint8_t DES_IP[64] = {58,50,42,34,26,18,10,2,60,52,44,36,28,20,12,4,62,54,46,38,30,22,14,6,64,56,48,40,32,24,16,8,
                                   57,49,41,33,25,17,9,1,59,51,43,35,27,19,11,3,61,53,45,37,29,21,13,5,63,55,47,39,31,23,15,7};
static const uint8_t DES_FP[64] = {40,8,48,16,56,24,64,32,39,7,47,15,55,23,63,31,38,6,46,14,54,22,62,30,37,5,45,13,53,21,61,29,
                                   36,4,44,12,52,20,60,28,35,3,43,11,51,19,59,27,34,2,42,10,50,18,58,26,33,1,41,9,49,17,57,25};
static const uint8_t DES_E[48] = {32,1,2,3,4,5,4,5,6,7,8,9,8,9,10,11,12,13,12,13,14,15,16,17,
                                  16,17,18,19,20,21,20,21,22,23,24,25,24,25,26,27,28,29,28,29,30,31,32,1};
static const uint8_t DES_P[32] = {16,7,20,21,29,12,28,17,1,15,23,26,5,18,31,10,2,8,24,14,32,27,3,9,19,13,30,6,22,11,4,25};
static const uint8_t DES_PC1[56] = {57,49,41,33,25,17,9,1,58,50,42,34,26,18,10,2,59,51,43,35,27,19,11,3,60,52,44,36,
                                    63,55,47,39,31,23,15,7,62,54,46,38,30,22,14,6,61,53,45,37,29,21,13,5,28,20,12,4};
static const uint8_t DES_PC2[48] = {14,17,11,24,1,5,3,28,15,6,21,10,23,19,12,4,26,8,16,7,27,20,13,2,
                                    41,52,31,37,47,55,30,40,51,45,33,48,44,49,39,56,34,53,46,42,50,36,29,32};
static const uint8_t DES_SHIFTS[16] = {1,1,2,2,2,2,2,2,1,2,2,2,2,2,2,1};
static const uint8_t DES_SBOX[8][64] = {
 {14,4,13,1,2,15,11,8,3,10,6,12,5,9,0,7, 0,15,7,4,14,2,13,1,10,6,12,11,9,5,3,8, 4,1,14,8,13,6,2,11,15,12,9,7,3,10,5,0, 15,12,8,2,4,9,1,7,5,11,3,14,10,0,6,13},
 {15,1,8,14,6,11,3,4,9,7,2,13,12,0,5,10, 3,13,4,7,15,2,8,14,12,0,1,10,6,9,11,5, 0,14,7,11,10,4,13,1,5,8,12,6,9,3,2,15, 13,8,10,1,3,15,4,2,11,6,7,12,0,5,14,9},
 {10,0,9,14,6,3,15,5,1,13,12,7,11,4,2,8, 13,7,0,9,3,4,6,10,2,8,5,14,12,11,15,1, 13,6,4,9,8,15,3,0,11,1,2,12,5,10,14,7, 1,10,13,0,6,9,8,7,4,15,14,3,11,5,2,12},
 {7,13,14,3,0,6,9,10,1,2,8,5,11,12,4,15, 13,8,11,5,6,15,0,3,4,7,2,12,1,10,14,9, 10,6,9,0,12,11,7,13,15,1,3,14,5,2,8,4, 3,15,0,6,10,1,13,8,9,4,5,11,12,7,2,14},
 {2,12,4,1,7,10,11,6,8,5,3,15,13,0,14,9, 14,11,2,12,4,7,13,1,5,0,15,10,3,9,8,6, 4,2,1,11,10,13,7,8,15,9,12,5,6,3,0,14, 11,8,12,7,1,14,2,13,6,15,0,9,10,4,5,3},
 {12,1,10,15,9,2,6,8,0,13,3,4,14,7,5,11, 10,15,4,2,7,12,9,5,6,1,13,14,0,11,3,8, 9,14,15,5,2,8,12,3,7,0,4,10,1,13,11,6, 4,3,2,12,9,5,15,10,11,14,1,7,6,0,8,13},
 {4,11,2,14,15,0,8,13,3,12,9,7,5,10,6,1, 13,0,11,7,4,9,1,10,14,3,5,12,2,15,8,6, 1,4,11,13,12,3,7,14,10,15,6,8,0,5,9,2, 6,11,13,8,1,4,10,7,9,5,0,15,14,2,3,12},
 {13,2,8,4,6,15,11,1,10,9,3,14,5,0,12,7, 1,15,13,8,10,3,7,4,12,5,6,11,0,14,9,2, 7,11,4,1,9,12,14,2,0,6,10,13,15,3,5,8, 2,1,14,7,4,10,8,13,15,12,9,0,3,5,6,11}};

static uint64_t permute(uint64_t in, int inbits, const uint8_t *tab, int n) {
    uint64_t out = 0;
    for (int i = 0; i < n; i++) out = (out << 1) | ((in >> (inbits - tab[i])) & 1);
    return out;
}

static void des_setkey(uint64_t sub[16], const uint8_t key[8]) {
    uint64_t k = 0;
    for (int i = 0; i < 8; i++) k = (k << 8) | key[i];
    uint64_t cd = permute(k, 64, DES_PC1, 56);
    uint32_t c = (uint32_t)(cd >> 28) & 0xfffffff, d = (uint32_t)cd & 0xfffffff;
    for (int r = 0; r < 16; r++) {
        for (int s = 0; s < DES_SHIFTS[r]; s++) {
            c = ((c << 1) | (c >> 27)) & 0xfffffff;
            d = ((d << 1) | (d >> 27)) & 0xfffffff;
        }
        sub[r] = permute(((uint64_t)c << 28) | d, 56, DES_PC2, 48);
    }
}

static uint32_t des_f(uint32_t r, uint64_t k) {
    uint64_t e = permute(r, 32, DES_E, 48) ^ k;
    uint32_t o = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t six = (uint32_t)(e >> (42 - 6 * i)) & 0x3f;
        uint32_t row = ((six >> 4) & 2) | (six & 1), col = (six >> 1) & 0xf;
        o = (o << 4) | DES_SBOX[i][row * 16 + col];
    }
    return (uint32_t)permute(o, 32, DES_P, 32);
}

static uint64_t des_block(const uint64_t sub[16], uint64_t in, int decrypt) {
    uint64_t x = permute(in, 64, DES_IP, 64);
    uint32_t l = (uint32_t)(x >> 32), r = (uint32_t)x;
    for (int i = 0; i < 16; i++) {
        uint32_t t = r;
        r = l ^ des_f(r, sub[decrypt ? 15 - i : i]);
        l = t;
    }
    return permute(((uint64_t)r << 32) | l, 64, DES_FP, 64);
}

static uint64_t load_be64(const uint8_t *p) { uint64_t v = 0; for (int i = 0; i < 8; i++) v = (v << 8) | p[i]; return v; }
static void store_be64(uint8_t *p, uint64_t v) { for (int i = 7; i >= 0; i--) { p[i] = (uint8_t)v; v >>= 8; } }

/* 3DES-EDE: E_K3(D_K2(E_K1(x))) / inverse */
static void tdes_enc(const ora_conn *c, const uint8_t in[8], uint8_t out[8]) {
    uint64_t v = load_be64(in);
    v = des_block(c->des[0], v, 0); v = des_block(c->des[1], v, 1); v = des_block(c->des[2], v, 0);
    store_be64(out, v);
}
static void tdes_dec(const ora_conn *c, const uint8_t in[8], uint8_t out[8]) {
    uint64_t v = load_be64(in);
    v = des_block(c->des[2], v, 1); v = des_block(c->des[1], v, 0); v = des_block(c->des[0], v, 1);
    store_be64(out, v);
}

/* ======================================================================= hashes */
#define ROL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha1_compress(uint32_t h[5], const uint8_t b[64]) {
    uint32_t w[80];
    for (int i = 0; i < 16; i++) w[i] = be32(b + 4 * i);
    for (int i = 16; i < 80; i++) w[i] = ROL(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; i++) {
        uint32_t f, k;
        if (i < 20) { f = (bb & c) | (~bb & d); k = 0x5A827999; }
        else if (i < 40) { f = bb ^ c ^ d; k = 0x6ED9EBA1; }
        else if (i < 60) { f = (bb & c) | (bb & d) | (c & d); k = 0x8F1BBCDC; }
        else { f = bb ^ c ^ d; k = 0xCA62C1D6; }
        uint32_t t = ROL(a, 5) + f + e + k + w[i];
        e = d; d = c; c = ROL(bb, 30); bb = a; a = t;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e;
}

static const uint32_t K256[64] = {
    0x428a2f98,0x71374491,0xb5c0fbcf,0xe9b5dba5,0x3956c25b,0x59f111f1,0x923f82a4,0xab1c5ed5,
    0xd807aa98,0x12835b01,0x243185be,0x550c7dc3,0x72be5d74,0x80deb1fe,0x9bdc06a7,0xc19bf174,
    0xe49b69c1,0xefbe4786,0x0fc19dc6,0x240ca1cc,0x2de92c6f,0x4a7484aa,0x5cb0a9dc,0x76f988da,
    0x983e5152,0xa831c66d,0xb00327c8,0xbf597fc7,0xc6e00bf3,0xd5a79147,0x06ca6351,0x14292967,
    0x27b70a85,0x2e1b2138,0x4d2c6dfc,0x53380d13,0x650a7354,0x766a0abb,0x81c2c92e,0x92722c85,
    0xa2bfe8a1,0xa81a664b,0xc24b8b70,0xc76c51a3,0xd192e819,0xd6990624,0xf40e3585,0x106aa070,
    0x19a4c116,0x1e376c08,0x2748774c,0x34b0bcb5,0x391c0cb3,0x4ed8aa4a,0x5b9cca4f,0x682e6ff3,
    0x748f82ee,0x78a5636f,0x84c87814,0x8cc70208,0x90befffa,0xa4506ceb,0xbef9a3f7,0xc67178f2};

static void sha256_compress(uint32_t h[8], const uint8_t b[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = be32(b + 4 * i);
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = hh + S1 + ch + K256[i] + w[i];
        uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
        uint32_t mj = (a & bb) ^ (a & c) ^ (bb & c);
        uint32_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static const uint32_t MD5K[64] = {
    0xd76aa478,0xe8c7b756,0x242070db,0xc1bdceee,0xf57c0faf,0x4787c62a,0xa8304613,0xfd469501,
    0x698098d8,0x8b44f7af,0xffff5bb1,0x895cd7be,0x6b901122,0xfd987193,0xa679438e,0x49b40821,
    0xf61e2562,0xc040b340,0x265e5a51,0xe9b6c7aa,0xd62f105d,0x02441453,0xd8a1e681,0xe7d3fbc8,
    0x21e1cde6,0xc33707d6,0xf4d50d87,0x455a14ed,0xa9e3e905,0xfcefa3f8,0x676f02d9,0x8d2a4c8a,
    0xfffa3942,0x8771f681,0x6d9d6122,0xfde5380c,0xa4beea44,0x4bdecfa9,0xf6bb4b60,0xbebfbc70,
    0x289b7ec6,0xeaa127fa,0xd4ef3085,0x04881d05,0xd9d4d039,0xe6db99e5,0x1fa27cf8,0xc4ac5665,
    0xf4292244,0x432aff97,0xab9423a7,0xfc93a039,0x655b59c3,0x8f0ccc92,0xffeff47d,0x85845dd1,
    0x6fa87e4f,0xfe2ce6e0,0xa3014314,0x4e0811a1,0xf7537e82,0xbd3af235,0x2ad7d2bb,0xeb86d391};
static const uint8_t MD5R[64] = {7,12,17,22,7,12,17,22,7,12,17,22,7,12,17,22,5,9,14,20,5,9,14,20,5,9,14,20,5,9,14,20,
                                 4,11,16,23,4,11,16,23,4,11,16,23,4,11,16,23,6,10,15,21,6,10,15,21,6,10,15,21,6,10,15,21};

static void md5_compress(uint32_t h[4], const uint8_t b[64]) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++) m[i] = le32(b + 4 * i);
    uint32_t a = h[0], bb = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f; int g;
        if (i < 16) { f = (bb & c) | (~bb & d); g = i; }
        else if (i < 32) { f = (d & bb) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = bb ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (bb | ~d); g = (7 * i) & 15; }
        uint32_t t = d; d = c; c = bb;
        uint32_t x = a + f + MD5K[i] + m[g];
        bb = bb + ROL(x, MD5R[i]);
        a = t;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d;
}

typedef struct { int alg; uint32_t h[8]; uint8_t buf[64]; uint64_t len; } hctx;

static int hash_dlen(int alg) { return alg == ORA_MAC_SHA1 ? 20 : alg == ORA_MAC_SHA256 ? 32 : 16; }

static void h_init(hctx *c, int alg) {
    static const uint32_t i1[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    static const uint32_t i256[8] = {0x6a09e667,0xbb67ae85,0x3c6ef372,0xa54ff53a,0x510e527f,0x9b05688c,0x1f83d9ab,0x5be0cd19};
    static const uint32_t i5[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
    c->alg = alg; c->len = 0;
    if (alg == ORA_MAC_SHA1) memcpy(c->h, i1, sizeof i1);
    else if (alg == ORA_MAC_SHA256) memcpy(c->h, i256, sizeof i256);
    else memcpy(c->h, i5, sizeof i5);
}
static void h_block(hctx *c, const uint8_t *b) {
    if (c->alg == ORA_MAC_SHA1) sha1_compress(c->h, b);
    else if (c->alg == ORA_MAC_SHA256) sha256_compress(c->h, b);
    else md5_compress(c->h, b);
}
static void h_update(hctx *c, const uint8_t *p, size_t n) {
    size_t fill = (size_t)(c->len & 63);
    c->len += n;
    if (fill) {
        size_t take = 64 - fill < n ? 64 - fill : n;
        memcpy(c->buf + fill, p, take); p += take; n -= take; fill += take;
        if (fill < 64) return;
        h_block(c, c->buf);
    }
    while (n >= 64) { h_block(c, p); p += 64; n -= 64; }
    memcpy(c->buf, p, n);
}
static void h_final(hctx *c, uint8_t *out) {
    uint64_t bits = c->len * 8;
    uint8_t pad[72] = {0x80};
    size_t fill = (size_t)(c->len & 63);
    size_t padn = (fill < 56 ? 56 - fill : 120 - fill);
    uint8_t lenb[8];
    for (int i = 0; i < 8; i++)
        lenb[i] = c->alg == ORA_MAC_MD5 ? (uint8_t)(bits >> (8 * i)) : (uint8_t)(bits >> (56 - 8 * i));
    h_update(c, pad, padn);
    h_update(c, lenb, 8);
    int dl = hash_dlen(c->alg);
    for (int i = 0; i < dl / 4; i++) {
        if (c->alg == ORA_MAC_MD5) put_le32(out + 4 * i, c->h[i]);
        else put_be32(out + 4 * i, c->h[i]);
    }
}

void ora_hash(int alg, const uint8_t *p, size_t n, uint8_t *out) {
    hctx c; h_init(&c, alg); h_update(&c, p, n); h_final(&c, out);
}

/* HMAC (RFC 2104) as CPython hmac.HMAC does it: keys longer than the block are
 * hashed first; tlslite MAC keys are 16..32 bytes so this never triggers.   */
void ora_hmac(int alg, const uint8_t *key, size_t klen, const uint8_t *msg, size_t n, uint8_t *out) {
    uint8_t k[64] = {0}, ip[64], op[64], inner[32];
    if (klen > 64) { ora_hash(alg, key, klen, k); } else memcpy(k, key, klen);
    for (int i = 0; i < 64; i++) { ip[i] = k[i] ^ 0x36; op[i] = k[i] ^ 0x5c; }
    hctx c; h_init(&c, alg); h_update(&c, ip, 64); h_update(&c, msg, n); h_final(&c, inner);
    h_init(&c, alg); h_update(&c, op, 64); h_update(&c, inner, (size_t)hash_dlen(alg)); h_final(&c, out);
}

/* P_hash (mathtls.py:24-35): A(0) = seed, A(i) = HMAC(secret, A(i-1)),
 * output HMAC(secret, A(i) || seed)...; XORed into out. */
static void p_hash_xor(int alg, const uint8_t *secret, size_t slen, const uint8_t *seed, size_t seedlen,
                       uint8_t *out, size_t length) {
    uint8_t a[32], blk[32], msg[32 + 256];
    size_t d = (size_t)hash_dlen(alg);
    ora_hmac(alg, secret, slen, seed, seedlen, a);
    for (size_t pos = 0; pos < length; pos += d) {
        memcpy(msg, a, d);
        memcpy(msg + d, seed, seedlen);
        ora_hmac(alg, secret, slen, msg, d + seedlen, blk);
        for (size_t i = 0; i < d && pos + i < length; i++) out[pos + i] ^= blk[i];
        ora_hmac(alg, secret, slen, a, d, a);
    }
}

/* PRF by protocol version: (3,0) PRF_SSL (mathtls.py:55-68; label unused),
 * (3,1)/(3,2) PRF = P_MD5(S1) ^ P_SHA1(S2) with S1/S2 the ceil/floor halves
 * (mathtls.py:37-50), (3,3) PRF_1_2 = P_SHA256 (mathtls.py:52-53).
 * label + seed <= 256 bytes. */
int ora_prf(int vmin, const uint8_t *secret, size_t slen, const uint8_t *label, size_t llen,
            const uint8_t *seed, size_t seedlen, uint8_t *out, size_t length) {
    uint8_t ls[256];
    if (llen + seedlen > sizeof ls || vmin < 0 || vmin > 3) return -1;
    memset(out, 0, length);
    if (vmin == 0) {
        uint8_t msg[26 + 64 + 256], inner[20], blk[16];
        if (26 + slen + seedlen > sizeof msg || length > 26 * 16) return -1;
        for (size_t x = 0, pos = 0; pos < length; x++, pos += 16) {
            size_t m = 0;
            for (size_t r = 0; r <= x; r++) msg[m++] = (uint8_t)('A' + x);
            memcpy(msg + m, secret, slen); m += slen;
            memcpy(msg + m, seed, seedlen); m += seedlen;
            ora_hash(ORA_MAC_SHA1, msg, m, inner);
            memcpy(msg, secret, slen);
            memcpy(msg + slen, inner, 20);
            ora_hash(ORA_MAC_MD5, msg, slen + 20, blk);
            for (size_t i = 0; i < 16 && pos + i < length; i++) out[pos + i] = blk[i];
        }
        return 0;
    }
    memcpy(ls, label, llen);
    memcpy(ls + llen, seed, seedlen);
    if (vmin == 3) {
        p_hash_xor(ORA_MAC_SHA256, secret, slen, ls, llen + seedlen, out, length);
    } else {
        size_t h1 = (slen + 1) / 2, h2 = slen / 2;
        p_hash_xor(ORA_MAC_MD5, secret, h1, ls, llen + seedlen, out, length);
        p_hash_xor(ORA_MAC_SHA1, secret + h2, slen - h2, ls, llen + seedlen, out, length);
    }
    return 0;
}

/* record MAC over seq||type||[ver]||len16||P: tlsrecordlayer.py:568-584,
 * SSL3 variant via MAC_SSL (mathtls.py:125-151): pad repeated 40 (SHA) / 48 (MD5) */
static void record_mac(const ora_conn *c, uint64_t seq, int ctype, const uint8_t *p, size_t n, uint8_t *out) {
    uint8_t hdr[13];
    int hl = 0;
    for (int i = 0; i < 8; i++) hdr[hl++] = (uint8_t)(seq >> (56 - 8 * i));
    hdr[hl++] = (uint8_t)ctype;
    if (!(c->vmaj == 3 && c->vmin == 0)) { hdr[hl++] = (uint8_t)c->vmaj; hdr[hl++] = (uint8_t)c->vmin; }
    hdr[hl++] = (uint8_t)(n >> 8);
    hdr[hl++] = (uint8_t)n;
    if (c->vmaj == 3 && c->vmin == 0) {
        int dl = hash_dlen(c->mac);
        int rep = (c->mac == ORA_MAC_MD5) ? 48 : 40;  /* mathtls.py:134-136 keys off digest_size 16 vs 20 */
        (void)dl;
        uint8_t pad1[48], pad2[48], inner[32];
        memset(pad1, 0x36, sizeof pad1); memset(pad2, 0x5c, sizeof pad2);
        hctx h; h_init(&h, c->mac);
        h_update(&h, c->mac_key, (size_t)c->mac_key_len); h_update(&h, pad1, (size_t)rep);
        h_update(&h, hdr, (size_t)hl); h_update(&h, p, n); h_final(&h, inner);
        h_init(&h, c->mac);
        h_update(&h, c->mac_key, (size_t)c->mac_key_len); h_update(&h, pad2, (size_t)rep);
        h_update(&h, inner, (size_t)hash_dlen(c->mac)); h_final(&h, out);
    } else {
        /* HMAC(K, hdr || P) without concatenating: stream both parts */
        uint8_t k[64] = {0}, ip[64], op[64], inner[32];
        memcpy(k, c->mac_key, (size_t)c->mac_key_len);
        for (int i = 0; i < 64; i++) { ip[i] = k[i] ^ 0x36; op[i] = k[i] ^ 0x5c; }
        hctx h; h_init(&h, c->mac); h_update(&h, ip, 64); h_update(&h, hdr, (size_t)hl); h_update(&h, p, n); h_final(&h, inner);
        h_init(&h, c->mac); h_update(&h, op, 64); h_update(&h, inner, (size_t)hash_dlen(c->mac)); h_final(&h, out);
    }
}

/* ======================================================================= RC4
 * KSA python_rc4.py:13-23; PRGA :25-38 (state carried across calls)        */
static void rc4_ksa(ora_conn *c, const uint8_t *key, size_t klen) {
    for (int i = 0; i < 256; i++) c->rc4_S[i] = (uint8_t)i;
    uint8_t j = 0;
    for (int i = 0; i < 256; i++) {
        j = (uint8_t)(j + c->rc4_S[i] + key[i % klen]);
        uint8_t t = c->rc4_S[i]; c->rc4_S[i] = c->rc4_S[j]; c->rc4_S[j] = t;
    }
    c->rc4_i = 0; c->rc4_j = 0;
}
static void rc4_xor(ora_conn *c, uint8_t *p, size_t n) {
    uint8_t i = (uint8_t)c->rc4_i, j = (uint8_t)c->rc4_j, *Sx = c->rc4_S;
    for (size_t x = 0; x < n; x++) {
        i = (uint8_t)(i + 1);
        j = (uint8_t)(j + Sx[i]);
        uint8_t t = Sx[i]; Sx[i] = Sx[j]; Sx[j] = t;
        p[x] ^= Sx[(uint8_t)(Sx[i] + Sx[j])];
    }
    c->rc4_i = i; c->rc4_j = j;
}

/* ======================================================================= conn */
int ora_conn_init(ora_conn *c, int cipher, int mac, int vmaj, int vmin,
                  const uint8_t *key, size_t klen, const uint8_t *iv, size_t ivlen,
                  const uint8_t *mac_key, size_t mklen, const uint8_t *fixed_iv, uint64_t seq) {
    memset(c, 0, sizeof *c);
    c->cipher = cipher; c->mac = mac; c->vmaj = vmaj; c->vmin = vmin; c->seq = seq;
    if (mklen > sizeof c->mac_key) return -1;
    memcpy(c->mac_key, mac_key, mklen); c->mac_key_len = (int)mklen;
    switch (cipher) {
    case ORA_CIPHER_AES128: case ORA_CIPHER_AES256:
        /* aes.py:7-13 */
        if (klen != (cipher == ORA_CIPHER_AES128 ? 16u : 32u) || ivlen != 16) return -1;
        aes_setkey(&c->aes, key, (int)klen);
        c->bs = 16; break;
    case ORA_CIPHER_3DES:
        if (klen != 24 || ivlen != 8) return -1;  /* tripledes.py:8-13 */
        for (int i = 0; i < 3; i++) des_setkey(c->des[i], key + 8 * i);
        c->bs = 8; break;
    case ORA_CIPHER_RC4:
        if (klen < 16 || klen > 256 || ivlen != 0) return -1;  /* rc4.py:9-10, cipherfactory.py:70-71 */
        rc4_ksa(c, key, klen);
        c->bs = 0; break;
    default: return -1;
    }
    if (ivlen) memcpy(c->iv, iv, ivlen);
    if (fixed_iv && c->bs) memcpy(c->fixed_iv, fixed_iv, (size_t)c->bs);
    return 0;
}

static void cbc_encrypt(ora_conn *c, uint8_t *b, size_t n) {  /* python_aes.py:20-45 */
    int bs = c->bs;
    for (size_t off = 0; off < n; off += (size_t)bs) {
        for (int y = 0; y < bs; y++) b[off + y] ^= c->iv[y];
        if (bs == 16) aes_enc_block(&c->aes, b + off, b + off); else tdes_enc(c, b + off, b + off);
        memcpy(c->iv, b + off, (size_t)bs);
    }
}
static void cbc_decrypt(ora_conn *c, uint8_t *b, size_t n) {  /* python_aes.py:47-69 */
    int bs = c->bs;
    uint8_t prev[16], cur[16];
    memcpy(prev, c->iv, (size_t)bs);
    for (size_t off = 0; off < n; off += (size_t)bs) {
        memcpy(cur, b + off, (size_t)bs);
        if (bs == 16) aes_dec_block(&c->aes, b + off, b + off); else tdes_dec(c, b + off, b + off);
        for (int y = 0; y < bs; y++) b[off + y] ^= prev[y];
        memcpy(prev, cur, (size_t)bs);
    }
    memcpy(c->iv, prev, (size_t)bs);
}

long ora_seal_len(const ora_conn *c, size_t n) {
    if (n == 0) return 0;
    size_t M = (size_t)hash_dlen(c->mac);
    if (!c->bs) return (long)(5 + n + M);
    size_t E = (c->vmaj == 3 && c->vmin >= 2) ? (size_t)c->bs : 0;
    size_t cur = E + n + M;
    size_t padl = (size_t)c->bs - 1 - (cur % (size_t)c->bs);
    return (long)(5 + cur + padl + 1);
}

/* _sendMsg seal block, tlsrecordlayer.py:538-617 (no BEAST split here: that is
 * write()-level, see ora_write_plan).  Returns wire length, 0 for an empty
 * record (no output, no seqnum consumed: :551-556), <0 on error.             */
long ora_seal(ora_conn *c, int ctype, const uint8_t *pt, size_t n, int fault, uint8_t *out, size_t cap) {
    if (n == 0) return 0;
    long wl = ora_seal_len(c, n);
    if ((size_t)wl > cap) return -2;
    if (wl - 5 > 0xffff) return -3;  /* RecordHeader3 length u16: codec.py:19-20 */
    uint8_t mac[32];
    size_t M = (size_t)hash_dlen(c->mac);
    record_mac(c, c->seq, ctype, pt, n, mac);
    c->seq++;
    if (fault & ORA_FAULT_BAD_MAC) mac[0] = (uint8_t)(mac[0] + 1);
    uint8_t *b = out + 5;
    size_t pos = 0;
    if (c->bs) {
        if (c->vmaj == 3 && c->vmin >= 2) { memcpy(b, c->fixed_iv, (size_t)c->bs); pos = (size_t)c->bs; }
        memcpy(b + pos, pt, n); pos += n;
        size_t cur = pos + M;
        size_t padl = (size_t)c->bs - 1 - (cur % (size_t)c->bs);
        memcpy(b + pos, mac, M); pos += M;
        for (size_t i = 0; i <= padl; i++) b[pos + i] = (uint8_t)padl;
        if (fault & ORA_FAULT_BAD_PADDING) b[pos] = (uint8_t)(b[pos] + 1);
        pos += padl + 1;
        cbc_encrypt(c, b, pos);
    } else {
        memcpy(b, pt, n); pos = n;
        memcpy(b + pos, mac, M); pos += M;
        rc4_xor(c, b, pos);
    }
    out[0] = (uint8_t)ctype; out[1] = (uint8_t)c->vmaj; out[2] = (uint8_t)c->vmin;
    out[3] = (uint8_t)(pos >> 8); out[4] = (uint8_t)pos;
    return (long)(pos + 5);
}

/* _decryptRecord, tlsrecordlayer.py:958-1044.  `b` is the record body (no
 * header), modified in place.  Returns plaintext length (plaintext at *pt_out
 * inside b) or an ORA_ALERT_* negative code.                                 */
long ora_open(ora_conn *c, int ctype, uint8_t *b, size_t n, size_t *pt_off) {
    size_t M = (size_t)hash_dlen(c->mac);
    size_t start = 0, len = n, totalPad = 0;
    int padGood = 1;
    if (c->bs) {
        if (n % (size_t)c->bs) return ORA_ALERT_DECRYPTION_FAILED;          /* :964-968 */
        cbc_decrypt(c, b, n);
        if (c->vmaj == 3 && c->vmin >= 2) {                                 /* :970-971 (b[bs:] of a shorter b is empty) */
            start = (size_t)c->bs;
            len = n > (size_t)c->bs ? n - (size_t)c->bs : 0;
        }
        if (len == 0) return ORA_ALERT_DECRYPTION_FAILED;                  /* :973-977 */
        uint8_t pl = b[start + len - 1];
        if ((size_t)pl + 1 > len) { padGood = 0; totalPad = 0; }
        else {
            totalPad = (size_t)pl + 1;
            if (!(c->vmaj == 3 && c->vmin == 0)) {
                size_t lo = len - totalPad;  /* slice b[-total:-1] taken once, :988 */
                for (size_t i = lo; i < len - 1; i++)
                    if (b[start + i] != pl) { padGood = 0; totalPad = 0; }
            }
        }
    } else {
        rc4_xor(c, b, n);
    }
    int macGood = 1;
    size_t endLen = M + totalPad;
    if (endLen > len) macGood = 0;
    else {
        size_t plen = len - endLen;
        uint8_t mac[32];
        record_mac(c, c->seq, ctype, b + start, plen, mac);
        c->seq++;
        if (memcmp(mac, b + start + plen, M)) macGood = 0;
        len = plen;
    }
    if (!(padGood && macGood)) return ORA_ALERT_BAD_RECORD_MAC;               /* :1038-1042 */
    *pt_off = start;
    return (long)len;
}

/* raw cipher-object encrypt/decrypt (python_aes.Python_AES / python_rc4 /
 * openssl_tripledes semantics: state carried across calls)                  */
int ora_cipher_encrypt(ora_conn *c, uint8_t *b, size_t n) {
    if (c->bs) { if (n % (size_t)c->bs) return -1; cbc_encrypt(c, b, n); }
    else rc4_xor(c, b, n);
    return 0;
}
int ora_cipher_decrypt(ora_conn *c, uint8_t *b, size_t n) {
    if (c->bs) { if (n % (size_t)c->bs) return -1; cbc_decrypt(c, b, n); }
    else rc4_xor(c, b, n);
    return 0;
}

void ora_conn_get_iv(const ora_conn *c, uint8_t *iv16) { memcpy(iv16, c->iv, 16); }
uint64_t ora_conn_get_seq(const ora_conn *c) { return c->seq; }
void ora_conn_get_rc4(const ora_conn *c, uint8_t *S256, int *i, int *j) { memcpy(S256, c->rc4_S, 256); *i = c->rc4_i; *j = c->rc4_j; }
size_t ora_conn_size(void) { return sizeof(ora_conn); }

/* ======================================================================= batch
 * The bench workload: records share key material from one
 * prototype connection but each record starts from its own CBC IV and seqnum
 * (cfg2/3/5), or a connection seals `per_conn` records in order (cfg4).
 * Threads split the independent chains.  Used only for cpu_baseline and for
 * full-size parity digests.                                                  */
typedef struct {
    ora_conn *protos;   /* one per chain */
    const uint8_t *pt;        /* plaintext arena */
    const uint64_t *pt_off; const uint32_t *pt_len; const uint64_t *wire_off;
    const uint8_t *ctype; const uint8_t *flags;
    uint8_t *wire;
    long *wire_len;
    const uint32_t *chain_begin; const uint32_t *chain_count;
    size_t nchains; int nthreads; int tid;
} batch_arg;

static void *batch_worker(void *p) {
    batch_arg *a = (batch_arg *)p;
    for (size_t ch = (size_t)a->tid; ch < a->nchains; ch += (size_t)a->nthreads) {
        ora_conn c = a->protos[ch];
        for (uint32_t k = 0; k < a->chain_count[ch]; k++) {
            size_t r = a->chain_begin[ch] + k;
            a->wire_len[r] = ora_seal(&c, a->ctype ? a->ctype[r] : 23, a->pt + a->pt_off[r], a->pt_len[r],
                                      a->flags ? a->flags[r] : 0,
                                      a->wire + a->wire_off[r], (size_t)1 << 20);
        }
        a->protos[ch] = c; /* the chain's state after its records (residue, RC4, seqnum) */
    }
    return NULL;
}

int ora_seal_batch(ora_conn *protos, size_t nchains, const uint32_t *chain_begin, const uint32_t *chain_count,
                   const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len, const uint8_t *ctype,
                   const uint8_t *flags, uint8_t *wire, const uint64_t *wire_off, long *wire_len, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    batch_arg args[256];
    for (int t = 0; t < nthreads; t++) {
        batch_arg a = {protos, pt, pt_off, pt_len, wire_off, ctype, flags, wire, wire_len, chain_begin, chain_count,
                       nchains, nthreads, t};
        args[t] = a;
        if (nthreads > 1) pthread_create(&th[t], NULL, batch_worker, &args[t]);
    }
    if (nthreads == 1) batch_worker(&args[0]);
    else for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* splitmix64-based fill, the deterministic synthetic-input generator shared
 * with the device (tlsgpu_fill_pattern): byte i = byte (i & 7) of
 * splitmix64(seed + (i >> 3)), little-endian.                               */
static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
void ora_fill_pattern(uint8_t *p, size_t n, uint64_t seed, uint64_t start) {
    for (size_t i = 0; i < n; i++) {
        uint64_t g = start + i;
        p[i] = (uint8_t)(splitmix64(seed + (g >> 3)) >> (8 * (g & 7)));
    }
}

// tg_derive.h -- batched post-handshake key derivation on the GPU: one lane
// per connection runs calcMasterSecret (mathtls.py:70-82, optional), the
// key-block PRF of _calcPendingStates (tlsrecordlayer.py:1097-1114: PRF_SSL
// mathtls.py:55-68, PRF mathtls.py:37-50 = P_MD5 ^ P_SHA1, PRF_1_2
// mathtls.py:52-53 = P_SHA256, P_hash mathtls.py:24-35), slices it
// (:1117-1126) and builds the pending write/read connection states
// (:1127-1149) with the same builder as the host (tg_keysched.h), directly in
// HBM where the seal/open kernels read them.
//
// This is control-plane work (tens of compressions per connection), not a
// byte stream: it is here so that thousands of connections (cfg4: 4096) get
// their states without a host round trip per connection.
#pragma once
#include "tg_device.h"
#include "tg_keysched.h"

namespace tg {

// Byte-fed Merkle-Damgard hasher (SHA-1 / SHA-256 big-endian words, MD5
// little-endian); messages here are < 200 bytes.
template <int MAC>
struct ByteHasher {
    using H = Hash<MAC>;
    uint32_t h[8];
    uint32_t w[16];
    uint32_t n;      // bytes in the current block
    uint32_t total;  // message bytes so far
    __device__ void init() {
        H::init(h);
        for (int i = 0; i < 16; i++) w[i] = 0;
        n = 0;
        total = 0;
    }
    __device__ void put_raw(uint8_t b) {
        const uint32_t sh = H::BE ? 24 - 8 * (n & 3) : 8 * (n & 3);
        w[n >> 2] |= (uint32_t)b << sh;
        if (++n == 64) {
            H::compress(h, w);
            for (int i = 0; i < 16; i++) w[i] = 0;
            n = 0;
        }
    }
    __device__ void put(const uint8_t* p, uint32_t len) {
        for (uint32_t i = 0; i < len; i++) put_raw(p[i]);
        total += len;
    }
    __device__ void put_byte_n(uint8_t b, uint32_t count) {
        for (uint32_t i = 0; i < count; i++) put_raw(b);
        total += count;
    }
    // FIPS 180-4 §5.1.1 / RFC 1321 §3.1-3.2 padding, then the digest bytes
    __device__ void final(uint8_t* out) {
        const uint64_t bits = (uint64_t)total * 8;
        put_raw(0x80);
        while (n != 56) put_raw(0);
        for (int i = 0; i < 8; i++) put_raw((uint8_t)(H::BE ? bits >> (56 - 8 * i) : bits >> (8 * i)));
        for (int i = 0; i < H::DLEN; i++) {
            const uint32_t v = h[i >> 2];
            out[i] = (uint8_t)(H::BE ? v >> (24 - 8 * (i & 3)) : v >> (8 * (i & 3)));
        }
    }
};

// HMAC-H(key, m1 | m2 | m3), key <= 64 bytes (hmac.HMAC, mathtls.py:116-117)
template <int MAC>
__device__ void hmac3(const uint8_t* key, uint32_t klen, const uint8_t* m1, uint32_t l1, const uint8_t* m2,
                      uint32_t l2, const uint8_t* m3, uint32_t l3, uint8_t* out) {
    ByteHasher<MAC> x;
    uint8_t pad[64];
    for (int i = 0; i < 64; i++) pad[i] = (uint8_t)(((uint32_t)i < klen ? key[i] : 0) ^ 0x36);
    x.init();
    x.put(pad, 64);
    x.put(m1, l1);
    x.put(m2, l2);
    x.put(m3, l3);
    uint8_t inner[32];
    x.final(inner);
    for (int i = 0; i < 64; i++) pad[i] ^= 0x36 ^ 0x5c;
    x.init();
    x.put(pad, 64);
    x.put(inner, Hash<MAC>::DLEN);
    x.final(out);
}

// P_hash (mathtls.py:24-35), output XORed into out[0..length)
template <int MAC>
__device__ void p_hash_xor(const uint8_t* secret, uint32_t slen, const uint8_t* label, uint32_t llen,
                           const uint8_t* seed, uint32_t seedlen, uint8_t* out, uint32_t length) {
    constexpr uint32_t D = Hash<MAC>::DLEN;
    uint8_t a[32], blk[32];
    hmac3<MAC>(secret, slen, label, llen, seed, seedlen, nullptr, 0, a);  // A(1) = HMAC(secret, A(0) = label|seed)
    for (uint32_t pos = 0; pos < length; pos += D) {
        hmac3<MAC>(secret, slen, a, D, label, llen, seed, seedlen, blk);
        for (uint32_t i = 0; i < D && pos + i < length; i++) out[pos + i] ^= blk[i];
        hmac3<MAC>(secret, slen, a, D, nullptr, 0, nullptr, 0, a);
    }
}

// PRF (TLS 1.0/1.1, mathtls.py:37-50) / PRF_1_2 (TLS 1.2, :52-53) / PRF_SSL (:55-68)
__device__ void tls_prf(int ver_minor, const uint8_t* secret, uint32_t slen, const uint8_t* label, uint32_t llen,
                        const uint8_t* seed, uint32_t seedlen, uint8_t* out, uint32_t length) {
    for (uint32_t i = 0; i < length; i++) out[i] = 0;
    if (ver_minor == 0) {
        // MD5(secret | SHA1(letter^(x+1) | secret | seed)), 16 bytes per x
        for (uint32_t x = 0, pos = 0; pos < length && x < 26; x++, pos += 16) {
            ByteHasher<TLSGPU_MAC_SHA1> s;
            s.init();
            s.put_byte_n((uint8_t)('A' + x), x + 1);
            s.put(secret, slen);
            s.put(seed, seedlen);
            uint8_t inner[20], blk[16];
            s.final(inner);
            ByteHasher<TLSGPU_MAC_MD5> m;
            m.init();
            m.put(secret, slen);
            m.put(inner, 20);
            m.final(blk);
            for (uint32_t i = 0; i < 16 && pos + i < length; i++) out[pos + i] = blk[i];
        }
    } else if (ver_minor == 3) {
        p_hash_xor<TLSGPU_MAC_SHA256>(secret, slen, label, llen, seed, seedlen, out, length);
    } else {
        const uint32_t h1 = (slen + 1) / 2, h2 = slen / 2;  // ceil / floor split, halves may share a byte
        p_hash_xor<TLSGPU_MAC_MD5>(secret, h1, label, llen, seed, seedlen, out, length);
        p_hash_xor<TLSGPU_MAC_SHA1>(secret + h2, slen - h2, label, llen, seed, seedlen, out, length);
    }
}

// CipherSuite -> (cipher, mac, key, iv, mac lengths) (tlsrecordlayer.py:1063-1095, constants.py:159-201)
__device__ bool suite_params(uint32_t suite, int& cipher, int& mac, uint32_t& kl, uint32_t& ivl, uint32_t& ml) {
    mac = TLSGPU_MAC_SHA1;
    switch (suite) {
        case 0x0004: cipher = TLSGPU_CIPHER_RC4; mac = TLSGPU_MAC_MD5; break;
        case 0x0005: cipher = TLSGPU_CIPHER_RC4; break;
        case 0x000a: case 0xc01a: case 0xc01b: cipher = TLSGPU_CIPHER_3DES; break;
        case 0x002f: case 0x0034: case 0xc01d: case 0xc01e: cipher = TLSGPU_CIPHER_AES128; break;
        case 0x0035: case 0x003a: case 0xc020: case 0xc021: cipher = TLSGPU_CIPHER_AES256; break;
        case 0x003c: cipher = TLSGPU_CIPHER_AES128; mac = TLSGPU_MAC_SHA256; break;
        case 0x003d: cipher = TLSGPU_CIPHER_AES256; mac = TLSGPU_MAC_SHA256; break;
        default: return false;
    }
    kl = cipher == TLSGPU_CIPHER_AES256 ? 32 : cipher == TLSGPU_CIPHER_3DES ? 24 : 16;
    ivl = cipher == TLSGPU_CIPHER_RC4 ? 0 : cipher == TLSGPU_CIPHER_3DES ? 8 : 16;
    ml = mac == TLSGPU_MAC_SHA256 ? 32 : mac == TLSGPU_MAC_MD5 ? 16 : 20;
    return true;
}

__global__ void __launch_bounds__(64) derive_kernel(const tlsgpu_derive_desc* __restrict__ descs, uint32_t n,
                                                    ConnState* __restrict__ wstates, ConnState* __restrict__ rstates,
                                                    uint8_t* __restrict__ master_out, uint8_t* __restrict__ kb_out,
                                                    int32_t* __restrict__ status) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tlsgpu_derive_desc d = descs[i];
    ConnState* ws = wstates + i;
    ConnState* rs = rstates + i;
    ks_zero(ws);
    ks_zero(rs);
    if (kb_out)
        for (int b = 0; b < TLSGPU_KEY_BLOCK_MAX; b++) kb_out[(size_t)i * TLSGPU_KEY_BLOCK_MAX + b] = 0;
    int cipher, mac;
    uint32_t kl, ivl, ml;
    if (!suite_params(d.suite, cipher, mac, kl, ivl, ml) || d.ver_major != 3 || d.ver_minor > 3 ||
        (mac == TLSGPU_MAC_SHA256 && d.ver_minor != 3)) {
        status[i] = TLSGPU_EINVAL;
        return;
    }
    uint8_t seed[64];
    uint8_t master[48];
    if (d.flags & TLSGPU_DERIVE_PREMASTER) {
        // calcMasterSecret: seed = clientRandom | serverRandom (mathtls.py:70-82)
        for (int b = 0; b < 32; b++) seed[b] = d.client_random[b], seed[32 + b] = d.server_random[b];
        const uint8_t label[13] = {'m', 'a', 's', 't', 'e', 'r', ' ', 's', 'e', 'c', 'r', 'e', 't'};
        tls_prf(d.ver_minor, d.secret, 48, label, 13, seed, 64, master, 48);
    } else {
        for (int b = 0; b < 48; b++) master[b] = d.secret[b];
    }
    if (master_out)
        for (int b = 0; b < 48; b++) master_out[(size_t)i * 48 + b] = master[b];
    // key block: seed = serverRandom | clientRandom (tlsrecordlayer.py:1099-1114)
    for (int b = 0; b < 32; b++) seed[b] = d.server_random[b], seed[32 + b] = d.client_random[b];
    const uint8_t label[13] = {'k', 'e', 'y', ' ', 'e', 'x', 'p', 'a', 'n', 's', 'i', 'o', 'n'};
    const uint32_t len = 2 * (ml + kl + ivl);
    uint8_t kb[TLSGPU_KEY_BLOCK_MAX];
    tls_prf(d.ver_minor, master, 48, label, 13, seed, 64, kb, len);
    if (kb_out)
        for (uint32_t b = 0; b < len; b++) kb_out[(size_t)i * TLSGPU_KEY_BLOCK_MAX + b] = kb[b];
    // slices: client MAC, server MAC, client key, server key, client IV, server IV (:1117-1126)
    const uint8_t* cmac = kb;
    const uint8_t* smac = kb + ml;
    const uint8_t* ckey = kb + 2 * ml;
    const uint8_t* skey = ckey + kl;
    const uint8_t* civ = skey + kl;
    const uint8_t* siv = civ + ivl;
    const bool client = d.client != 0;
    // the sender's fixedIVBlock (:1146-1149); the receiver only strips the explicit IV
    const bool need_fiv = d.ver_minor >= 2 && ivl != 0;
    uint8_t zero_iv[16] = {0};
    int rc = build_conn_state(ws, cipher, mac, 3, d.ver_minor, client ? ckey : skey, kl, client ? civ : siv, ivl,
                              client ? cmac : smac, ml, need_fiv ? d.fixed_iv : nullptr, need_fiv ? ivl : 0, 0,
                              c_aes.sbox, c_aes.im0);
    if (!rc)
        rc = build_conn_state(rs, cipher, mac, 3, d.ver_minor, client ? skey : ckey, kl, client ? siv : civ, ivl,
                              client ? smac : cmac, ml, need_fiv ? zero_iv : nullptr, need_fiv ? ivl : 0, 0,
                              c_aes.sbox, c_aes.im0);
    status[i] = rc ? TLSGPU_EINVAL : TLSGPU_OK;
}

}  // namespace tg

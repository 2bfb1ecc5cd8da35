// tg_keysched.h -- connection-state construction shared by the host entry
// point (tlsgpu_conn_state_init, tg_api.hip) and the batched device key
// derivation (derive_kernel, tg_derive.h), so both write byte-identical
// 2 KiB states.  This is _calcPendingStates' cipher/MAC object creation
// (tlsrecordlayer.py:1127-1149): createAES/createRC4/createTripleDES
// (cipherfactory.py:31-102) + createHMAC / createMAC_SSL (mathtls.py:116-151).
// The AES S-box / InvMixColumn tables are passed in: h_aes on the host,
// the __constant__ c_aes copy on the device.
#pragma once
#include "tg_common.h"
#include "tg_hash.h"

namespace tg {

// error codes of build_conn_state (host maps them to messages)
enum : int {
    KS_OK = 0,
    KS_AES192_SUITE,
    KS_VERSION,
    KS_MAC,
    KS_SHA256_VERSION,
    KS_AES_KEY,
    KS_3DES_KEY,
    KS_RC4_KEY,
    KS_CIPHER,
    KS_FIXED_IV,
    KS_MAC_KEY,
    KS_SSL3_SHA_KEY,
    KS_SSL3_MD5_KEY,
    KS_SSL3_MAC,
    KS_NCODES
};

TG_HD uint32_t ks_bswap(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}
TG_HD uint32_t ks_rotl(uint32_t x, int n) { return n ? (x << n) | (x >> (32 - n)) : x; }
TG_HD uint32_t ks_le_word(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
TG_HD uint32_t ks_be_word(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
TG_HD uint8_t ks_xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

// FIPS-197 §5.2 key expansion; stored as LE column words (+ equivalent
// inverse cipher keys, §5.3.5).  Same result as rijndael.py:206-276.
TG_HD void aes_expand(ConnState* st, const uint8_t* key, int klen, const uint8_t* sbox, const uint32_t* im0) {
    const int nk = klen / 4, nr = nk + 6, total = 4 * (nr + 1);
    uint32_t w[60];
    for (int i = 0; i < nk; i++) w[i] = ks_be_word(key + 4 * i);
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = w[i - 1];
        if (i % nk == 0) {
            t = ((uint32_t)sbox[(t >> 16) & 0xff] << 24) | ((uint32_t)sbox[(t >> 8) & 0xff] << 16) |
                ((uint32_t)sbox[t & 0xff] << 8) | sbox[t >> 24];
            t ^= (uint32_t)rcon << 24;
            rcon = ks_xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = ((uint32_t)sbox[t >> 24] << 24) | ((uint32_t)sbox[(t >> 16) & 0xff] << 16) |
                ((uint32_t)sbox[(t >> 8) & 0xff] << 8) | sbox[t & 0xff];
        }
        w[i] = w[i - nk] ^ t;
    }
    for (int i = 0; i < total; i++) st->ek[i] = ks_bswap(w[i]);
    for (int r = 0; r <= nr; r++)
        for (int c = 0; c < 4; c++) {
            uint32_t x = st->ek[4 * (nr - r) + c];
            if (r > 0 && r < nr)
                x = im0[x & 0xff] ^ ks_rotl(im0[(x >> 8) & 0xff], 8) ^ ks_rotl(im0[(x >> 16) & 0xff], 16) ^
                    ks_rotl(im0[x >> 24], 24);
            st->dk[4 * r + c] = x;
        }
}

// FIPS 46-3 key schedule, packed for the kernels' rotated-domain rounds:
// even word = K8 | K6<<8 | K4<<16 | K2<<24, odd word = K7 | K5<<8 | K3<<16 | K1<<24
TG_HD uint64_t ks_permute_bits(uint64_t in, int inbits, const uint8_t* tab, int n) {
    uint64_t out = 0;
    for (int i = 0; i < n; i++) out = (out << 1) | ((in >> (inbits - tab[i])) & 1);
    return out;
}
TG_HD void des_schedule(uint32_t* out, const uint8_t* key) {
    uint64_t k = 0;
    for (int i = 0; i < 8; i++) k = (k << 8) | key[i];
    uint64_t cd = ks_permute_bits(k, 64, DesConst::PC1, 56);
    uint32_t c = (uint32_t)(cd >> 28) & 0xfffffff, d = (uint32_t)cd & 0xfffffff;
    for (int r = 0; r < 16; r++) {
        for (int s = 0; s < DesConst::SHIFTS[r]; s++) {
            c = ((c << 1) | (c >> 27)) & 0xfffffff;
            d = ((d << 1) | (d >> 27)) & 0xfffffff;
        }
        uint64_t sub = ks_permute_bits(((uint64_t)c << 28) | d, 56, DesConst::PC2, 48);
        uint32_t K[8];
        for (int i = 0; i < 8; i++) K[i] = (uint32_t)(sub >> (42 - 6 * i)) & 63;
        out[2 * r] = K[7] | (K[5] << 8) | (K[3] << 16) | (K[1] << 24);
        out[2 * r + 1] = K[6] | (K[4] << 8) | (K[2] << 16) | (K[0] << 24);
    }
}

// python_rc4.py:13-23
TG_HD void rc4_ksa(ConnState* st, const uint8_t* key, size_t klen) {
    for (int i = 0; i < 256; i++) st->rc4_S[i] = (uint8_t)i;
    uint32_t j = 0;
    for (int i = 0; i < 256; i++) {
        j = (j + st->rc4_S[i] + key[i % klen]) & 255;
        uint8_t t = st->rc4_S[i];
        st->rc4_S[i] = st->rc4_S[j];
        st->rc4_S[j] = t;
    }
    st->rc4_i = st->rc4_j = 0;
}

template <int MAC>
TG_HD void ks_midstate(uint32_t* out, const uint8_t* block) {
    using H = Hash<MAC>;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0}, w[16];
    H::init(h);
    for (int i = 0; i < 16; i++) w[i] = H::BE ? ks_be_word(block + 4 * i) : ks_le_word(block + 4 * i);
    H::compress(h, w);
    for (int i = 0; i < 8; i++) out[i] = h[i];
}
TG_HD void ks_midstate_any(int mac, uint32_t* out, const uint8_t* block) {
    if (mac == TLSGPU_MAC_SHA1) ks_midstate<TLSGPU_MAC_SHA1>(out, block);
    else if (mac == TLSGPU_MAC_SHA256) ks_midstate<TLSGPU_MAC_SHA256>(out, block);
    else ks_midstate<TLSGPU_MAC_MD5>(out, block);
}

TG_HD void ks_pack_le(uint32_t* dst, const uint8_t* src, size_t n) {
    for (size_t i = 0; i < (n + 3) / 4; i++) {
        uint32_t v = 0;
        for (size_t b = 0; b < 4 && 4 * i + b < n; b++) v |= (uint32_t)src[4 * i + b] << (8 * b);
        dst[i] = v;
    }
}

TG_HD void ks_zero(ConnState* st) {
    uint32_t* p = reinterpret_cast<uint32_t*>(st);
    for (int i = 0; i < (int)(sizeof(ConnState) / 4); i++) p[i] = 0;
}

// createAES / createTripleDES / createRC4 argument checks (aes.py:8-13,
// tripledes.py:8-13, rc4.py:9-10, cipherfactory.py:70-71) + key setup
TG_HD int cipher_setup(ConnState* st, int cipher, const uint8_t* key, size_t key_len, const uint8_t* iv,
                       size_t iv_len, const uint8_t* sbox, const uint32_t* im0) {
    st->cipher = (uint32_t)cipher;
    switch (cipher) {
        case TLSGPU_CIPHER_AES128:
        case TLSGPU_CIPHER_AES192:
        case TLSGPU_CIPHER_AES256:
            if (key_len != (cipher == TLSGPU_CIPHER_AES128 ? 16u : cipher == TLSGPU_CIPHER_AES192 ? 24u : 32u) ||
                iv_len != 16 || !key || !iv)
                return KS_AES_KEY;
            aes_expand(st, key, (int)key_len, sbox, im0);
            st->bs = 16;
            ks_pack_le(st->iv, iv, 16);
            return KS_OK;
        case TLSGPU_CIPHER_3DES:
            if (key_len != 24 || iv_len != 8 || !key || !iv) return KS_3DES_KEY;
            for (int i = 0; i < 3; i++) des_schedule(st->des[i], key + 8 * i);
            st->bs = 8;
            ks_pack_le(st->iv, iv, 8);
            return KS_OK;
        case TLSGPU_CIPHER_RC4:
            if (key_len < 16 || key_len > 256 || iv_len != 0 || !key) return KS_RC4_KEY;
            rc4_ksa(st, key, key_len);
            st->bs = 0;
            return KS_OK;
        default:
            return KS_CIPHER;
    }
}

// The whole _ConnectionState of one direction: cipher + MAC context +
// version-dependent framing flags.  st must be zeroed by the caller.
TG_HD int build_conn_state(ConnState* st, int cipher, int mac, int ver_major, int ver_minor, const uint8_t* key,
                           size_t key_len, const uint8_t* iv, size_t iv_len, const uint8_t* mac_key,
                           size_t mac_key_len, const uint8_t* fixed_iv, size_t fixed_iv_len, uint64_t seqnum,
                           const uint8_t* sbox, const uint32_t* im0) {
    if (cipher == TLSGPU_CIPHER_AES192) return KS_AES192_SUITE;
    if (ver_major != 3 || ver_minor < 0 || ver_minor > 3) return KS_VERSION;  // handshakesettings.py:174-178
    if (mac != TLSGPU_MAC_SHA1 && mac != TLSGPU_MAC_SHA256 && mac != TLSGPU_MAC_MD5) return KS_MAC;
    if (mac == TLSGPU_MAC_SHA256 && ver_minor != 3) return KS_SHA256_VERSION;  // constants.py:204-210
    int rc = cipher_setup(st, cipher, key, key_len, iv, iv_len, sbox, im0);
    if (rc) return rc;
    st->mac = (uint32_t)mac;
    st->vmaj = (uint8_t)ver_major;
    st->vmin = (uint8_t)ver_minor;
    st->ssl3 = ver_minor == 0;
    st->seqnum = seqnum;
    st->maclen = (uint8_t)(mac == TLSGPU_MAC_SHA1 ? 20 : mac == TLSGPU_MAC_SHA256 ? 32 : 16);
    st->explicit_iv = (ver_minor >= 2 && cipher != TLSGPU_CIPHER_RC4) ? 1u : 0u;
    if (st->explicit_iv) {
        if (!fixed_iv || fixed_iv_len != st->bs) return KS_FIXED_IV;
        ks_pack_le(st->fixed_iv, fixed_iv, fixed_iv_len);
    }
    if (mac_key_len > 64 || (!mac_key && mac_key_len)) return KS_MAC_KEY;
    st->mac_key_len = (uint32_t)mac_key_len;
    uint8_t blk[64];
    if (st->ssl3) {
        // MAC_SSL (mathtls.py:125-151): H(K | pad2 | H(K | pad1 | m)), pads 40 (SHA) / 48 (MD5) bytes
        if (mac == TLSGPU_MAC_SHA1) {
            if (mac_key_len != 20) return KS_SSL3_SHA_KEY;
            for (int i = 0; i < 5; i++) st->mac_key[i] = ks_be_word(mac_key + 4 * i);
        } else if (mac == TLSGPU_MAC_MD5) {
            if (mac_key_len != 16) return KS_SSL3_MD5_KEY;
            for (int i = 0; i < 16; i++) blk[i] = mac_key[i];
            for (int i = 16; i < 64; i++) blk[i] = 0x36;
            ks_midstate_any(mac, st->mac_in, blk);
            for (int i = 16; i < 64; i++) blk[i] = 0x5c;
            ks_midstate_any(mac, st->mac_out, blk);
        } else {
            return KS_SSL3_MAC;
        }
    } else {
        // HMAC (RFC 2104) ipad/opad midstates, as hmac.HMAC does (mathtls.py:116-117)
        for (int i = 0; i < 64; i++) blk[i] = (uint8_t)((i < (int)mac_key_len ? mac_key[i] : 0) ^ 0x36);
        ks_midstate_any(mac, st->mac_in, blk);
        for (int i = 0; i < 64; i++) blk[i] = (uint8_t)((i < (int)mac_key_len ? mac_key[i] : 0) ^ 0x5c);
        ks_midstate_any(mac, st->mac_out, blk);
    }
    return KS_OK;
}

}  // namespace tg

// tg_api.hip -- extern "C" entry points of libtlsgpu.so (declared in
// include/tlsgpu.h).  Host-side connection-state construction (the
// _calcPendingStates equivalent, tlsrecordlayer.py:1061-1149), memory /
// stream / event plumbing, and argument validation in front of the kernels.
#include <string.h>
#include <stdio.h>
#include "tg_common.h"
#include "tg_hash.h"
#include "tg_launch.h"

using namespace tg;

namespace {

thread_local char g_err[256] = "";

int fail_hip(hipError_t e, const char* what) {
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return TLSGPU_EHIP;
}
int fail(int code, const char* what) {
    snprintf(g_err, sizeof g_err, "%s", what);
    return code;
}
#define TG_HIP(call)                                   \
    do {                                               \
        hipError_t e_ = (call);                        \
        if (e_ != hipSuccess) return fail_hip(e_, #call); \
    } while (0)

constexpr AesTables h_aes{};

inline uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
inline uint32_t rotl(uint32_t x, int n) { return n ? (x << n) | (x >> (32 - n)) : x; }
inline uint32_t le_word(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline uint32_t be_word(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// FIPS-197 §5.2 key expansion; stored as LE column words (+ equivalent
// inverse cipher keys, §5.3.5).  Same result as rijndael.py:206-276.
void aes_expand(ConnState* st, const uint8_t* key, int klen) {
    const int nk = klen / 4, nr = nk + 6, total = 4 * (nr + 1);
    uint32_t w[60];
    for (int i = 0; i < nk; i++) w[i] = be_word(key + 4 * i);
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = w[i - 1];
        if (i % nk == 0) {
            t = ((uint32_t)h_aes.sbox[(t >> 16) & 0xff] << 24) | ((uint32_t)h_aes.sbox[(t >> 8) & 0xff] << 16) |
                ((uint32_t)h_aes.sbox[t & 0xff] << 8) | h_aes.sbox[t >> 24];
            t ^= (uint32_t)rcon << 24;
            rcon = gf_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = ((uint32_t)h_aes.sbox[t >> 24] << 24) | ((uint32_t)h_aes.sbox[(t >> 16) & 0xff] << 16) |
                ((uint32_t)h_aes.sbox[(t >> 8) & 0xff] << 8) | h_aes.sbox[t & 0xff];
        }
        w[i] = w[i - nk] ^ t;
    }
    for (int i = 0; i < total; i++) st->ek[i] = bswap(w[i]);
    for (int r = 0; r <= nr; r++)
        for (int c = 0; c < 4; c++) {
            uint32_t x = st->ek[4 * (nr - r) + c];
            if (r > 0 && r < nr)
                x = h_aes.im0[x & 0xff] ^ rotl(h_aes.im0[(x >> 8) & 0xff], 8) ^
                    rotl(h_aes.im0[(x >> 16) & 0xff], 16) ^ rotl(h_aes.im0[x >> 24], 24);
            st->dk[4 * r + c] = x;
        }
}

// FIPS 46-3 key schedule, packed for the kernels' rotated-domain rounds:
// even word = K8 | K6<<8 | K4<<16 | K2<<24, odd word = K7 | K5<<8 | K3<<16 | K1<<24
uint64_t permute_bits(uint64_t in, int inbits, const uint8_t* tab, int n) {
    uint64_t out = 0;
    for (int i = 0; i < n; i++) out = (out << 1) | ((in >> (inbits - tab[i])) & 1);
    return out;
}
void des_schedule(uint32_t out[32], const uint8_t key[8]) {
    uint64_t k = 0;
    for (int i = 0; i < 8; i++) k = (k << 8) | key[i];
    uint64_t cd = permute_bits(k, 64, DesConst::PC1, 56);
    uint32_t c = (uint32_t)(cd >> 28) & 0xfffffff, d = (uint32_t)cd & 0xfffffff;
    for (int r = 0; r < 16; r++) {
        for (int s = 0; s < DesConst::SHIFTS[r]; s++) {
            c = ((c << 1) | (c >> 27)) & 0xfffffff;
            d = ((d << 1) | (d >> 27)) & 0xfffffff;
        }
        uint64_t sub = permute_bits(((uint64_t)c << 28) | d, 56, DesConst::PC2, 48);
        uint32_t K[8];
        for (int i = 0; i < 8; i++) K[i] = (uint32_t)(sub >> (42 - 6 * i)) & 63;
        out[2 * r] = K[7] | (K[5] << 8) | (K[3] << 16) | (K[1] << 24);
        out[2 * r + 1] = K[6] | (K[4] << 8) | (K[2] << 16) | (K[0] << 24);
    }
}

// python_rc4.py:13-23
void rc4_ksa(ConnState* st, const uint8_t* key, size_t klen) {
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
void midstate(uint32_t out[8], const uint8_t block[64]) {
    using H = Hash<MAC>;
    uint32_t h[8] = {0}, w[16];
    H::init(h);
    for (int i = 0; i < 16; i++) w[i] = H::BE ? be_word(block + 4 * i) : le_word(block + 4 * i);
    H::compress(h, w);
    for (int i = 0; i < 8; i++) out[i] = h[i];
}
void midstate_any(int mac, uint32_t out[8], const uint8_t block[64]) {
    if (mac == TLSGPU_MAC_SHA1) midstate<TLSGPU_MAC_SHA1>(out, block);
    else if (mac == TLSGPU_MAC_SHA256) midstate<TLSGPU_MAC_SHA256>(out, block);
    else midstate<TLSGPU_MAC_MD5>(out, block);
}

void pack_le(uint32_t* dst, const uint8_t* src, size_t n) {
    for (size_t i = 0; i < (n + 3) / 4; i++) {
        uint32_t v = 0;
        for (size_t b = 0; b < 4 && 4 * i + b < n; b++) v |= (uint32_t)src[4 * i + b] << (8 * b);
        dst[i] = v;
    }
}

int cipher_setup(ConnState* st, int cipher, const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len) {
    st->cipher = (uint32_t)cipher;
    switch (cipher) {
        case TLSGPU_CIPHER_AES128:
        case TLSGPU_CIPHER_AES192:
        case TLSGPU_CIPHER_AES256:
            // aes.py:8-13
            if (key_len != (cipher == TLSGPU_CIPHER_AES128 ? 16u : cipher == TLSGPU_CIPHER_AES192 ? 24u : 32u) ||
                iv_len != 16 || !key || !iv)
                return fail(TLSGPU_EINVAL, "AES needs a 16/24/32-byte key and a 16-byte IV");
            aes_expand(st, key, (int)key_len);
            st->bs = 16;
            pack_le(st->iv, iv, 16);
            break;
        case TLSGPU_CIPHER_3DES:
            // tripledes.py:8-13
            if (key_len != 24 || iv_len != 8 || !key || !iv)
                return fail(TLSGPU_EINVAL, "3DES needs a 24-byte key and an 8-byte IV");
            for (int i = 0; i < 3; i++) des_schedule(st->des[i], key + 8 * i);
            st->bs = 8;
            pack_le(st->iv, iv, 8);
            break;
        case TLSGPU_CIPHER_RC4:
            // rc4.py:9-10; cipherfactory.py:70-71
            if (key_len < 16 || key_len > 256 || iv_len != 0 || !key)
                return fail(TLSGPU_EINVAL, "RC4 needs a 16..256-byte key and no IV");
            rc4_ksa(st, key, key_len);
            st->bs = 0;
            break;
        default:
            return fail(TLSGPU_EINVAL, "unknown cipher");
    }
    return 0;
}

inline ConnState* S(tlsgpu_conn_state* p) { return reinterpret_cast<ConnState*>(p); }
inline const ConnState* S(const tlsgpu_conn_state* p) { return reinterpret_cast<const ConnState*>(p); }
inline hipStream_t HS(tlsgpu_stream s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

extern "C" {

int tlsgpu_abi_version(void) { return TLSGPU_ABI_VERSION; }
const char* tlsgpu_last_error(void) { return g_err; }

int tlsgpu_device_count(int* n) {
    if (!n) return fail(TLSGPU_EINVAL, "null");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        return fail_hip(e, "hipGetDeviceCount");
    }
    *n = c;
    return 0;
}
int tlsgpu_set_device(int ordinal) {
    TG_HIP(hipSetDevice(ordinal));
    return 0;
}
int tlsgpu_get_device(int* ordinal) {
    TG_HIP(hipGetDevice(ordinal));
    return 0;
}
int tlsgpu_device_synchronize(void) {
    TG_HIP(hipDeviceSynchronize());
    return 0;
}
int tlsgpu_device_arch(int ordinal, char* name, size_t cap) {
    hipDeviceProp_t p;
    TG_HIP(hipGetDeviceProperties(&p, ordinal));
    snprintf(name, cap, "%s", p.gcnArchName);
    return 0;
}

int tlsgpu_malloc(void** dptr, size_t bytes) {
    TG_HIP(hipMalloc(dptr, bytes ? bytes : 1));
    return 0;
}
int tlsgpu_free(void* dptr) {
    TG_HIP(hipFree(dptr));
    return 0;
}
int tlsgpu_host_alloc(void** hptr, size_t bytes) {
    TG_HIP(hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault));
    return 0;
}
int tlsgpu_host_free(void* hptr) {
    TG_HIP(hipHostFree(hptr));
    return 0;
}
int tlsgpu_memcpy_h2d(void* dst, const void* src, size_t bytes, tlsgpu_stream s) {
    TG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, HS(s)));
    return 0;
}
int tlsgpu_memcpy_d2h(void* dst, const void* src, size_t bytes, tlsgpu_stream s) {
    TG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, HS(s)));
    return 0;
}
int tlsgpu_memcpy_d2d(void* dst, const void* src, size_t bytes, tlsgpu_stream s) {
    TG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, HS(s)));
    return 0;
}
int tlsgpu_memset(void* dptr, int value, size_t bytes, tlsgpu_stream s) {
    TG_HIP(hipMemsetAsync(dptr, value, bytes, HS(s)));
    return 0;
}

int tlsgpu_stream_create(tlsgpu_stream* s) {
    hipStream_t h;
    TG_HIP(hipStreamCreateWithFlags(&h, hipStreamNonBlocking));
    *s = reinterpret_cast<tlsgpu_stream>(h);
    return 0;
}
int tlsgpu_stream_destroy(tlsgpu_stream s) {
    TG_HIP(hipStreamDestroy(HS(s)));
    return 0;
}
int tlsgpu_stream_synchronize(tlsgpu_stream s) {
    TG_HIP(hipStreamSynchronize(HS(s)));
    return 0;
}
int tlsgpu_event_create(tlsgpu_event* e) {
    hipEvent_t h;
    TG_HIP(hipEventCreate(&h));
    *e = reinterpret_cast<tlsgpu_event>(h);
    return 0;
}
int tlsgpu_event_destroy(tlsgpu_event e) {
    TG_HIP(hipEventDestroy(reinterpret_cast<hipEvent_t>(e)));
    return 0;
}
int tlsgpu_event_record(tlsgpu_event e, tlsgpu_stream s) {
    TG_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(e), HS(s)));
    return 0;
}
int tlsgpu_event_synchronize(tlsgpu_event e) {
    TG_HIP(hipEventSynchronize(reinterpret_cast<hipEvent_t>(e)));
    return 0;
}
int tlsgpu_event_elapsed_ms(float* ms, tlsgpu_event a, tlsgpu_event b) {
    TG_HIP(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(a), reinterpret_cast<hipEvent_t>(b)));
    return 0;
}

int tlsgpu_conn_state_init(tlsgpu_conn_state* out, int cipher, int mac, int ver_major, int ver_minor,
                           const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                           const uint8_t* mac_key, size_t mac_key_len, const uint8_t* fixed_iv,
                           size_t fixed_iv_len, uint64_t seqnum) {
    if (!out) return fail(TLSGPU_EINVAL, "null state");
    if (cipher == TLSGPU_CIPHER_AES192) return fail(TLSGPU_EINVAL, "no TLS suite uses AES-192");
    memset(out, 0, sizeof *out);
    ConnState* st = S(out);
    if (ver_major != 3 || ver_minor < 0 || ver_minor > 3)
        return fail(TLSGPU_EINVAL, "version must be (3,0)..(3,3)");  // handshakesettings.py:174-178
    if (mac != TLSGPU_MAC_SHA1 && mac != TLSGPU_MAC_SHA256 && mac != TLSGPU_MAC_MD5)
        return fail(TLSGPU_EINVAL, "unknown MAC");
    if (mac == TLSGPU_MAC_SHA256 && ver_minor != 3)
        return fail(TLSGPU_EINVAL, "SHA256 suites need TLS 1.2");  // constants.py:204-210
    int rc = cipher_setup(st, cipher, key, key_len, iv, iv_len);
    if (rc) return rc;
    st->mac = (uint32_t)mac;
    st->vmaj = (uint8_t)ver_major;
    st->vmin = (uint8_t)ver_minor;
    st->ssl3 = ver_minor == 0;
    st->seqnum = seqnum;
    st->maclen = (uint8_t)(mac == TLSGPU_MAC_SHA1 ? 20 : mac == TLSGPU_MAC_SHA256 ? 32 : 16);
    st->explicit_iv = (ver_minor >= 2 && cipher != TLSGPU_CIPHER_RC4) ? 1u : 0u;
    if (st->explicit_iv) {
        if (!fixed_iv || fixed_iv_len != st->bs)
            return fail(TLSGPU_EINVAL, "TLS>=1.1 block cipher needs fixed_iv of the block size");
        pack_le(st->fixed_iv, fixed_iv, fixed_iv_len);
    }
    if (mac_key_len > 64 || (!mac_key && mac_key_len)) return fail(TLSGPU_EINVAL, "MAC key longer than 64 bytes");
    st->mac_key_len = (uint32_t)mac_key_len;
    if (st->ssl3) {
        // MAC_SSL (mathtls.py:125-151): H(K | pad2 | H(K | pad1 | m)), pads 40 (SHA) / 48 (MD5) bytes
        if (mac == TLSGPU_MAC_SHA1) {
            if (mac_key_len != 20) return fail(TLSGPU_EINVAL, "SSL3 SHA MAC key must be 20 bytes");
            for (int i = 0; i < 5; i++) st->mac_key[i] = be_word(mac_key + 4 * i);
        } else if (mac == TLSGPU_MAC_MD5) {
            if (mac_key_len != 16) return fail(TLSGPU_EINVAL, "SSL3 MD5 MAC key must be 16 bytes");
            uint8_t blk[64];
            memcpy(blk, mac_key, 16);
            memset(blk + 16, 0x36, 48);
            midstate_any(mac, st->mac_in, blk);
            memset(blk + 16, 0x5c, 48);
            midstate_any(mac, st->mac_out, blk);
        } else {
            return fail(TLSGPU_EINVAL, "SSL3 supports SHA1/MD5 MACs only");
        }
    } else {
        // HMAC (RFC 2104) ipad/opad midstates, as hmac.HMAC does (mathtls.py:116-117)
        uint8_t k[64] = {0}, blk[64];
        if (mac_key_len) memcpy(k, mac_key, mac_key_len);
        for (int i = 0; i < 64; i++) blk[i] = k[i] ^ 0x36;
        midstate_any(mac, st->mac_in, blk);
        for (int i = 0; i < 64; i++) blk[i] = k[i] ^ 0x5c;
        midstate_any(mac, st->mac_out, blk);
    }
    return 0;
}

int tlsgpu_cipher_state_init(tlsgpu_conn_state* out, int cipher, const uint8_t* key, size_t key_len,
                             const uint8_t* iv, size_t iv_len) {
    if (!out) return fail(TLSGPU_EINVAL, "null state");
    memset(out, 0, sizeof *out);
    ConnState* st = S(out);
    int rc = cipher_setup(st, cipher, key, key_len, iv, iv_len);
    if (rc) return rc;
    st->raw = 1;
    return 0;
}

int tlsgpu_conn_state_set_seqnum(tlsgpu_conn_state* st, uint64_t seqnum) {
    S(st)->seqnum = seqnum;
    return 0;
}
int tlsgpu_conn_state_set_iv(tlsgpu_conn_state* st, const uint8_t* iv, size_t iv_len) {
    ConnState* s = S(st);
    if (iv_len != s->bs || !s->bs) return fail(TLSGPU_EINVAL, "IV length must equal the block size");
    pack_le(s->iv, iv, iv_len);
    return 0;
}
int tlsgpu_conn_state_get_seqnum(const tlsgpu_conn_state* st, uint64_t* seqnum) {
    *seqnum = S(st)->seqnum;
    return 0;
}
int tlsgpu_conn_state_get_iv(const tlsgpu_conn_state* st, uint8_t* iv, size_t cap, size_t* iv_len) {
    const ConnState* s = S(st);
    size_t n = s->bs;
    if (cap < n) return fail(TLSGPU_EINVAL, "buffer too small");
    for (size_t i = 0; i < n; i++) iv[i] = (uint8_t)(s->iv[i / 4] >> (8 * (i % 4)));
    *iv_len = n;
    return 0;
}
int tlsgpu_conn_state_get_rc4(const tlsgpu_conn_state* st, uint8_t Sx[256], uint32_t* i, uint32_t* j) {
    const ConnState* s = S(st);
    if (s->cipher != TLSGPU_CIPHER_RC4) return fail(TLSGPU_EINVAL, "not an RC4 state");
    memcpy(Sx, s->rc4_S, 256);
    *i = s->rc4_i;
    *j = s->rc4_j;
    return 0;
}
int tlsgpu_conn_state_variant(const tlsgpu_conn_state* st, uint32_t* variant) {
    const ConnState* s = S(st);
    *variant = TLSGPU_VARIANT(s->cipher, s->mac, s->ssl3);
    return 0;
}
int tlsgpu_seal_wire_len(const tlsgpu_conn_state* st, uint32_t pt_len, uint32_t* wire_len) {
    const ConnState* s = S(st);
    if (pt_len == 0) {
        *wire_len = 0;
        return 0;
    }
    uint32_t body;
    if (s->bs == 0) {
        body = pt_len + s->maclen;
    } else {
        uint32_t cur = (s->explicit_iv ? s->bs : 0) + pt_len + s->maclen;
        body = cur + (s->bs - cur % s->bs);
    }
    if (body > 0xffff) return fail(TLSGPU_ETOOBIG, "record body exceeds 65535 bytes");
    *wire_len = body + 5;
    return 0;
}

size_t tlsgpu_seal_workspace_bytes(uint32_t nrecords) { return seal_workspace_bytes(nrecords); }

// library-owned workspace: per device and per kind, grow-only (calls that use it must not
// run concurrently on several streams: pass a workspace for that)
static int own_workspace(int kind, size_t need, uint8_t** out) {
    static thread_local void* own[2][64] = {{nullptr}};
    static thread_local size_t own_bytes[2][64] = {{0}};
    int dev = 0;
    (void)hipGetDevice(&dev);
    dev &= 63;
    if (own_bytes[kind][dev] < need) {
        if (own[kind][dev]) TG_HIP(hipFree(own[kind][dev]));
        own[kind][dev] = nullptr;
        own_bytes[kind][dev] = 0;
        TG_HIP(hipMalloc(&own[kind][dev], need));
        own_bytes[kind][dev] = need;
    }
    *out = static_cast<uint8_t*>(own[kind][dev]);
    return 0;
}

static uint32_t next_epoch() {
    static uint32_t epoch_ctr = 0;
    return __atomic_add_fetch(&epoch_ctr, 1, __ATOMIC_RELAXED);
}

int tlsgpu_seal_dev(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* records, uint32_t nrecords,
                    const uint8_t* pt, uint8_t* wire, tlsgpu_conn_state* states, int32_t* wire_len, uint32_t variant,
                    void* workspace, size_t workspace_bytes, tlsgpu_stream s) {
    if (nchains == 0) return 0;
    if (!chains || !records || !pt || !wire || !states || !wire_len) return fail(TLSGPU_EINVAL, "null pointer");
    uint8_t* ws = static_cast<uint8_t*>(workspace);
    if (seal_needs_workspace(variant)) {
        const size_t need = seal_workspace_bytes(nrecords);
        if (ws && workspace_bytes < need) return fail(TLSGPU_EINVAL, "workspace too small");
        if (!ws) {
            int rc = own_workspace(0, need, &ws);
            if (rc) return rc;
        }
    }
    bool known = false;
    hipError_t e = launch_seal(variant, chains, nchains, records, nrecords, pt, wire, S(states), wire_len, ws,
                               next_epoch(), HS(s), &known);
    if (!known) return fail(TLSGPU_EINVAL, "unsupported seal variant");
    if (e != hipSuccess) return fail_hip(e, "seal launch");
    return 0;
}

// ---------------------------------------------------------------- pipeline
struct tlsgpu_pipeline_s {
    int dev;
    hipStream_t mac_s, cbc_s;
    hipEvent_t mac_done[2], cbc_done[2];
    void* ws[2];
    size_t ws_bytes;
    uint64_t k;
};

int tlsgpu_pipeline_create(tlsgpu_pipeline* out, uint32_t max_records) {
    if (!out) return fail(TLSGPU_EINVAL, "null");
    tlsgpu_pipeline p = new tlsgpu_pipeline_s();
    TG_HIP(hipGetDevice(&p->dev));
    TG_HIP(hipStreamCreateWithFlags(&p->mac_s, hipStreamNonBlocking));
    TG_HIP(hipStreamCreateWithFlags(&p->cbc_s, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) {
        TG_HIP(hipEventCreateWithFlags(&p->mac_done[i], hipEventDisableTiming));
        TG_HIP(hipEventCreateWithFlags(&p->cbc_done[i], hipEventDisableTiming));
    }
    p->ws_bytes = seal_workspace_bytes(max_records ? max_records : 1);
    for (int i = 0; i < 2; i++) TG_HIP(hipMalloc(&p->ws[i], p->ws_bytes));
    p->k = 0;
    *out = p;
    return 0;
}

int tlsgpu_pipeline_destroy(tlsgpu_pipeline p) {
    if (!p) return 0;
    (void)hipStreamSynchronize(p->mac_s);
    (void)hipStreamSynchronize(p->cbc_s);
    for (int i = 0; i < 2; i++) {
        (void)hipFree(p->ws[i]);
        (void)hipEventDestroy(p->mac_done[i]);
        (void)hipEventDestroy(p->cbc_done[i]);
    }
    (void)hipStreamDestroy(p->mac_s);
    (void)hipStreamDestroy(p->cbc_s);
    delete p;
    return 0;
}

int tlsgpu_pipeline_synchronize(tlsgpu_pipeline p) {
    TG_HIP(hipStreamSynchronize(p->mac_s));
    TG_HIP(hipStreamSynchronize(p->cbc_s));
    return 0;
}

int tlsgpu_pipeline_seal(tlsgpu_pipeline p, const tlsgpu_chain* chains, uint32_t nchains,
                         const tlsgpu_record* records, uint32_t nrecords, const uint8_t* pt, uint8_t* wire,
                         tlsgpu_conn_state* states, int32_t* wire_len, uint32_t variant, tlsgpu_event cipher_start,
                         tlsgpu_event cipher_stop) {
    if (!p) return fail(TLSGPU_EINVAL, "null pipeline");
    if (nchains == 0) return 0;
    if (!chains || !records || !pt || !wire || !states || !wire_len) return fail(TLSGPU_EINVAL, "null pointer");
    if (seal_workspace_bytes(nrecords) > p->ws_bytes) return fail(TLSGPU_EINVAL, "nrecords > pipeline max_records");
    static uint32_t epoch_ctr = 0x80000000u;
    const uint32_t epoch = __atomic_add_fetch(&epoch_ctr, 1, __ATOMIC_RELAXED);
    const int i = (int)(p->k & 1);
    // workspace i was last read by the cipher phase of call k-2
    if (p->k >= 2) TG_HIP(hipStreamWaitEvent(p->mac_s, p->cbc_done[i], 0));
    bool known = false;
    hipError_t e = hipSuccess;
    if (seal_needs_workspace(variant)) {
        e = launch_seal_phases(variant, chains, nchains, records, nrecords, pt, wire, S(states), wire_len,
                               static_cast<uint8_t*>(p->ws[i]), epoch, p->mac_s, p->mac_done[i], p->cbc_s,
                               reinterpret_cast<hipEvent_t>(cipher_start), reinterpret_cast<hipEvent_t>(cipher_stop),
                               &known);
    } else {
        // single-kernel variants run on the cipher stream, in order with earlier calls
        if (cipher_start) TG_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(cipher_start), p->cbc_s));
        e = launch_seal(variant, chains, nchains, records, nrecords, pt, wire, S(states), wire_len, nullptr, epoch,
                        p->cbc_s, &known);
        if (e == hipSuccess && cipher_stop) e = hipEventRecord(reinterpret_cast<hipEvent_t>(cipher_stop), p->cbc_s);
    }
    if (!known) return fail(TLSGPU_EINVAL, "unsupported seal variant");
    if (e != hipSuccess) return fail_hip(e, "pipeline seal");
    TG_HIP(hipEventRecord(p->cbc_done[i], p->cbc_s));
    p->k++;
    return 0;
}

int tlsgpu_cipher_dev(const tlsgpu_span* spans, uint32_t nspans, const uint8_t* in, uint8_t* out,
                      tlsgpu_conn_state* states, int cipher, int decrypt, tlsgpu_stream s) {
    if (nspans == 0) return 0;
    if (!spans || !in || !out || !states) return fail(TLSGPU_EINVAL, "null pointer");
    bool known = false;
    hipError_t e = launch_cipher(cipher, decrypt, spans, nspans, in, out, S(states), HS(s), &known);
    if (!known) return fail(TLSGPU_EINVAL, "unknown cipher");
    if (e != hipSuccess) return fail_hip(e, "cipher launch");
    return 0;
}

size_t tlsgpu_open_workspace_bytes(uint32_t nrecords) { return open_workspace_bytes(nrecords); }

int tlsgpu_open_dev(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_open_record* records,
                    uint32_t nrecords, const uint8_t* wire, uint8_t* pt, tlsgpu_conn_state* states, int32_t* status,
                    uint32_t variant, void* workspace, size_t workspace_bytes, tlsgpu_stream s) {
    if (nchains == 0) return 0;
    if (!chains || !records || !wire || !pt || !states || !status) return fail(TLSGPU_EINVAL, "null pointer");
    uint8_t* ws = static_cast<uint8_t*>(workspace);
    if (open_needs_workspace(variant)) {
        const size_t need = open_workspace_bytes(nrecords);
        if (ws && workspace_bytes < need) return fail(TLSGPU_EINVAL, "workspace too small");
        if (!ws) {
            int rc = own_workspace(1, need, &ws);
            if (rc) return rc;
        }
    }
    bool known = false;
    hipError_t e = launch_open(variant, chains, nchains, records, nrecords, wire, pt, S(states), status, ws,
                               next_epoch(), HS(s), &known);
    if (!known) return fail(TLSGPU_EINVAL, "unsupported open variant");
    if (e != hipSuccess) return fail_hip(e, "open launch");
    return 0;
}

int tlsgpu_fill_pattern(uint8_t* dptr, size_t bytes, uint64_t seed, uint64_t start, tlsgpu_stream s) {
    hipError_t e = launch_fill(dptr, bytes, seed, start, HS(s));
    if (e != hipSuccess) return fail_hip(e, "fill launch");
    return 0;
}

}  // extern "C"

// tg_api.hip -- extern "C" entry points of libtlsgpu.so (declared in
// include/tlsgpu.h).  Host-side connection-state construction (the
// _calcPendingStates equivalent, tlsrecordlayer.py:1061-1149), memory /
// stream / event plumbing, and argument validation in front of the kernels.
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <map>
#include <set>
#include <mutex>
#include <thread>
#include <vector>
#include <stdint.h>
#include "tg_common.h"
#include "tg_hash.h"
#include "tg_keysched.h"
#include "tg_launch.h"
#include <tg_config.h>

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

const char* const KS_MSG[KS_NCODES] = {
    "ok",
    "no TLS suite uses AES-192",
    "version must be (3,0)..(3,3)",
    "unknown MAC",
    "SHA256 suites need TLS 1.2",
    "AES needs a 16/24/32-byte key and a 16-byte IV",
    "3DES needs a 24-byte key and an 8-byte IV",
    "RC4 needs a 16..256-byte key and no IV",
    "unknown cipher",
    "TLS>=1.1 block cipher needs fixed_iv of the block size",
    "MAC key longer than 64 bytes",
    "SSL3 SHA MAC key must be 20 bytes",
    "SSL3 MD5 MAC key must be 16 bytes",
    "SSL3 supports SHA1/MD5 MACs only",
};
int ks_fail(int code) { return code ? fail(TLSGPU_EINVAL, KS_MSG[code]) : 0; }

inline ConnState* S(tlsgpu_conn_state* p) { return reinterpret_cast<ConnState*>(p); }
inline const ConnState* S(const tlsgpu_conn_state* p) { return reinterpret_cast<const ConnState*>(p); }
inline hipStream_t HS(tlsgpu_stream s) { return reinterpret_cast<hipStream_t>(s); }
// A pipeline's calls run on the device it was created on (its streams, events and buffers live
// there) whatever device the calling thread has current; the caller's device is restored after.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
            return;
        }
        if (prev == dev) {
            prev = -1;
        } else if (hipSetDevice(dev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

hipError_t own_release_stream(hipStream_t s);

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
int tlsgpu_device_cu_count(int ordinal, int* n) {
    if (!n) return fail(TLSGPU_EINVAL, "null pointer");
    TG_HIP(hipDeviceGetAttribute(n, hipDeviceAttributeMultiprocessorCount, ordinal));
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
int tlsgpu_stream_create_priority(tlsgpu_stream* s, int high) {
    if (!s) return fail(TLSGPU_EINVAL, "null pointer");
    int least = 0, greatest = 0;
    TG_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t h;
    TG_HIP(hipStreamCreateWithPriority(&h, hipStreamNonBlocking, high ? greatest : least));
    *s = reinterpret_cast<tlsgpu_stream>(h);
    return 0;
}
int tlsgpu_stream_destroy(tlsgpu_stream s) {
    if (!s) return fail(TLSGPU_EINVAL, "the null stream cannot be destroyed");
    TG_HIP(hipStreamSynchronize(HS(s)));
    // the library-owned workspaces of this stream go with it
    hipError_t e = own_release_stream(HS(s));
    if (e != hipSuccess) return fail_hip(e, "tlsgpu_stream_destroy: workspace release");
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
    memset(out, 0, sizeof *out);
    return ks_fail(build_conn_state(S(out), cipher, mac, ver_major, ver_minor, key, key_len, iv, iv_len, mac_key,
                                    mac_key_len, fixed_iv, fixed_iv_len, seqnum, h_aes.sbox, h_aes.im0));
}

int tlsgpu_cipher_state_init(tlsgpu_conn_state* out, int cipher, const uint8_t* key, size_t key_len,
                             const uint8_t* iv, size_t iv_len) {
    if (!out) return fail(TLSGPU_EINVAL, "null state");
    memset(out, 0, sizeof *out);
    ConnState* st = S(out);
    int rc = ks_fail(cipher_setup(st, cipher, key, key_len, iv, iv_len, h_aes.sbox, h_aes.im0));
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
    ks_pack_le(s->iv, iv, iv_len);
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

int tlsgpu_seal_cipher_kernel(uint32_t variant, uint32_t nchains, char* name, size_t cap) {
    if (!name || !cap) return fail(TLSGPU_EINVAL, "null name buffer");
    const std::string k = seal_cipher_kernel(variant, nchains);
    if (k.empty()) return fail(TLSGPU_EINVAL, "unsupported seal variant");
    snprintf(name, cap, "%s", k.c_str());
    return k.size() < cap ? 0 : fail(TLSGPU_EINVAL, "name buffer too small");
}


// library-owned workspace: one grow-only buffer per (kind, device, stream), so calls
// on different streams never share one and calls on one stream are ordered by it.  The
// device is the stream's (hipStreamGetDevice).  tlsgpu_stream_destroy frees the buffers of
// the stream it destroys (a later stream that reuses the handle value starts without
// one); tlsgpu_release_workspaces() frees them all.
}  // extern "C"
namespace {
struct OwnKey {
    int kind, dev;
    hipStream_t s;
    bool operator<(const OwnKey& o) const {
        return kind != o.kind ? kind < o.kind : dev != o.dev ? dev < o.dev : s < o.s;
    }
};
struct OwnBuf {
    void* p = nullptr;
    size_t bytes = 0;
};
std::mutex own_mu;
std::map<OwnKey, OwnBuf> own_bufs;

// frees the buffers `pick` selects and erases their entries whatever fails on the way (an
// entry is never left pointing at freed memory); returns the first error
template <class Pick>
hipError_t own_release(Pick pick, bool sync_device) {
    hipError_t first = hipSuccess;
    std::set<int> synced;
    for (auto it = own_bufs.begin(); it != own_bufs.end();) {
        if (!pick(it->first)) {
            ++it;
            continue;
        }
        const int dev = it->first.dev;
        DeviceGuard guard(dev);
        // the buffer's stream may already be gone: wait for its whole device once
        if (sync_device && !synced.count(dev)) {
            hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess && first == hipSuccess) first = e;
            synced.insert(dev);
        }
        hipError_t e = it->second.p ? hipFree(it->second.p) : hipSuccess;
        if (e != hipSuccess && first == hipSuccess) first = e;
        it = own_bufs.erase(it);
    }
    return first;
}
}  // namespace

namespace {
hipError_t own_release_stream(hipStream_t s) {
    std::lock_guard<std::mutex> g(own_mu);
    return own_release([s](const OwnKey& k) { return k.s == s; }, false);  // s is synchronised
}
}  // namespace
extern "C" {

int tlsgpu_release_workspaces(void) {
    hipError_t e;
    {
        std::lock_guard<std::mutex> g(own_mu);
        e = own_release([](const OwnKey&) { return true; }, true);
    }
    const hipError_t e2 = release_open_aux();  // the split open's second streams and events
    if (e == hipSuccess) e = e2;
    if (e != hipSuccess) return fail_hip(e, "tlsgpu_release_workspaces");
    return 0;
}

size_t tlsgpu_owned_workspace_count(void) {
    std::lock_guard<std::mutex> g(own_mu);
    return own_bufs.size();
}

size_t tlsgpu_owned_stream_count(void) { return open_aux_count(); }

int tlsgpu_set_open_parts(int mode, int64_t min_records) {
    if (set_open_parts(mode, min_records) != 0) return fail(TLSGPU_EINVAL, "open split mode must be 0..3");
    return 0;
}

static int own_workspace(int kind, size_t need, hipStream_t stream, uint8_t** out) {
    const int dev = stream_device(stream);
    std::lock_guard<std::mutex> g(own_mu);
    OwnBuf& b = own_bufs[OwnKey{kind, dev, stream}];
    if (b.bytes < need) {
        DeviceGuard guard(dev);
        if (b.p) {
            TG_HIP(hipStreamSynchronize(stream));  // earlier calls on this stream may still read it
            void* old = b.p;
            b.p = nullptr;
            b.bytes = 0;
            TG_HIP(hipFree(old));
        }
        TG_HIP(hipMalloc(&b.p, need));
        b.bytes = need;
    }
    *out = static_cast<uint8_t*>(b.p);
    return 0;
}

static uint32_t next_epoch() {
    static uint32_t epoch_ctr = 0;
    return __atomic_add_fetch(&epoch_ctr, 1, __ATOMIC_RELAXED);
}

int tlsgpu_seal_dev(const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* records, uint32_t nrecords,
                    const uint8_t* pt, size_t pt_bytes, uint8_t* wire, size_t wire_bytes, tlsgpu_conn_state* states,
                    uint32_t nstates, int32_t* wire_len, uint32_t variant, void* workspace, size_t workspace_bytes,
                    tlsgpu_stream s) {
    if (nchains == 0) return 0;
    if (!chains || !records || !pt || !wire || !states || !wire_len) return fail(TLSGPU_EINVAL, "null pointer");
    uint8_t* ws = static_cast<uint8_t*>(workspace);
    if (seal_needs_workspace(variant)) {
        const size_t need = seal_workspace_bytes(nrecords);
        if (ws && workspace_bytes < need) return fail(TLSGPU_EINVAL, "workspace too small");
        if (!ws) {
            int rc = own_workspace(0, need, HS(s), &ws);
            if (rc) return rc;
        }
    }
    Bounds b;
    b.pt_cap = pt_bytes;
    b.wire_cap = wire_bytes;
    b.nstates = nstates;
    bool known = false;
    hipError_t e = launch_seal(variant, chains, nchains, records, nrecords, pt, wire, S(states), wire_len, ws,
                               next_epoch(), HS(s), &known, b);
    if (!known) return fail(TLSGPU_EINVAL, "unsupported seal variant");
    if (e != hipSuccess) return fail_hip(e, "seal launch");
    return 0;
}

// ---------------------------------------------------------------- pipeline
// Workspaces in rotation: the MAC phase of call k reuses the workspace of call k - PIPE_WS,
// so the MAC stream may run up to PIPE_WS - 1 calls ahead of the cipher stream.
constexpr int PIPE_WS = CFG_PIPE_WS;
struct tlsgpu_pipeline_s {
    int dev;
    hipStream_t mac_s, cbc_s;
    hipEvent_t mac_done[PIPE_WS], cbc_done[PIPE_WS];
    void* ws[PIPE_WS];
    size_t ws_bytes;
    uint64_t k;
};

int tlsgpu_pipeline_create(tlsgpu_pipeline* out, uint32_t max_records) {
    if (!out) return fail(TLSGPU_EINVAL, "null");
    tlsgpu_pipeline p = new tlsgpu_pipeline_s();
    TG_HIP(hipGetDevice(&p->dev));
    TG_HIP(hipStreamCreateWithFlags(&p->mac_s, hipStreamNonBlocking));
    // The cipher stream at high priority (round 4).  The runtime spreads a process's streams
    // over a few hardware queues (GPU_MAX_HW_QUEUES, 4 here), kept per priority level, and
    // the kernels of one queue run in submission order: when the MAC and cipher streams
    // landed on one queue the phases ran one after the other instead of side by side (one
    // idle stream created before the pipeline was enough: cfg2 805 instead of 982 GiB/s).
    // At different priorities they can never share a queue: 981 GiB/s with that extra
    // stream, 979-980 without (profiles/r04/ab/ab_stream_priority.txt).
    {
        int lo_prio = 0, hi_prio = 0;
        TG_HIP(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
        TG_HIP(hipStreamCreateWithPriority(&p->cbc_s, hipStreamNonBlocking, hi_prio));
    }
    for (int i = 0; i < PIPE_WS; i++) {
        TG_HIP(hipEventCreateWithFlags(&p->mac_done[i], hipEventDisableTiming));
        TG_HIP(hipEventCreateWithFlags(&p->cbc_done[i], hipEventDisableTiming));
    }
    p->ws_bytes = seal_workspace_bytes(max_records ? max_records : 1);
    for (int i = 0; i < PIPE_WS; i++) TG_HIP(hipMalloc(&p->ws[i], p->ws_bytes));
    p->k = 0;
    *out = p;
    return 0;
}

int tlsgpu_pipeline_destroy(tlsgpu_pipeline p) {
    if (!p) return 0;
    DeviceScope scope_(p->dev);
    (void)hipStreamSynchronize(p->mac_s);
    (void)hipStreamSynchronize(p->cbc_s);
    for (int i = 0; i < PIPE_WS; i++) {
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
                         const tlsgpu_record* records, uint32_t nrecords, const uint8_t* pt, size_t pt_bytes,
                         uint8_t* wire, size_t wire_bytes, tlsgpu_conn_state* states, uint32_t nstates,
                         int32_t* wire_len, uint32_t variant, tlsgpu_event cipher_start, tlsgpu_event cipher_stop) {
    if (!p) return fail(TLSGPU_EINVAL, "null pipeline");
    DeviceScope scope_(p->dev);
    if (nchains == 0) return 0;
    if (!chains || !records || !pt || !wire || !states || !wire_len) return fail(TLSGPU_EINVAL, "null pointer");
    if (seal_workspace_bytes(nrecords) > p->ws_bytes) return fail(TLSGPU_EINVAL, "nrecords > pipeline max_records");
    static uint32_t epoch_ctr = 0x80000000u;
    const uint32_t epoch = __atomic_add_fetch(&epoch_ctr, 1, __ATOMIC_RELAXED);
    const int i = (int)(p->k % PIPE_WS);
    Bounds b;
    b.pt_cap = pt_bytes;
    b.wire_cap = wire_bytes;
    b.nstates = nstates;
    // workspace i was last read by the cipher phase of call k - PIPE_WS
    if (p->k >= (uint64_t)PIPE_WS) TG_HIP(hipStreamWaitEvent(p->mac_s, p->cbc_done[i], 0));
    bool known = false;
    hipError_t e = hipSuccess;
    if (seal_needs_workspace(variant)) {
        e = launch_seal_phases(variant, chains, nchains, records, nrecords, pt, wire, S(states), wire_len,
                               static_cast<uint8_t*>(p->ws[i]), epoch, p->mac_s, p->mac_done[i], p->cbc_s,
                               reinterpret_cast<hipEvent_t>(cipher_start), reinterpret_cast<hipEvent_t>(cipher_stop),
                               &known, b);
    } else {
        // single-kernel variants run on the cipher stream, in order with earlier calls
        if (cipher_start) TG_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(cipher_start), p->cbc_s));
        e = launch_seal(variant, chains, nchains, records, nrecords, pt, wire, S(states), wire_len, nullptr, epoch,
                        p->cbc_s, &known, b);
        if (e == hipSuccess && cipher_stop) e = hipEventRecord(reinterpret_cast<hipEvent_t>(cipher_stop), p->cbc_s);
    }
    if (!known) return fail(TLSGPU_EINVAL, "unsupported seal variant");
    if (e != hipSuccess) return fail_hip(e, "pipeline seal");
    TG_HIP(hipEventRecord(p->cbc_done[i], p->cbc_s));
    p->k++;
    return 0;
}

// ---------------------------------------------------------------- host-buffer pipeline
namespace {
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (bytes >= need && p) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
        }
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, need ? need : 1);
        if (e == hipSuccess) bytes = need;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};
struct PinBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (bytes >= need && p) return hipSuccess;
        if (p) {
            hipError_t e = hipHostFree(p);
            if (e != hipSuccess) return e;
        }
        p = nullptr;
        bytes = 0;
        hipError_t e = hipHostMalloc(&p, need ? need : 1, hipHostMallocDefault);
        if (e == hipSuccess) bytes = need;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};
// host memory the DMA engines can read directly (hipHostMalloc / hipHostRegister)
bool host_pinned(const void* ptr) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}
// Pinned host memory the GPU can store into at its own address (ROCm maps pinned host memory at
// the same virtual address on the device): that address, or nullptr (the copy engine only)
uint8_t* host_store_ptr(void* h) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, h) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.hostPointer || !a.devicePointer) return nullptr;
    // h's device address, whether the runtime reports the allocation's base or h itself
    uint8_t* d = static_cast<uint8_t*>(a.devicePointer) + (static_cast<uint8_t*>(h) - static_cast<uint8_t*>(a.hostPointer));
    return d == h ? d : nullptr;
}
// Staging copies between pageable host memory and the pinned buffers: one thread moves
// ~10 GB/s, below the link's 57 GB/s per direction, so large copies are split over a few
// threads (at most 8: the job's share of host cores on the GPU box is 16).
void stage_copy(void* dst, const void* src, size_t n) {
    const size_t piece = (size_t)4 << 20;
    unsigned hc = std::thread::hardware_concurrency();
    unsigned T = (unsigned)((n + piece - 1) / piece);
    T = T > 8 ? 8 : T;
    T = hc && T > hc ? hc : T;
    if (T <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t per = (n / T + 63) & ~(size_t)63;
    std::vector<std::thread> th;
    for (unsigned i = 1; i < T; i++) {
        const size_t a = i * per, e = a + per < n ? a + per : n;
        if (a < e) th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, e - a); });
    }
    memcpy(dst, src, per < n ? per : n);
    for (auto& t : th) t.join();
}
struct SubBatch {
    uint32_t c0, c1;  // chains [c0, c1)
    uint32_t r0, r1;  // records its chains use: [r0, r1)
    size_t p0, p1;    // plaintext bytes copied H2D
    size_t w0, w1;    // wire bytes copied D2H
};
}  // namespace

// Four streams, chained per sub-batch by events: h2d (plaintext copies) and d2h (wire
// copies), one per copy direction so both directions run at once (pinned: 57 GB/s each
// way, 97 GB/s both at once on the MI355X box, tools/pcie_probe.hip), and the seal's
// two phases on mac (prefix + MAC kernels) and cbc (cipher kernel), so the MAC phase of
// sub-batch i+1 runs beside the cipher phase of sub-batch i as in tlsgpu_pipeline_seal.
// A sub-batch of a few thousand single-record chains is a latency-bound seal (~0.4 ms
// MAC + ~0.5 ms CBC for 16 KiB records whatever the chain count up to ~64 per CU), so
// the phases must overlap for the seals to keep up with the copies.  Separate streams
// per kernel kind, not per slot: the runtime spreads streams over only a few hardware
// queues, and kernels of streams that share a queue run in submission order.
// `depth` sub-batches are in flight: slot i % depth's staging buffers and workspace are
// reused once sub-batch i - depth is done.
struct tlsgpu_host_pipeline_s {
    int dev = 0;
    int depth = 2;
    size_t chunk = 0;
    hipStream_t h2d = nullptr, mac = nullptr, cbc = nullptr, d2h = nullptr;
    hipStream_t frs = nullptr;  // receive framing: its own (high-priority) queue, never behind an open
    std::vector<hipEvent_t> mac_done;
    std::vector<hipEvent_t> in_done, seal_done, out_done;
    DevBuf pt, wire, recs, chains, len;
    std::vector<DevBuf> ws;
    std::vector<PinBuf> pt_stage, wire_stage;
    // receive direction (tlsgpu_host_pipeline_open): the received bytes and the opened
    // plaintext (device arenas mirroring the host ones), the connections' spans and framing
    // results, and per slot the framed descriptors, statuses and workspaces of one sub-batch
    DevBuf rx, opt, conns, rchains, consumed, fstatus, totals;
    std::vector<DevBuf> rrecs, rstat, rws, fws;
    std::vector<PinBuf> rx_stage, opt_stage, recs_stage, stat_stage;
    PinBuf h_totals;
    std::vector<hipEvent_t> framed, opened;
    std::vector<hipEvent_t> rx_in;  // per sub-batch of a receive call: its H2D copy is done
    int d2h_path = -1;              // D2H by: -1 not chosen yet, 0 the copy engine, 1 the GPU's stores
};

// The host pipelines' big D2H copies (wire / plaintext ranges) go by the copy engine or by the
// GPU's own stores (host_store_kernel).  On most boxes the engine is the faster one beside the
// H2D copies (56 + 48 GB/s against 43 + 50), but in about one process in four its D2H runs at
// 30 GB/s where the stores still reach 55 (profiles/r06/hostpipe/NOTES.md).  So each pipeline
// times them once, on its first call (32 MiB each, best of 3, ~4 ms), and takes the stores only
// when the engine's D2H runs at < 0.7x its own H2D rate and the stores are >= 1.5x faster.  TLSGPU_HOST_D2H=engine|kernel forces a path (tests).
static int choose_d2h_path(tlsgpu_host_pipeline p) {
    if (p->d2h_path >= 0) return 0;
    const char* env = getenv("TLSGPU_HOST_D2H");
    if (env && !strcmp(env, "engine")) {
        p->d2h_path = 0;
        return 0;
    }
    if (env && !strcmp(env, "kernel")) {
        p->d2h_path = 1;
        return 0;
    }
    const size_t n = (size_t)32 << 20;
    DevBuf src;
    PinBuf dst;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float best[3] = {1e30f, 1e30f, 1e30f};  // engine D2H, stores D2H, engine H2D (ms for n bytes)
    hipError_t e = src.ensure(n);
    if (e == hipSuccess) e = dst.ensure(n);
    uint8_t* dd = e == hipSuccess ? host_store_ptr(dst.p) : nullptr;
    if (dd) {  // else the copy engine (no device address for the stores)
        e = hipEventCreate(&e0);
        if (e == hipSuccess) e = hipEventCreate(&e1);
        if (e == hipSuccess) e = hipMemsetAsync(src.p, 0, n, p->d2h);
        for (int rep = 0; rep < 4 && e == hipSuccess; rep++)
            for (int k = 0; k < 3 && e == hipSuccess; k++) {
                e = hipEventRecord(e0, p->d2h);
                if (e == hipSuccess)
                    e = k == 1   ? launch_host_store(src.u8(), dd, n, p->d2h)
                        : k == 0 ? hipMemcpyAsync(dst.p, src.p, n, hipMemcpyDeviceToHost, p->d2h)
                                 : hipMemcpyAsync(src.p, dst.p, n, hipMemcpyHostToDevice, p->d2h);
                if (e == hipSuccess) e = hipEventRecord(e1, p->d2h);
                if (e == hipSuccess) e = hipEventSynchronize(e1);
                float ms = 0;
                if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
                if (e == hipSuccess && rep) best[k] = ms < best[k] ? ms : best[k];
            }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e == hipSuccess) e = hipStreamSynchronize(p->d2h);  // before the buffers go
    src.release();
    dst.release();
    if (e != hipSuccess) return fail_hip(e, "host pipeline D2H calibration");
    // The anomaly the stores path is for: the engine's D2H at about half its H2D rate (30 vs 57
    // GB/s) while the stores reach 55.  Both conditions, so that copies of other processes on a
    // shared link -- which slow the engine's two directions alike -- do not pick the stores (8
    // ranks on one GPU: engine 40.8 vs stores 33.5 GiB/s, profiles/r06/hostpipe/NOTES.md).
    p->d2h_path = (best[0] > 1.4f * best[2] && best[1] * 1.5f < best[0]) ? 1 : 0;
    return 0;
}

// one big D2H range of a host pipeline: dst is pinned host memory (the caller's or a stage) at
// the same address mod 16 as src; by the GPU's stores where chosen and possible
static hipError_t pipeline_d2h(tlsgpu_host_pipeline p, uint8_t* dst, uint8_t* dst_dev, const uint8_t* src, size_t n) {
    if (p->d2h_path == 1 && dst_dev && !(((uintptr_t)src ^ (uintptr_t)dst_dev) & 15))
        return launch_host_store(src, dst_dev, n, p->d2h);
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, p->d2h);
}

int tlsgpu_host_pipeline_d2h_path(tlsgpu_host_pipeline p, int* path) {
    if (!p || !path) return fail(TLSGPU_EINVAL, "null");
    *path = p->d2h_path;
    return 0;
}

int tlsgpu_host_store(void* dst_host, const void* src_dev, size_t bytes, tlsgpu_stream s) {
    if (!bytes) return 0;
    if (!dst_host || !src_dev) return fail(TLSGPU_EINVAL, "null pointer");
    uint8_t* dd = host_store_ptr(dst_host);
    if (!dd) return fail(TLSGPU_EINVAL, "destination is not pinned host memory the device can store into");
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, src_dev) != hipSuccess || a.type != hipMemoryTypeDevice) {
        (void)hipGetLastError();
        return fail(TLSGPU_EINVAL, "source is not device memory");
    }
    if (((uintptr_t)dd ^ (uintptr_t)src_dev) & 15) return fail(TLSGPU_EINVAL, "source and destination differ mod 16");
    hipError_t e = launch_host_store(static_cast<const uint8_t*>(src_dev), dd, bytes, HS(s));
    if (e != hipSuccess) return fail_hip(e, "host store launch");
    return 0;
}

int tlsgpu_host_pipeline_create(tlsgpu_host_pipeline* out, size_t chunk_bytes, int depth) {
    if (!out) return fail(TLSGPU_EINVAL, "null");
    if (depth < 1 || depth > 16) return fail(TLSGPU_EINVAL, "depth must be 1..16");
    tlsgpu_host_pipeline p = new tlsgpu_host_pipeline_s();
    TG_HIP(hipGetDevice(&p->dev));
    p->depth = depth;
    p->chunk = chunk_bytes ? chunk_bytes : ((size_t)64 << 20);
    p->in_done.resize(depth);
    p->seal_done.resize(depth);
    p->out_done.resize(depth);
    p->ws.resize(depth);
    p->pt_stage.resize(depth);
    p->wire_stage.resize(depth);
    p->mac_done.resize(depth);
    p->rrecs.resize(depth);
    p->rstat.resize(depth);
    p->rws.resize(depth);
    p->fws.resize(depth);
    p->rx_stage.resize(depth);
    p->opt_stage.resize(depth);
    p->recs_stage.resize(depth);
    p->stat_stage.resize(depth);
    p->framed.resize(depth);
    p->opened.resize(depth);
    // The runtime spreads streams over a few hardware queues per priority, and a copy holds
    // its queue until it completes (kernels queued behind it wait; with the MAC stream
    // behind the H2D copies on one queue the call took 31.9 instead of 24.6 ms): the copy
    // streams are created at high priority, away from the kernel streams' queues.
    int lo_prio = 0, hi_prio = 0;
    TG_HIP(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
    TG_HIP(hipStreamCreateWithPriority(&p->h2d, hipStreamNonBlocking, hi_prio));
    TG_HIP(hipStreamCreateWithPriority(&p->d2h, hipStreamNonBlocking, hi_prio));
    TG_HIP(hipStreamCreateWithPriority(&p->frs, hipStreamNonBlocking, hi_prio));
    TG_HIP(hipStreamCreateWithFlags(&p->mac, hipStreamNonBlocking));
    TG_HIP(hipStreamCreateWithFlags(&p->cbc, hipStreamNonBlocking));
    for (int i = 0; i < depth; i++) {
        TG_HIP(hipEventCreateWithFlags(&p->mac_done[i], hipEventDisableTiming));
        TG_HIP(hipEventCreateWithFlags(&p->in_done[i], hipEventDisableTiming));
        TG_HIP(hipEventCreateWithFlags(&p->seal_done[i], hipEventDisableTiming));
        TG_HIP(hipEventCreateWithFlags(&p->out_done[i], hipEventDisableTiming));
        TG_HIP(hipEventCreateWithFlags(&p->framed[i], hipEventDisableTiming));
        TG_HIP(hipEventCreateWithFlags(&p->opened[i], hipEventDisableTiming));
    }
    *out = p;
    return 0;
}

int tlsgpu_host_pipeline_destroy(tlsgpu_host_pipeline p) {
    if (!p) return 0;
    DeviceScope scope_(p->dev);
    for (hipStream_t s : {p->h2d, p->mac, p->cbc, p->d2h, p->frs}) (void)hipStreamSynchronize(s);
    p->pt.release();
    p->wire.release();
    p->recs.release();
    p->chains.release();
    p->len.release();
    for (DevBuf* b : {&p->rx, &p->opt, &p->conns, &p->rchains, &p->consumed, &p->fstatus, &p->totals}) b->release();
    p->h_totals.release();
    for (int i = 0; i < p->depth; i++) {
        p->ws[i].release();
        p->pt_stage[i].release();
        p->wire_stage[i].release();
        p->rrecs[i].release();
        p->rstat[i].release();
        p->rws[i].release();
        p->fws[i].release();
        p->rx_stage[i].release();
        p->opt_stage[i].release();
        p->recs_stage[i].release();
        p->stat_stage[i].release();
        (void)hipEventDestroy(p->in_done[i]);
        (void)hipEventDestroy(p->seal_done[i]);
        (void)hipEventDestroy(p->out_done[i]);
        (void)hipEventDestroy(p->mac_done[i]);
        (void)hipEventDestroy(p->framed[i]);
        (void)hipEventDestroy(p->opened[i]);
    }
    for (hipEvent_t e : p->rx_in) (void)hipEventDestroy(e);
    for (hipStream_t s : {p->h2d, p->mac, p->cbc, p->d2h, p->frs}) (void)hipStreamDestroy(s);
    delete p;
    return 0;
}

// Largest record a seal of this variant can write for pt_len plaintext bytes: the 5-byte
// header and the body [explicit IV] | P | MAC | padding (tlsrecordlayer.py:594-606), taking
// the explicit IV (TLS >= 1.1, a state field the host does not see) when it makes the body
// longer.  0 for an unknown variant.
static uint64_t sealed_max_bytes(uint32_t variant, uint64_t n) {
    const uint32_t c = variant & 0xff, m = (variant >> 8) & 0xff;
    const uint64_t dl = m == TLSGPU_MAC_SHA1 ? 20 : m == TLSGPU_MAC_SHA256 ? 32 : m == TLSGPU_MAC_MD5 ? 16 : 0;
    if (!dl) return 0;
    if (c == TLSGPU_CIPHER_RC4) return 5 + n + dl;
    const uint64_t bs = c == TLSGPU_CIPHER_3DES ? 8 : (c == TLSGPU_CIPHER_AES128 || c == TLSGPU_CIPHER_AES256) ? 16 : 0;
    if (!bs) return 0;
    uint64_t body = 0;
    for (uint64_t e : {(uint64_t)0, bs}) {
        const uint64_t cur = e + n + dl, b = cur + (bs - (cur & (bs - 1)));
        body = b > body ? b : body;
    }
    return 5 + body;
}

int tlsgpu_host_pipeline_seal(tlsgpu_host_pipeline p, const tlsgpu_chain* chains, uint32_t nchains,
                              const tlsgpu_record* records, uint32_t nrecords, const uint8_t* pt_host,
                              size_t pt_bytes, uint8_t* wire_host, size_t wire_bytes, tlsgpu_conn_state* states,
                              uint32_t nstates, int32_t* wire_len_host, uint32_t variant) {
    if (!p) return fail(TLSGPU_EINVAL, "null pipeline");
    DeviceScope scope_(p->dev);
    if (nchains == 0) return 0;
    if (!chains || !records || !pt_host || !wire_host || !states || !wire_len_host)
        return fail(TLSGPU_EINVAL, "null pointer");
    if (!sealed_max_bytes(variant, 0)) return fail(TLSGPU_EINVAL, "unsupported seal variant");
    const bool need_ws = seal_needs_workspace(variant);
    // sub-batches of consecutive chains, about p->chunk plaintext bytes each
    std::vector<SubBatch> sub;
    std::vector<size_t> pmin, wmin, pend, wend;  // per sub-batch extremes over its records
    {
        SubBatch cur = {0, 0, UINT32_MAX, 0, 0, 0, 0, 0};
        size_t acc = 0, lo_p = SIZE_MAX, lo_w = SIZE_MAX, hi_p = 0, hi_w = 0;
        for (uint32_t c = 0; c < nchains; c++) {
            const tlsgpu_chain& ch = chains[c];
            if ((uint64_t)ch.first + ch.count > nrecords) return fail(TLSGPU_EINVAL, "chain outside the records");
            if (ch.state >= nstates) return fail(TLSGPU_EINVAL, "chain state outside the states array");
            if (ch.count) {
                cur.r0 = ch.first < cur.r0 ? ch.first : cur.r0;
                cur.r1 = ch.first + ch.count > cur.r1 ? ch.first + ch.count : cur.r1;
            }
            for (uint32_t k = 0; k < ch.count; k++) {
                const tlsgpu_record& R = records[ch.first + k];
                // A record's wire slot must hold its sealed form, not just 5 + P: the kernels
                // write the tail, MAC and padding past it.  RC4's size is known here; a CBC
                // record's depends on the state's explicit-IV flag (device-resident), so the
                // prefix kernel checks its exact end against wire_bytes (SealBounds) and this
                // check only needs the header and the plaintext length in range.
                const uint64_t wext = (uint64_t)R.wire_off + (need_ws ? 5 + (uint64_t)R.pt_len
                                                                      : sealed_max_bytes(variant, R.pt_len));
                if ((uint64_t)R.pt_off + R.pt_len > pt_bytes || wext > wire_bytes)
                    return fail(TLSGPU_EINVAL, "record outside the host arenas");
                lo_p = R.pt_off < lo_p ? R.pt_off : lo_p;
                lo_w = R.wire_off < lo_w ? R.wire_off : lo_w;
                hi_p = R.pt_off + R.pt_len > hi_p ? R.pt_off + R.pt_len : hi_p;
                hi_w = wext > hi_w ? wext : hi_w;
                acc += R.pt_len;
            }
            cur.c1 = c + 1;
            if (acc >= p->chunk || c + 1 == nchains) {
                sub.push_back(cur);
                pmin.push_back(lo_p == SIZE_MAX ? 0 : lo_p);
                wmin.push_back(lo_w == SIZE_MAX ? 0 : lo_w);
                pend.push_back(hi_p);
                wend.push_back(hi_w);
                cur.c0 = c + 1;
                cur.r0 = UINT32_MAX;
                cur.r1 = 0;
                acc = 0;
                lo_p = lo_w = SIZE_MAX;
                hi_p = hi_w = 0;
            }
        }
        // copy ranges: from this sub-batch's first offset to the next one's; a layout that is
        // not monotone in chain order (ranges would overlap) is sealed as one sub-batch
        bool mono = true;
        for (size_t i = 0; i + 1 < sub.size(); i++)
            if (pend[i] > pmin[i + 1] || wend[i] > wmin[i + 1] || pmin[i + 1] < pmin[i] || wmin[i + 1] < wmin[i])
                mono = false;
        if (!mono) {
            sub.assign(1, SubBatch{0, nchains, 0, nrecords, 0, 0, 0, 0});
            pmin.assign(1, 0);
            wmin.assign(1, 0);
        }
        for (size_t i = 0; i < sub.size(); i++) {
            sub[i].p0 = mono ? pmin[i] : 0;
            sub[i].w0 = mono ? wmin[i] : 0;
            sub[i].p1 = (mono && i + 1 < sub.size()) ? pmin[i + 1] : pt_bytes;
            sub[i].w1 = (mono && i + 1 < sub.size()) ? wmin[i + 1] : wire_bytes;
        }
    }
    const int D = p->depth;
    const bool pt_direct = host_pinned(pt_host), wire_direct = host_pinned(wire_host);
    {
        int rc = choose_d2h_path(p);
        if (rc) return rc;
    }
    uint8_t* wire_dev = wire_direct ? host_store_ptr(wire_host) : nullptr;
    size_t max_p = 0, max_w = 0;
    for (const SubBatch& b : sub) {
        max_p = b.p1 - b.p0 > max_p ? b.p1 - b.p0 : max_p;
        max_w = b.w1 - b.w0 > max_w ? b.w1 - b.w0 : max_w;
    }
    TG_HIP(p->pt.ensure(pt_bytes));
    TG_HIP(p->wire.ensure(wire_bytes));
    // the D2H ranges include the gaps between records: they come back as zeros, never as
    // bytes an earlier batch left in the device arena (h2d stream: before every seal kernel)
    TG_HIP(hipMemsetAsync(p->wire.p, 0, wire_bytes, p->h2d));
    TG_HIP(p->recs.ensure((size_t)nrecords * sizeof(tlsgpu_record)));
    TG_HIP(p->chains.ensure((size_t)nchains * sizeof(tlsgpu_chain)));
    TG_HIP(p->len.ensure((size_t)nrecords * 4));
    for (int i = 0; i < D; i++) {
        if (need_ws) TG_HIP(p->ws[i].ensure(seal_workspace_bytes(nrecords)));
        if (!pt_direct) TG_HIP(p->pt_stage[i].ensure(max_p));
        if (!wire_direct) TG_HIP(p->wire_stage[i].ensure(max_w + 16));  // + the range's offset mod 16
    }
    // descriptors once (small), on the h2d stream ahead of the first sub-batch's plaintext
    TG_HIP(hipMemcpyAsync(p->recs.p, records, (size_t)nrecords * sizeof(tlsgpu_record), hipMemcpyHostToDevice, p->h2d));
    TG_HIP(hipMemcpyAsync(p->chains.p, chains, (size_t)nchains * sizeof(tlsgpu_chain), hipMemcpyHostToDevice, p->h2d));
    const tlsgpu_chain* d_chains = static_cast<const tlsgpu_chain*>(p->chains.p);
    const tlsgpu_record* d_recs = static_cast<const tlsgpu_record*>(p->recs.p);
    // finish sub-batch j (CPU): wait for its D2H copy, then unstage it
    auto drain = [&](size_t j) -> int {
        const int t = (int)(j % D);
        TG_HIP(hipEventSynchronize(p->out_done[t]));
        if (!wire_direct)
            stage_copy(wire_host + sub[j].w0, p->wire_stage[t].u8() + (sub[j].w0 & 15), sub[j].w1 - sub[j].w0);
        return 0;
    };
    // Pinned arenas: everything is enqueued at once and ordered on the GPU (slot t's seal
    // stream keeps its workspace in order), the calling thread only waits at the end.
    // Staged arenas: before refilling slot t's plaintext stage the thread waits for the
    // H2D copy of sub-batch i - D, and before enqueueing the D2H copy into slot t's wire
    // stage it unstages sub-batch i - D.
    for (size_t i = 0; i < sub.size(); i++) {
        const SubBatch& b = sub[i];
        const int t = (int)(i % D);
        const uint8_t* src = pt_host + b.p0;
        if (!pt_direct) {
            if (i >= (size_t)D) TG_HIP(hipEventSynchronize(p->in_done[t]));
            stage_copy(p->pt_stage[t].u8(), src, b.p1 - b.p0);
            src = p->pt_stage[t].u8();
        }
        // (CFG_HOST_H2D_LEAD) sub-batch i - L's seal_done is slot (i - L) % D's latest record for L <= D
        const size_t lead = CFG_HOST_H2D_LEAD < 1 ? 0 : CFG_HOST_H2D_LEAD > D ? (size_t)D : (size_t)CFG_HOST_H2D_LEAD;
        if (pt_direct && lead && i >= lead) TG_HIP(hipStreamWaitEvent(p->h2d, p->seal_done[(i - lead) % D], 0));
        if (b.p1 > b.p0) TG_HIP(hipMemcpyAsync(p->pt.u8() + b.p0, src, b.p1 - b.p0, hipMemcpyHostToDevice, p->h2d));
        TG_HIP(hipEventRecord(p->in_done[t], p->h2d));
        TG_HIP(hipStreamWaitEvent(p->mac, p->in_done[t], 0));
        // slot t's workspace: the cipher phase of sub-batch i - D has read it
        if (i >= (size_t)D) TG_HIP(hipStreamWaitEvent(p->mac, p->seal_done[t], 0));
        bool known = false;
        hipError_t e;
        if (need_ws) {
            Bounds sb;
            sb.rec_lo = b.r0 < b.r1 ? b.r0 : 0;
            sb.rec_hi = b.r0 < b.r1 ? b.r1 : 0;
            sb.pt_cap = pt_bytes;
            sb.wire_cap = wire_bytes;
            sb.nstates = nstates;
            e = launch_seal_phases(variant, d_chains + b.c0, b.c1 - b.c0, d_recs, nrecords, p->pt.u8(), p->wire.u8(),
                                   S(states), static_cast<int32_t*>(p->len.p), p->ws[t].u8(), next_epoch(), p->mac,
                                   p->mac_done[t], p->cbc, nullptr, nullptr, &known, sb);
        } else {  // single-kernel variants (RC4) on the cipher stream
            TG_HIP(hipStreamWaitEvent(p->cbc, p->in_done[t], 0));
            Bounds rb;
            rb.pt_cap = pt_bytes;
            rb.wire_cap = wire_bytes;
            rb.nstates = nstates;
            e = launch_seal(variant, d_chains + b.c0, b.c1 - b.c0, d_recs, nrecords, p->pt.u8(), p->wire.u8(),
                            S(states), static_cast<int32_t*>(p->len.p), nullptr, next_epoch(), p->cbc, &known, rb);
        }
        if (!known) return fail(TLSGPU_EINVAL, "unsupported seal variant");
        if (e != hipSuccess) return fail_hip(e, "host pipeline seal");
        TG_HIP(hipEventRecord(p->seal_done[t], p->cbc));
        if (!wire_direct && i >= (size_t)D) {
            int rc = drain(i - D);
            if (rc) return rc;
        }
        TG_HIP(hipStreamWaitEvent(p->d2h, p->seal_done[t], 0));
        // the stage holds the range at the same offset mod 16 as the device arena (stores path)
        uint8_t* dst = wire_direct ? wire_host + b.w0 : p->wire_stage[t].u8() + (b.w0 & 15);
        uint8_t* dst_dev = wire_direct ? (wire_dev ? wire_dev + b.w0 : nullptr) : host_store_ptr(p->wire_stage[t].p);
        if (dst_dev && !wire_direct) dst_dev += b.w0 & 15;
        if (b.w1 > b.w0) TG_HIP(pipeline_d2h(p, dst, dst_dev, p->wire.u8() + b.w0, b.w1 - b.w0));
        TG_HIP(hipEventRecord(p->out_done[t], p->d2h));
    }
    if (wire_direct) {
        TG_HIP(hipStreamSynchronize(p->d2h));
    } else {
        for (size_t j = sub.size() > (size_t)D ? sub.size() - D : 0; j < sub.size(); j++) {
            int rc = drain(j);
            if (rc) return rc;
        }
    }
    // wire_len: ordered after every seal (each seal_done precedes its D2H copy, all drained)
    TG_HIP(hipMemcpy(wire_len_host, p->len.p, (size_t)nrecords * 4, hipMemcpyDeviceToHost));
    return 0;
}

// Receive path from host socket buffers (ABI 7): sub-batches of consecutive connections, about
// p->chunk received bytes each, flow H2D copy (h2d stream) -> device framing -> open (one of
// the two kernel streams, alternating per sub-batch) -> D2H of the opened plaintext, the framed
// descriptors and the statuses (d2h stream), `depth` sub-batches in flight.  The open needs the
// sub-batch's record count on the host (grids, workspace), so the host reads each framing's
// total (4 bytes into pinned memory) before it enqueues that sub-batch's open: the wait falls
// under the next sub-batch's H2D copy, which is enqueued first, so the copy engines -- the
// bound of this path -- never wait for it.  A sub-batch's framing may use at most its share of
// max_records (what the sub-batches before it left), so records are cut exactly where one
// tlsgpu_frame_dev call over every connection would cut them.
namespace {
struct RxSub {
    uint32_t c0, c1;   // connections [c0, c1)
    size_t b0, b1;     // received bytes copied H2D, plaintext copied D2H: [b0, b1)
    uint64_t bound;    // records its framing can produce at most (sum of span lengths / 5)
};
}  // namespace

int tlsgpu_host_pipeline_open(tlsgpu_host_pipeline p, const uint8_t* rx_host, size_t rx_bytes,
                              const tlsgpu_span* conns, uint32_t n, uint32_t chain_flags, uint8_t* pt_host,
                              size_t pt_bytes, tlsgpu_conn_state* states, uint32_t nstates, uint32_t variant,
                              tlsgpu_open_record* records_host, uint32_t max_records, tlsgpu_chain* chains_host,
                              uint32_t* consumed_host, int32_t* frame_status_host, int32_t* status_host,
                              uint32_t* total_host) {
    if (!p) return fail(TLSGPU_EINVAL, "null pipeline");
    DeviceScope scope_(p->dev);
    if (!total_host) return fail(TLSGPU_EINVAL, "null pointer");
    *total_host = 0;
    if (n == 0) return 0;
    if (!rx_host || !conns || !pt_host || !states || !chains_host || !consumed_host || !frame_status_host ||
        (max_records && (!records_host || !status_host)))
        return fail(TLSGPU_EINVAL, "null pointer");
    if (n > (1u << 26)) return fail(TLSGPU_EINVAL, "too many connections");
    if (pt_bytes < rx_bytes) return fail(TLSGPU_EINVAL, "plaintext arena smaller than the received bytes");
    {
        const uint32_t c = variant & 0xff, m = (variant >> 8) & 0xff;
        const bool cbc = c == TLSGPU_CIPHER_AES128 || c == TLSGPU_CIPHER_AES256 || c == TLSGPU_CIPHER_3DES;
        const bool ok = (cbc && m == TLSGPU_MAC_SHA1) || (cbc && c != TLSGPU_CIPHER_3DES && m == TLSGPU_MAC_SHA256) ||
                        (c == TLSGPU_CIPHER_RC4 && (m == TLSGPU_MAC_SHA1 || m == TLSGPU_MAC_MD5));
        if (!ok || (variant >> 17)) return fail(TLSGPU_EINVAL, "unsupported open variant");
    }
    // sub-batches of consecutive connections; spans outside the arena are refused by the
    // framing (status EINVAL) and take no part in the copy ranges
    std::vector<RxSub> sub;
    {
        RxSub cur = {0, 0, SIZE_MAX, 0, 0};
        size_t acc = 0;
        for (uint32_t c = 0; c < n; c++) {
            const tlsgpu_span& sp = conns[c];
            if (in_arena(sp.off, sp.len, rx_bytes) && sp.len) {
                cur.b0 = sp.off < cur.b0 ? sp.off : cur.b0;
                cur.b1 = sp.off + sp.len > cur.b1 ? sp.off + sp.len : cur.b1;
                cur.bound += sp.len / 5;
                acc += sp.len;
            }
            cur.c1 = c + 1;
            if (acc >= p->chunk || c + 1 == n) {
                if (cur.b0 == SIZE_MAX) cur.b0 = cur.b1 = 0;
                sub.push_back(cur);
                cur = {c + 1, c + 1, SIZE_MAX, 0, 0};
                acc = 0;
            }
        }
        // copy ranges must follow each other; otherwise everything is one sub-batch
        bool mono = true;
        size_t end = 0;
        for (const RxSub& b : sub) {
            if (b.b1 > b.b0 && b.b0 < end) mono = false;
            end = b.b1 > end ? b.b1 : end;
        }
        if (!mono) {
            RxSub all = {0, n, SIZE_MAX, 0, 0};
            for (const RxSub& b : sub) {
                if (b.b1 > b.b0) {
                    all.b0 = b.b0 < all.b0 ? b.b0 : all.b0;
                    all.b1 = b.b1 > all.b1 ? b.b1 : all.b1;
                }
                all.bound += b.bound;
            }
            if (all.b0 == SIZE_MAX) all.b0 = all.b1 = 0;
            sub.assign(1, all);
        }
    }
    const int D = p->depth;
    const size_t nsub = sub.size();
    const bool rx_direct = host_pinned(rx_host), pt_direct = host_pinned(pt_host);
    {
        int rc = choose_d2h_path(p);
        if (rc) return rc;
    }
    uint8_t* pt_dev = pt_direct ? host_store_ptr(pt_host) : nullptr;
    const bool out_direct = max_records == 0 || (host_pinned(records_host) && host_pinned(status_host));
    const bool need_ws = open_needs_workspace(variant);
    uint64_t cap_max = 1, span_max = 0;
    uint32_t nc_max = 1;
    for (const RxSub& b : sub) {
        const uint64_t c = b.bound + 1 < max_records ? b.bound + 1 : max_records;
        cap_max = c > cap_max ? c : cap_max;
        span_max = b.b1 - b.b0 > span_max ? b.b1 - b.b0 : span_max;
        nc_max = b.c1 - b.c0 > nc_max ? b.c1 - b.c0 : nc_max;
    }
    TG_HIP(p->rx.ensure(rx_bytes));
    TG_HIP(p->opt.ensure(rx_bytes));
    TG_HIP(p->conns.ensure((size_t)n * sizeof(tlsgpu_span)));
    TG_HIP(p->rchains.ensure((size_t)n * sizeof(tlsgpu_chain)));
    TG_HIP(p->consumed.ensure((size_t)n * 4));
    TG_HIP(p->fstatus.ensure((size_t)n * 4));
    TG_HIP(p->totals.ensure((size_t)D * 4));
    while (p->rx_in.size() < nsub) {
        hipEvent_t e = nullptr;
        TG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        p->rx_in.push_back(e);
    }
    TG_HIP(p->h_totals.ensure((size_t)D * 4));
    for (int t = 0; t < D; t++) {
        TG_HIP(p->rrecs[t].ensure(cap_max * sizeof(tlsgpu_open_record)));
        TG_HIP(p->rstat[t].ensure(cap_max * 4));
        if (need_ws) TG_HIP(p->rws[t].ensure(open_workspace_bytes((uint32_t)cap_max)));
        TG_HIP(p->fws[t].ensure(frame_workspace_bytes(nc_max)));
        if (!rx_direct) TG_HIP(p->rx_stage[t].ensure(span_max));
        if (!pt_direct) TG_HIP(p->opt_stage[t].ensure(span_max + 16));  // + the range's offset mod 16
    }
    // the D2H ranges come back zero outside the opened bodies, never bytes of an earlier call
    TG_HIP(hipMemsetAsync(p->opt.p, 0, rx_bytes, p->h2d));
    TG_HIP(hipMemcpyAsync(p->conns.p, conns, (size_t)n * sizeof(tlsgpu_span), hipMemcpyHostToDevice, p->h2d));
    const tlsgpu_span* d_conns = static_cast<const tlsgpu_span*>(p->conns.p);
    tlsgpu_chain* d_chains = static_cast<tlsgpu_chain*>(p->rchains.p);
    uint32_t* d_tot = static_cast<uint32_t*>(p->totals.p);
    volatile uint32_t* h_tot = static_cast<volatile uint32_t*>(p->h_totals.p);
    std::vector<uint32_t> base(nsub, 0), tot(nsub, 0);
    uint32_t running = 0;
    auto kstream = [&](size_t i) { return (i & 1) ? p->cbc : p->mac; };
    // H2D of sub-batch i's received bytes (pageable: through slot t's pinned stage, whose
    // previous copy -- sub-batch i - D's, drained by unstage before -- is done)
    auto in_enq = [&](size_t i) -> int {
        const RxSub& b = sub[i];
        const int t = (int)(i % D);
        if (b.b1 > b.b0) {
            const uint8_t* src = rx_host + b.b0;
            if (!rx_direct) {
                stage_copy(p->rx_stage[t].u8(), src, b.b1 - b.b0);
                src = p->rx_stage[t].u8();
            }
            TG_HIP(hipMemcpyAsync(p->rx.u8() + b.b0, src, b.b1 - b.b0, hipMemcpyHostToDevice, p->h2d));
        }
        TG_HIP(hipEventRecord(p->rx_in[i], p->h2d));
        return 0;
    };
    // framing of sub-batch i into slot t (after its bytes arrived and slot t's previous
    // outputs left), its record count to pinned host memory
    auto frame_enq = [&](size_t i) -> int {
        const RxSub& b = sub[i];
        const int t = (int)(i % D);
        hipStream_t ks = p->frs;
        TG_HIP(hipStreamWaitEvent(ks, p->rx_in[i], 0));
        if (i >= (size_t)D) TG_HIP(hipStreamWaitEvent(ks, p->out_done[t], 0));
        const uint64_t left = (uint64_t)max_records - running;
        const uint32_t cap = (uint32_t)(b.bound + 1 < left ? b.bound + 1 : left);
        hipError_t e = launch_frame(p->rx.u8(), rx_bytes, d_conns + b.c0, b.c1 - b.c0,
                                    static_cast<tlsgpu_open_record*>(p->rrecs[t].p), cap, d_chains + b.c0,
                                    chain_flags, static_cast<uint32_t*>(p->consumed.p) + b.c0,
                                    static_cast<int32_t*>(p->fstatus.p) + b.c0, d_tot + t, p->fws[t].u8(), ks);
        if (e != hipSuccess) return fail_hip(e, "host pipeline framing");
        TG_HIP(hipMemcpyAsync((void*)(h_tot + t), d_tot + t, 4, hipMemcpyDeviceToHost, ks));
        TG_HIP(hipEventRecord(p->framed[t], ks));
        return 0;
    };
    // open of sub-batch i once its count is known, then its D2H copies
    auto finish = [&](size_t i) -> int {
        const RxSub& b = sub[i];
        const int t = (int)(i % D);
        hipStream_t ks = kstream(i);
        TG_HIP(hipEventSynchronize(p->framed[t]));
        const uint32_t T = h_tot[t];
        tot[i] = T;
        base[i] = running;
        running += T;
        TG_HIP(hipStreamWaitEvent(ks, p->framed[t], 0));
        if (T) {
            Bounds ob;
            ob.wire_cap = rx_bytes;
            ob.pt_cap = rx_bytes;
            ob.nstates = nstates;
            bool known = false;
            hipError_t e = launch_open(variant, d_chains + b.c0, b.c1 - b.c0,
                                       static_cast<const tlsgpu_open_record*>(p->rrecs[t].p), T, p->rx.u8(),
                                       p->opt.u8(), S(states), static_cast<int32_t*>(p->rstat[t].p), p->rws[t].u8(),
                                       next_epoch(), ks, &known, ob);
            if (!known) return fail(TLSGPU_EINVAL, "unsupported open variant");
            if (e != hipSuccess) return fail_hip(e, "host pipeline open");
        }
        TG_HIP(hipEventRecord(p->opened[t], ks));
        TG_HIP(hipStreamWaitEvent(p->d2h, p->opened[t], 0));
        if (b.b1 > b.b0) {
            uint8_t* dst = pt_direct ? pt_host + b.b0 : p->opt_stage[t].u8() + (b.b0 & 15);
            uint8_t* dst_dev = pt_direct ? (pt_dev ? pt_dev + b.b0 : nullptr) : host_store_ptr(p->opt_stage[t].p);
            if (dst_dev && !pt_direct) dst_dev += b.b0 & 15;
            TG_HIP(pipeline_d2h(p, dst, dst_dev, p->opt.u8() + b.b0, b.b1 - b.b0));
        }
        if (T) {
            void* rd = records_host + base[i];
            void* sd = status_host + base[i];
            if (!out_direct) {
                TG_HIP(p->recs_stage[t].ensure((size_t)T * sizeof(tlsgpu_open_record)));
                TG_HIP(p->stat_stage[t].ensure((size_t)T * 4));
                rd = p->recs_stage[t].p;
                sd = p->stat_stage[t].p;
            }
            TG_HIP(hipMemcpyAsync(rd, p->rrecs[t].p, (size_t)T * sizeof(tlsgpu_open_record), hipMemcpyDeviceToHost,
                                  p->d2h));
            TG_HIP(hipMemcpyAsync(sd, p->rstat[t].p, (size_t)T * 4, hipMemcpyDeviceToHost, p->d2h));
        }
        TG_HIP(hipEventRecord(p->out_done[t], p->d2h));
        return 0;
    };
    // sub-batch j's staged outputs to the caller's arrays (after its D2H copies)
    auto unstage = [&](size_t j) -> int {
        const int t = (int)(j % D);
        TG_HIP(hipEventSynchronize(p->out_done[t]));
        if (!pt_direct && sub[j].b1 > sub[j].b0)
            stage_copy(pt_host + sub[j].b0, p->opt_stage[t].u8() + (sub[j].b0 & 15), sub[j].b1 - sub[j].b0);
        if (!out_direct && tot[j]) {
            memcpy(records_host + base[j], p->recs_stage[t].p, (size_t)tot[j] * sizeof(tlsgpu_open_record));
            memcpy(status_host + base[j], p->stat_stage[t].p, (size_t)tot[j] * 4);
        }
        return 0;
    };
    // H2D copies run ahead of the framing: pinned received bytes are all enqueued at once (each
    // sub-batch has its own device range and event); pageable ones one sub-batch ahead, as far
    // as the pinned stages allow (slot (i + 1) % D's previous copy, i + 1 - D's, is done once
    // sub-batch i - 1's framing has been seen).
    const bool staged = !pt_direct || !out_direct;
    size_t issued = 0;
    auto issue_upto = [&](size_t lim) -> int {
        for (; issued < lim && issued < nsub; issued++) {
            int rc = in_enq(issued);
            if (rc) return rc;
        }
        return 0;
    };
    {
        int rc = issue_upto(rx_direct ? nsub : 1);
        if (rc) return rc;
    }
    for (size_t i = 0; i < nsub; i++) {
        int rc;
        // sub-batch i - 1's count: the wait falls under sub-batch i's H2D copy, already queued
        // (with one slot, i - 1 must also be copied out before i reuses the slot)
        if (i >= 1 && (rc = finish(i - 1))) return rc;
        if (staged && i >= (size_t)D && (rc = unstage(i - D))) return rc;  // slot t's stages free again
        if (!rx_direct && (rc = issue_upto(D == 1 ? i + 1 : i + 2))) return rc;
        if ((rc = frame_enq(i))) return rc;
    }
    {
        int rc = finish(nsub - 1);
        if (rc) return rc;
    }
    TG_HIP(hipStreamSynchronize(p->d2h));
    if (staged)
        for (size_t j = nsub > (size_t)D ? nsub - D : 0; j < nsub; j++) {
            int rc = unstage(j);
            if (rc) return rc;
        }
    // per-connection results (every framing is done: each open waited for its framing, and
    // the d2h stream for each open)
    TG_HIP(hipMemcpy(chains_host, d_chains, (size_t)n * sizeof(tlsgpu_chain), hipMemcpyDeviceToHost));
    TG_HIP(hipMemcpy(consumed_host, p->consumed.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    TG_HIP(hipMemcpy(frame_status_host, p->fstatus.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nsub; i++)
        for (uint32_t c = sub[i].c0; c < sub[i].c1; c++) chains_host[c].first += base[i];
    *total_host = running;
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
                    uint32_t nrecords, const uint8_t* wire, size_t wire_bytes, uint8_t* pt, size_t pt_bytes,
                    tlsgpu_conn_state* states, uint32_t nstates, int32_t* status, uint32_t variant, void* workspace,
                    size_t workspace_bytes, tlsgpu_stream s) {
    if (nchains == 0) return 0;
    if (!chains || !records || !wire || !pt || !states || !status) return fail(TLSGPU_EINVAL, "null pointer");
    uint8_t* ws = static_cast<uint8_t*>(workspace);
    if (open_needs_workspace(variant)) {
        const size_t need = open_workspace_bytes(nrecords);
        if (ws && workspace_bytes < need) return fail(TLSGPU_EINVAL, "workspace too small");
        if (!ws) {
            int rc = own_workspace(1, need, HS(s), &ws);
            if (rc) return rc;
        }
    }
    Bounds b;
    b.pt_cap = pt_bytes;
    b.wire_cap = wire_bytes;
    b.nstates = nstates;
    bool known = false;
    hipError_t e = launch_open(variant, chains, nchains, records, nrecords, wire, pt, S(states), status, ws,
                               next_epoch(), HS(s), &known, b);
    if (!known) return fail(TLSGPU_EINVAL, "unsupported open variant");
    if (e != hipSuccess) return fail_hip(e, "open launch");
    return 0;
}

size_t tlsgpu_frame_workspace_bytes(uint32_t n) { return frame_workspace_bytes(n); }

int tlsgpu_frame_dev(const uint8_t* stream, size_t stream_bytes, const tlsgpu_span* conns, uint32_t n,
                     tlsgpu_open_record* records, uint32_t max_records, tlsgpu_chain* chains, uint32_t chain_flags,
                     uint32_t* consumed, int32_t* status, uint32_t* total, void* workspace, size_t workspace_bytes,
                     tlsgpu_stream s) {
    if (n == 0) {  // nothing framed: total = 0 (stream-ordered, as the kernels would write it)
        if (total) TG_HIP(hipMemsetAsync(total, 0, 4, HS(s)));
        return 0;
    }
    if (!stream || !conns || !chains || !consumed || !status || !total || !workspace || (!records && max_records))
        return fail(TLSGPU_EINVAL, "null pointer");
    if (n > (1u << 26)) return fail(TLSGPU_EINVAL, "too many connections");
    if (workspace_bytes < frame_workspace_bytes(n)) return fail(TLSGPU_EINVAL, "workspace too small");
    hipError_t e = launch_frame(stream, stream_bytes, conns, n, records, max_records, chains, chain_flags, consumed,
                                status, total, static_cast<uint8_t*>(workspace), HS(s));
    if (e != hipSuccess) return fail_hip(e, "frame launch");
    return 0;
}

int tlsgpu_derive_states_dev(const tlsgpu_derive_desc* descs, uint32_t n, tlsgpu_conn_state* write_states,
                             tlsgpu_conn_state* read_states, uint8_t* master_out, uint8_t* key_block_out,
                             int32_t* status, tlsgpu_stream s) {
    if (n && (!descs || !write_states || !read_states || !status)) return fail(TLSGPU_EINVAL, "null argument");
    if (n > (1u << 26)) return fail(TLSGPU_EINVAL, "too many connections");
    hipError_t e = launch_derive(descs, n, S(write_states), S(read_states), master_out, key_block_out, status, HS(s));
    if (e != hipSuccess) return fail_hip(e, "derive launch");
    return 0;
}

int tlsgpu_fill_pattern(uint8_t* dptr, size_t bytes, uint64_t seed, uint64_t start, tlsgpu_stream s) {
    hipError_t e = launch_fill(dptr, bytes, seed, start, HS(s));
    if (e != hipSuccess) return fail_hip(e, "fill launch");
    return 0;
}

}  // extern "C"

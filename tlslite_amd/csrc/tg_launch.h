// tg_launch.h -- kernel launchers exported from tg_kernels.hip to the C ABI
// layer (tg_api.hip).
#pragma once
#include "tg_common.h"
#include <string>

namespace tg {

constexpr int SEAL_BLOCK = 256;  // one lane per chain, 4 waves per workgroup

// The device of a stream (the current device for the null stream): launch plumbing keys
// its per-device caches and allocations on it, not on the calling thread's current device.
int stream_device(hipStream_t s);
// Makes `dev` the current device for a scope and restores the previous one.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        int cur = 0;
        if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

size_t seal_workspace_bytes(uint32_t nrecords);
// What a seal / open launch may touch (ABI 6): the caller's arena sizes and state count,
// checked per record / chain in the prefix kernels -- a record whose plaintext or wire range
// leaves its arena, or a chain whose state index is >= nstates, is refused with
// TLSGPU_EINVAL in wire_len / status: nothing of it is written, its state is not read or
// touched, no seqnum is consumed -- and, for a host-pipeline sub-batch, the window of records
// its chains use ([rec_lo, rec_hi): the MAC phase's grid and meta clear cover only it).
struct Bounds {
    uint32_t rec_lo = 0, rec_hi = 0xffffffffu;
    uint64_t pt_cap = ~(uint64_t)0;    // bytes of the plaintext arena
    uint64_t wire_cap = ~(uint64_t)0;  // bytes of the wire arena
    uint32_t nstates = 0xffffffffu;    // connection states in the states array
};

bool seal_needs_workspace(uint32_t variant);
std::string seal_cipher_kernel(uint32_t variant, uint32_t nchains);
hipError_t launch_seal(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                       uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states, int32_t* wire_len,
                       uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known, const Bounds& b);
hipError_t launch_seal_phases(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                              const tlsgpu_record* recs, uint32_t nrecords, const uint8_t* pt, uint8_t* wire,
                              ConnState* states, int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s1,
                              hipEvent_t mac_done, hipStream_t s2, hipEvent_t cbc_start, hipEvent_t cbc_stop,
                              bool* known, const Bounds& b);
hipError_t launch_cipher(int cipher, int dec, const tlsgpu_span* spans, uint32_t n, const uint8_t* in, uint8_t* out,
                         ConnState* states, hipStream_t s, bool* known);
size_t open_workspace_bytes(uint32_t nrecords);
bool open_needs_workspace(uint32_t variant);
// receive framing (tg_frame.h)
size_t frame_workspace_bytes(uint32_t n);
hipError_t launch_frame(const uint8_t* stream, uint64_t cap, const tlsgpu_span* conns, uint32_t n,
                        tlsgpu_open_record* recs, uint32_t max_records, tlsgpu_chain* chains, uint32_t chain_flags,
                        uint32_t* consumed, int32_t* status, uint32_t* total, uint8_t* ws, hipStream_t s);
hipError_t launch_open(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                       const tlsgpu_open_record* recs, uint32_t nrecords, const uint8_t* wire, uint8_t* pt,
                       ConnState* states, int32_t* status, uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known,
                       const Bounds& b);
// the split open's library-owned second streams and events (one per device and priority)
hipError_t release_open_aux();
size_t open_aux_count();
// the open's split form and record threshold (tlsgpu_set_open_parts); -1 for a bad mode
int set_open_parts(int mode, long long min_records);
hipError_t launch_derive(const tlsgpu_derive_desc* descs, uint32_t n, ConnState* ws, ConnState* rs,
                         uint8_t* master_out, uint8_t* kb_out, int32_t* status, hipStream_t s);
hipError_t launch_fill(uint8_t* p, size_t bytes, uint64_t seed, uint64_t start, hipStream_t s);
// D2H copy by device stores: dst_dev = the device address of pinned host memory, same address
// mod 16 as src (hipErrorInvalidValue otherwise)
hipError_t launch_host_store(const uint8_t* src, uint8_t* dst_dev, size_t n, hipStream_t s);

}  // namespace tg

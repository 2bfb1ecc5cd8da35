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
// What a split-path seal launch may touch besides its chains: the window of records its
// chains use ([rec_lo, rec_hi): the MAC phase's grid and meta clear cover only it) and the
// wire arena's size (a record whose sealed form would end past wire_cap is refused with
// wire_len = TLSGPU_EINVAL, nothing written, no seqnum consumed).
struct SealBounds {
    uint32_t rec_lo = 0, rec_hi = 0xffffffffu;
    uint64_t wire_cap = ~(uint64_t)0;
};
bool seal_needs_workspace(uint32_t variant);
std::string seal_cipher_kernel(uint32_t variant, uint32_t nchains);
hipError_t launch_seal(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains, const tlsgpu_record* recs,
                       uint32_t nrecords, const uint8_t* pt, uint8_t* wire, ConnState* states, int32_t* wire_len,
                       uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known);
hipError_t launch_seal_phases(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                              const tlsgpu_record* recs, uint32_t nrecords, const uint8_t* pt, uint8_t* wire,
                              ConnState* states, int32_t* wire_len, uint8_t* ws, uint32_t epoch, hipStream_t s1,
                              hipEvent_t mac_done, hipStream_t s2, hipEvent_t cbc_start, hipEvent_t cbc_stop,
                              bool* known, const SealBounds& sb = SealBounds());
hipError_t launch_cipher(int cipher, int dec, const tlsgpu_span* spans, uint32_t n, const uint8_t* in, uint8_t* out,
                         ConnState* states, hipStream_t s, bool* known);
size_t open_workspace_bytes(uint32_t nrecords);
bool open_needs_workspace(uint32_t variant);
hipError_t launch_open(uint32_t variant, const tlsgpu_chain* chains, uint32_t nchains,
                       const tlsgpu_open_record* recs, uint32_t nrecords, const uint8_t* wire, uint8_t* pt,
                       ConnState* states, int32_t* status, uint8_t* ws, uint32_t epoch, hipStream_t s, bool* known);
hipError_t launch_derive(const tlsgpu_derive_desc* descs, uint32_t n, ConnState* ws, ConnState* rs,
                         uint8_t* master_out, uint8_t* kb_out, int32_t* status, hipStream_t s);
hipError_t launch_fill(uint8_t* p, size_t bytes, uint64_t seed, uint64_t start, hipStream_t s);

}  // namespace tg

// tg_frame.h -- receive framing on the device (round 5): _getNextRecord's record-header parse
// (tlsrecordlayer.py:832-876; RecordHeader3.parse, messages.py:44-49) for many connections'
// received byte streams at once, producing the tlsgpu_open_record / tlsgpu_chain descriptors
// tlsgpu_open_dev takes -- so received bytes go to plaintext without a host pass.
//
// A connection's records are serial (each header's length locates the next), connections are
// independent: one lane walks one connection.  Three launches:
//   frame_count_kernel  256 connections per block: each lane counts its complete records;
//                       the block's total goes to the workspace
//   frame_scan_kernel   one block: exclusive scan of the block totals (and the grand total)
//   frame_write_kernel  each lane's first record index (block scan + the block's offset),
//                       clamped to max_records, then the walk again, writing descriptors
#pragma once
#include "tg_common.h"

namespace tg {

constexpr uint32_t FRAME_MAX_BODY = 16384 + 2048;  // tlsrecordlayer.py:871
constexpr int FRAME_BLOCK = 256;

struct FrameWalk {
    uint32_t count;  // records framed
    uint64_t pos;    // first byte after them
    int32_t code;    // 0, or the error that stopped the walk there
};

// Walk [off, off + len) of the arena, at most `limit` records; with `out`, write their
// descriptors.  The checks in the reference's order: the first byte of a header must be a
// content type as soon as it arrives (:850-857, SyntaxError otherwise -- an SSLv2 header, 128,
// belongs to the handshake), then the 5-byte header, its length against 18432 (:871-873), then
// the body: an empty one ends the connection (the body loop's sock.recv(0) returns b"" and
// raises TLSAbruptCloseError, :877-889; ABI 7), else it must be complete.
__device__ __forceinline__ FrameWalk frame_walk(const uint8_t* __restrict__ s, uint64_t off, uint64_t len,
                                                uint32_t limit, tlsgpu_open_record* __restrict__ out) {
    uint64_t pos = off;
    const uint64_t end = off + len;
    uint32_t c = 0;
    int32_t code = 0;
    while (c < limit && pos < end) {
        const uint32_t t = s[pos];
        if (t - 20u >= 4u) {  // ContentType.all = 20..23
            code = TLSGPU_EFRAME;
            break;
        }
        if (end - pos < 5) break;  // header incomplete: left for the next call
        const uint32_t L = ((uint32_t)s[pos + 3] << 8) | s[pos + 4];
        if (L > FRAME_MAX_BODY) {
            code = TLSGPU_ALERT_RECORD_OVERFLOW;
            break;
        }
        if (L == 0) {
            code = TLSGPU_EABRUPT;
            break;
        }
        if (end - pos - 5 < L) break;  // body incomplete
        if (out) {
            tlsgpu_open_record R;
            R.ct_off = pos + 5;
            R.pt_off = pos + 5;
            R.ct_len = L;
            R.content_type = (uint8_t)t;
            R.reserved[0] = R.reserved[1] = R.reserved[2] = 0;
            out[c] = R;
        }
        c++;
        pos += 5 + L;
    }
    return {c, pos, code};
}

__global__ void __launch_bounds__(FRAME_BLOCK) frame_count_kernel(const uint8_t* __restrict__ s, uint64_t cap,
                                                                 const tlsgpu_span* __restrict__ conns, uint32_t n,
                                                                 uint32_t* __restrict__ counts,
                                                                 uint64_t* __restrict__ block_sums) {
    // 64-bit sums: 256 connections' spans may overlap and frame more than 2^32 records
    __shared__ uint64_t red[FRAME_BLOCK / 64];
    const uint32_t i = blockIdx.x * FRAME_BLOCK + threadIdx.x;
    uint32_t c = 0;
    if (i < n) {
        const tlsgpu_span sp = conns[i];
        if (in_arena(sp.off, sp.len, cap)) c = frame_walk(s, sp.off, sp.len, 0xffffffffu, nullptr).count;
        counts[i] = c;
    }
    uint64_t w = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) w += (uint64_t)__shfl_xor((unsigned long long)w, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int k = 0; k < FRAME_BLOCK / 64; k++) t += red[k];
        block_sums[blockIdx.x] = t;
    }
}

// exclusive scan of nb block totals in place (one block of 1024 threads, each a contiguous
// piece), the grand total to *total (64-bit sums: 2^26 connections of up to 2^32 records)
__global__ void __launch_bounds__(1024) frame_scan_kernel(uint64_t* __restrict__ block_sums, uint32_t nb,
                                                        uint32_t* __restrict__ total, uint32_t max_records) {
    __shared__ uint64_t part[1024];
    const uint32_t per = (nb + 1023) / 1024, a = threadIdx.x * per, b = min(nb, a + per);
    uint64_t sum = 0;
    for (uint32_t k = a; k < b; k++) sum += block_sums[k];
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {  // 1,024 partial sums, once
        uint64_t run = 0;
        for (int k = 0; k < 1024; k++) {
            const uint64_t v = part[k];
            part[k] = run;
            run += v;
        }
        *total = (uint32_t)min<uint64_t>(run, max_records);
    }
    __syncthreads();
    uint64_t run = part[threadIdx.x];
    for (uint32_t k = a; k < b; k++) {
        const uint64_t v = block_sums[k];
        block_sums[k] = run;
        run += v;
    }
}

__global__ void __launch_bounds__(FRAME_BLOCK) frame_write_kernel(
    const uint8_t* __restrict__ s, uint64_t cap, const tlsgpu_span* __restrict__ conns, uint32_t n,
    const uint32_t* __restrict__ counts, const uint64_t* __restrict__ block_off, tlsgpu_open_record* __restrict__ recs,
    uint32_t max_records, tlsgpu_chain* __restrict__ chains, uint32_t chain_flags, uint32_t* __restrict__ consumed,
    int32_t* __restrict__ status) {
    __shared__ uint64_t wsum[FRAME_BLOCK / 64];
    const uint32_t i = blockIdx.x * FRAME_BLOCK + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t c = i < n ? counts[i] : 0u;
    // inclusive scan of c over the wave, then over the block's waves
    uint64_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t before = 0;
    for (uint32_t k = 0; k < wv; k++) before += wsum[k];
    if (i >= n) return;
    const uint64_t first = block_off[blockIdx.x] + before + (x - c);
    const tlsgpu_span sp = conns[i];
    tlsgpu_chain ch;
    ch.state = sp.state;
    ch.flags = chain_flags;
    ch.first = (uint32_t)min<uint64_t>(first, max_records);
    if (!in_arena(sp.off, sp.len, cap)) {
        ch.count = 0;
        chains[i] = ch;
        consumed[i] = 0;
        status[i] = TLSGPU_EINVAL;
        return;
    }
    const uint32_t room = first >= max_records ? 0u : (uint32_t)min<uint64_t>(c, max_records - first);
    // not cut short by max_records: walk on to where the count pass stopped, to see its error
    const FrameWalk w = frame_walk(s, sp.off, sp.len, room < c ? room : 0xffffffffu, recs + ch.first);
    ch.count = w.count;
    chains[i] = ch;
    consumed[i] = (uint32_t)(w.pos - sp.off);
    status[i] = w.code ? w.code : (int32_t)w.count;
}

}  // namespace tg

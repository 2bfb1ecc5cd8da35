// tg_config.h -- the product's tuning constants (one place, no switches).
//
// Every value here was chosen by a same-box A/B on the MI355X (the
// measurements are under profiles/).  The kernels include this header as <tg_config.h>,
// so an experiment build (tools/build_ab.sh) puts tools/ab_overlay/ first on the include
// path and its tg_config.h -- the same names, overridable with -D flags -- replaces this
// one.  The product library is always built from this file.
#pragma once

namespace tg {

// cbc_kernel (quad layout, the few-chains regime, cfg4): waves per CU (16 x 16 chains)
constexpr int CFG_CBC_WAVES = 16;
// wave priorities: the cipher waves (latency-bound CBC chains) above the MAC waves
// (issue-bound), so when the pipeline runs the MAC phase of batch k+1 beside the cipher
// phase of batch k the cipher waves win issue arbitration
constexpr int CFG_MAC_PRIO = 0;
constexpr int CFG_CBC_PRIO = 1;
// mac_kernel: 64-B chunks the quad-cooperative loop prefetches; launch bound in 256-thread
// blocks per CU (3: <= 168 VGPRs, one MAC wave per SIMD fits beside the cipher waves)
constexpr int CFG_MAC_PF = 2;
constexpr int CFG_MAC_LB = 3;
// the many-chains MAC kernel (cfg3): <= 128 VGPRs, one-chunk prefetch
constexpr int CFG_MAC_LB_MANY = 4;
constexpr int CFG_MAC_PF_MANY = 1;
// LDS bytes the many-chains MAC launch reserves per 256-thread workgroup: none (the kernel
// uses no LDS).  Experiment builds set it to what an LDS staging of each record's current
// 128-B plaintext line would take (8 KiB), to measure that occupancy cost alone (round 6).
constexpr int CFG_MAC_MANY_LDS = 0;
// cbc_pair_kernel: waves per CU in the many-chains regime; prefetch group (blocks) in the
// one-generation (cfg2) and many-chains (cfg3) regimes
constexpr int CFG_PAIR_WAVES_MANY = 8;
constexpr int CFG_PAIR_G1 = 8;
constexpr int CFG_PAIR_GM = 4;
// seal pipeline: workspaces in rotation (the MAC stream may run PIPE_WS - 1 calls ahead)
constexpr int CFG_PIPE_WS = 3;
// open MAC: batches of at most this many records per CU take the cooperative-load, one-wave-
// workgroup form (the receive pipeline's sub-batches, round 6)
constexpr int CFG_OPEN_MAC_COOP_PER_CU = 64;
// host seal pipeline, pinned arenas: 0 = every sub-batch's H2D copy enqueued at once; L > 0 =
// sub-batch i's H2D copy waits until sub-batch i - L's D2H copy may start (its seal is done),
// so the H2D direction cannot run far ahead of the D2H one (experiment knob, round 6)
constexpr int CFG_HOST_H2D_LEAD = 0;

}  // namespace tg

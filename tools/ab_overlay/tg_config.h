// tools/ab_overlay/tg_config.h -- experiment build of the product's tuning constants.
// tools/build_ab.sh puts this directory ahead of tlslite_amd/csrc on the include path, so
// this file replaces tlslite_amd/csrc/tg_config.h; each constant takes its -D override
// (e.g. -DTG_AB_PAIR_G1=4) or the product value.  Never used by the product build.
#pragma once

#ifndef TG_AB_CBC_WAVES
#define TG_AB_CBC_WAVES 16
#endif
#ifndef TG_AB_MAC_PRIO
#define TG_AB_MAC_PRIO 0
#endif
#ifndef TG_AB_CBC_PRIO
#define TG_AB_CBC_PRIO 1
#endif
#ifndef TG_AB_MAC_PF
#define TG_AB_MAC_PF 2
#endif
#ifndef TG_AB_MAC_LB
#define TG_AB_MAC_LB 3
#endif
#ifndef TG_AB_MAC_LB_MANY
#define TG_AB_MAC_LB_MANY 4
#endif
#ifndef TG_AB_MAC_PF_MANY
#define TG_AB_MAC_PF_MANY 1
#endif
#ifndef TG_AB_MAC_MANY_LDS
#define TG_AB_MAC_MANY_LDS 0
#endif
#ifndef TG_AB_PAIR_WM
#define TG_AB_PAIR_WM 8
#endif
#ifndef TG_AB_PAIR_G1
#define TG_AB_PAIR_G1 8
#endif
#ifndef TG_AB_PAIR_GM
#define TG_AB_PAIR_GM 4
#endif
#ifndef TG_AB_PIPE_WS
#define TG_AB_PIPE_WS 3
#endif

#ifndef TG_AB_H2D_LEAD
#define TG_AB_H2D_LEAD 0
#endif
#ifndef TG_AB_OPEN_COOP
#define TG_AB_OPEN_COOP 64
#endif
namespace tg {
constexpr int CFG_CBC_WAVES = TG_AB_CBC_WAVES;
constexpr int CFG_MAC_PRIO = TG_AB_MAC_PRIO;
constexpr int CFG_CBC_PRIO = TG_AB_CBC_PRIO;
constexpr int CFG_MAC_PF = TG_AB_MAC_PF;
constexpr int CFG_MAC_LB = TG_AB_MAC_LB;
constexpr int CFG_MAC_LB_MANY = TG_AB_MAC_LB_MANY;
constexpr int CFG_MAC_PF_MANY = TG_AB_MAC_PF_MANY;
constexpr int CFG_MAC_MANY_LDS = TG_AB_MAC_MANY_LDS;
constexpr int CFG_PAIR_WAVES_MANY = TG_AB_PAIR_WM;
constexpr int CFG_PAIR_G1 = TG_AB_PAIR_G1;
constexpr int CFG_PAIR_GM = TG_AB_PAIR_GM;
constexpr int CFG_PIPE_WS = TG_AB_PIPE_WS;
constexpr int CFG_HOST_H2D_LEAD = TG_AB_H2D_LEAD;
constexpr int CFG_OPEN_MAC_COOP_PER_CU = TG_AB_OPEN_COOP;
}  // namespace tg

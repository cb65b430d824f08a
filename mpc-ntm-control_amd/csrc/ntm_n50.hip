// ntm_n50.hip — the N = 50 specialisation of the hot-path kernels (BASELINE
// config 5) in a translation unit of its own, so that its LDS contractions can
// batch a different number of terms per round trip than the other horizons.
// Measured on the MI355X (B = 5e4, ms per step, mode 2 / mode 3, all-LDS workspace):
//   CH = 4: 119.9 / 273.3   CH = 8: 120.3 / 276.5   CH = 10: 109.0 / 260.2
//   CH = 16: 126.6 / 282.4  CH = 25: 119.6 / 271.8
// 10 divides 50 (no masked tail chunk) and 5 chunks per horizon loop unroll
// without spilling.  Re-measured on the round-3 build (far workspace, MFMA Gram,
// B = 1e5, mode 2 / mode 3): CH = 10 140.4 / 297.3, CH = 25 141.0 / 299.2,
// CH = 5 149.0 / 309.8, CH = 10 unrolled twice 147.2 / 306.8, CH = 5 twice 152.0 / 317.7.
#ifdef NTM_N50_UNROLL
#define NTM_CHUNK_UNROLL NTM_N50_UNROLL
#endif
#ifndef NTM_N50_CH
#define NTM_N50_CH 10
#endif
#undef NTM_CH
#define NTM_CH NTM_N50_CH
// modes 0-2: without the three-hole null-space path, which only input-rate rows use
// and which costs this kernel's register allocation 3.8% (config 5 mode 2: 76.6 vs
// 79.5 ms, A/B on one box); mode 3 launches ntm_n50m3.hip
#ifndef NTM_COLL3
#define NTM_COLL3 0
#endif
#include "ntm_step.h"

NTM_DEFINE_LAYOUT_LAUNCHERS(n50, 50, true)

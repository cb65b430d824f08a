// ntm_n50m3.hip — the N = 50 specialisation for input-rate rows (NTM_MODE_FULL_DU,
// config 5's mode 3): ntm_n50.hip's batch settings plus the three-hole null-space
// path (NTM_COLL3: k = 2 sets with one collision, which mode 3 meets 0.44 times per
// MPC step and which took the bordered elimination: 99.8 -> 90.0 ms per step-batch,
// A/B on one box).  The host launches this build for mode 3 only (ntm_kernels.hip).
#ifdef NTM_N50_UNROLL
#define NTM_CHUNK_UNROLL NTM_N50_UNROLL
#endif
#ifndef NTM_N50_CH
#define NTM_N50_CH 10
#endif
#undef NTM_CH
#define NTM_CH NTM_N50_CH
#ifndef NTM_COLL3
#define NTM_COLL3 1
#endif
// the certificate's sparse pass over the active general rows by readlane (round 6: mode 3
// 76.9 -> 76.3 ms per step-batch; the modes 0-2 TU ran 64.9 -> 65.6 ms with it, so off there)
#ifndef NTM_SUB_LANEIDX
#define NTM_SUB_LANEIDX 1
#endif
#include "ntm_step.h"

NTM_DEFINE_LAYOUT_LAUNCHERS(n50m3, 50, true)

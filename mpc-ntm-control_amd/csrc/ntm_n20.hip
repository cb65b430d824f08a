// ntm_n20.hip — the N = 20 specialisation of the hot-path kernels (BASELINE
// configs 2-4, the headline) in a translation unit of its own, for its own LDS
// batch size.  With the far workspace and 3 waves per SIMD (168 VGPRs), measured
// on the MI355X (B = 1e5, ms per step-batch over steps 6-25, A/B on one box):
//   CH = 2: 11.53   CH = 3: 11.10   CH = 4: 11.24   CH = 5: 11.03
// (at 2 waves per SIMD and 256 VGPRs CH = 4 and 5 were equal, 10.90 / 10.92).
// The chunk loops are unrolled twice, not fully: at 168 VGPRs full unrolling
// spills 68 VGPRs (276 B of scratch per lane), unroll 2 spills 28 (132 B):
//   CH = 5, full unroll: 10.83   unroll 1: 10.61   unroll 2: 10.38 ms
// Round 5, the slim layout at 4 waves per SIMD (128 VGPRs), default scheduler:
//   CH = 5, unroll 2: 6.68   unroll 1: 6.78   unroll 3: 10.08   CH = 6: 9.33
//   CH = 4: 10.86   CH = 3: 10.07 ms (the last two with the max-memory-clause scheduler)
#ifndef NTM_N20_CH
#define NTM_N20_CH 5
#endif
#ifndef NTM_N20_UNROLL
#define NTM_N20_UNROLL 2
#endif
#if NTM_N20_UNROLL > 0
#define NTM_CHUNK_UNROLL NTM_N20_UNROLL
#endif
// chunk loops with a runtime trip count are left alone (the pragma is a hint)
#pragma clang diagnostic ignored "-Wpass-failed"
#undef NTM_CH
#define NTM_CH NTM_N20_CH
#include "ntm_step.h"

// the far layout is what the host side attaches a far block for (ws_far(20)); the
// all-LDS N = 20 kernel is ntm_n20near.hip, so this TU requires NTM_FAR_N20
#if !NTM_FAR_N20
#error "ntm_n20.hip is the far-workspace N = 20 build: NTM_FAR_N20=0 applies to single-TU builds only"
#endif
NTM_DEFINE_LAYOUT_LAUNCHERS(n20, 20, ntm::ws_far(20))

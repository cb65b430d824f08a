// ntm_n20near.hip — the all-LDS N = 20 build (2 waves per SIMD, 256 VGPRs, the
// round-2 layout) for batches the far 3-wave build cannot fill (BASELINE config
// 2: B = 1024; ntm_ctx_set_small_batch), in a translation unit of its own so that
// it keeps its own batch settings: 4 terms per LDS round trip and fully unrolled
// chunk loops, which suit a 256-VGPR kernel (round 2: CH = 4 and 5 equal, full
// unrolling ahead of unroll 1 by 9%).
#ifndef NTM_N20NEAR_CH
#define NTM_N20NEAR_CH 4
#endif
#undef NTM_CH
#define NTM_CH NTM_N20NEAR_CH
#include "ntm_step.h"

NTM_DEFINE_LAYOUT_LAUNCHERS(n20near, 20, false)

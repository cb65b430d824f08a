// ntm_n20near1w.hip — the all-LDS N = 20 build with a one-wave-per-SIMD register
// budget (512 registers: no spills), for batches of at most 4 scenarios per CU
// (one wave per SIMD, BASELINE config 2: B = 1024), where that build's occupancy
// of 2 waves per SIMD cannot be used.  Same source and batch settings as
// ntm_n20near.hip; measured (round 6, A/B on one box): config 2 0.198 -> 0.1925 ms,
// B = 1024 mode 2 0.480 -> 0.467 ms per step-batch; at B = 2048 the budget halves
// the occupancy (round 5: 28% slower), so the host launches it only below 4 per CU
// (ntm_ctx_set_one_wave_batch).  Results are bit-identical to ntm_n20near.hip's
// (tests/test_gpu_parity.py::test_one_wave_build_bitwise).
#ifndef NTM_N20NEAR_CH
#define NTM_N20NEAR_CH 4
#endif
#undef NTM_CH
#define NTM_CH NTM_N20NEAR_CH
#define NTM_HOT_WAVES_PER_EU 1
#include "ntm_step.h"

NTM_DEFINE_LAYOUT_LAUNCHERS(n20near1w, 20, false)

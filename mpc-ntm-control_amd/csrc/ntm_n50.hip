// ntm_n50.hip — the N = 50 specialisation of the hot-path kernels (BASELINE
// config 5) in a translation unit of its own, so that its LDS contractions can
// batch a different number of terms per round trip than the other horizons.
// Measured on the MI355X (B = 5e4, ms per step, mode 2 / mode 3):
//   CH = 4: 119.9 / 273.3   CH = 8: 120.3 / 276.5   CH = 10: 109.0 / 260.2
//   CH = 16: 126.6 / 282.4  CH = 25: 119.6 / 271.8
// 10 divides 50 (no masked tail chunk) and 5 chunks per horizon loop unroll
// without spilling.  At N = 20 CH = 4 stays best (10.90 vs 10.92 at CH = 5 and
// 10.97 at CH = 10), so ntm_kernels.hip keeps the default.
#ifdef NTM_N50_UNROLL
#define NTM_CHUNK_UNROLL NTM_N50_UNROLL
#endif
#ifndef NTM_N50_CH
#define NTM_N50_CH 10
#endif
#define NTM_CH NTM_N50_CH
#include "ntm_step.h"

namespace {
template <typename K>
hipError_t lds_opt_in(K kern, size_t lds) {
    if (lds <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds);
}
}  // namespace

hipError_t ntm_launch_step_n50(const ntm::Prob& pb, int64_t B, const double* x_k, double* rho, double* U_old,
                               double* U, double* x_pred, double* x_next, int32_t* exitflag, int32_t* inner_iters,
                               int32_t* active_ws, size_t lds, hipStream_t st) {
    const bool gen = pb.g.phys_on || pb.g.dist_on;
    hipError_t e = gen ? lds_opt_in(k_mpc_step<64, 50, true>, lds) : lds_opt_in(k_mpc_step<64, 50, false>, lds);
    if (e != hipSuccess) return e;
    if (B <= 0) return hipSuccess;
    if (gen)
        hipLaunchKernelGGL((k_mpc_step<64, 50, true>), dim3((unsigned)B), dim3(64), lds, st, pb, B, x_k, rho, U_old, U,
                           x_pred, x_next, exitflag, inner_iters, active_ws);
    else
        hipLaunchKernelGGL((k_mpc_step<64, 50, false>), dim3((unsigned)B), dim3(64), lds, st, pb, B, x_k, rho, U_old,
                           U, x_pred, x_next, exitflag, inner_iters, active_ws);
    return hipGetLastError();
}

hipError_t ntm_launch_run_n50(const ntm::Prob& pb, int64_t B, int k_sim, const double* x0, double* xk, double* uk,
                              double* Uk, double* wpred, int32_t* exitflag, int32_t* inner_iters, size_t lds,
                              hipStream_t st) {
    hipError_t e = lds_opt_in(k_mpc_run<64, 50>, lds);
    if (e != hipSuccess) return e;
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_mpc_run<64, 50>), dim3((unsigned)B), dim3(64), lds, st, pb, B, k_sim, x0, xk, uk, Uk, wpred,
                       exitflag, inner_iters);
    return hipGetLastError();
}

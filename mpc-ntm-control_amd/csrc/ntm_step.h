// ntm_step.h — the hot-path kernels k_mpc_step / k_mpc_run (one fused launch
// per MPC time step, or per closed loop, for the whole scenario batch) and
// their per-scenario helpers.  Included by ntm_kernels.hip and, for the N = 50
// specialisation, by ntm_n50.hip: a translation unit of its own so that its
// chunk loops can be built without unrolling (NTM_CHUNK_UNROLL) while the
// other horizons keep the compiler's choice.  Each group of P lanes runs the
// complete NTM_MPC_Sim.m:94-130 body for one scenario out of LDS.
#pragma once
#include <hip/hip_runtime.h>

#include "ntm_device.h"

namespace {

using namespace ntm;

template <int P, class W>
__device__ __forceinline__ void load_state(const W& w, int64_t B, int64_t s, const double* rho,
                                           const double* U_old, int l) {
    const int N = w.n();
    const double* rs = rho + s * (3 * N);
    for (int e = l; e < 3 * N; e += P) w.rho()[e] = rs[e];
    if (l < N) w.Uold()[l] = U_old[s * N + l];
    NTM_WSYNC();
}

__device__ __forceinline__ bool is16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// One scenario's record of n doubles from LDS to HBM.  With a 16-byte aligned
// destination and an even n, lanes store two doubles each (16-B stores: every
// request carries whole 16-B granules); otherwise one double per lane.
template <int P>
__device__ __forceinline__ void store_record(double* dst, const double* src, int n, int l) {
    if (is16(dst) && (n & 1) == 0) {
        for (int e = 2 * l; e < n; e += 2 * P)
            *reinterpret_cast<double2*>(dst + e) = make_double2(src[e], src[e + 1]);
    } else {
        for (int e = l; e < n; e += P) dst[e] = src[e];
    }
}

// XCD-aware block order (bijective): blocks are dealt round-robin over the 8
// XCDs, so block b is given the k-th slot of XCD b%8's contiguous range of
// scenario blocks.  Neighbouring scenarios share the cache lines at the ends
// of their (scenario-major) records; this keeps each line's users on one L2.
__device__ __forceinline__ int64_t xcd_swizzle(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

// Warm-start workspace (ntm_mpc_step_ws): the active sets of the previous
// step's last two QPs, 2 slots x (N ids + count) per scenario, in/out.  It is
// only a hint (every candidate is re-solved exactly and KKT-certified), but it
// comes from the caller, so each slot is validated before use: count in
// [0, N], ids in [0, rows), no repeats; anything else disables the slot.
template <int P, class W>
__device__ __forceinline__ void load_candidates(const Prob& pb, const W& w, int64_t B, int64_t s, const int32_t* ws, int l) {
    const int N = w.n();
    const int nrows = StructRows(pb).rows();
    const int32_t* wss = ws + s * (2 * (N + 1));
    for (int e = l; e < 2 * (N + 1); e += P) w.cand()[e] = wss[e];
    for (int i = l; i < nrows; i += P) w.aflag()[i] = 0;
    NTM_WSYNC();
    for (int slot = 0; slot < 2; ++slot) {
        int* c = w.cand() + slot * (N + 1);
        const int q = uni<P>(c[N]);
        if (q < 0) continue;
        bool bad = q > N || nrows == 0;
        if (!bad) {
            int lb = 0;
            if (l < q) lb = (c[l] < 0 || c[l] >= nrows) ? 1 : 0;
            bad = gmaxi<P>(lb) != 0;
        }
        if (!bad) {
            int lb = 0;
            for (int i = 0; i < q; ++i) {         // lane l < q checks its id against the earlier ones
                const int ci = c[i];
                if (l < q && i < l && ci == c[l]) lb = 1;
            }
            bad = gmaxi<P>(lb) != 0;
        }
        if (bad && l == 0) c[N] = -1;
        NTM_WSYNC();
    }
}

// 1: the rollout of a certified plan is the lifted prediction e + Gamma U (rollout_phase)
#ifndef NTM_ROLL_LIFTED
#define NTM_ROLL_LIFTED 1
#endif
// one MPC step on LDS-resident state; returns exit flag, sets *iters
template <int P, class W>
__device__ __forceinline__ int mpc_step_dev(const Prob& pb, const W& w, double x0, double x1, int l, int* iters,
                            int64_t B = 0, int64_t s = 0) {
    int flag = NTM_EXIT_OPTIMAL, it;
    int n_qp = 0, n_gi = 0, n_act = 0, n_gen = 0, n_try = 0, n_girun = 0;
#ifdef NTM_STAMPS
    // exact 2-cycle study (diagnostic build): is the state after iteration it
    // (rho and U) bit-identical to the state after iteration it-2?  A necessary
    // condition for the LPV loop to repeat exactly from there on
    double cr[2][3] = {{0, 0, 0}, {0, 0, 0}}, cu[2] = {0, 0};
    int cyc = 0;
#endif
    for (it = 1; it <= pb.i_sim; ++it) {
        int qi = 0, qa = 0, ns = 0;
        bool yv = false;
        flag = qp_phase<P>(pb, w, x0, x1, l, &qi, &qa, &ns, (it - 1) & 1, &n_try, &n_girun, it, &yv);
        ++n_qp;
        n_gi += qi;
        n_act += qa;
        n_gen += ns;
        NTM_T0(tr);
        bool conv = rollout_phase<P>(pb, w, x0, x1, l, NTM_ROLL_LIFTED && yv);
        NTM_ACC(ST_ROLL, tr);
#ifdef NTM_STAMPS
        {
            double r0 = 0.0, r1 = 0.0, r2 = 0.0, u = 0.0;
            if (l < w.n()) { r0 = w.rho()[3 * l]; r1 = w.rho()[3 * l + 1]; r2 = w.rho()[3 * l + 2]; u = w.U()[l]; }
            const int sl = it & 1;
            int ne = (it < 3) || (l < w.n() && (r0 != cr[sl][0] || r1 != cr[sl][1] || r2 != cr[sl][2] || u != cu[sl]));
            ne = gmaxi<P>(ne);
            if (!ne && !cyc) {
                cyc = it;
                NTM_CNT(CN_CYC_HIT);
                if ((threadIdx.x & 63) == 0) ntm_lds_stamps[CN_CYC_SKIP] += (unsigned long long)(pb.i_sim - it);
            }
            cr[sl][0] = r0; cr[sl][1] = r1; cr[sl][2] = r2; cu[sl] = u;
        }
#endif
        if (conv) break;
    }
    *iters = it > pb.i_sim ? pb.i_sim : it;
    if (pb.stats && l == 0) {
        pb.stats[s] += n_qp;
        pb.stats[B + s] += n_gi;
        pb.stats[2 * B + s] += n_act;
        pb.stats[3 * B + s] += n_gen;
        pb.stats[4 * B + s] += n_try;
        pb.stats[5 * B + s] += n_girun;
    }
    return flag;
}

#ifndef NTM_HOT_WAVES_PER_EU
#define NTM_HOT_WAVES_PER_EU 2
#endif
#ifndef NTM_N20_WAVES_PER_EU
#define NTM_N20_WAVES_PER_EU (NTM_FAR_N20 ? (NTM_SLIM20 ? 4 : 3) : 2)
#endif
// Long horizons (NN > 32): the LDS workspace already limits a CU to fewer waves
// than SIMDs, so the register budget of one wave per SIMD costs no occupancy and
// removes the spills of the fully unrolled horizon loops.  N = 20: three waves per
// SIMD (the far workspace fits 12 scenarios per CU); 168 VGPRs spill ~60 of them,
// and the third wave still wins (11.92 -> 11.03 ms per step-batch, A/B on one box).
// FAR = false at N = 20: the all-LDS build (2 waves per SIMD, 256 VGPRs), which
// runs each wave faster and is launched for batches that fill no more than its
// 8 scenarios per CU (small_batch in ntm_kernels.hip)
#define NTM_WAVES_PER_EU(NN, FAR) \
    ((NN) > 32 ? 1 : ((NN) == 20 && (FAR) ? NTM_N20_WAVES_PER_EU : NTM_HOT_WAVES_PER_EU))
// two scenarios per wave at N = 20 (far layout, 24 KB of LDS per wave): at most 6
// waves per CU fit, so the register budget of 2 waves per SIMD costs nothing
#define NTM_WAVES_PER_EU_P(P, NN, FAR) ((P) < 64 && (NN) == 20 ? 2 : NTM_WAVES_PER_EU(NN, FAR))
// NTM_STATIC_LDS=1: compile-time horizons with one scenario per wave keep their
// workspace in a static __shared__ array (the launch passes no dynamic LDS), so
// every workspace address is a constant the backend folds into the ds_read /
// ds_write offset field (the dynamic-LDS base is an opaque value: the layout's
// loop-invariant addresses are held in VGPRs and spilled).  It cuts the N = 20
// kernel's scratch from 88 to 56 B per lane, yet measured 0.6% slower (9.96 vs
// 9.90 ms per step-batch, A/B on one box), so it stays off
#ifndef NTM_STATIC_LDS
#define NTM_STATIC_LDS 0
#endif
template <int P, int NN>
__host__ __device__ constexpr bool static_lds() { return NTM_STATIC_LDS && P == 64 && NN > 0; }

template <int P, int NN, bool GEN, bool FAR = ws_far(NN)>
__global__ __launch_bounds__(64, NTM_WAVES_PER_EU_P(P, NN, FAR)) void k_mpc_step(Prob pb, int64_t B, const double* __restrict__ x_k,
                                                 double* __restrict__ rho, double* __restrict__ U_old,
                                                 double* __restrict__ U, double* __restrict__ x_pred,
                                                 double* __restrict__ x_next, int32_t* __restrict__ exitflag,
                                                 int32_t* __restrict__ inner_iters, int32_t* __restrict__ active_ws) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int G = 64 / P;
    const int g = threadIdx.x / P, l = threadIdx.x % P;
    const int64_t s = xcd_swizzle(blockIdx.x, gridDim.x) * G + g;
    const int N = NN > 0 ? NN : pb.N;
    NTM_STAMPS_INIT();
    NTM_TRACE_SET(s, g, l);
    if (s >= B) return;
    char* sbase = smem + g * ws_bytes(N, FAR);
    if constexpr (static_lds<P, NN>()) {
        __shared__ __attribute__((aligned(16))) char smem_s[ws_bytes(NN > 0 ? NN : 1, FAR)];
        sbase = smem_s;
    }
    auto w = ws_carve<NN, GEN, FAR>(sbase, N, &pb, s);
#ifdef NTM_POISON
    // debug build (make poison): the workspace starts as NTM_POISON-valued doubles, so
    // a read of LDS this launch never wrote shows up as a run-to-run difference
    // (tools/determinism.py + compare_runs.py; this found the x_0-row read of rinfo[-1])
    for (int e = l; e < ws_bytes(N, FAR) / 8; e += P) w.base[e] = NTM_POISON;
    NTM_WSYNC();
#endif
    const double x0 = x_k[2 * s], x1 = x_k[2 * s + 1];
    if (active_ws) {
        load_candidates<P>(pb, w, B, s, active_ws, l);
    } else if (l < 2) {
        w.cand()[l * (N + 1) + N] = -1;
    }
    load_state<P>(w, B, s, rho, U_old, l);
    scn_store(pb, w, pb.g.first_id + s, l);           // this scenario's plasma (generator)
    NTM_WSYNC();
    int its;
    int flag = mpc_step_dev<P>(pb, w, x0, x1, l, &its, B, s);
    // scenario-major outputs: each wave writes its scenario's contiguous records
    store_record<P>(rho + s * (3 * N), w.rho(), 3 * N, l);
    store_record<P>(U_old + s * N, w.Uold(), N, l);
    store_record<P>(U + s * N, w.U(), N, l);
    store_record<P>(x_pred + s * (2 * (N + 1)), w.xp(), 2 * (N + 1), l);
    {
        double n0, n1;
        plant_step<GEN>(pb, scn_coef(pb, w), x0, x1, w.U()[0], n0, n1, pb.g.first_id + s, pb.g.k0);
        if (is16(x_next)) {
            if (l == 0) *reinterpret_cast<double2*>(x_next + 2 * s) = make_double2(n0, n1);
        } else if (l < 2) {
            x_next[2 * s + l] = l ? n1 : n0;
        }
    }
    if (l == 0) {
        exitflag[s] = flag;
        inner_iters[s] = its;
    }
    if (active_ws)
        for (int e = l; e < 2 * (N + 1); e += P) active_ws[s * (2 * (N + 1)) + e] = w.cand()[e];
    NTM_STAMPS_FLUSH();
}

template <int P, int NN, bool FAR = ws_far(NN)>
__global__ __launch_bounds__(64, NTM_WAVES_PER_EU_P(P, NN, FAR)) void k_mpc_run(Prob pb, int64_t B, int k_sim, const double* __restrict__ x0v,
                                                double* xk, double* uk, double* Uk, double* wpred,
                                                int32_t* exitflag, int32_t* inner_iters) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int G = 64 / P;
    const int g = threadIdx.x / P, l = threadIdx.x % P;
    const int64_t s = xcd_swizzle(blockIdx.x, gridDim.x) * G + g;
    const int N = NN > 0 ? NN : pb.N;
    if (s >= B) return;
    char* sbase = smem + g * ws_bytes(N, FAR);
    if constexpr (static_lds<P, NN>()) {
        __shared__ __attribute__((aligned(16))) char smem_s[ws_bytes(NN > 0 ? NN : 1, FAR)];
        sbase = smem_s;
    }
    auto w = ws_carve<NN, true, FAR>(sbase, N, &pb, s);
    double x0 = x0v[2 * s], x1 = x0v[2 * s + 1];
    if (l < 2) w.cand()[l * (N + 1) + N] = -1;
    scn_store(pb, w, pb.g.first_id + s, l);           // this scenario's plasma (generator)
    NTM_WSYNC();
    {   // Rho = repmat(rho(x0), 1, N) (NTM_MPC_Sim.m:63-65); Uold = +inf (D14)
        double r1, r2, r3;
        rho_eval(scn_coef(pb, w), x0, x1, r1, r2, r3);
        if (l < N) {
            w.rho()[3 * l] = r1;
            w.rho()[3 * l + 1] = r2;
            w.rho()[3 * l + 2] = r3;
            w.Uold()[l] = kInf;
        }
        NTM_WSYNC();
    }
    if (xk && l == 0) { xk[s * 2 * (k_sim + 1)] = x0; xk[s * 2 * (k_sim + 1) + 1] = x1; }
    for (int kk = 0; kk < k_sim; ++kk) {
        int its;
        int flag = mpc_step_dev<P>(pb, w, x0, x1, l, &its, B, s);
        if (Uk && l < N) Uk[(s * k_sim + kk) * N + l] = w.U()[l];
        if (wpred) for (int i = l; i <= N; i += P) wpred[(s * k_sim + kk) * (N + 1) + i] = w.xp()[2 * i];
        double n0, n1;
        plant_step<true>(pb, scn_coef(pb, w), x0, x1, w.U()[0], n0, n1, pb.g.first_id + s, pb.g.k0 + kk);
        if (l == 0) {
            if (uk) uk[s * k_sim + kk] = w.U()[0];
            if (exitflag) exitflag[s * k_sim + kk] = flag;
            if (inner_iters) inner_iters[s * k_sim + kk] = its;
            if (xk) { xk[s * 2 * (k_sim + 1) + 2 * kk + 2] = n0; xk[s * 2 * (k_sim + 1) + 2 * kk + 3] = n1; }
        }
        x0 = n0;
        x1 = n1;
        NTM_WSYNC();
    }
}

}  // namespace

// Launchers of one horizon's one-wave-per-scenario kernels (grid of one 64-lane
// block per scenario, lds bytes each), instantiated by the translation unit that
// owns that horizon (ntm_n20.hip, ntm_n50.hip: each sets its own LDS batch size).
// Internal linkage: two translation units that build the same horizon with
// different settings (ntm_n50.hip and ntm_n50m3.hip) instantiate these templates
// with the same arguments, and external (COMDAT) instances would be folded into
// one of the two builds at link time
namespace {
template <typename K>
hipError_t ntm_lds_opt_in(K kern, size_t lds) {
    if (lds <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds);
}
template <int NN, bool FAR>
hipError_t ntm_launch_step_v(const ntm::Prob& pb, int64_t B, const double* x_k, double* rho, double* U_old, double* U,
                             double* x_pred, double* x_next, int32_t* exitflag, int32_t* inner_iters,
                             int32_t* active_ws, size_t lds, hipStream_t st) {
    const bool gen = pb.g.phys_on || pb.g.dist_on;     // the generator's build only when it is used
    if (static_lds<64, NN>()) lds = 0;                 // the workspace is the kernel's static LDS
    hipError_t e = gen ? ntm_lds_opt_in(k_mpc_step<64, NN, true, FAR>, lds)
                       : ntm_lds_opt_in(k_mpc_step<64, NN, false, FAR>, lds);
    if (e != hipSuccess) return e;
    if (B <= 0) return hipSuccess;
    if (gen)
        hipLaunchKernelGGL((k_mpc_step<64, NN, true, FAR>), dim3((unsigned)B), dim3(64), lds, st, pb, B, x_k, rho,
                           U_old, U, x_pred, x_next, exitflag, inner_iters, active_ws);
    else
        hipLaunchKernelGGL((k_mpc_step<64, NN, false, FAR>), dim3((unsigned)B), dim3(64), lds, st, pb, B, x_k, rho,
                           U_old, U, x_pred, x_next, exitflag, inner_iters, active_ws);
    return hipGetLastError();
}
template <int NN, bool FAR>
hipError_t ntm_launch_run_v(const ntm::Prob& pb, int64_t B, int k_sim, const double* x0, double* xk, double* uk,
                            double* Uk, double* wpred, int32_t* exitflag, int32_t* inner_iters, size_t lds,
                            hipStream_t st) {
    if (static_lds<64, NN>()) lds = 0;                 // the workspace is the kernel's static LDS
    hipError_t e = ntm_lds_opt_in(k_mpc_run<64, NN, FAR>, lds);
    if (e != hipSuccess) return e;
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_mpc_run<64, NN, FAR>), dim3((unsigned)B), dim3(64), lds, st, pb, B, k_sim, x0, xk, uk, Uk,
                       wpred, exitflag, inner_iters);
    return hipGetLastError();
}
}  // namespace
// One translation unit per (horizon, layout): ntm_n20.hip (far), ntm_n20near.hip (the
// all-LDS N = 20 build for small batches, its own batch settings), ntm_n50.hip (far,
// modes 0-2) and ntm_n50m3.hip (far, input-rate rows: mode 3)
#define NTM_DECLARE_LAYOUT_LAUNCHERS(NAME)                                                                         \
    hipError_t ntm_launch_step_##NAME(const ntm::Prob& pb, int64_t B, const double* x_k, double* rho,             \
                                      double* U_old, double* U, double* x_pred, double* x_next, int32_t* exitflag, \
                                      int32_t* inner_iters, int32_t* active_ws, size_t lds, hipStream_t st);       \
    hipError_t ntm_launch_run_##NAME(const ntm::Prob& pb, int64_t B, int k_sim, const double* x0, double* xk,     \
                                     double* uk, double* Uk, double* wpred, int32_t* exitflag,                     \
                                     int32_t* inner_iters, size_t lds, hipStream_t st);
#define NTM_DEFINE_LAYOUT_LAUNCHERS(NAME, NNV, FARV)                                                               \
    hipError_t ntm_launch_step_##NAME(const ntm::Prob& pb, int64_t B, const double* x_k, double* rho,             \
                                      double* U_old, double* U, double* x_pred, double* x_next, int32_t* exitflag, \
                                      int32_t* inner_iters, int32_t* active_ws, size_t lds, hipStream_t st) {      \
        return ntm_launch_step_v<NNV, FARV>(pb, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters,     \
                                            active_ws, lds, st);                                                   \
    }                                                                                                              \
    hipError_t ntm_launch_run_##NAME(const ntm::Prob& pb, int64_t B, int k_sim, const double* x0, double* xk,     \
                                     double* uk, double* Uk, double* wpred, int32_t* exitflag,                     \
                                     int32_t* inner_iters, size_t lds, hipStream_t st) {                           \
        return ntm_launch_run_v<NNV, FARV>(pb, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, lds, st);  \
    }
NTM_DECLARE_LAYOUT_LAUNCHERS(n20)
NTM_DECLARE_LAYOUT_LAUNCHERS(n20near)
NTM_DECLARE_LAYOUT_LAUNCHERS(n20near1w)
NTM_DECLARE_LAYOUT_LAUNCHERS(n50)
NTM_DECLARE_LAYOUT_LAUNCHERS(n50m3)

// ntm_device.h — device-side building blocks of the batched LPV-MPC hot path
// (gfx950 / CDNA4).  One scenario is owned by a GROUP of P lanes of a wave
// (P = 16, 32 or 64; 64/P scenarios per wave).  Lane l of a group owns index
// l of every length-N vector (decision variable u_l, prediction step l).
// All per-scenario matrices live in the group's slice of LDS; cross-lane
// traffic is LDS broadcast reads plus ds_bpermute shuffles inside the group.
// Every control decision is a group reduction, so control flow is
// group-uniform and the 64/P groups of a wave may diverge freely.
//
// Reference map (file:line of the MATLAB reference):
//   rho_eval          rho1.m:2, rho2.m:2, rho3.m:2-3
//   lift_phase        A.m:2, B.m:2, Rho_to_PhiGammaLambda.m:17-52 (CANON D4/D6)
//   cost_phase        NTM_MPC_Sim.m:67-73, 120-121 (CANON D8/D12)
//   StructRows        getWLc.m:9-59 rows, never materialised (implicit rows)
//   gi_solve          quadprog call NTM_MPC_Sim.m:97 (Goldfarb-Idnani)
//   rollout_phase     NTM_MPC_Sim.m:110-117, 123-127
//   plant_phase       NTM_MPC_Sim.m:130 (CANON D13)
//
// Every phase is __forceinline__: left to its heuristics the inliner outlines
// whichever phase crosses its size threshold, and an outlined phase is a real
// call on gfx950 (the Prob and WS references copied to scratch, the caller's
// live VGPRs saved around it): 15.9 -> 14.7 ms per step-batch at B=1e5, N=20
// once everything was inlined again.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ntm_mpc.h"

namespace ntm {

// ---------------------------------------------------------------------------
// launch-constant problem description (derived on the host, see ntm_capi.hip)
// ---------------------------------------------------------------------------
struct Coef {
    double a11c;    // (4/3)(kappa rs/(0.82 tau_r)) Ts           A.m:2
    double za3;     // zeta * a^3 (D19, divides rho2*Ts)         A.m:2
    double a22;     // 1 - Ts/tau_E                              A.m:2
    double bc;      // kappa Ts eta_CD / w_dep                   B.m:2
    double C1, C2;  // NTM_MPC_Sim.m:37
    double wmarg2;  // w_marg^2                                  rho1.m:2
    double wdep;    // w_dep                                     rho3.m:2
    double Ts;
    int rho1_sq;    // D18 switch
};

// Scenario generator (ntm_ctx_set_scenarios): per-scenario plasma parameters
// and per-step plant disturbances, counter-based on (seed, global scenario id,
// time index), so any sharding or batching reproduces the same realisations.
struct Gen {
    uint64_t seed;
    int64_t first_id;   // global id of the launch's scenario 0
    int k0;             // time index of the launch's first plant step
    int dist_on;        // sigma_w or sigma_omega non-zero
    int phys_on;        // a parameter spread non-zero
    double sw, so;      // disturbance standard deviations (w [m], omega [rad/s])
    double sj, sd;      // j_BS / w_dep spreads
    // host-computed pieces of NTM_MPC_Sim.m:24,37 and B.m:2 the per-scenario
    // C1 and b coefficient are rebuilt from (same expression order as make_prob)
    double kTs, wsat, den, jbs, kte, wdep;
};

struct Prob {
    Coef k;
    int N, i_sim, mode, flags;
    double xmin[2], xmax[2], umin, umax, Q[4], r[2], eps;
    double du;        // input-rate bound (NTM_MODE_FULL_DU)
    int32_t* stats;  // optional per-scenario counters (4 x B, SoA): QP solves,
                      // GI iterations, final active rows, general (state) active rows
    Gen g;
    double* far;      // far workspace (HBM, far_doubles(N) per scenario) of the kernels
                      // whose WS keeps J/R out of LDS (ws_far); null otherwise
    double Ru;        // input weight (ABI v5): G = 2 Gamma' Om Gamma + 2 Ru I; read by the
                      // generic (NN = 0) kernels only, the host sends Ru != 0 there (ru_on);
                      // last, so the specialised kernels' argument layout is unchanged
};

constexpr double kInf = __builtin_huge_val();

// ---------------------------------------------------------------------------
// Counter-based scenario generator (host and device share this code, so the
// library's host-side sampler ntm_scenario_sample returns the device's values)
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// uniform [0, 1) from (seed, global scenario id, time index k, channel ch < 256)
__host__ __device__ __forceinline__ double gen_u01(uint64_t seed, int64_t sid, uint32_t k, uint32_t ch) {
    uint64_t h = splitmix64(seed ^ 0xD1B54A32D192ED03ull);
    h = splitmix64(h ^ (uint64_t)sid);
    h = splitmix64(h ^ (((uint64_t)k << 8) | ch));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}
// unit-variance, zero-mean Irwin-Hall(4) sample (bounded at +-2 sqrt(3)); only
// + and * so host and device agree bit for bit.  Channel c uses sub-channels 4c..4c+3.
__host__ __device__ __forceinline__ double gen_normal(uint64_t seed, int64_t sid, uint32_t k, uint32_t c) {
    double s = gen_u01(seed, sid, k, 4 * c);
    s = s + gen_u01(seed, sid, k, 4 * c + 1);
    s = s + gen_u01(seed, sid, k, 4 * c + 2);
    s = s + gen_u01(seed, sid, k, 4 * c + 3);
    return (s - 2.0) * 1.7320508075688772;
}
constexpr uint32_t kGenParamK = 0xFFFFFFFFu;   // time index of the per-scenario parameters
// per-scenario factor 1 + spread (2u - 1) of parameter channel c (0 j_BS, 1 w_dep)
// (an explicit fused multiply-add: compilers may or may not contract 1 + a b, so the
// generator fixes the rounding itself and every implementation agrees bit for bit)
__host__ __device__ __forceinline__ double gen_factor(uint64_t seed, int64_t sid, uint32_t c, double spread) {
    return fma(spread, 2.0 * gen_u01(seed, sid, kGenParamK, c) - 1.0, 1.0);
}
// scenario sid's plasma (j_BS, w_dep) into the coefficients that depend on them:
// C1 (NTM_MPC_Sim.m:37), the B.m:2 gain and rho3's w_dep (rho3.m:2)
__host__ __device__ __forceinline__ void gen_apply_physics(Prob& p, int64_t sid) {
    const Gen& g = p.g;
    const double jbs = g.jbs * gen_factor(g.seed, sid, 0, g.sj);
    const double wdep = g.wdep * gen_factor(g.seed, sid, 1, g.sd);
    p.k.C1 = -4.0 / 3.0 * (g.kTs * jbs * g.wsat) / g.den;
    p.k.bc = g.kte / wdep;
    p.k.wdep = wdep;
}


// 1/sqrt(x) for x > 0: v_rsq_f64 plus two Newton steps (full fp64 accuracy;
// the pivots of the small Cholesky factorisations sit on their sequential
// critical path, where the IEEE sqrt + division expansions cost ~25 dependent ops)
__device__ __forceinline__ double rsqrt_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = fma(y, fma(-h * y, y, 0.5), y);
    y = fma(y, fma(-h * y, y, 0.5), y);
    return y;
}

// Trace build only (make trace NTM_DEBUG_SCEN=s): printf GI's iterations for
// one scenario.  The production library compiles every trace away.
#ifdef NTM_DEBUG_SCEN
__shared__ int ntm_trace_grp;   // group (of this one-wave block) that owns the traced scenario
#define NTM_TRACE_SET(s, g, l)                                                  \
    do {                                                                        \
        if (threadIdx.x == 0) ntm_trace_grp = -1;                               \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");                 \
        __builtin_amdgcn_wave_barrier();                                        \
        if ((l) == 0 && (s) == NTM_DEBUG_SCEN) ntm_trace_grp = (g);             \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");                 \
        __builtin_amdgcn_wave_barrier();                                        \
    } while (0)
#define NTM_TRACE(...) \
    do { if (ntm_trace_grp == (int)((threadIdx.x & 63) / P) && l == 0) printf(__VA_ARGS__); } while (0)
#else
#define NTM_TRACE_SET(s, g, l) (void)0
#define NTM_TRACE(...) (void)0
#endif

// Diagnostic build only (-DNTM_STAMPS): per-phase s_memtime cycle totals,
// summed over waves into ntm_stamps[] (read with ntm_debug_stamps).  The
// production library compiles every stamp away.
#define NTM_NSTAMPS 104
#ifdef NTM_STAMPS
extern __device__ unsigned long long ntm_stamps[NTM_NSTAMPS];
__shared__ unsigned long long ntm_lds_stamps[NTM_NSTAMPS];   // per block (= per wave), flushed once
#define NTM_T0(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define NTM_ACC(i, v)                                                                   \
    do {                                                                                \
        unsigned long long t1_ = __builtin_amdgcn_s_memtime();                         \
        if ((threadIdx.x & 63) == 0) ntm_lds_stamps[i] += t1_ - (v);                   \
        v = t1_;                                                                        \
    } while (0)
#define NTM_CNT(i) \
    do { if ((threadIdx.x & 63) == 0) ntm_lds_stamps[i] += 1ull; } while (0)
#define NTM_STAMPS_INIT() \
    do { for (int i_ = threadIdx.x; i_ < NTM_NSTAMPS; i_ += blockDim.x) ntm_lds_stamps[i_] = 0; __syncthreads(); } while (0)
#define NTM_STAMPS_FLUSH() \
    do { __syncthreads(); for (int i_ = threadIdx.x; i_ < NTM_NSTAMPS; i_ += blockDim.x) atomicAdd(&ntm_stamps[i_], ntm_lds_stamps[i_]); } while (0)
#else
#define NTM_T0(v) (void)0
#define NTM_ACC(i, v) (void)0
#define NTM_CNT(i) (void)0
#define NTM_STAMPS_INIT() (void)0
#define NTM_STAMPS_FLUSH() (void)0
#endif
enum { ST_LIFT, ST_COST, ST_SCALE, ST_CAND, ST_REGRAM, ST_GI, ST_POLISH, ST_ROLL, ST_GI_FACT, ST_GI_CHECK,
       ST_GI_DIR, ST_GI_ADD, ST_GI_DROP, CN_CHECK, CN_CAND, CN_HIT,
       ST_P_CLASS, ST_P_GRAM, ST_P_CHOL, ST_P_SCHUR, ST_P_BWD, ST_P_KKT, CN_REPAIR, CN_GIRUN,
       ST_S_E, ST_S_Y, ST_S_K, ST_S_CHOL, ST_S_SOLVE, CN_TRY_EARLY, CN_FAIL_EARLY, CN_FAIL_LATE,
       CN_FAIL_IT1, CN_FAIL_IT2, CN_GI_IT1, CN_GI_IT2, CN_GI_LATE, CN_TRY_IT1, CN_TRY_IT2, CN_WARM_TRY, CN_WARM_OK, CN_WARM_DEP, CN_WARM_NEG, CN_WARM_FULL, CN_ALT_TRY, CN_ALT_HIT,
       ST_K_Y, ST_K_CHK, ST_K_GRAD, ST_K_MU, ST_K_SUB, ST_C_A, ST_C_B, ST_C_Y, ST_C_SQ,
       ST_SC_COL, ST_SC_ROW, ST_SC_END, ST_L_COEF, ST_L_LOOP, CN_CYC_HIT, CN_CYC_SKIP,
       CN_FK_DUAL, CN_FK_PRIMAL, CN_FK_SING, CN_FK_BOTH, ST_GI_WARM,
       CN_CDP_DROP, CN_CDP_RES, CN_CDP_PART, CN_CDP_DIR, CN_CDP_GI,
       CN_CDPX_SING0, CN_CDPX_SING1, CN_CDPX_BUDGET, CN_CDPX_DIR, CN_CDPX_NOVIOL, CN_CDPX_FULLDUAL, CN_CDPX_TINF,
       CN_BORD_K0, CN_BORD_K1, CN_BORD_K2, CN_BORD_K3, CN_BORD_K4P, CN_SQ_K0, CN_SQ_K1, CN_SQ_K2, CN_SQ_COLL,
       CN_CDPX_NAN, CN_NAN_BORD, CN_NAN_K0, CN_NAN_K1, CN_NAN_K2, CN_NAN_COLL, CN_NAN_COLL2, CN_NAN_PRIMFAIL,
       CN_NAN_V, CN_BX_O1, CN_BX_O2, CN_BX_O3P, CN_BX_NEG, CN_BX_NOCLASS, CN_CDP_SKIP, CN_CDP_SKIPDIR };
constexpr double kDepTol = 1e-8;   // GI linear-dependence threshold (oracle GI_DEP_TOL)
#ifndef NTM_MAX_NT
#define NTM_MAX_NT 32
#endif
constexpr int kMaxNT = NTM_MAX_NT; // explicit R^{-1} in GI up to this horizon (WS::useT)
#ifndef NTM_REPAIRS
#define NTM_REPAIRS 8
#endif
constexpr int kRepairs = NTM_REPAIRS;
// NTM_CDP=1: a failed candidate continues on Goldfarb-Idnani's dual path with certified
// re-solves (qp_phase); up to N + kCdpExtra re-solves before GI itself takes over
#ifndef NTM_CDP
#define NTM_CDP 1
#endif
#ifndef NTM_CDP_EXTRA
#define NTM_CDP_EXTRA 8
#endif
constexpr int kCdpExtra = NTM_CDP_EXTRA;
#ifndef NTM_SPLIT_SCALE
#define NTM_SPLIT_SCALE 1
#endif
#ifndef NTM_SPLIT_FAR
#define NTM_SPLIT_FAR 0
#endif
#ifndef NTM_SPLIT_PRAGMA
#define NTM_SPLIT_PRAGMA NTM_CHUNK_PRAGMA
#endif
// The re-solve's Gamma passes split over idle lanes (gamma_rows_split /
// gamma_col_split; N = 20): bit 0 the row passes (Gamma U_B, the k = 1 line's
// Gamma U_0 and Gamma D Z, the certificate's Gamma U), bit 1 the certificate's
// gradient column pass.  NTM_SPLIT_CERT for the all-LDS build, _FAR for the far one
#ifndef NTM_SPLIT_CERT
#define NTM_SPLIT_CERT 0
#endif
#ifndef NTM_SPLIT_CERT_FAR
#define NTM_SPLIT_CERT_FAR 0
#endif
// the dual path's skip of a row whose A + {p} end point is non-finite (long horizons)
#ifndef NTM_CDP_SKIP
#define NTM_CDP_SKIP 1
#endif
#ifndef NTM_FUSE_LOCAL_E
#define NTM_FUSE_LOCAL_E 0 // 1: the fused column sums run the free-response recursion on every lane
#endif
#ifndef NTM_SUB_PRESCALE
#define NTM_SUB_PRESCALE 0 // 1: long horizons, echelon substitutions on accumulators scaled by 1/E[l][l] (slower)
#endif
#ifndef NTM_MU_AHEAD
#define NTM_MU_AHEAD 0     // long horizons: steps ahead the multipliers' back substitution loads E (0: none)
#endif
#ifndef NTM_SUB_AHEAD
#define NTM_SUB_AHEAD 1    // long horizons: steps ahead the echelon forward substitution loads E
#endif
#ifndef NTM_SUB_LANEIDX
#define NTM_SUB_LANEIDX 0  // 1: the certificate's sparse pass takes rows and z by readlane (long horizons;
#endif                     // on in the mode-3 TU: 76.9 -> 76.3 ms, while mode 2 ran 64.9 -> 65.6 ms)
#ifndef NTM_E_LANEIDX
#define NTM_E_LANEIDX 1    // row-per-lane E build: pivot columns' variables and D_j by readlane
#endif
#ifndef NTM_CY_LATE
#define NTM_CY_LATE 1      // long horizons: Gamma U_B at an echelon set's general rows only (polish_compact)
#endif
#ifndef NTM_CDP_SKIPDIR
#define NTM_CDP_SKIPDIR 1  // long horizons: no violated row but skipped ones -> the last one's dual-only step
#endif
#ifndef NTM_CDP_HINT
#define NTM_CDP_HINT 1
#endif
#ifndef NTM_BOX_REPAIRS
#define NTM_BOX_REPAIRS 16
#endif
constexpr int kBoxRepairs = NTM_BOX_REPAIRS;   // box-only QPs: single-row exchanges before GI (qp_phase)   // also at N = 50: 16 / 32 were no faster in mode 2, 6% / 10% slower in mode 3
// A constant row (Lin_i = 0: the x_0 rows of getWLc, state rows Gamma doesn't
// reach) is violated when b_i < -kConstTol (D22, oracle CONST_ROW_TOL): the same
// absolute 1e-9 the KKT certificate allows on a unit-scale row.  An exact test
// turned a state that the plant step leaves one ulp outside a bound the
// previous plan held it at (x_{k+1} = xmin - ulp) into an infeasible QP.
constexpr double kConstTol = 1e-9;
constexpr int kRowMulti = 256;     // WS::rinfo flag: the state row has two or more non-zeros
constexpr int kGiWarmRejected = 100;   // gi_solve: the warm-start set was not dual feasible (caller reruns cold)

// Terms per batch of the LDS contractions (loads issued ahead of their uses);
// a translation unit may set its own (ntm_n50.hip)
#ifndef NTM_CH
#define NTM_CH 4
#endif
// Unroll count of the CH-batched chunk loops: empty (the compiler's choice, full
// unrolling at the BASELINE horizons) unless a build sets NTM_CHUNK_UNROLL
#define NTM_STR_(x) #x
#define NTM_STR(x) NTM_STR_(x)
#ifdef NTM_CHUNK_UNROLL
#define NTM_CHUNK_PRAGMA _Pragma(NTM_STR(unroll NTM_CHUNK_UNROLL))
#else
#define NTM_CHUNK_PRAGMA
#endif

#define NTM_WSYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
    } while (0)

// ---------------------------------------------------------------------------
// group collectives (width-P segments of the 64-lane wave)
//
// Butterflies run on DPP / permlane VALU ops, not ds_bpermute: quad_perm
// (xor 1, xor 2), row_half_mirror (pairs the quads of an 8-lane group),
// row_mirror (pairs the 8-lane halves of a row), v_permlane16_swap (pairs
// the 16-lane rows of a 32-lane group) and v_permlane32_swap (pairs the wave
// halves).  Every pairing step combines the two operands symmetrically, so
// each lane of a group ends with the bit-identical result and every control
// decision taken on it stays group-uniform.  Callers must be in
// group-uniform control flow (all P lanes active).
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    int2 a = __builtin_bit_cast(int2, v);
    a.x = __builtin_amdgcn_update_dpp(0, a.x, CTRL, 0xF, 0xF, false);
    a.y = __builtin_amdgcn_update_dpp(0, a.y, CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, a);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }

// (lower-row value, upper-row value) of a 16-lane (S=16) or 32-lane (S=32) pairing, same in both partners
template <int S>
__device__ __forceinline__ void pair_d(double v, double& lo, double& hi) {
    int2 a = __builtin_bit_cast(int2, v);
    int2 x, y;
    if constexpr (S == 16) {
        auto r0 = __builtin_amdgcn_permlane16_swap(a.x, a.x, false, false);
        auto r1 = __builtin_amdgcn_permlane16_swap(a.y, a.y, false, false);
        x.x = r0[0]; x.y = r1[0]; y.x = r0[1]; y.y = r1[1];
    } else {
        auto r0 = __builtin_amdgcn_permlane32_swap(a.x, a.x, false, false);
        auto r1 = __builtin_amdgcn_permlane32_swap(a.y, a.y, false, false);
        x.x = r0[0]; x.y = r1[0]; y.x = r0[1]; y.y = r1[1];
    }
    lo = __builtin_bit_cast(double, x);
    hi = __builtin_bit_cast(double, y);
}
template <int S>
__device__ __forceinline__ void pair_i(int v, int& lo, int& hi) {
    if constexpr (S == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        lo = r[0]; hi = r[1];
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        lo = r[0]; hi = r[1];
    }
}

// P = 64 (one scenario per wave): results of group reductions are identical
// in every lane; readfirstlane makes that visible to the compiler, so the
// branches they feed become scalar branches and loop counters live in SGPRs.
template <int P>
__device__ __forceinline__ int uni(int v) {
    if constexpr (P == 64) return __builtin_amdgcn_readfirstlane(v);
    else return v;
}
template <int P>
__device__ __forceinline__ double uni(double v) {
    if constexpr (P == 64) {
        int2 a = __builtin_bit_cast(int2, v);
        a.x = __builtin_amdgcn_readfirstlane(a.x);
        a.y = __builtin_amdgcn_readfirstlane(a.y);
        return __builtin_bit_cast(double, a);
    } else {
        return v;
    }
}
template <int P>
__device__ __forceinline__ double gsum(double v) {
    v = v + dpp_d<0xB1>(v);                       // quad_perm [1,0,3,2]
    v = v + dpp_d<0x4E>(v);                       // quad_perm [2,3,0,1]
    if constexpr (P >= 8) v = v + dpp_d<0x141>(v);   // row_half_mirror
    if constexpr (P >= 16) v = v + dpp_d<0x140>(v);  // row_mirror
    if constexpr (P >= 32) { double a, b; pair_d<16>(v, a, b); v = a + b; }
    if constexpr (P >= 64) { double a, b; pair_d<32>(v, a, b); v = a + b; }
    return uni<P>(v);
}
template <int P>
__device__ __forceinline__ double gmax(double v) {
    v = fmax(v, dpp_d<0xB1>(v));
    v = fmax(v, dpp_d<0x4E>(v));
    if constexpr (P >= 8) v = fmax(v, dpp_d<0x141>(v));
    if constexpr (P >= 16) v = fmax(v, dpp_d<0x140>(v));
    if constexpr (P >= 32) { double a, b; pair_d<16>(v, a, b); v = fmax(a, b); }
    if constexpr (P >= 64) { double a, b; pair_d<32>(v, a, b); v = fmax(a, b); }
    return uni<P>(v);
}
template <int P>
__device__ __forceinline__ int gmaxi(int v) {
    v = max(v, dpp_i<0xB1>(v));
    v = max(v, dpp_i<0x4E>(v));
    if constexpr (P >= 8) v = max(v, dpp_i<0x141>(v));
    if constexpr (P >= 16) v = max(v, dpp_i<0x140>(v));
    if constexpr (P >= 32) { int a, b; pair_i<16>(v, a, b); v = max(a, b); }
    if constexpr (P >= 64) { int a, b; pair_i<32>(v, a, b); v = max(a, b); }
    return uni<P>(v);
}
// broadcast lane `src` of the group (src group-uniform)
template <int P>
__device__ __forceinline__ double gbcast(double v, int src) {
    if constexpr (P == 64) {
        int2 a = __builtin_bit_cast(int2, v);
        a.x = __builtin_amdgcn_readlane(a.x, src);
        a.y = __builtin_amdgcn_readlane(a.y, src);
        return __builtin_bit_cast(double, a);
    } else {
        return __shfl(v, src, P);
    }
}

// argmin over (v, id) with ties broken towards the smaller id; carries two
// payload doubles.  Identical result in every lane of the group.
__device__ __forceinline__ void amin_sel(double& v, int& id, double& a, double& b, double ov, int oid, double oa,
                                         double ob) {
    if (ov < v || (ov == v && oid < id)) { v = ov; id = oid; a = oa; b = ob; }
}
template <int CTRL>
__device__ __forceinline__ void amin_dpp(double& v, int& id, double& a, double& b) {
    amin_sel(v, id, a, b, dpp_d<CTRL>(v), dpp_i<CTRL>(id), dpp_d<CTRL>(a), dpp_d<CTRL>(b));
}
template <int S>
__device__ __forceinline__ void amin_pair(double& v, int& id, double& a, double& b) {
    double v0, v1, a0, a1, b0, b1;
    int i0, i1;
    pair_d<S>(v, v0, v1);
    pair_i<S>(id, i0, i1);
    pair_d<S>(a, a0, a1);
    pair_d<S>(b, b0, b1);
    v = v0; id = i0; a = a0; b = b0;
    amin_sel(v, id, a, b, v1, i1, a1, b1);
}
template <int P>
__device__ __forceinline__ void gargmin(double& v, int& id, double& a, double& b) {
    amin_dpp<0xB1>(v, id, a, b);
    amin_dpp<0x4E>(v, id, a, b);
    if constexpr (P >= 8) amin_dpp<0x141>(v, id, a, b);
    if constexpr (P >= 16) amin_dpp<0x140>(v, id, a, b);
    if constexpr (P >= 32) amin_pair<16>(v, id, a, b);
    if constexpr (P >= 64) amin_pair<32>(v, id, a, b);
    v = uni<P>(v);
    id = uni<P>(id);
    a = uni<P>(a);
    b = uni<P>(b);
}
template <int P>
__device__ __forceinline__ void gargmin(double& v, int& id) {
    double a = 0.0, b = 0.0;
    gargmin<P>(v, id, a, b);
}

// ---------------------------------------------------------------------------
// L0 / L1: scheduling parameters and LPV coefficients
// ---------------------------------------------------------------------------
// rho1.m:2, rho2.m:2, rho3.m:2-3 (same operation order as the oracle)
__device__ __forceinline__ void rho_eval(const Coef& k, double w, double om,
                                         double& r1, double& r2, double& r3) {
    r1 = 1.0 / ((k.rho1_sq ? w * w : w) + k.wmarg2);
    r2 = (w * w) / om;
    double ws = w / k.wdep;
    r3 = (0.25 + 0.24 * ws) / (1 + 1.5 * ws + 0.43 * (ws * ws) + 0.64 * (ws * ws * ws));
}
// A.m:2 entries a11, a21 (a12 = 0, a22 = k.a22); B.m:2 as the column [b; 0] (D5)
__device__ __forceinline__ double coef_a11(const Coef& k, double r1) { return k.a11c * r1 + 1; }
__device__ __forceinline__ double coef_a21(const Coef& k, double r2) { return (r2 * k.Ts) / k.za3; }
__device__ __forceinline__ double coef_b(const Coef& k, double r3) { return k.bc * r3; }

// ---------------------------------------------------------------------------
// per-scenario LDS workspace (all offsets in doubles; see ws_doubles())
// ---------------------------------------------------------------------------
// NN > 0: horizon fixed at compile time (strides become immediates, loops
// unroll); NN == 0: runtime horizon (generic kernels).
// GEN: the kernel is built with the scenario generator (per-scenario plasma in
// the workspace, plant disturbances); without it those paths are compiled out
// (they cost the N=20 step kernel 2% through register allocation even when off)
//
// FAR (ws_far: N = 20 and N > 32): the J/R(/T) block (GI's factors and the
// bordered KKT factor) lives in a per-scenario HBM block (Prob::far, L2-resident
// while the wave runs) instead of LDS, and the echelon re-solve's sorted E moves
// to an LDS block of its own, packed lower triangular (row t at t(t+1)/2).  The
// certified re-solve of an echelon set, the common path, stays LDS-only; GI and
// the bordered elimination read and write HBM.  More scenarios fit a CU:
//   N = 50: 78.5 -> 47.9 KB, 3 scenarios per CU instead of 2 (one wave on each
//           of 3 SIMDs instead of 2; the kernel has the 512-register budget of
//           one wave per SIMD either way);
//   N = 20: 20.4 -> 12.0 KB, 12 scenarios per CU instead of 8, i.e. 3 waves per
//           SIMD, which the kernel is built for (168 VGPRs, NTM_WAVES_PER_EU).
// Neither pays without the occupancy: at 2 waves per SIMD the N = 20 kernel is 6%
// slower with its GI in HBM.  NTM_FAR_N20=0 builds the all-LDS N = 20 kernel.
#ifndef NTM_FAR_N20
#define NTM_FAR_N20 1
#endif
#ifndef NTM_FAR_JB
#define NTM_FAR_JB 0         // columns per trip of the bordered elimination's loads in the far block (0: two, loaded as used)
#endif
#ifndef NTM_GI_LDS
#define NTM_GI_LDS 3         // far layouts: GI's G~ / L (bit 0) and R (bit 1) in the LDS E block (WS::gr)
#endif
#ifndef NTM_FAR_COLMAJOR
#define NTM_FAR_COLMAJOR 0   // 1: J, T and the bordered factor column-major in the far block (slower)
#endif
__host__ __device__ constexpr bool ws_far(int NN) { return NN > 32 || (NTM_FAR_N20 && NN == 20); }
// The slim far layout (N = 20 far, round 5): 16 scenarios per CU (4 waves per SIMD,
// <= 10,240 B of LDS each) instead of 12.  What leaves LDS: the A/B coefficient
// arrays (each lane keeps its stage's in registers, broadcast by readlane in the
// lift), Phi and Lambda (the lift runs the free response e = Phi x_k + Lambda as a
// recursion of its own, one more lane; 2N of the old Phi stay as the re-solve's
// scratch), the hoisted V-space box (vlo / vhi, recomputed from D), and the
// diagonal reciprocals of the bordered factor and GI's Cholesky (ldi / kdi), which
// move to the far block with the rate-row norms (idun, mode 3 never runs here).
// The Om products are the identity (qi_on), so the certificate's Om y is y itself.
#ifndef NTM_SLIM20
#define NTM_SLIM20 1
#endif
#ifndef NTM_SLIM50
#define NTM_SLIM50 1
#endif
// The slim N = 50 layout (round 5): 4 scenarios per CU (one wave on each SIMD) instead
// of 3, <= 40,960 B each.  Besides the N = 20 slim changes (its Om is general: the
// certificate's Om y goes to the 2N of scratch), rho, U_old and the two carried
// active sets move to the far block (touched once or twice per LPV iteration).
__host__ __device__ constexpr bool ws_slim(int N, bool far) {
    return far && ((NTM_SLIM20 && N == 20) || (NTM_SLIM50 && N == 50));
}
__host__ __device__ constexpr bool slim_far(int N, bool far) { return ws_slim(N, far) && N == 50; }
// NTM_SLIM_AB: the slim layout keeps a11 / a21 in LDS after all (2N doubles, paid for by
// active-row flags for the 6N+4 getWLc rows only: mode 3 never runs on these kernels)
#ifndef NTM_SLIM_AB
#define NTM_SLIM_AB 1
#endif
__host__ __device__ constexpr int slim_ab(int N, bool far) { return NTM_SLIM_AB && N == 20 && ws_slim(N, far) ? 2 : 0; }

template <int NN, bool GEN = false, bool FAR = ws_far(NN)>
struct WS {
    static constexpr int kNN = NN;
    static constexpr bool kGen = GEN;
    static constexpr bool kFar = FAR;
    static constexpr bool kSlim = ws_slim(NN, FAR);
    int N_rt;
    double* base;
    double* far;       // kFar: this scenario's J/R block in HBM
    __device__ __forceinline__ int n() const { return NN > 0 ? NN : N_rt; }
    __device__ __forceinline__ int ldj() const { return n() | 1; }
    __device__ __forceinline__ int ldg() const { return 2 * n(); }
    // double offsets of each array (n() is launch-uniform, so these fold to scalar math)
    static constexpr int kAB = slim_ab(NN, FAR);           // kSlim: a11 / a21 (N each) in LDS
    static constexpr bool kSF = slim_far(NN, FAR);          // rho, U_old, cand in the far block
    static constexpr int kRL = kSF ? 0 : 3;                 // kSlim: rho's N-vectors in LDS
    __device__ __forceinline__ int oJ() const { return (kSlim ? kRL + 4 + kAB : 14) * n() + n() * (n() + 1); }
    __device__ __forceinline__ int oR() const { return oJ() + n() * ldj(); }
    // T = R^{-1} is kept for N <= kMaxNT only: at long horizons its N^2 doubles would
    // halve the scenarios per CU, and the dual direction falls back to back substitution.
    // The far layouts keep no T either: maintaining it in HBM (a column per add, a
    // Givens sweep and a row shift per drop) cost more than the back substitution
    // on R saves (N = 20, 3 waves per SIMD: 10.09 -> 9.99 ms per step-batch without it)
    __device__ __forceinline__ bool useT() const { return !kFar && n() <= kMaxNT; }
    __device__ __forceinline__ int oT() const { return oR() + (n() + 1) * ldj(); }
    // kFar: the E block (packed lower-triangular E, then 2(N+1) ints) replaces J/R/T in LDS
    __device__ __forceinline__ int oV() const {
        if constexpr (kFar) return oJ() + (n() * (n() + 1)) / 2 + (n() + 1);
        else return oT() + (useT() ? n() * ldj() : 0);   // vector block
    }
    __device__ __forceinline__ double* rho() const {                                  // 3N (3xN col-major)
        if constexpr (kSF) return far + n() * ldj() + (n() + 1) * ldj() + 3 * n();
        else return base;
    }
    // (kSlim: no a11 / a21 / bb / Lam, Phi is 2N of scratch; never called there)
    __device__ __forceinline__ double* a11() const { return base + 3 * n(); }         // n()
    __device__ __forceinline__ double* a21() const { return base + 4 * n(); }         // n()
    __device__ __forceinline__ double* bb() const { return base + 5 * n(); }          // n()
    __device__ __forceinline__ double* Phi() const { return base + (kSlim ? kRL + kAB : 6) * n(); }   // 4N Phi_i (2x2 col-major)
    __device__ __forceinline__ double* Lam() const { return base + 10 * n(); }        // 2N
    __device__ __forceinline__ double* e() const { return base + (kSlim ? kRL + 2 + kAB : 12) * n(); }    // 2N free response
    // Gamma, block-lower-triangular and packed by column: column j holds rows 2j..2N-1
    __device__ __forceinline__ double* Gt() const { return base + (kSlim ? kRL + 4 + kAB : 14) * n(); }   // n()(n()+1)
    __device__ __forceinline__ int gidx(int r, int j) const { return j * (2 * n() - j + 1) + r - 2 * j; }
    __device__ __forceinline__ double& gt(int r, int j) const { return Gt()[gidx(r, j)]; }   // r >= 2j
    __device__ __forceinline__ double* J() const {                                   // n() x ldj() row-major
        if constexpr (kFar) return far;
        else return base + oJ();
    }
    // R: n() rows x (n()+1) columns col-major; the polish keeps its Schur complement
    // K in the strict upper triangle: K(a, c), a >= c, at R[c + (a+1) ldj()]
    __device__ __forceinline__ double* R() const {
        if constexpr (kFar) return far + n() * ldj();
        else return base + oR();
    }
    // T = R^{-1} of the GI factorisation (upper triangular, row-major n() x ldj();
    // zero outside the leading q x q block), so the dual direction is a matvec
    __device__ __forceinline__ double* T() const {
        if constexpr (kFar) return far;   // never dereferenced: far layouts keep no T (useT)
        else return base + oT();
    }
    // element (r, c) of J (and of T) at J()[r jr() + c jc()]: row-major in LDS,
    // column-major in HBM (kFar), where the common access, each lane walking its own
    // row, is then one coalesced load per column instead of 64 cache lines
    static constexpr bool kCol = kFar && NTM_FAR_COLMAJOR;
    __device__ __forceinline__ int jr() const { return kCol ? 1 : ldj(); }
    __device__ __forceinline__ int jc() const { return kCol ? ldj() : 1; }
    // packed bordered KKT factor (rows 0..nt, row nt the right-hand side), entry
    // (r, c), c <= r, at J()[brow(r) + bcol(c, nt)]: row-major (row r at r(r+1)/2) in
    // LDS, column-major (column c at c(nt+1) - c(c-1)/2) in HBM, where a lane owns a
    // row and the elimination walks the columns
    __device__ __forceinline__ int brow(int r) const { return kCol ? r : (r * (r + 1)) / 2; }
    __device__ __forceinline__ int bcol(int c, int nt) const {
        return kCol ? c * (nt + 1) - (c * (c - 1)) / 2 - c : c;
    }
    // echelon re-solve: sorted E (entry (t, u), u <= t, at Ep()[eidx(t, u)]) and the
    // GI's triangular factor R (and, before it, the scaled Gram G~ and its Cholesky
    // factor L): element (i, j) at R()[i + j ldj()], or, in the far layouts
    // (kGiLds), in the LDS E block, which is dead while GI runs (the echelon
    // re-solve's sorted E is rebuilt by every re-solve): the lower triangle row-major
    // packed (row i at i(i+1)/2, so G~ / L rows are contiguous), the upper triangle
    // column-major packed in the same slots ((i, j) and (j, i) share one: the lower
    // triangle is dead once R is being built, the factor below R's subdiagonal is
    // never touched), and R's superdiagonal (i, i+1) apart after the triangle, so
    // that a drop's upper-Hessenberg subdiagonal (i+1, i) does not collide with it.
    // N(N+1)/2 + N-1 doubles <= the E block's N(N+1)/2 + N+1.  GI's back and forward
    // substitutions, adds and drops then run on LDS instead of the HBM far block
    // (J stays there)
    // (NTM_GI_LDS bit 0: G~ and L, bit 1: R; the two phases never overlap, so each
    // may live in either place)
    static constexpr bool kGiLdsL = FAR && (NTM_GI_LDS & 1);
    static constexpr bool kGiLds = FAR && (NTM_GI_LDS & 2);
    __device__ __forceinline__ int gio(int i, int j) const {
        if (i >= j) return (i * (i + 1)) / 2 + j;
        if (i == j - 1) return (n() * (n() + 1)) / 2 + i;
        return (j * (j + 1)) / 2 + i;
    }
    __device__ __forceinline__ double& gr(int i, int j) const {
        if constexpr (kGiLds) return Ep()[gio(i, j)];
        else return R()[i + j * ldj()];
    }
    __device__ __forceinline__ double& grL(int i, int j) const {   // lower triangle, i >= j
        if constexpr (kGiLdsL) return Ep()[(i * (i + 1)) / 2 + j];
        else return R()[i + j * ldj()];
    }
    // row i of the lower triangle (elements (i, 0..i) at stride grs())
    __device__ __forceinline__ double* grow(int i) const {
        if constexpr (kGiLdsL) return Ep() + (i * (i + 1)) / 2;
        else return R() + i;
    }
    __device__ __forceinline__ int grs() const { return kGiLdsL ? 1 : ldj(); }
    // row permutation / column owner ints (2(N+1)); in the J/R block unless kFar
    __device__ __forceinline__ double* Ep() const {
        if constexpr (kFar) return base + oJ();
        else return J();
    }
    __device__ __forceinline__ int eidx(int t, int u) const {
        if constexpr (kFar) return (t * (t + 1)) / 2 + u;
        else return t * ldj() + u;
    }
    __device__ __forceinline__ int* permi() const {
        if constexpr (kFar) return reinterpret_cast<int*>(base + oJ() + (n() * (n() + 1)) / 2);
        else return reinterpret_cast<int*>(R());
    }
    // 2N ints (in 2N doubles of space): per state row r, (last column j with
    // Gamma_rj != 0) + 1, plus kRowMulti if it has two or more non-zeros
    __device__ __forceinline__ int* rinfo() const { return reinterpret_cast<int*>(base + oV()); }
    // kSlim: the 2N rinfo ints take N doubles, and vlo / vhi / ldi / kdi / idun leave LDS
    static constexpr int kRi = kSlim ? 1 : 2;                // doubles of rinfo per N
    __device__ __forceinline__ double* F() const { return base + oV() + kRi * n(); }         // n()  F~
    __device__ __forceinline__ double* D() const { return base + oV() + (kRi + 1) * n(); }   // n()  Jacobi scaling
    __device__ __forceinline__ double* V() const { return base + oV() + (kRi + 2) * n(); }   // n()  scaled variables
    __device__ __forceinline__ double* d() const { return base + oV() + (kRi + 3) * n(); }   // n()
    __device__ __forceinline__ double* np() const { return base + oV() + (kRi + 4) * n(); }  // n()  GI normal
    __device__ __forceinline__ double* hv() const { return base + oV() + (kRi + 5) * n(); }  // n()  Householder / polish
    __device__ __forceinline__ double* Vb() const { return base + oV() + (kRi + 6) * n(); }  // n()  polish fixed (V)
    __device__ __forceinline__ double* Uf() const { return base + oV() + (kRi + 7) * n(); }  // n()  polish fixed (U)
    __device__ __forceinline__ double* uu() const { return base + oV() + (kRi + 8) * n(); }  // n()+1 multipliers
    __device__ __forceinline__ double* xp() const { return base + oV() + (kRi + 9) * n() + 1; }    // 2(n()+1) rollout
    __device__ __forceinline__ double* U() const { return base + oV() + (kRi + 11) * n() + 3; }    // n()
    static constexpr int kUo = kSF ? 0 : 1;                  // U_old's N-vector in LDS
    __device__ __forceinline__ double* Uold() const {                                              // n()
        if constexpr (kSF) return rho() + 3 * n();
        else return base + oV() + (kRi + 12) * n() + 3;
    }
    __device__ __forceinline__ double* dr() const { return base + oV() + (kRi + 12 + kUo) * n() + 3; }    // N: d masked to b < q (GI)
    __device__ __forceinline__ double* irn() const { return base + oV() + (kRi + 13 + kUo) * n() + 3; }   // 2N: 1/rn_r (0: const row)
    __device__ __forceinline__ double* ssg() const { return base + oV() + (kRi + 15 + kUo) * n() + 3; }   // N: sign of general row s
    // per-QP constants hoisted out of the solver loops (not kSlim: recomputed from D)
    __device__ __forceinline__ double* vlo() const { return base + oV() + (kRi + 17) * n() + 3; }   // N: umin/D_j
    __device__ __forceinline__ double* vhi() const { return base + oV() + (kRi + 18) * n() + 3; }   // N: umax/D_j
    // 1/L(k,k) (Cholesky), 1/K(k,k) (Schur), contiguous; 1/|D (e_i - e_{i-1})|: in the far block when kSlim
    __device__ __forceinline__ double* ldi() const {
        if constexpr (kSlim) return far + n() * ldj() + (n() + 1) * ldj();
        else return base + oV() + (kRi + 19) * n() + 3;
    }
    __device__ __forceinline__ double* kdi() const { return ldi() + n(); }
    __device__ __forceinline__ double* idun() const {
        if constexpr (kSlim) return ldi() + 2 * n();
        else return base + oV() + (kRi + 21) * n() + 3;
    }
    static constexpr int kVec = kSlim ? 17 + kUo : 24;        // N-vectors of the block (+ 3 + 3 scn)
    // this scenario's C1, B.m gain and w_dep (scenario generator; read only when pb.g.phys_on)
    __device__ __forceinline__ double* scn() const { return base + oV() + kVec * n() + 3; }
    __device__ __forceinline__ int* act() const { return reinterpret_cast<int*>(base + oV() + kVec * n() + 6); }
    __device__ __forceinline__ int* sidx() const { return act() + n() + 1; }
    static constexpr int kCL = kSF ? 0 : 2;                  // the carried sets' (N+1)-int tables in LDS
    __device__ __forceinline__ int* cand() const {                                   // 2(n()+1): last two active sets
        if constexpr (kSF) return reinterpret_cast<int*>(Uold() + n());
        else return act() + 2 * (n() + 1);
    }
    __device__ __forceinline__ int* fidx() const { return act() + (2 + kCL) * (n() + 1); }   // n()+1: free variables (polish)
    __device__ __forceinline__ int* srw() const { return act() + (3 + kCL) * (n() + 1); }    // n()+1: state row of general row s
    __device__ __forceinline__ unsigned char* fx() const {
        return reinterpret_cast<unsigned char*>(act() + (4 + kCL) * (n() + 1));
    }
    __device__ __forceinline__ unsigned char* aflag() const { return fx() + n(); }
};

__host__ __device__ constexpr int ldj_of(int N) { return N | 1; }
// the J/R block of a far layout, in HBM per scenario (no T: WS::useT)
__host__ __device__ constexpr int far_doubles(int N) {
    // + ldi, kdi, idun (slim); + rho, U_old and the carried sets' 2(N+1) ints (slim_far)
    return N * ldj_of(N) + (N + 1) * ldj_of(N) + (ws_slim(N, true) ? 3 * N : 0) +
           (slim_far(N, true) ? 4 * N + (N + 1) : 0);
}
__host__ __device__ constexpr int ws_doubles(int N, bool far = false) {
    // LDS: the E block (far), or J, R and (N <= kMaxNT) T
    const int jr = far ? (N * (N + 1)) / 2 + (N + 1) : (N <= kMaxNT ? 2 : 1) * N * ldj_of(N) + (N + 1) * ldj_of(N);
    const int rl = slim_far(N, far) ? 0 : 3, uo = slim_far(N, far) ? 0 : 1;
    return ws_slim(N, far) ? (rl + 4 + slim_ab(N, far)) * N + N * (N + 1) + jr + (17 + uo) * N + 6
                           : 14 * N + N * (N + 1) + jr + 24 * N + 6;
}
// workspace bytes with room for `rows` active-row flags: the structured rows of
// the MPC step are at most 8N+2 (getWLc 6N+4 plus 2(N-1) rate rows); a dense
// quadprog problem (k_qp) may carry more
__host__ __device__ constexpr int ws_bytes_rows(int N, int rows, bool far = false) {
    const int fmin = slim_ab(N, far) ? 6 * N + 4 : 8 * N + 4;      // (slim_ab: no rate rows)
    const int flags = rows > fmin ? rows : fmin;
    int b = ws_doubles(N, far) * 8 + (slim_far(N, far) ? 4 : 6) * (N + 1) * 4 + N + flags;   // ..., fx (N), aflag
    return (b + 15) & ~15;
}
__host__ __device__ constexpr int ws_bytes(int N, bool far = false) {
    return ws_bytes_rows(N, slim_ab(N, far) ? 6 * N + 4 : 8 * N + 4, far);
}
static_assert(!ws_slim(20, true) || 16 * ws_bytes(20, true) <= 160 * 1024, "slim N = 20: 16 scenarios per CU");
static_assert(!ws_slim(50, true) || 4 * ws_bytes(50, true) <= 160 * 1024, "slim N = 50: 4 scenarios per CU");

// s: the scenario's index in the launch (its far block, when the WS has one)
template <int NN, bool GEN = false, bool FAR = ws_far(NN)>
__device__ inline WS<NN, GEN, FAR> ws_carve(char* base, int N, const Prob* pb = nullptr, int64_t s = 0) {
    WS<NN, GEN, FAR> w;
    w.N_rt = N;
    w.base = reinterpret_cast<double*>(base);
    w.far = nullptr;
    if constexpr (FAR) w.far = pb->far + s * (int64_t)far_doubles(N);
    return w;
}

// The scenario's LPV coefficients: the launch constants, with C1, the B.m gain and
// w_dep taken from the workspace when the scenario generator varies the plasma
// (written once per launch by scn_store).  Keeping the launch constants in the
// kernel arguments matters: a copy of the whole Prob per scenario cost the N=20
// step kernel 100 B of scratch per lane and 20 more spilled SGPRs.
// The input weight R_u: its term 2 Ru I of the Hessian enters the
// Gram diagonal (scaling, GI's full G~, the re-solve's G~_FF), the echelon k = 1 line
// search and the certificate's gradient.  Compiled into the generic kernels only
// (ru_on): the specialised N = 10 / 20 / 50 kernels keep their register allocation,
// and the host dispatches a launch with Ru != 0 to the generic ones (as D4 / D6)
template <class W>
__device__ __forceinline__ constexpr bool ru_on() { return W::kNN == 0; }
template <class W>
__device__ __forceinline__ double ru_of(const Prob& pb) {
    if constexpr (ru_on<W>()) return pb.Ru;
    else return 0.0;
}
// The reference's stage weight is Q = I (NTM_MPC_Sim.m:59, Omega = blkdiag(Q, ...)).
// The specialised kernels (compile-time horizons) assume it, so their Om products
// are the identity (bit for bit what 1 x + 0 y gives for finite data) and the
// weight's four launch constants leave their scalar registers; a launch with any
// other Q runs on the generic kernels (host dispatch, like Ru and D4 / D6).
#ifndef NTM_QI_MAXN
#define NTM_QI_MAXN 32     // compile-time horizons up to this one assume Q = I (qi_on): N = 10, 20 (at
                           // N = 50 it cost 11% through register allocation, A/B on one box)
#endif
template <class W>
__device__ __forceinline__ constexpr bool qi_on() { return W::kNN > 0 && NTM_QI_MAXN >= W::kNN; }
template <bool QI>
struct OmQ {                       // x -> Q x for one stage's 2-vector
    double q00, q01, q10, q11;
    __device__ __forceinline__ explicit OmQ(const double* Q) {
        if constexpr (QI) { q00 = 1.0; q01 = 0.0; q10 = 0.0; q11 = 1.0; }
        else { q00 = Q[0]; q01 = Q[1]; q10 = Q[2]; q11 = Q[3]; }
    }
    __device__ __forceinline__ double o0(double x0, double x1) const {
        if constexpr (QI) return x0;
        else return q00 * x0 + q01 * x1;
    }
    __device__ __forceinline__ double o1(double x0, double x1) const {
        if constexpr (QI) return x1;
        else return q10 * x0 + q11 * x1;
    }
};
__device__ __forceinline__ bool gen_phys(const Prob& pb) { return pb.g.phys_on != 0; }
__device__ __forceinline__ bool gen_dist(const Prob& pb) { return pb.g.dist_on != 0; }
template <class W>
__device__ __forceinline__ Coef scn_coef(const Prob& pb, const W& w) {
    Coef k = pb.k;
    if (W::kGen && gen_phys(pb)) {
        k.C1 = w.scn()[0];
        k.bc = w.scn()[1];
        k.wdep = w.scn()[2];
    }
    return k;
}
template <class W>
__device__ __forceinline__ void scn_store(const Prob& pb, const W& w, int64_t gid, int l) {
    if (W::kGen && gen_phys(pb) && l == 0) {
        Prob q = pb;
        gen_apply_physics(q, gid);
        w.scn()[0] = q.k.C1;
        w.scn()[1] = q.k.bc;
        w.scn()[2] = q.k.wdep;
    }
}

// ---------------------------------------------------------------------------
// Batched LDS contractions.  The long masked fixed-trip loops below are LDS
// latency chains when the scheduler interleaves each load with its use (the
// 256-VGPR kernels leave it no room to hoist); these helpers issue CH rows of
// loads, fence the scheduler, then consume them, so one LDS round trip serves
// CH terms.  Same terms in the same order as the plain loops.  Loads of the
// tail chunk past n are skipped (zero), never read out of the workspace.
// ---------------------------------------------------------------------------
// sum_{imin <= i < n} a_i' Q b_i over 2-vectors stored at stride 2
template <int CH, class OM>
__device__ __forceinline__ double qdot_rows(const double* a, const double* b, int n, int imin, const OM& om) {
    double s = 0.0;
    NTM_CHUNK_PRAGMA
    for (int i0 = 0; i0 < n; i0 += CH) {
        double a0[CH], a1[CH], b0[CH], b1[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = i0 + u;
            const bool in = i < n;
            a0[u] = in ? a[2 * i] : 0.0;
            a1[u] = in ? a[2 * i + 1] : 0.0;
            b0[u] = in ? b[2 * i] : 0.0;
            b1[u] = in ? b[2 * i + 1] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = i0 + u;
            const double o0 = om.o0(b0[u], b1[u]);
            const double o1 = om.o1(b0[u], b1[u]);
            const double t = a0[u] * o0 + a1[u] * o1;
            s += (i >= imin && i < n) ? t : 0.0;
        }
    }
    return s;
}
// sum_{j < n} a[j sa] b[j sb] (strided LDS vectors)
template <int CH>
__device__ __forceinline__ double dot_batched(const double* a, int sa, const double* b, int sb, int n) {
    double y = 0.0;
    NTM_CHUNK_PRAGMA
    for (int j0 = 0; j0 < n; j0 += CH) {
        double x[CH], z[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int j = j0 + u;
            const bool in = j < n;
            x[u] = in ? a[j * sa] : 0.0;
            z[u] = in ? b[j * sb] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) y += x[u] * z[u];
    }
    return y;
}
// sum_{lo <= j < hi} a[j sa] b[j sb] (per-lane bounds; terms added in index order)
template <int CH>
__device__ __forceinline__ double dot_range(const double* a, int sa, const double* b, int sb, int lo, int hi) {
    double y = 0.0;
    NTM_CHUNK_PRAGMA
    for (int j0 = lo; j0 < hi; j0 += CH) {
        double x[CH], z[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int j = j0 + u;
            const bool in = j < hi;
            x[u] = in ? a[j * sa] : 0.0;
            z[u] = in ? b[j * sb] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) y += x[u] * z[u];
    }
    return y;
}
// s - sum_{lo <= j < hi} a[j sa] b[j sb], the terms subtracted one by one in index order
template <int CH>
__device__ __forceinline__ double sub_dot(double s, const double* a, int sa, const double* b, int sb, int lo, int hi) {
    NTM_CHUNK_PRAGMA
    for (int j0 = lo; j0 < hi; j0 += CH) {
        double x[CH], z[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int j = j0 + u;
            const bool in = j < hi;
            x[u] = in ? a[j * sa] : 0.0;
            z[u] = in ? b[j * sb] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) s -= x[u] * z[u];
    }
    return s;
}
// a[j] -= f b[j] for lo <= j < hi, the loads of CH entries issued ahead of their stores
template <int CH>
__device__ __forceinline__ void axpy_sub(double* a, const double* b, double f, int lo, int hi, int sa = 1) {
    NTM_CHUNK_PRAGMA
    for (int j0 = lo; j0 < hi; j0 += CH) {
        double x[CH], z[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int j = j0 + u;
            const bool in = j < hi;
            x[u] = in ? a[j * sa] : 0.0;
            z[u] = in ? b[j] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (j0 + u < hi) a[(j0 + u) * sa] = x[u] - f * z[u];
    }
}
// Gamma_r v restricted to j <= r/2 (row r of the packed block-lower-triangular Gamma)
template <int CH, class W>
__device__ __forceinline__ double gamma_row_dot(const W& w, int r, const double* v) {
    const int n = w.n(), jm = r >> 1;
    const double* gr = w.Gt() + r;                        // gt(r, j) = gr[gidx(0, j)]
    double y = 0.0;
    NTM_CHUNK_PRAGMA
    for (int j0 = 0; j0 < n; j0 += CH) {
        double g[CH], x[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int j = j0 + u;
            const bool in = j < n;
            g[u] = in ? gr[w.gidx(0, j)] : 0.0;
            x[u] = in ? v[j] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int j = j0 + u;
            y += (j <= jm ? g[u] : 0.0) * x[u];
        }
    }
    return y;
}

// Gamma_r v1 and Gamma_r v2 in one pass over row r (its loads shared)
template <int CH, class W>
__device__ __forceinline__ void gamma_row_dot2(const W& w, int r, const double* v1, const double* v2, double& y1,
                                               double& y2) {
    const int n = w.n(), jm = r >> 1;
    const double* gr = w.Gt() + r;
    y1 = 0.0;
    y2 = 0.0;
    NTM_CHUNK_PRAGMA
    for (int j0 = 0; j0 < n; j0 += CH) {
        double g[CH], x1[CH], x2[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int j = j0 + u;
            const bool in = j < n;
            g[u] = in ? gr[w.gidx(0, j)] : 0.0;
            x1[u] = in ? v1[j] : 0.0;
            x2[u] = in ? v2[j] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const double gm = (j0 + u <= jm) ? g[u] : 0.0;
            y1 += gm * x1[u];
            y2 += gm * x2[u];
        }
    }
}

// ---------------------------------------------------------------------------
// Row and column passes over Gamma split in two halves on otherwise idle lanes
// (compile-time horizons with 4N - 2H <= 64, H = ceil(N/2): N = 20), as the
// all-LDS build's scaling pass does (diag_scale_phase).  Row pass: lane l < 2N
// sums the j < H terms of row r = l; lane 2N <= l < 4N - 2H the j >= H terms of
// row r = l - 2N + 2H (the rows r >= 2H, the only ones that have such terms);
// row r's value, (first half) + (second half), ends on lane r.  Column pass:
// lane l < N takes stages i < H of column l, lane N + l stages i >= H; column
// l's value ends on lane l.  The wave runs H trips instead of N.
// ---------------------------------------------------------------------------
template <int P, class W>
__device__ __forceinline__ constexpr bool split_ok() {
    return P == 64 && W::kNN > 0 && 4 * W::kNN - 2 * ((W::kNN + 1) / 2) <= 64;
}
// (Gamma_r v_k for the NV vectors v_k) on lane r < 2N
template <int CH, int NV, class W>
__device__ __forceinline__ void gamma_rows_split(const W& w, const double* const (&v)[NV], double (&y)[NV], int l) {
    constexpr int NN = W::kNN, H = (NN + 1) / 2;
    const bool lo = l < 2 * NN, hi = !lo && l < 4 * NN - 2 * H;
    const int r = lo ? l : (hi ? l - 2 * NN + 2 * H : 0);
    const int jb = lo ? 0 : H, jm = r >> 1;
    const double* gr = w.Gt() + r;                        // gt(r, j) = gr[gidx(0, j)]
    double s[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) s[k] = 0.0;
    if (lo || hi) {
        NTM_SPLIT_PRAGMA
        for (int u0 = 0; u0 < H; u0 += CH) {
            double g[CH], x[NV][CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int j = jb + u0 + u;
                const bool in = u0 + u < H && j < NN;
                g[u] = in ? gr[w.gidx(0, j)] : 0.0;
#pragma unroll
                for (int k = 0; k < NV; ++k) x[k][u] = in ? v[k][j] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int j = jb + u0 + u;
                const double gm = (u0 + u < H && j <= jm) ? g[u] : 0.0;
#pragma unroll
                for (int k = 0; k < NV; ++k) s[k] += gm * x[k][u];
            }
        }
    }
    const int src = (l >= 2 * H && l < 2 * NN) ? l + 2 * NN - 2 * H : l;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const double s2 = __shfl(s[k], src & 63, 64);
        y[k] = (src != l) ? s[k] + s2 : s[k];
    }
}
// sum_{i >= l} Gamma_{2i,l} c_{2i} + Gamma_{2i+1,l} c_{2i+1} on lane l < N
template <int CH, class W>
__device__ __forceinline__ double gamma_col_split(const W& w, const double* c, int l) {
    constexpr int NN = W::kNN, H = (NN + 1) / 2;
    const bool lo = l < NN, hi = !lo && l < 2 * NN;
    const int col = lo ? l : (hi ? l - NN : 0);
    const int ib = lo ? 0 : H;
    const double* cl = w.Gt() + w.gidx(2 * col, col) - 2 * col;   // cl[r] = gt(r, col), r >= 2 col
    double s = 0.0;
    if (lo || hi) {
        NTM_SPLIT_PRAGMA
        for (int u0 = 0; u0 < H; u0 += CH) {
            double a0[CH], a1[CH], c0[CH], c1[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = ib + u0 + u;
                const bool in = u0 + u < H && i < NN;
                a0[u] = in ? cl[2 * i] : 0.0;
                a1[u] = in ? cl[2 * i + 1] : 0.0;
                c0[u] = in ? c[2 * i] : 0.0;
                c1[u] = in ? c[2 * i + 1] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = ib + u0 + u;
                const double t = a0[u] * c0[u] + a1[u] * c1[u];
                s += (u0 + u < H && i >= col && i < NN) ? t : 0.0;
            }
        }
    }
    const double s2 = __shfl(s, (l + NN) & 63, 64);
    return lo ? s + s2 : s;
}

// ---------------------------------------------------------------------------
// L2: lifted prediction  (Rho_to_PhiGammaLambda.m:17-52, CANON D4/D6)
// ---------------------------------------------------------------------------
// Literal-reference lift (D4 / D6; generic kernels only, the host dispatches any
// launch that sets these flags there): D6 takes A(rho_{i-j}) for Gamma_ij, i.e.
// the coefficient index i - j - 1 counted from 0 (Rho_to_PhiGammaLambda.m:32);
// D4 right-multiplies Phi_i = Phi_{i-1} A_i (:21).  Same arithmetic as
// oracle/ntm_oracle.c orc_lift.  Lane j < N runs Gamma's column j; lane 0 then
// runs Phi and Lambda.  Kept apart from lift_phase so that the specialised hot
// kernels compile exactly as before (folding the switches into lift_phase cost
// the N=20 kernel 72 B of scratch per lane although they are constant there).
template <int P, class W>
__device__ __forceinline__ void lift_literal(const Prob& pb, const W& w, const Coef& k, int l) {
    const int N = w.n();
    const bool d6 = (pb.flags & NTM_LITERAL_GAMMA_INDEX) != 0, d4 = (pb.flags & NTM_LITERAL_PHI_RIGHTMUL) != 0;
    for (int j = l; j < N; j += P) {
        double* col = w.Gt() + w.gidx(2 * j, j) - 2 * j;
        double g0 = w.bb()[j], g1 = 0.0;
        col[2 * j] = g0;
        col[2 * j + 1] = g1;
        for (int i = j + 1; i < N; ++i) {
            const int ai = d6 ? i - j - 1 : i;
            const double n0 = w.a11()[ai] * g0;
            const double n1 = w.a21()[ai] * g0 + k.a22 * g1;
            g0 = n0;
            g1 = n1;
            col[2 * i] = g0;
            col[2 * i + 1] = g1;
        }
    }
    if (l == 0) {
        double p00 = w.a11()[0], p10 = w.a21()[0], p01 = 0.0, p11 = k.a22;
        double l0 = k.C1, l1 = k.C2;
        w.Phi()[0] = p00; w.Phi()[1] = p10; w.Phi()[2] = p01; w.Phi()[3] = p11;
        w.Lam()[0] = l0; w.Lam()[1] = l1;
        for (int i = 1; i < N; ++i) {
            const double a11 = w.a11()[i], a21 = w.a21()[i];
            double q00, q01, q10, q11;
            if (d4) {                                  // Phi_{i-1} A_i
                q00 = p00 * a11 + p01 * a21;
                q01 = p01 * k.a22;
                q10 = p10 * a11 + p11 * a21;
                q11 = p11 * k.a22;
            } else {                                   // A_i Phi_{i-1}
                q00 = a11 * p00;
                q01 = a11 * p01;
                q10 = a21 * p00 + k.a22 * p10;
                q11 = a21 * p01 + k.a22 * p11;
            }
            p00 = q00; p01 = q01; p10 = q10; p11 = q11;
            const double m0 = a11 * l0 + k.C1;
            const double m1 = (a21 * l0 + k.a22 * l1) + k.C2;
            l0 = m0; l1 = m1;
            w.Phi()[4 * i] = p00; w.Phi()[4 * i + 1] = p10; w.Phi()[4 * i + 2] = p01; w.Phi()[4 * i + 3] = p11;
            w.Lam()[2 * i] = l0; w.Lam()[2 * i + 1] = l1;
        }
    }
    NTM_WSYNC();
}

#ifndef NTM_ROW_PAIRS
#define NTM_ROW_PAIRS 0    // 1: long horizons, the scaling pass's row norms two rows per lane (slower)
#endif
#ifndef NTM_FUSE_COLSUM
#define NTM_FUSE_COLSUM 1  // the lift accumulates the scaling pass's column sums (ColSums): bit 0
#endif                     // long horizons (N = 50), bit 1 the far N = 20 kernel, bit 2 the all-LDS N = 20 one
// The scaling pass's column sums, accumulated by the slim lift (NTM_FUSE_COLSUM):
// lane l < N walks Gamma's column l stage by stage, so it can add G_ll's and F_l's
// terms as it produces them (the free response e_i is lane N's value at the same
// stage, read by readlane), instead of the scaling pass reading the column back
// from LDS.  Same terms in the same order as the pass (diag_scale_phase).  Round 6,
// A/B on one box: config 5 mode 2 73.9 -> 70.9 ms per step-batch; the far N = 20
// kernel 6.31 -> 6.50 ms (its register allocation again) and the all-LDS one (config
// 2 0.193 -> 0.210 ms: e_i takes six lane reads there), so N = 50 only.
struct ColSums {
    double s = 0.0, f = 0.0;   // sum_i Gamma_il' Om Gamma_il and sum_i Gamma_il' Om (e_i - r)
    int bad = 0;               // a non-finite Gamma entry
};
template <class W>
__device__ __forceinline__ constexpr bool fuse_colsum() {
    if constexpr (W::kSlim) return W::kNN > 32 ? (NTM_FUSE_COLSUM & 1) != 0 : (NTM_FUSE_COLSUM & 2) != 0;
    // the all-LDS N = 20 build (lanes N, N+1 and N+2 hold Phi's columns and Lambda)
    else return !W::kFar && W::kNN == 20 && (NTM_FUSE_COLSUM & 4) != 0;
}

template <int P, class W>
__device__ __forceinline__ void lift_phase(const Prob& pb, const W& w, int l, double x0 = 0.0, double x1 = 0.0,
                                           ColSums* cs = nullptr) {
    const int N = w.n();
    const Coef k = scn_coef(pb, w);
    if constexpr (W::kSlim) {
        // lane l < N keeps stage l's A/B coefficients in registers; the loop takes
        // stage i's by readlane.  Lanes < N: Gamma columns (as below); lane N: the
        // free response e = Phi x_k + Lambda as its own recursion e_i = A_i e_{i-1} + C
        // with e_{-1} = x_k (CANON D4: Phi_i = A_i Phi_{i-1}; the same states as
        // Phi x_k + Lambda to rounding), written straight to w.e()
        double ra = 0.0, rc = 0.0, rbb = 0.0;
        if (l < N) {
            ra = coef_a11(k, w.rho()[3 * l]);
            rc = coef_a21(k, w.rho()[3 * l + 1]);
            rbb = coef_b(k, w.rho()[3 * l + 2]);
            if constexpr (W::kAB) { w.a11()[l] = ra; w.a21()[l] = rc; }
        }
        if constexpr (W::kAB) NTM_WSYNC();
        const double a0 = gbcast<P>(ra, 0), c0v = gbcast<P>(rc, 0);
        NTM_T0(tlf);
        if (l <= N) {
            const bool gam = l < N;
            double g0 = gam ? rbb : (a0 * x0 + k.C1);
            double g1 = gam ? 0.0 : ((c0v * x0 + k.a22 * x1) + k.C2);
            const double c0 = gam ? 0.0 : k.C1, c1 = gam ? 0.0 : k.C2;
            double* const rec = gam ? w.Gt() + w.gidx(2 * l, l) - 2 * l : w.e();
            rec[2 * (gam ? l : 0)] = g0;
            rec[2 * (gam ? l : 0) + 1] = g1;
            // stage i's terms of the column sums (lane N holds e_i): the scaling pass's
            // and free_response's expressions
            double cs_s = 0.0, cs_f = 0.0;
            int cs_bad = 0;
            const OmQ<qi_on<W>()> cq(pb.Q);
            // NTM_FUSE_LOCAL_E: every lane runs lane N's free-response recursion itself (the
            // same operations on the same coefficients), so e_i needs no lane read per stage
            constexpr bool kLocalE = fuse_colsum<W>() && NTM_FUSE_LOCAL_E;
            double ee0 = kLocalE ? (a0 * x0 + k.C1) : 0.0;
            double ee1 = kLocalE ? ((c0v * x0 + k.a22 * x1) + k.C2) : 0.0;
            auto col_terms = [&](int i) {
                if constexpr (fuse_colsum<W>()) {
                    const double e0 = kLocalE ? ee0 : gbcast<P>(g0, N), e1 = kLocalE ? ee1 : gbcast<P>(g1, N);
                    const double d0 = e0 - pb.r[0], d1 = e1 - pb.r[1];
                    const double ea = cq.o0(d0, d1), eb = cq.o1(d0, d1);
                    const double o0 = cq.o0(g0, g1), o1 = cq.o1(g0, g1);
                    const double t = g0 * o0 + g1 * o1;
                    const double tf = g0 * ea + g1 * eb;
                    const bool on = gam && i >= l;
                    if (on) cs_bad |= !isfinite(g0) || !isfinite(g1);
                    cs_s += on ? t : 0.0;
                    cs_f += on ? tf : 0.0;
                }
            };
            col_terms(0);
            constexpr int CH = NTM_CH;
            NTM_CHUNK_PRAGMA
            for (int i0 = 1; i0 < N; i0 += CH) {
                double ca[CH], cb[CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const int i = i0 + u;
                    if constexpr (W::kAB) {
                        ca[u] = i < N ? w.a11()[i] : 0.0;
                        cb[u] = i < N ? w.a21()[i] : 0.0;
                    } else {
                        ca[u] = i < N ? gbcast<P>(ra, i) : 0.0;
                        cb[u] = i < N ? gbcast<P>(rc, i) : 0.0;
                    }
                }
                if constexpr (W::kAB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const int i = i0 + u;
                    if (i < N) {
                        const double n0 = ca[u] * g0 + c0;
                        const double n1 = (cb[u] * g0 + k.a22 * g1) + c1;
                        const bool live = !gam || i > l;
                        g0 = live ? n0 : g0;
                        g1 = live ? n1 : g1;
                        const int at = live ? i : l;
                        rec[2 * at] = g0;
                        rec[2 * at + 1] = g1;
                        if constexpr (kLocalE) {
                            const double m0 = ca[u] * ee0 + k.C1;
                            const double m1 = (cb[u] * ee0 + k.a22 * ee1) + k.C2;
                            ee0 = m0;
                            ee1 = m1;
                        }
                        col_terms(i);
                    }
                }
            }
            if (cs) { cs->s = cs_s; cs->f = cs_f; cs->bad = cs_bad; }
        }
        NTM_ACC(ST_L_LOOP, tlf);
        NTM_WSYNC();
        return;
    } else {
    if (l < N) {
        w.a11()[l] = coef_a11(k, w.rho()[3 * l]);
        w.a21()[l] = coef_a21(k, w.rho()[3 * l + 1]);
        w.bb()[l] = coef_b(k, w.rho()[3 * l + 2]);
    }
    NTM_WSYNC();
    if constexpr (W::kNN == 0) {
        if (pb.flags & (NTM_LITERAL_PHI_RIGHTMUL | NTM_LITERAL_GAMMA_INDEX)) {
            lift_literal<P>(pb, w, k, l);
            return;
        }
    }
    NTM_T0(tlf);
    // Gamma: lane j owns column j: Gamma_jj = B_j, Gamma_ij = A_i Gamma_{i-1,j} (D6).
    // Lanes N and N+1 run the same 2-vector recursion for the two columns of
    // Phi_i = A_i Phi_{i-1} (D4), lane N+2 for Lambda_i = A_i Lambda_{i-1} + C,
    // all in the one loop (the group has the idle lanes for N + 3 <= P).
    const bool extra = N + 3 <= P;
    if (l < N || (extra && l < N + 3)) {
        const bool gam = l < N;
        const int ph = l - N;                          // 0, 1: Phi column; 2: Lambda
        double g0, g1;
        if (gam) { g0 = w.bb()[l]; g1 = 0.0; }
        else if (ph == 0) { g0 = w.a11()[0]; g1 = w.a21()[0]; }
        else if (ph == 1) { g0 = 0.0; g1 = k.a22; }
        else { g0 = k.C1; g1 = k.C2; }
        const double c0 = (ph == 2) ? k.C1 : 0.0, c1 = (ph == 2) ? k.C2 : 0.0;
        // this lane's record, stage i at rec[st i]: its Gamma column (col[r], r >= 2l),
        // its Phi column (stride 4) or Lambda; one address for the three kinds of
        // lanes, so every step is one pair of stores with no divergent branches
        double* const rec = gam ? w.Gt() + w.gidx(2 * l, l) - 2 * l : (ph < 2 ? w.Phi() + 2 * ph : w.Lam());
        const int st = (gam || ph == 2) ? 2 : 4;
        auto put = [&](int i) {
            rec[st * i] = g0;
            rec[st * i + 1] = g1;
        };
        put(gam ? l : 0);
        // stage i's terms of the scaling pass's column sums (ColSums): e_i = Phi_i x_k +
        // Lambda_i from lanes N, N+1 (Phi's columns) and N+2 (Lambda), free_response's
        // expressions
        double cs_s = 0.0, cs_f = 0.0;
        int cs_bad = 0;
        const OmQ<qi_on<W>()> cq(pb.Q);
        auto col_terms = [&](int i) {
            if constexpr (fuse_colsum<W>()) {
                const double p00 = gbcast<P>(g0, N), p10 = gbcast<P>(g1, N);
                const double p01 = gbcast<P>(g0, N + 1), p11 = gbcast<P>(g1, N + 1);
                const double l0 = gbcast<P>(g0, N + 2), l1 = gbcast<P>(g1, N + 2);
                const double e0 = (p00 * x0 + p01 * x1) + l0;
                const double e1 = (p10 * x0 + p11 * x1) + l1;
                const double d0 = e0 - pb.r[0], d1 = e1 - pb.r[1];
                const double ea = cq.o0(d0, d1), eb = cq.o1(d0, d1);
                const double o0 = cq.o0(g0, g1), o1 = cq.o1(g0, g1);
                const double t = g0 * o0 + g1 * o1;
                const double tf = g0 * ea + g1 * eb;
                const bool on = gam && i >= l;
                if (on) cs_bad |= !isfinite(g0) || !isfinite(g1);
                cs_s += on ? t : 0.0;
                cs_f += on ? tf : 0.0;
            }
        };
        col_terms(0);
        // fixed trip count (unrolls), branch-free: Gamma rows i <= l keep (B_l, 0) and
        // rewrite the diagonal.  The coefficients of CH steps are loaded ahead of the
        // chunk's stores (the stores cannot be proven not to alias them, so per-step
        // loads would wait for the previous step's stores: one LDS round trip a step)
        constexpr int CH = NTM_CH;
        NTM_CHUNK_PRAGMA
        for (int i0 = 1; i0 < N; i0 += CH) {
            double ca[CH], cb[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = i0 + u;
                ca[u] = i < N ? w.a11()[i] : 0.0;
                cb[u] = i < N ? w.a21()[i] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = i0 + u;
                if (i < N) {
                    const double n0 = ca[u] * g0 + c0;
                    const double n1 = (cb[u] * g0 + k.a22 * g1) + c1;
                    const bool live = !gam || i > l;
                    g0 = live ? n0 : g0;
                    g1 = live ? n1 : g1;
                    put(live ? i : l);
                    col_terms(i);
                }
            }
        }
        if (cs) { cs->s = cs_s; cs->f = cs_f; cs->bad = cs_bad; }
    }
    NTM_ACC(ST_L_LOOP, tlf);
    // Phi and Lambda on lane 0 when the group has no idle lanes
    if (!extra && l == 0) {
        double p00 = w.a11()[0], p10 = w.a21()[0], p01 = 0.0, p11 = k.a22;
        double l0 = k.C1, l1 = k.C2;
        w.Phi()[0] = p00; w.Phi()[1] = p10; w.Phi()[2] = p01; w.Phi()[3] = p11;
        w.Lam()[0] = l0; w.Lam()[1] = l1;
        for (int i = 1; i < N; ++i) {
            double a11 = w.a11()[i], a21 = w.a21()[i];
            double q00 = a11 * p00, q01 = a11 * p01;
            double q10 = a21 * p00 + k.a22 * p10, q11 = a21 * p01 + k.a22 * p11;
            p00 = q00; p01 = q01; p10 = q10; p11 = q11;
            double m0 = a11 * l0 + k.C1;
            double m1 = (a21 * l0 + k.a22 * l1) + k.C2;
            l0 = m0; l1 = m1;
            w.Phi()[4 * i] = p00; w.Phi()[4 * i + 1] = p10; w.Phi()[4 * i + 2] = p01; w.Phi()[4 * i + 3] = p11;
            w.Lam()[2 * i] = l0; w.Lam()[2 * i + 1] = l1;
        }
    }
    NTM_WSYNC();
    }
}

// free response e = Phi x_k + Lambda (the x-dependent part of NTM_MPC_Sim.m:121
// and of c + W x_k at :97)
template <int P, class W>
__device__ __forceinline__ void free_response(const W& w, double x0, double x1, int l, const Prob* pw = nullptr) {
    for (int i = l; i < w.n(); i += P) {
        double e0, e1;
        if constexpr (W::kSlim) {                // the lift wrote e itself
            e0 = w.e()[2 * i];
            e1 = w.e()[2 * i + 1];
        } else {
            const double* Ph = w.Phi() + 4 * i;
            e0 = (Ph[0] * x0 + Ph[2] * x1) + w.Lam()[2 * i];
            e1 = (Ph[1] * x0 + Ph[3] * x1) + w.Lam()[2 * i + 1];
            w.e()[2 * i] = e0;
            w.e()[2 * i + 1] = e1;
        }
        if (pw) {
            // Om (e_i - r) per stage for the scaling pass's F (scratch in w.xp(): the
            // rollout consumed it and rewrites it; the re-solve recomputes it)
            const double d0 = e0 - pw->r[0], d1 = e1 - pw->r[1];
            const OmQ<qi_on<W>()> om(pw->Q);
            w.xp()[2 * i] = om.o0(d0, d1);
            w.xp()[2 * i + 1] = om.o1(d0, d1);
        }
    }
    NTM_WSYNC();
}

// sum_{imin <= i < n} a_i' c_i over 2-vectors stored at stride 2 (c = Om b precomputed)
template <int CH>
__device__ __forceinline__ double dot_rows2(const double* a, const double* c, int n, int imin) {
    double s = 0.0;
    NTM_CHUNK_PRAGMA
    for (int i0 = 0; i0 < n; i0 += CH) {
        double a0[CH], a1[CH], c0[CH], c1[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = i0 + u;
            const bool in = i < n;
            a0[u] = in ? a[2 * i] : 0.0;
            a1[u] = in ? a[2 * i + 1] : 0.0;
            c0[u] = in ? c[2 * i] : 0.0;
            c1[u] = in ? c[2 * i + 1] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = i0 + u;
            const double t = a0[u] * c0[u] + a1[u] * c1[u];
            s += (i >= imin && i < n) ? t : 0.0;
        }
    }
    return s;
}

// ---------------------------------------------------------------------------
// Gram of Gamma columns on the matrix cores (long horizons): for the columns
// j_a = col_of(a), a < nc, S(a, c) = X_a' (I (x) Q) X_c with X_a = Gamma(:, j_a),
// i.e. S = X' Y with Y = (I (x) Q) X, the (nc x 2N) x (2N x nc) contraction of
// NTM_MPC_Sim.m:120 restricted to those columns.  V_MFMA_F64_16X16X4F64 on
// 16 x 16 tiles, K = 4 rows of Gamma per instruction (2N / 4 steps; NN even):
// lane l holds A = X(r, 16 t + (l & 15)) and B = Y(r, 16 t + (l & 15)) with
// r = 4 s + (l >> 4), both from the two Gamma rows of stage r / 2 (two LDS
// loads); the lower tile pairs accumulate in registers and put(a, c, S) takes
// every entry a >= c (D layout: column l & 15, row (l >> 4) + 4 i).  Same terms
// as qdot_rows / gram_rows, summed in the matrix core's order.  P = 64 only,
// called in wave-uniform control flow.
// ---------------------------------------------------------------------------
typedef double ntm_d4 __attribute__((ext_vector_type(4)));
#ifndef NTM_MFMA_FF
#define NTM_MFMA_FF 0      // the re-solve's compact G~_FF (bordered path): measured slower, off
#endif
#ifndef NTM_PLANE
#define NTM_PLANE 1        // k = 2 echelon sets on the null-space path (long horizons, generic kernels)
#endif
#ifndef NTM_COLL2
#define NTM_COLL2 1        // square sets with two collisions on the null-space path (long horizons, generic)
#endif
#ifndef NTM_COLL3
#define NTM_COLL3 1        // k = 2 sets with one collision (three holes) on the null-space path (round 6)
#endif
#ifndef NTM_ROWE_ALL
#define NTM_ROWE_ALL 0     // 1: the echelon re-solve builds E one sorted row per lane at every horizon
#endif
#ifndef NTM_MFMA_FULL
#define NTM_MFMA_FULL 1    // GI's full G~
#endif
template <int NN, class W, class ColOf, class Put>
__device__ __forceinline__ void gram_mfma(const Prob& pb, const W& w, int nc, ColOf col_of, Put put, int l) {
    static_assert(NN > 0 && NN % 2 == 0, "gram_mfma: compile-time even horizon");
    constexpr int TM = (NN + 15) / 16;                 // tiles of 16 columns
    constexpr int NP = TM * (TM + 1) / 2;              // lower tile pairs
    const OmQ<qi_on<W>()> om(pb.Q);
    const int li = l & 15, lk = l >> 4;
    const int T = (nc + 15) >> 4;
    int base[TM], r0[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
        const int a = 16 * t + li;
        const bool on = a < nc;
        const int j = on ? col_of(a) : 0;
        base[t] = w.gidx(2 * j, j) - 2 * j;             // Gamma(r, j) = Gt[base + r], r >= 2j
        r0[t] = on ? 2 * j : 2 * NN;                    // rows above the block diagonal are zero
    }
    ntm_d4 acc[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p] = ntm_d4{0.0, 0.0, 0.0, 0.0};
    const double* const G = w.Gt();
#pragma unroll 1
    for (int s = 0; s < NN / 2; ++s) {                  // not unrolled: the accumulators stay the only long-lived registers
        const int re = 4 * s + (lk & ~1);               // the even row of this lane's stage
        double xa[TM], yb[TM];
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            const bool in = re >= r0[t];
            const double x0 = in ? G[base[t] + re] : 0.0, x1 = in ? G[base[t] + re + 1] : 0.0;
            xa[t] = (lk & 1) ? x1 : x0;
            yb[t] = (lk & 1) ? om.o1(x0, x1) : om.o0(x0, x1);
        }
        int p = 0;
#pragma unroll
        for (int ta = 0; ta < TM; ++ta)
#pragma unroll
            for (int tc = 0; tc <= ta; ++tc, ++p)
                if (ta < T) acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[ta], yb[tc], acc[p], 0, 0, 0);
    }
    int p = 0;
#pragma unroll
    for (int ta = 0; ta < TM; ++ta)
#pragma unroll
        for (int tc = 0; tc <= ta; ++tc, ++p) {
            if (ta >= T) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int a = 16 * ta + lk + 4 * i, c = 16 * tc + li;
                if (a < nc && c <= a) put(a, c, acc[p][i]);
            }
        }
}

// ---------------------------------------------------------------------------
// condensed cost G = 2 Gamma' Om Gamma (lower triangle into dst, col-major),
// F = 2 Gamma' Om (e - R)      NTM_MPC_Sim.m:120-121 (CANON D8, D12)
// ---------------------------------------------------------------------------
template <int P, class W, class Put>
__device__ __forceinline__ void gram_rows_put(const Prob& pb, const W& w, Put put, int l) {
    const int N = w.n();
    if constexpr (NTM_MFMA_FULL && W::kNN > 32 && P == 64) {   // the matrix cores (gram_mfma)
        gram_mfma<W::kNN>(pb, w, N, [](int a) { return a; }, [&](int j, int kk, double sg) { put(j, kk, 2 * sg); },
                          l);
        return;
    }
    const OmQ<qi_on<W>()> om(pb.Q);
    // one (j, kk) entry per lane; fixed-trip masked dot (column reads below the
    // packed column start stay inside Gt, see StructRows::check)
    const int npair = N * (N + 1) / 2;
    for (int idx = l; idx < npair; idx += P) {
        int j = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
        if ((j + 1) * (j + 2) / 2 <= idx) ++j;
        if (j * (j + 1) / 2 > idx) --j;
        const int kk = idx - j * (j + 1) / 2;
        const double* cj = w.Gt() + w.gidx(2 * j, j) - 2 * j;
        const double* ck = w.Gt() + w.gidx(2 * kk, kk) - 2 * kk;
        double s = 0.0;
        for (int i = 0; i < N; ++i) {
            const double g0 = ck[2 * i], g1 = ck[2 * i + 1];
            const double o0 = om.o0(g0, g1);
            const double o1 = om.o1(g0, g1);
            const double t = cj[2 * i] * o0 + cj[2 * i + 1] * o1;
            s += (i >= j) ? t : 0.0;
        }
        double gv = 2 * s;
        if constexpr (ru_on<W>()) gv = (j == kk) ? gv + 2 * pb.Ru : gv;   // + 2 Ru I (ABI v5)
        put(j, kk, gv);             // G(j, kk), j >= kk
    }
}
template <int P, class W>
__device__ __forceinline__ void gram_rows(const Prob& pb, const W& w, double* dst, int l) {
    const int LD = w.ldj();
    gram_rows_put<P>(pb, w, [&](int j, int kk, double v) { dst[j + kk * LD] = v; }, l);
}

template <int P, class W>
__device__ __forceinline__ void cost_phase(const Prob& pb, const W& w, int l) {
    const int N = w.n();
    const double q00 = pb.Q[0], q01 = pb.Q[1], q10 = pb.Q[2], q11 = pb.Q[3];
    gram_rows<P>(pb, w, w.R(), l);
    if (l < N) {
        const double* cj = w.Gt() + w.gidx(2 * l, l) - 2 * l;
        double f = 0.0;
        for (int i = l; i < N; ++i) {
            double e0 = w.e()[2 * i] - pb.r[0], e1 = w.e()[2 * i + 1] - pb.r[1];
            double o0 = q00 * e0 + q01 * e1;
            double o1 = q10 * e0 + q11 * e1;
            f += cj[2 * i] * o0 + cj[2 * i + 1] * o1;
        }
        w.F()[l] = 2 * f;
    }
    NTM_WSYNC();
}

// G~ = D G D in place (lower triangle, col-major); the same expression order
// is used when the polish recomputes G~ (so both copies are bit-identical).
template <int P, class W>
__device__ __forceinline__ int scale_gram(const W& w, double* G, int l) {
    int bad = 0;
    if (l < w.n()) {
        double Dl = w.D()[l];
        for (int kk = 0; kk <= l; ++kk) {
            double v = G[l + kk * w.ldj()] * Dl * w.D()[kk];
            bad |= !isfinite(v);
            G[l + kk * w.ldj()] = v;
        }
    }
    return bad;
}

// ---------------------------------------------------------------------------
// Jacobi scaling U = D V with D = diag(G)^{-1/2}, computed from the Gram
// diagonal only (same summation order as gram_rows, so D is bit-identical to
// what the full G would give); F~ = D F; norms of the scaled state rows
// ||Gamma_r D||.  Gamma stays unscaled (D is applied on the fly).  The full
// G~ is only formed when the Goldfarb-Idnani fallback runs (full_gram).
// Returns (group-uniform) 2 if any datum is non-finite, else 1 if a constant
// row is violated (the x_0 rows and state rows Gamma does not reach: D15, D22,
// StructRows::feasible_const's test, folded into the row pass that finds them
// and into the one reduction, round 6), else 0.
// ---------------------------------------------------------------------------
// The far N = 20 build keeps the separate test (qp_phase calls feasible_const):
// folded in, it cost that kernel 1.3% through register allocation (6.30 -> 6.38 ms)
// while config 2 (0.201 -> 0.199 ms) and config 5 (74.2 -> 73.7 ms) gained.
template <class W>
__device__ __forceinline__ constexpr bool fold_const() { return !(W::kFar && W::kNN == 20); }
template <int P, class W>
__device__ __forceinline__ int diag_scale_phase(const Prob& pb, const W& w, int l, bool with_state_rows,
                                                double x0 = 0.0, double x1 = 0.0, const ColSums* cs = nullptr) {
    const int N = w.n();
    const OmQ<qi_on<W>()> qw(pb.Q);
    int bad = 0, infe = 0;
    auto const_row = [&](int r) {                         // 0 <= b on a constant state row, to kConstTol
        if constexpr (!fold_const<W>()) return;
        const int c = r & 1;
        const double er = w.e()[r];
        infe |= (er - pb.xmin[c]) < -kConstTol;
        infe |= (pb.xmax[c] - er) < -kConstTol;
    };
    if (fold_const<W>() && with_state_rows && l == 0) {   // the x_0 rows (D15)
        infe |= (x0 - pb.xmin[0]) < -kConstTol;
        infe |= (x1 - pb.xmin[1]) < -kConstTol;
        infe |= (pb.xmax[0] - x0) < -kConstTol;
        infe |= (pb.xmax[1] - x1) < -kConstTol;
    }
    NTM_T0(tsc);
    // Short horizons (2N <= 64, N = 20): the column pass and the row pass each split
    // their sums in two halves at H = ceil(N/2) on otherwise idle lanes, so the wave
    // runs H trips instead of N (lanes N..2N-1 take the columns' i >= H terms; lanes
    // 2N.. the j >= H terms of rows with r >= 2H).  The sums are then (first half) +
    // (second half) instead of one sequential pass.  The all-LDS build only (config 2,
    // B = 1024: 0.208 -> 0.199 ms; mode 2 at B = 1024: 0.545 -> 0.526 ms).  The far
    // build's register allocation does not absorb it: 6.36 -> 7.98 ms per step-batch
    // at B = 1e5 with the chunk unroll, 6.41 ms without; the column pass alone 7.11 ms,
    // the row pass alone 9.66 ms (A/B on one box, NTM_SPLIT_FAR)
    constexpr int NNs = W::kNN, Hs = (NNs + 1) / 2;
    constexpr bool kSplit = NTM_SPLIT_SCALE && P == 64 && NNs > 0 && 4 * NNs - 2 * Hs <= 64;
    // NTM_SPLIT_FAR (far build): bit 0 the column pass, bit 1 the row pass
    constexpr bool kSC = kSplit && (!W::kFar || (NTM_SPLIT_FAR & 1));
    constexpr bool kSR = kSplit && (!W::kFar || (NTM_SPLIT_FAR & 2));
    constexpr int TC = kSC ? Hs : NNs, TR = kSR ? Hs : NNs;   // trips of each pass
    if constexpr (kSC || kSR) {
        double s = 0.0, fs = 0.0;
        const int col = l < N ? l : l - N;
        const int base = l < N ? 0 : Hs;
        const bool fc = fuse_colsum<W>() && cs != nullptr;   // summed by the lift (one sequential sum)
        if (fc) {
            if (l < N) { s = cs->s; fs = cs->f; bad |= cs->bad; }
        } else if (l < (kSC ? 2 * N : N)) {
            const double* cj = w.Gt() + w.gidx(2 * col, col) - 2 * col;
            const double* om = w.xp();
            constexpr int CH = NTM_CH;
            NTM_SPLIT_PRAGMA
            for (int u0 = 0; u0 < TC; u0 += CH) {
                double ga[CH], gb[CH], ea[CH], eb[CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const int i = base + u0 + u;
                    const bool in = u0 + u < TC && i < N;
                    ga[u] = in ? cj[2 * i] : 0.0;
                    gb[u] = in ? cj[2 * i + 1] : 0.0;
                    ea[u] = in ? om[2 * i] : 0.0;
                    eb[u] = in ? om[2 * i + 1] : 0.0;
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const int i = base + u0 + u;
                    const double g0 = ga[u], g1 = gb[u];
                    const double o0 = qw.o0(g0, g1);
                    const double o1 = qw.o1(g0, g1);
                    const double t = g0 * o0 + g1 * o1;
                    const double tf = g0 * ea[u] + g1 * eb[u];
                    const bool on = u0 + u < TC && i >= col && i < N;
                    if (on) bad |= !isfinite(g0) || !isfinite(g1);
                    s += on ? t : 0.0;
                    fs += on ? tf : 0.0;
                }
            }
        }
        const double s2 = (kSC && !fc) ? __shfl(s, (l + N) & 63, 64) : 0.0;
        const double f2 = (kSC && !fc) ? __shfl(fs, (l + N) & 63, 64) : 0.0;
        if (l < N) {
            double g = (kSC && !fc) ? 2 * (s + s2) : 2 * s;
            if constexpr (ru_on<W>()) g = g + 2 * pb.Ru;   // G_ll + 2 Ru (ABI v5)
            const double Dl = (g > 0.0 && g < kInf) ? rsqrt_nr(g) : 1.0;
            w.D()[l] = Dl;
            const double f = ((kSC && !fc) ? 2 * (fs + f2) : 2 * fs) * Dl;
            bad |= !isfinite(f) || !isfinite(Dl);
            w.F()[l] = f;
            if constexpr (!W::kSlim) {
                w.vlo()[l] = -((-pb.umin) / Dl);
                w.vhi()[l] = pb.umax / Dl;
            }
        }
        NTM_WSYNC();
        NTM_ACC(ST_SC_COL, tsc);
        if (pb.mode == NTM_MODE_FULL_DU && l >= 1 && l < N) {
            const double a = w.D()[l], b = w.D()[l - 1];
            w.idun()[l] = 1.0 / sqrt(a * a + b * b);
        }
        if (with_state_rows) {
            const bool lo = l < 2 * N, hi = kSR && !lo && l < 4 * N - 2 * Hs;
            const int r = lo ? l : (hi ? l - 2 * N + 2 * Hs : 0);
            const int jb = lo ? 0 : Hs;
            const int jmax = r >> 1;
            double rs = 0.0;
            int last = -1, cnt = 0;
            if (lo || hi) {
                constexpr int CH = NTM_CH;
                NTM_SPLIT_PRAGMA
                for (int u0 = 0; u0 < TR; u0 += CH) {
                    double g[CH], dd[CH];
#pragma unroll
                    for (int u = 0; u < CH; ++u) {
                        const int j = jb + u0 + u;
                        const bool in = u0 + u < TR && j < N;
                        g[u] = in ? w.gt(r, j) : 0.0;
                        dd[u] = in ? w.D()[j] : 0.0;
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < CH; ++u) {
                        const int j = jb + u0 + u;
                        const double v = g[u] * dd[u];
                        const bool in = u0 + u < TR && j <= jmax;
                        rs += in ? v * v : 0.0;
                        if (in && g[u] != 0.0) { last = j; ++cnt; }
                    }
                }
            }
            // the row's second half sits on lane 2N + r - 2H (rows r >= 2H)
            const int src = (kSR && l >= 2 * Hs && l < 2 * N) ? l + 2 * N - 2 * Hs : l;
            const double rs2 = kSR ? __shfl(rs, src & 63, 64) : 0.0;
            const int last2 = kSR ? __shfl(last, src & 63, 64) : -1;
            const int cnt2 = kSR ? __shfl(cnt, src & 63, 64) : 0;
            if (lo) {
                const bool two = src != l;
                const double sr = two ? rs + rs2 : rs;
                const int lr = (two && last2 >= 0) ? last2 : last;
                const int cr = two ? cnt + cnt2 : cnt;
                bad |= !isfinite(sr) || !isfinite(w.e()[r]);
                const double ir = (sr > 0.0 && sr < kInf) ? rsqrt_nr(sr) : 0.0;
                w.irn()[r] = ir;
                w.rinfo()[r] = (lr + 1) | (cr > 1 ? kRowMulti : 0);
                if (ir == 0.0) const_row(r);
            }
            NTM_WSYNC();
        }
        NTM_ACC(ST_SC_ROW, tsc);
        const int code = fold_const<W>() ? gmaxi<P>(bad ? 2 : infe) : (gmaxi<P>(bad) != 0 ? 2 : 0);
        NTM_ACC(ST_SC_END, tsc);
        return code;
    }
    if (l < N) {
        // one pass over Gamma's column l: the Gram diagonal G_ll and F_l = 2 Gamma_l' Om (e - r)
        const double* cj = w.Gt() + w.gidx(2 * l, l) - 2 * l;
        const double* om = w.xp();               // Om (e_i - r), from free_response
        double s = 0.0, fs = 0.0;
        constexpr int CH = NTM_CH;
        if (fuse_colsum<W>() && cs) {           // summed by the lift
            s = cs->s;
            fs = cs->f;
            bad |= cs->bad;
        } else {
        NTM_CHUNK_PRAGMA
        for (int i0 = 0; i0 < N; i0 += CH) {     // fixed trip count, terms i < l masked; batched loads
            double ga[CH], gb[CH], ea[CH], eb[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = i0 + u;
                const bool in = i < N;
                ga[u] = in ? cj[2 * i] : 0.0;
                gb[u] = in ? cj[2 * i + 1] : 0.0;
                ea[u] = in ? om[2 * i] : 0.0;
                eb[u] = in ? om[2 * i + 1] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = i0 + u;
                const double g0 = ga[u], g1 = gb[u];
                const double o0 = qw.o0(g0, g1);
                const double o1 = qw.o1(g0, g1);
                const double t = g0 * o0 + g1 * o1;
                const double tf = g0 * ea[u] + g1 * eb[u];
                const bool on = i >= l && i < N;
                if (on) bad |= !isfinite(g0) || !isfinite(g1);
                s += on ? t : 0.0;
                fs += on ? tf : 0.0;
            }
        }
        }
        double g = 2 * s;
        if constexpr (ru_on<W>()) g = g + 2 * pb.Ru;   // G_ll + 2 Ru (ABI v5)
        double Dl = (g > 0.0 && g < kInf) ? rsqrt_nr(g) : 1.0;
        w.D()[l] = Dl;
        double f = (2 * fs) * Dl;
        bad |= !isfinite(f) || !isfinite(Dl);
        w.F()[l] = f;
        // V-space box of u_l (bc of the two u rows; same expressions as the oracle's b/rn)
        if constexpr (!W::kSlim) {
            w.vlo()[l] = -((-pb.umin) / Dl);
            w.vhi()[l] = pb.umax / Dl;
        }
    }
    NTM_WSYNC();
    NTM_ACC(ST_SC_COL, tsc);
    if (pb.mode == NTM_MODE_FULL_DU && l >= 1 && l < N) {      // rate-row norms |D (e_l - e_{l-1})|
        const double a = w.D()[l], b = w.D()[l - 1];
        w.idun()[l] = 1.0 / sqrt(a * a + b * b);
    }
    // Long horizons (P < 2N <= 2P): lane l takes state rows l and l + P in one pass
    // (both rows' loads of a chunk issued together, D_j loaded once) instead of two
    // passes (NTM_ROW_PAIRS).  Each row's terms are summed in the same order as below.
    constexpr bool kRowPairs = NTM_ROW_PAIRS && P == 64 && W::kNN > 32 && W::kNN <= 64;
    if (kRowPairs && with_state_rows) {
        const int r1 = l, r2 = l + P;
        const bool two = r2 < 2 * N;
        const int jmax1 = r1 >> 1, jmax2 = two ? (r2 >> 1) : -1;
        double s1 = 0.0, s2 = 0.0;
        int last1 = -1, cnt1 = 0, last2 = -1, cnt2 = 0;
        constexpr int CH = NTM_CH;
        NTM_CHUNK_PRAGMA
        for (int j0 = 0; j0 < N; j0 += CH) {     // fixed trip count, j > jmax masked; batched loads
            double g1[CH], g2[CH], dd[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int j = j0 + u;
                g1[u] = j < N ? w.gt(r1, j) : 0.0;
                g2[u] = (two && j < N) ? w.gt(r2, j) : 0.0;
                dd[u] = j < N ? w.D()[j] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const double v1 = g1[u] * dd[u], v2 = g2[u] * dd[u];
                const bool in1 = j0 + u <= jmax1, in2 = j0 + u <= jmax2;
                s1 += in1 ? v1 * v1 : 0.0;
                s2 += in2 ? v2 * v2 : 0.0;
                if (in1 && g1[u] != 0.0) { last1 = j0 + u; ++cnt1; }
                if (in2 && g2[u] != 0.0) { last2 = j0 + u; ++cnt2; }
            }
        }
        bad |= !isfinite(s1) || !isfinite(w.e()[r1]);
        const double ir1 = (s1 > 0.0 && s1 < kInf) ? rsqrt_nr(s1) : 0.0;
        w.irn()[r1] = ir1;
        w.rinfo()[r1] = (last1 + 1) | (cnt1 > 1 ? kRowMulti : 0);
        if (ir1 == 0.0) const_row(r1);
        if (two) {
            bad |= !isfinite(s2) || !isfinite(w.e()[r2]);
            const double ir2 = (s2 > 0.0 && s2 < kInf) ? rsqrt_nr(s2) : 0.0;
            w.irn()[r2] = ir2;
            w.rinfo()[r2] = (last2 + 1) | (cnt2 > 1 ? kRowMulti : 0);
            if (ir2 == 0.0) const_row(r2);
        }
        NTM_WSYNC();
    } else if (with_state_rows) {
        for (int r = l; r < 2 * N; r += P) {
            double s = 0.0;
            const int jmax = r >> 1;
            int last = -1, cnt = 0;
            constexpr int CH = NTM_CH;
            NTM_CHUNK_PRAGMA
            for (int j0 = 0; j0 < N; j0 += CH) { // fixed trip count, j > jmax masked; batched loads
                double g[CH], dd[CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const int j = j0 + u;
                    g[u] = j < N ? w.gt(r, j) : 0.0;
                    dd[u] = j < N ? w.D()[j] : 0.0;
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const double v = g[u] * dd[u];
                    const bool in = j0 + u <= jmax;
                    s += in ? v * v : 0.0;
                    if (in && g[u] != 0.0) { last = j0 + u; ++cnt; }
                }
            }
            bad |= !isfinite(s) || !isfinite(w.e()[r]);
            const double ir = (s > 0.0 && s < kInf) ? rsqrt_nr(s) : 0.0;
            w.irn()[r] = ir;                     // 1/|Gamma_r D| (0: constant row)
            w.rinfo()[r] = (last + 1) | (cnt > 1 ? kRowMulti : 0);
            if (ir == 0.0) const_row(r);
        }
        NTM_WSYNC();
    }
    NTM_ACC(ST_SC_ROW, tsc);
    const int code = fold_const<W>() ? gmaxi<P>(bad ? 2 : infe) : (gmaxi<P>(bad) != 0 ? 2 : 0);
    NTM_ACC(ST_SC_END, tsc);
    return code;
}

// the full scaled Hessian G~ (lower triangle, WS::gr) for the GI fallback
template <int P, class W>
__device__ __forceinline__ bool full_gram(const Prob& pb, const W& w, int l) {
    int bad = 0;
    if constexpr (W::kGiLdsL) {
        gram_rows_put<P>(pb, w, [&](int j, int kk, double v) { w.grL(j, kk) = v; }, l);
        NTM_WSYNC();
        if (l < w.n()) {                      // scale_gram's expression order
            const double Dl = w.D()[l];
            for (int kk = 0; kk <= l; ++kk) {
                const double v = w.grL(l, kk) * Dl * w.D()[kk];
                bad |= !isfinite(v);
                w.grL(l, kk) = v;
            }
        }
    } else {
        gram_rows<P>(pb, w, w.R(), l);
        NTM_WSYNC();
        bad = scale_gram<P>(w, w.R(), l);
    }
    NTM_WSYNC();
    return gmaxi<P>(bad) == 0;
}

// kept for the dense-row entry point (ntm_qp_device): G~ = D G D in place,
// F~ = D F (G given in w.R()); no state rows
template <int P, class W>
__device__ __forceinline__ bool scale_phase(const W& w, int l, bool /*with_state_rows*/) {
    const int N = w.n(), LD = w.ldj();
    if (l < N) {
        double g = w.R()[l + l * LD];
        w.D()[l] = (g > 0.0) ? 1.0 / sqrt(g) : 1.0;
    }
    NTM_WSYNC();
    int bad = scale_gram<P>(w, w.R(), l);
    if (l < N) {
        double f = w.F()[l] * w.D()[l];
        bad |= !isfinite(f);
        w.F()[l] = f;
    }
    NTM_WSYNC();
    return gmaxi<P>(bad) == 0;
}

// ---------------------------------------------------------------------------
// Constraint-row providers (Lin U <= b form, getWLc.m row convention).  Row
// ids follow the oracle: box mode rows 0..N-1 are u_j >= umin, N..2N-1 are
// u_j <= umax; full mode rows follow getWLc.m:9-59 block by block (6 per
// step, 4 terminal).  In the solver each row is scaled and normalised:
//   GI normal n = -(Lin D)/rn,  GI rhs bc = -b/rn,  slack s = n'V - bc.
// ---------------------------------------------------------------------------
struct Pick {
    int p;        // row id (-1 none)
    double s;     // normalised slack (GI form n'V - bc)
    double bc;    // normalised GI right-hand side
};

// aflag bits per constraint row
constexpr unsigned char kActiveRow = 1;   // in GI's active set
constexpr unsigned char kCandRow = 2;     // row of a failed warm-start candidate (GI adds these first)
constexpr unsigned char kSkipRow = 4;     // dual path (long horizons): p left out until the active set changes

// Implicit getWLc rows: u-bounds are -+e_j, state rows are -+Gamma_r; the
// rows are never materialised.
struct StructRows {
    static constexpr bool kHasUnitRows = true;
    int N, mode;  // NTM_MODE_BOX, NTM_MODE_FULL or NTM_MODE_FULL_DU (NONE: no rows)
    double umin, umax, xmin0, xmin1, xmax0, xmax1, du;

    __device__ __forceinline__ StructRows(const Prob& p)
        : N(p.N), mode(p.mode), umin(p.umin), umax(p.umax), xmin0(p.xmin[0]), xmin1(p.xmin[1]),
          xmax0(p.xmax[0]), xmax1(p.xmax[1]), du(p.du) {}
    __device__ __forceinline__ bool has_state() const { return mode >= NTM_MODE_FULL; }
    __device__ __forceinline__ bool has_rate() const { return mode == NTM_MODE_FULL_DU; }
    __device__ __forceinline__ double xmin(int c) const { return c ? xmin1 : xmin0; }
    __device__ __forceinline__ double xmax(int c) const { return c ? xmax1 : xmax0; }

    __device__ __forceinline__ int rows() const {
        return mode == NTM_MODE_NONE ? 0 : (mode == NTM_MODE_BOX ? 2 * N : (mode == NTM_MODE_FULL_DU ? 8 * N + 2 : 6 * N + 4));
    }

    // decode a row id: kind 0 = u lower, 1 = u upper, 2 = state min, 3 = state max,
    // 4 = rate up (U_j - U_{j-1} <= du), 5 = rate down (U_{j-1} - U_j <= du);
    // j = variable (u and rate rows) or state row r (state rows); -1 for x_0 rows.
    // Rate rows follow the 6N+4 getWLc rows: id = 6N+4 + 2(j-1) + {0 up, 1 down}.
    __device__ __forceinline__ void decode(int id, int N, int& kind, int& j) const {
        if (mode == NTM_MODE_FULL_DU && id >= 6 * N + 4) {
            const int t = id - (6 * N + 4);
            kind = 4 + (t & 1);
            j = (t >> 1) + 1;
            return;
        }
        if (mode == NTM_MODE_BOX) {
            kind = id < N ? 0 : 1;
            j = id < N ? id : id - N;
            return;
        }
        int blk = id / 6, rr = id - 6 * blk;
        if (blk < N && rr < 2) { kind = rr; j = blk; return; }
        int i, c;
        bool upper;
        if (blk < N) { i = blk; c = (rr - 2) & 1; upper = rr >= 4; }
        else { i = N; c = rr & 1; upper = rr >= 2; }
        kind = upper ? 3 : 2;
        j = (i == 0) ? -1 : 2 * (i - 1) + c;
    }
    // u-bound row: its variable j and the sign of its GI normal (+1 lower, -1 upper); -1 otherwise
    __device__ __forceinline__ int unit_row(int id, int Nn, double& sg) const {
        int kind, j;
        decode(id, Nn, kind, j);
        sg = (kind == 0) ? 1.0 : -1.0;
        return kind < 2 ? j : -1;
    }
    template <class W>
    __device__ __forceinline__ double lin(const W& w, int id, int col) const {          // Lin[id][col]
        int kind, j;
        decode(id, w.n(), kind, j);
        if (kind < 2) return (col == j) ? (kind == 0 ? -1.0 : 1.0) : 0.0;
        if (kind >= 4) {
            const double sg = kind == 4 ? 1.0 : -1.0;
            return col == j ? sg : (col == j - 1 ? -sg : 0.0);
        }
        if (j < 0 || col > (j >> 1)) return 0.0;
        double g = w.gt(j, col);
        return kind == 2 ? -g : g;
    }
    template <class W>
    __device__ __forceinline__ double bval(const W& w, int id) const {                  // b[id]
        int kind, j;
        decode(id, w.n(), kind, j);
        if (kind == 0) return -umin;
        if (kind == 1) return umax;
        if (kind >= 4) return du;
        int c = j & 1;
        return kind == 2 ? (-xmin(c) + w.e()[j]) : (xmax(c) - w.e()[j]);
    }
    template <class W>
    __device__ __forceinline__ double rnorm(const W& w, int id) const {
        int kind, j;
        decode(id, w.n(), kind, j);
        if (kind >= 4) return 1.0 / w.idun()[j];
        return kind < 2 ? w.D()[j] : 1.0 / w.irn()[j];
    }

    // constant rows (x_0 rows; state rows with Gamma_r == 0): 0 <= b, to kConstTol,
    // or infeasible (D15, D22)
    template <int P, class W>
    __device__ __forceinline__ bool feasible_const(const W& w, double x0, double x1, int l) const {
        int bad = 0;
        if (has_state()) {
            if (l == 0) {
                bad |= (x0 - xmin(0)) < -kConstTol;
                bad |= (x1 - xmin(1)) < -kConstTol;
                bad |= (xmax(0) - x0) < -kConstTol;
                bad |= (xmax(1) - x1) < -kConstTol;
            }
            for (int r = l; r < 2 * w.n(); r += P) {
                if (w.irn()[r] == 0.0) {
                    int c = r & 1;
                    bad |= (w.e()[r] - xmin(c)) < -kConstTol;
                    bad |= (xmax(c) - w.e()[r]) < -kConstTol;
                }
            }
        }
        return gmaxi<P>(bad) == 0;
    }

    // Most violated inactive row (verify = false), or, with verify = true,
    // whether EVERY row has slack >= -tol * max(vmax, |bc|) (returned in .p).
    // Rows flagged kCandRow (the rows of a warm-start candidate that failed
    // its certificate) are taken first while any of them is violated beyond
    // GI's stopping tolerance: GI may add any violated row, so this only
    // steers it towards the nearby active set.
    template <int P, class W>
    __device__ __forceinline__ Pick check(const W& w, double Vl, int l, bool verify = false, double vmax = 1.0,
                                          const double* y_pre = nullptr) const {   // y_pre[r] = Gamma_r U if given
        const int N = w.n();
        if (mode == NTM_MODE_NONE) { Pick none; none.p = verify ? 0 : -1; none.s = 0.0; none.bc = 0.0; return none; }
        double bv = kInf, bs = 0.0, bbc = 0.0;
        int bid = 0x7fffffff, bad = 0;
        auto consider = [&](double s, int id, double bcv) {
            if (verify) { bad |= s < -1e-9 * fmax(vmax, fabs(bcv)); return; }
            const unsigned char fl = w.aflag()[id];
            constexpr unsigned char kOut = (W::kNN > 32 || W::kNN == 0) ? (kActiveRow | kSkipRow) : kActiveRow;
            if (fl & kOut) return;
            const double key = ((fl & kCandRow) && s < -1e-12 * fmax(vmax, fabs(bcv))) ? s - 1e200 : s;
            if (key < bv || (key == bv && id < bid)) { bv = key; bid = id; bs = s; bbc = bcv; }
        };
        if (l < N) {
            double lo, hi;
            if constexpr (W::kSlim) {                         // (diag_scale_phase's expressions)
                const double Dl = w.D()[l];
                lo = -((-umin) / Dl);
                hi = umax / Dl;
            } else {
                lo = w.vlo()[l];
                hi = w.vhi()[l];
            }
            int idl = (mode == NTM_MODE_BOX) ? l : 6 * l;
            int idh = (mode == NTM_MODE_BOX) ? N + l : 6 * l + 1;
            consider(Vl - lo, idl, lo);
            consider(hi - Vl, idh, -hi);
        }
        if (has_rate() && l >= 1 && l < N) {                 // rate rows on lane j
            const double ir = w.idun()[l];
            const double dU = w.U()[l] - w.U()[l - 1];
            const int id0 = 6 * N + 4 + 2 * (l - 1);
            consider((du - dU) * ir, id0, -(du * ir));
            consider((du + dU) * ir, id0 + 1, -(du * ir));
        }
        if (has_state()) {
            for (int r = l; r < 2 * N; r += P) {
                double ir = w.irn()[r];
                if (ir > 0.0) {
                    int jmax = r >> 1;
                    const double* gr = w.Gt() + r;           // gt(r, j) = gr[gidx(0, j)]
                    double xh = 0.0;
                    if (y_pre) {
                        xh = y_pre[r];
                    } else {
                        // fixed trip count, entries j > jmax masked.  The packed reads stay
                        // inside Gt: gidx(0, j) + r = j(2N-j-1) + r < N(N+1)
                        (void)gr;
                        xh = gamma_row_dot<NTM_CH>(w, r, w.U());
                    }
                    const double er = w.e()[r];
                    xh += er;
                    int c = r & 1, i = jmax + 1;
                    int idmin = (i < N) ? 6 * i + 2 + c : 6 * N + c;
                    consider((xh - xmin(c)) * ir, idmin, (xmin(c) - er) * ir);
                    consider((xmax(c) - xh) * ir, idmin + 2, -((xmax(c) - er) * ir));
                }
            }
        }
        Pick pk;
        if (verify) {
            pk.p = gmaxi<P>(bad);
            pk.s = 0.0;
            pk.bc = 0.0;
            return pk;
        }
        gargmin<P>(bv, bid, bs, bbc);
        pk.p = (bv < kInf) ? bid : -1;
        pk.s = bs;
        pk.bc = bbc;
        return pk;
    }

    // GI normal n_p into w.np(); returns bc_p
    template <int P, class W>
    __device__ __forceinline__ double load_np(const W& w, int p, int l) const {
        double rn = rnorm(w, p);
        if (l < w.n()) w.np()[l] = -((lin(w, p, l) * w.D()[l]) / rn);
        NTM_WSYNC();
        return -(bval(w, p) / rn);
    }
};

// Explicit dense rows Lin U <= b (batched SoA in global memory) for the
// quadprog-level entry point ntm_qp_device.
struct DenseRows {
    static constexpr bool kHasUnitRows = false;
    __device__ int unit_row(int, int, double& sg) const { sg = 0.0; return -1; }
    const double* Lin;  // element (i, j) of scenario s at [s*m*N + i + j*m] (scenario-major)
    const double* b;    // [s*m + i]
    double* rnrm;       // LDS, m entries
    int64_t nv, s;      // variables per scenario (N), scenario index
    int m;

    __device__ int rows() const { return m; }
    template <class W>
    __device__ double lin(const W&, int i, int j) const { return Lin[s * ((int64_t)m * nv) + i + (int64_t)j * m]; }
    template <class W>
    __device__ double bval(const W&, int i) const { return b[s * m + i]; }
    template <class W>
    __device__ double rnorm(const W&, int i) const { return rnrm[i]; }

    template <int P, class W>
    __device__ int prepare_code(const W& w, int l) {
        int bad = 0;
        for (int i = l; i < m; i += P) {
            double ss = 0.0;
            for (int j = 0; j < w.n(); ++j) { double v = lin(w, i, j) * w.D()[j]; ss += v * v; }
            double bi = bval(w, i);
            if (!isfinite(ss) || !isfinite(bi)) bad |= 1;
            rnrm[i] = ss > 0.0 ? sqrt(ss) : 0.0;
            if (!(ss > 0.0) && bi < -kConstTol) bad |= 2;   // constant row violated (D15, D22)
        }
        NTM_WSYNC();
        return gmaxi<P>(bad);
    }
    template <int P, class W>
    __device__ Pick check(const W& w, double Vl, int l, bool verify = false, double vmax = 1.0) const {
        double bvv = kInf, bs = 0.0, bbc = 0.0;
        int bid = 0x7fffffff, bad = 0;
        for (int i = l; i < m; i += P) {
            double rn = rnrm[i];
            if (rn > 0.0 && (verify || !(w.aflag()[i] & kActiveRow))) {
                double sl = 0.0;
                for (int j = 0; j < w.n(); ++j) sl -= ((lin(w, i, j) * w.D()[j]) / rn) * w.V()[j];
                double bi = bval(w, i) / rn;
                sl += bi;
                if (verify) bad |= sl < -1e-9 * fmax(vmax, fabs(bi));
                else if (sl < bvv || (sl == bvv && i < bid)) { bvv = sl; bid = i; bs = sl; bbc = -bi; }
            }
        }
        Pick pk;
        if (verify) {
            pk.p = gmaxi<P>(bad);
            pk.s = 0.0;
            pk.bc = 0.0;
            return pk;
        }
        gargmin<P>(bvv, bid, bs, bbc);
        pk.p = (bvv < kInf) ? bid : -1;
        pk.s = bs;
        pk.bc = bbc;
        return pk;
    }
    template <int P, class W>
    __device__ double load_np(const W& w, int p, int l) const {
        double rn = rnrm[p];
        if (l < w.n()) w.np()[l] = -((lin(w, p, l) * w.D()[l]) / rn);
        NTM_WSYNC();
        return -(bval(w, p) / rn);
    }
};

// ---------------------------------------------------------------------------
// small dense kernels on a group's LDS matrices (col-major, leading dim LD)
// ---------------------------------------------------------------------------
// Element (i, j) of a small matrix lives at A[i*RS + j*CS] (col-major: RS = 1,
// CS = LD; the polish's K is stored transposed: RS = LD, CS = 1).
// left-looking Cholesky of the n x n lower triangle of A, in place; the
// reciprocals of the diagonal go to rdiag[0..n) (the triangular solves then
// multiply instead of divide); false if not PD
template <int P>
__device__ __forceinline__ bool chol_inplace(double* A, int n, int RS, int CS, int l, double* rdiag) {
    for (int k = 0; k < n; ++k) {
        double s = 0.0;
        if (l >= k && l < n) {
            s = sub_dot<NTM_CH>(A[l * RS + k * CS], A + l * RS, CS, A + k * RS, CS, 0, k);
        }
        double dk = gbcast<P>(s, k);
        if (!(dk > 0.0) || !(dk < kInf)) return false;
        const double il = rsqrt_nr(dk);
        const double lk = dk * il;
        if (l > k && l < n) A[l * RS + k * CS] = s * il;
        if (l == k) { A[k * RS + k * CS] = lk; rdiag[k] = il; }
        NTM_WSYNC();
    }
    return true;
}
// chol_inplace on GI's factor storage (WS::gr / grow: rows of the lower triangle)
template <int P, class W>
__device__ __forceinline__ bool chol_gr(const W& w, int n, int l, double* rdiag) {
    if constexpr (!W::kGiLdsL) {
        return chol_inplace<P>(w.R(), n, 1, w.ldj(), l, rdiag);
    } else {
        for (int k = 0; k < n; ++k) {
            double s = 0.0;
            if (l >= k && l < n) s = sub_dot<NTM_CH>(w.grL(l, k), w.grow(l), 1, w.grow(k), 1, 0, k);
            const double dk = gbcast<P>(s, k);
            if (!(dk > 0.0) || !(dk < kInf)) return false;
            const double il = rsqrt_nr(dk);
            const double lk = dk * il;
            if (l > k && l < n) w.grL(l, k) = s * il;
            if (l == k) { w.grL(k, k) = lk; rdiag[k] = il; }
            NTM_WSYNC();
        }
        return true;
    }
}
// lane i holds b_i in `v`; returns x_i of L x = b (L lower, rdiag = 1/diag)
template <int P>
__device__ __forceinline__ double fwd_lanes(const double* L, const double* rdiag, int n, int RS, int CS, double v, int l) {
    double acc = (l < n) ? v : 0.0, x = 0.0;
    for (int k = 0; k < n; ++k) {
        double xk = gbcast<P>(acc, k) * rdiag[k];
        if (l == k) x = xk;
        if (l > k && l < n) acc -= L[l * RS + k * CS] * xk;
    }
    return x;
}
// lane i holds b_i in `v`; returns x_i of L' x = b (L lower, rdiag = 1/diag)
template <int P>
__device__ __forceinline__ double bwd_lanes(const double* L, const double* rdiag, int n, int RS, int CS, double v, int l) {
    double acc = (l < n) ? v : 0.0, x = 0.0;
    for (int k = n - 1; k >= 0; --k) {
        double xk = gbcast<P>(acc, k) * rdiag[k];
        if (l == k) x = xk;
        if (l < k) acc -= L[k * RS + l * CS] * xk;
    }
    return x;
}

// ---------------------------------------------------------------------------
// Goldfarb-Idnani dual active set on the Jacobi-scaled problem.
//   min 1/2 V'G~V + F~'V  s.t.  n_i'V >= bc_i (rows from the provider)
// Pre:  w.R() holds G~ (lower, col-major), w.F() holds F~, w.aflag() cleared.
// Post: w.V() holds V, w.act()[0..*q_out) the active rows; returns the quadprog
// exit flag.  Adds use a Householder reflector on J's trailing columns (one
// reduction instead of a Givens chain); drops restore R with a Givens sweep
// (Goldfarb & Idnani 1983, section 3).
// ---------------------------------------------------------------------------
template <int P, class Rows, class W>
__device__ __forceinline__ int gi_solve(const W& w, const Rows rows, bool has_rows, int nrows, int l, int* iters_out, int* q_out,
                        int nwarm = 0) {
    const int N = w.n();
    const int JR = w.jr(), JC = w.jc();     // J(r, c) at r JR + c JC (T alike)
    *iters_out = 0;
    *q_out = 0;
    NTM_T0(tg);
    // 1. Cholesky G~ = L L' (in place in w.R())
    if (!chol_gr<P>(w, N, l, w.ldi())) return NTM_EXIT_NONFINITE;
    // 2. J = L^{-T}: lane c computes row c of J (= column c of L^{-1})
    if (l < N) {
        for (int i = 0; i < N; ++i) {
            double x = 0.0;
            if (i >= l) {
                x = sub_dot<NTM_CH>((i == l) ? 1.0 : 0.0, w.grow(i), w.grs(), w.J() + l * JR, JC, l, i);
                x *= w.ldi()[i];
            }
            w.J()[l * JR + i * JC] = x;
        }
    }
    NTM_WSYNC();
    // 3. unconstrained minimiser V = -J J' F~
    double Vl = 0.0;
    {
        double t = 0.0;
        if (l < N) t = dot_batched<NTM_CH>(w.J() + l * JC, JR, w.F(), 1, N);
        if (l < N) w.d()[l] = t;
        NTM_WSYNC();
        if (l < N) {
            const double v = dot_batched<NTM_CH>(w.J() + l * JR, JC, w.d(), 1, N);
            Vl = -v;
            w.V()[l] = Vl;
            w.U()[l] = w.D()[l] * Vl;
        }
        NTM_WSYNC();
    }
    NTM_ACC(ST_GI_FACT, tg);
    if (!has_rows) return NTM_EXIT_OPTIMAL;
    const bool useT = w.useT();
    if (useT && l < N) for (int b = 0; b < N; ++b) w.T()[l * JR + b * JC] = 0.0;
    const int max_iter = 10 * (N + nrows) + 50;
    int q = 0, it = 0;
    // Warm start: the rows w.sidx()[0..nwarm) of a failed
    // candidate are added first without primal steps (Householder on J, R and T
    // gain their columns), then V is set to the equality-constrained optimum on
    // that set, V = -J2 J2' F~ + J1 R^{-T} bc, with multipliers
    // u = R^{-1} (R^{-T} bc + J1' F~) (matvecs with T = R^{-1} for N <= 32,
    // triangular solves on R above).
    // Rows dependent on those already added are skipped (a failed candidate often
    // holds a state row and a bound row that fix the same variable).  If every
    // u >= 0 the pair satisfies GI's invariant (optimal for the active set, dual
    // feasible) and the iteration continues from it; otherwise the caller
    // re-forms G~ and runs GI cold.
    if (nwarm > 0 && has_rows) {
        NTM_CNT(CN_WARM_TRY);
        bool okw = true;
        for (int a = 0; a < nwarm; ++a) {
            const int p = uni<P>(w.sidx()[a]);
            int ej = -1;
            double esg = 0.0, bcp, dl = 0.0;
            if constexpr (Rows::kHasUnitRows) {
                ej = uni<P>(rows.unit_row(p, N, esg));
                esg = uni<P>(esg);
            }
            if (ej >= 0) {                        // u-bound row: n_p = -+e_j, d = J' n_p a signed row of J
                bcp = uni<P>(-(rows.bval(w, p) / rows.rnorm(w, p)));
                if (l < N) dl = esg * w.J()[ej * JR + l * JC];
            } else {
                bcp = uni<P>(rows.template load_np<P>(w, p, l));
                if (l < N) dl = dot_batched<NTM_CH>(w.J() + l * JC, JR, w.np(), 1, N);
            }
            if (l < N) { w.d()[l] = (l >= q) ? dl : 0.0; w.dr()[l] = (l < q) ? dl : 0.0; }
            NTM_WSYNC();
            double rl = 0.0;
            if (useT && l < N) rl = dot_batched<NTM_CH>(w.T() + l * JR, JC, w.dr(), 1, N);
            const double zn = gsum<P>((l >= q && l < N) ? dl * dl : 0.0);
            const double dnrm = gsum<P>(dl * dl);
            if (q >= N) { NTM_CNT(CN_WARM_FULL); break; }
            if (zn <= 1e-300 || zn <= (kDepTol * kDepTol) * dnrm) {   // dependent on the rows added: skip it
                NTM_CNT(CN_WARM_DEP);
                NTM_WSYNC();
                continue;
            }
            const double nrm = sqrt(zn);
            const double dqv = gbcast<P>(dl, q);
            double h = dqv;
            if (q < N - 1) {
                h = (dqv >= 0.0) ? -nrm : nrm;
                double vl = (l == q) ? dl - h : ((l > q && l < N) ? dl : 0.0);
                if (l < N) w.hv()[l] = vl;
                double vtv = gsum<P>(vl * vl);
                NTM_WSYNC();
                if (l < N) {
                    const double dot = dot_batched<NTM_CH>(w.J() + l * JR, JC, w.hv(), 1, N);
                    const double f = 2.0 * dot / vtv;
                    axpy_sub<NTM_CH>(w.J() + l * JR, w.hv(), f, q, N, JC);
                }
            }
            const double ih = 1.0 / h;
            if (l < q) {
                w.gr(l, q) = dl;
                if (useT) w.T()[l * JR + q * JC] = -rl * ih;
            }
            if (l == q) {
                w.gr(q, q) = h;
                if (useT) w.T()[q * JR + q * JC] = ih;
                w.act()[q] = p;
                w.aflag()[p] = kActiveRow;
                w.Vb()[q] = bcp;                     // bc of active row q (scratch)
            }
            ++q;
            NTM_WSYNC();
        }
        if (okw) {
            // c = J' F~ (lane k), wv = (T' bc)_k for k < q
            double c = 0.0, wv = 0.0;
            if (l < N) c = dot_batched<NTM_CH>(w.J() + l * JC, JR, w.F(), 1, N);
            if (useT) {
                if (l < q) wv = dot_range<NTM_CH>(w.T() + l * JC, JR, w.Vb(), 1, 0, l + 1);
            } else {                                 // long horizons: R' wv = bc by forward substitution
                double acc = (l < q) ? w.Vb()[l] : 0.0;
                for (int k2 = 0; k2 < q; ++k2) {
                    const double xk = gbcast<P>(acc, k2) / w.gr(k2, k2);
                    if (l == k2) wv = xk;
                    if (l > k2 && l < q) acc -= w.gr(k2, l) * xk;
                }
            }
            if (l < N) {
                w.d()[l] = (l >= q) ? c : 0.0;
                w.dr()[l] = (l < q) ? wv : 0.0;
                w.np()[l] = (l < q) ? wv + c : 0.0;
            }
            NTM_WSYNC();
            double v = 0.0, u = 0.0;
            if (l < N) for (int k2 = 0; k2 < N; ++k2) v += w.J()[l * JR + k2 * JC] * (w.dr()[k2] - w.d()[k2]);
            if (useT) {
                if (l < q) u = dot_range<NTM_CH>(w.T() + l * JR, JC, w.np(), 1, l, q);
            } else {                                 // R u = wv + c1 by back substitution
                double acc = (l < q) ? w.np()[l] : 0.0;
                for (int b = q - 1; b >= 0; --b) {
                    const double ub = gbcast<P>(acc, b) / w.gr(b, b);
                    if (l == b) u = ub;
                    if (l < b) acc -= w.gr(l, b) * ub;
                }
            }
            const double uabs = gmax<P>(l < q ? fabs(u) : 0.0);
            const double umin = -gmax<P>(l < q ? -u : -kInf);
            okw = !(umin < -1e-9 * fmax(1.0, uabs)) && gmaxi<P>((l < N && !isfinite(v)) ? 1 : 0) == 0;
            if (!okw) {
                NTM_CNT(CN_WARM_NEG);
                // the added rows whose multipliers are >= 0: the caller's second warm pass
                const int lane = threadIdx.x & 63;
                const unsigned long long gm = (P == 64) ? ~0ull : (((1ull << P) - 1ull) << (lane & ~(P - 1)));
                const bool keep = l < q && u >= 0.0;
                const unsigned long long bk = __ballot(keep) & gm;
                const int id = (l < q) ? w.act()[l] : 0;
                NTM_WSYNC();
                if (keep) w.sidx()[__popcll(bk & ((1ull << lane) - 1ull))] = id;
                *q_out = uni<P>((int)__popcll(bk));
            }
            if (okw) {
                Vl = (l < N) ? v : 0.0;
                if (l < N) { w.V()[l] = Vl; w.U()[l] = w.D()[l] * Vl; }
                if (l < q) w.uu()[l] = fmax(0.0, u);
                NTM_CNT(CN_WARM_OK);
            }
            NTM_WSYNC();
        }
        if (!okw) {
            if (l < q) w.aflag()[w.act()[l]] = kCandRow;   // back to steering flags
            NTM_WSYNC();
            return kGiWarmRejected;                        // *q_out: rows kept in w.sidx() (0: none)
        }
    }
    NTM_ACC(ST_GI_WARM, tg);                               // the warm start's adds (not the first check)
    for (;;) {
        const double vmax = gmax<P>(l < N ? fabs(Vl) : 0.0);
        Pick pk = rows.template check<P>(w, Vl, l, false, fmax(1.0, vmax));
        NTM_ACC(ST_GI_CHECK, tg);
        NTM_CNT(CN_CHECK);
        NTM_TRACE("GI it %d q %d pick %d s %.6e bc %.6e\n", it, q, pk.p, pk.s, pk.bc);
        if (pk.p < 0 || pk.s >= -1e-12 * fmax(fmax(1.0, vmax), fabs(pk.bc))) {
            *iters_out = it;
            *q_out = q;
            return NTM_EXIT_OPTIMAL;
        }
        const int p = pk.p;
        const double bcp = uni<P>(rows.template load_np<P>(w, p, l));
        // u-bound rows have n_p = -+e_j: d = J' n_p is then a signed row of J
        int ej = -1;
        double esg = 0.0;
        if constexpr (Rows::kHasUnitRows) {
            ej = uni<P>(rows.unit_row(p, N, esg));
            esg = uni<P>(esg);
        }
        double upq = 0.0;   // multiplier of the constraint being added
        for (;;) {
            if (++it > max_iter) { *iters_out = it; *q_out = q; return NTM_EXIT_MAXITER; }
            // d = J' n_p
            double dl = 0.0;
            if (ej >= 0) {
                if (l < N) dl = esg * w.J()[ej * JR + l * JC];
            } else if (l < N) {
                dl = dot_batched<NTM_CH>(w.J() + l * JC, JR, w.np(), 1, N);
            }
            // d split at q: d2 = d[q:N] (w.d) and d1 = d[0:q] (w.dr), zero elsewhere, so
            // both matvecs run full fixed-length rows (unrolled, loads batched)
            if (l < N) { w.d()[l] = (l >= q) ? dl : 0.0; w.dr()[l] = (l < q) ? dl : 0.0; }
            NTM_WSYNC();
            // z = J2 d2 (primal direction) and r = T d1 = R^{-1} d1 (negative dual direction)
            double zl = 0.0, rl = 0.0;
            if (l < N) {
                zl = dot_batched<NTM_CH>(w.J() + l * JR, JC, w.d(), 1, N);
                if (useT) rl = dot_batched<NTM_CH>(w.T() + l * JR, JC, w.dr(), 1, N);
            }
            if (!useT) {                       // long horizons: back substitution on R
                double acc = (l < q) ? dl : 0.0;
                for (int b = q - 1; b >= 0; --b) {
                    const double rb = gbcast<P>(acc, b) / w.gr(b, b);
                    if (l == b) rl = rb;
                    if (l < b) acc -= w.gr(l, b) * rb;
                }
            }
            // partial (dual) step length t1
            double ratio = (l < q && rl > 0.0) ? w.uu()[l] / rl : kInf;
            int li = l;
            gargmin<P>(ratio, li);
            const double t1 = ratio;
            // full (primal) step length t2.  z'n_p = |d2|^2 exactly (z = J2 d2),
            // never negative; n_p counts as dependent on the active rows when
            // |d2| <= kDepTol |d|
            double npl = (l < N) ? w.np()[l] : 0.0;
            double zn = gsum<P>((l >= q && l < N) ? dl * dl : 0.0);
            double sp = gsum<P>(npl * Vl) - bcp;
            double dnrm = gsum<P>(dl * dl);
            double t2 = (zn <= 1e-300 || zn <= (kDepTol * kDepTol) * dnrm) ? kInf : -sp / zn;
            double t = fmin(t1, t2);
            NTM_TRACE("   dir: t1 %.6e (pos %d) t2 %.6e zn %.6e dn %.6e sp %.6e\n", t1, li, t2, zn, dnrm, sp);
            NTM_ACC(ST_GI_DIR, tg);
            if (!(t < kInf)) { *iters_out = it; *q_out = q; return NTM_EXIT_INFEASIBLE; }
            if (l < q) w.uu()[l] = fmax(0.0, w.uu()[l] - t * rl);
            upq += t;
            if (t2 < kInf) {
                Vl += t * zl;
                if (l < N) { w.V()[l] = Vl; w.U()[l] = w.D()[l] * Vl; }
                if (t == t2) {
                    // ---- add p: Householder on d[q:N] -> J(:, q:N) ----
                    double dq2 = (l >= q && l < N) ? dl * dl : 0.0;
                    double nrm = sqrt(gsum<P>(dq2));
                    double dqv = gbcast<P>(dl, q);
                    double h = dqv;
                    if (q < N - 1 && nrm > 0.0) {
                        h = (dqv >= 0.0) ? -nrm : nrm;
                        double vl = (l == q) ? dl - h : ((l > q && l < N) ? dl : 0.0);
                        if (l < N) w.hv()[l] = vl;          // zero for l < q
                        double vtv = gsum<P>(vl * vl);
                        NTM_WSYNC();
                        if (l < N) {
                            const double dot = dot_batched<NTM_CH>(w.J() + l * JR, JC, w.hv(), 1, N);
                            const double f = 2.0 * dot / vtv;
                            axpy_sub<NTM_CH>(w.J() + l * JR, w.hv(), f, q, N, JC);
                        }
                    }
                    // R gains column q = [d1; h]; T = R^{-1} gains column q = [-r/h; 1/h]
                    const double ih = 1.0 / h;
                    if (l < q) {
                        w.gr(l, q) = dl;
                        if (useT) w.T()[l * JR + q * JC] = -rl * ih;
                    }
                    if (l == q) {
                        w.gr(q, q) = h;
                        if (useT) w.T()[q * JR + q * JC] = ih;
                        w.act()[q] = p;
                        w.aflag()[p] = kActiveRow;
                        w.uu()[q] = upq;
                    }
                    ++q;
                    NTM_WSYNC();
                    NTM_ACC(ST_GI_ADD, tg);
                    break;
                }
            }
            // ---- drop active position li (partial or dual-only step) ----
            const int l0 = li;
            const int dropped = uni<P>(w.act()[l0]);
            NTM_WSYNC();
            if (l < q) {
                // column shift: rows l <= c + 1 (R upper, plus the subdiagonal the shift
                // creates); the rows below are zero and, in the packed LDS storage
                // (kGiLds), share their slots with the upper triangle
                for (int c = l0; c < q - 1; ++c)
                    if (!W::kGiLds || l <= c + 1) w.gr(l, c) = w.gr(l, c + 1);
                w.gr(l, q - 1) = 0.0;
            }
            {
                int an = 0;
                double un = 0.0;
                if (l >= l0 && l < q) { an = w.act()[l + 1]; un = w.uu()[l + 1]; }
                NTM_WSYNC();
                if (l >= l0 && l < q) { w.act()[l] = an; w.uu()[l] = un; }
                if (l == 0) w.aflag()[dropped] = 0;
            }
            NTM_WSYNC();
            for (int j = l0; j < q - 1; ++j) {
                double a = uni<P>(w.gr(j, j)), bq = uni<P>(w.gr(j + 1, j));
                double hh = hypot(a, bq);
                double cc = 1.0, ss = 0.0;
                if (hh != 0.0) { cc = a / hh; ss = bq / hh; }
                NTM_WSYNC();
                if (l >= j && l < q - 1) {
                    double r1 = w.gr(j, l), r2 = w.gr(j + 1, l);
                    double nr = cc * r1 + ss * r2;
                    w.gr(j, l) = nr;
                    w.gr(j + 1, l) = (l == j) ? 0.0 : (-ss * r1 + cc * r2);
                }
                if (l < N) {
                    double j1 = w.J()[l * JR + j * JC], j2 = w.J()[l * JR + (j + 1) * JC];
                    w.J()[l * JR + j * JC] = cc * j1 + ss * j2;
                    w.J()[l * JR + (j + 1) * JC] = -ss * j1 + cc * j2;
                }
                if (useT && l < q) {   // T <- T G_j' (the columns rotate like J's)
                    double t1v = w.T()[l * JR + j * JC], t2v = w.T()[l * JR + (j + 1) * JC];
                    w.T()[l * JR + j * JC] = cc * t1v + ss * t2v;
                    w.T()[l * JR + (j + 1) * JC] = -ss * t1v + cc * t2v;
                }
                NTM_WSYNC();
            }
            // R'^{-1} = (T Q) without row l0 and column q-1.  Lane c owns column c:
            // rows l0+1..q-1 move up one; the discarded column q-1 is cleared
            if (useT && l < q - 1) {
                for (int a = l0; a < q - 1; ++a) w.T()[a * JR + l * JC] = w.T()[(a + 1) * JR + l * JC];
                w.T()[(q - 1) * JR + l * JC] = 0.0;
            } else if (useT && l == q - 1) {
                for (int a = 0; a < q; ++a) w.T()[a * JR + l * JC] = 0.0;
            }
            NTM_WSYNC();
            --q;
            NTM_ACC(ST_GI_DROP, tg);
        }
    }
}

// ---------------------------------------------------------------------------
// Exact re-solve on GI's final active set (oracle: polish_active_set).
//   Rows with a single non-zero fix their variable exactly (U_j = b/Lin_j);
//   the other active rows S are equality constraints on the free variables:
//   masked Cholesky of G~ (fixed rows/cols -> identity), Schur complement
//   K = E G~_FF^{-1} E', then V_F.  Accepted only if the KKT certificate
//   holds; otherwise w.U() keeps GI's solution.  Pre: w.V() = GI solution.
//   Writes w.U() (unscaled U).  G~ comes from Gamma (gram, structured rows) or
//   from Gsave (a copy taken before the GI factorisation, dense rows).
// ---------------------------------------------------------------------------
template <int P, class Rows, class W>
__device__ __forceinline__ bool polish_phase(const Prob& pb, const W& w, const Rows* rows, int q, int l,
                             const double* Gsave, bool g_in_R, bool verify_only, int* ns_out) {
    const int N = w.n(), LD = w.ldj(), LDJ = w.ldj();
    const double Vgi = (l < N) ? w.V()[l] : 0.0;
    // --- classify active rows ---
    if (l < N) w.fx()[l] = 0;
    NTM_WSYNC();
    int isgen = 0, fixj = -1;
    double ufix = 0.0;
    int id = -1;
    if (l < q) {
        id = w.act()[l];
        int nnz = 0;
        for (int j = 0; j < N; ++j) if (rows->lin(w, id, j) != 0.0) { ++nnz; fixj = j; }
        if (nnz == 1) ufix = rows->bval(w, id) / rows->lin(w, id, fixj);
        else isgen = 1;
    }
    double nfix = 0.0;   // GI normal entry of the single-entry row (for its multiplier)
    if (l < q && !isgen) nfix = -((rows->lin(w, id, fixj) * w.D()[fixj]) / rows->rnorm(w, id));
    const unsigned long long gmask = (P == 64) ? ~0ull : (((1ull << P) - 1ull) << ((threadIdx.x & 63) & ~(P - 1)));
    const unsigned long long bal = __ballot(isgen) & gmask;
    const int nS = __popcll(bal);
    const int spos = __popcll(bal & ((1ull << (threadIdx.x & 63)) - 1ull));
    if (l < q) {
        if (isgen) w.sidx()[spos] = id;
        else { w.fx()[fixj] = 1; w.Uf()[fixj] = ufix; w.hv()[fixj] = nfix; }
    }
    NTM_WSYNC();
    const bool fixed = (l < N) && w.fx()[l];
    const double vb = fixed ? w.Uf()[l] / w.D()[l] : 0.0;
    if (l < N) w.Vb()[l] = vb;
    if (ns_out) *ns_out = nS;
    // --- G~ again (bit-identical to the GI's copy), g = F~ + G~_{:,B} V_B ---
    if (g_in_R) {
        // candidate verification: G~ is still intact in w.R()
    } else if (Gsave) {
        if (l < N) for (int j = 0; j <= l; ++j) w.R()[l + j * LD] = Gsave[l + j * LD];
    } else {
        gram_rows<P>(pb, w, w.R(), l);
        NTM_WSYNC();
        (void)scale_gram<P>(w, w.R(), l);
    }
    NTM_WSYNC();
    double gl = 0.0;
    if (l < N) {
        gl = w.F()[l];
        for (int j = 0; j < N; ++j)
            if (w.fx()[j]) gl += ((j <= l) ? w.R()[l + j * LD] : w.R()[j + l * LD]) * w.Vb()[j];
        if (fixed) gl = 0.0;
    }
    NTM_WSYNC();
    if (l < N) {   // mask fixed rows/cols to identity (row l, columns <= l)
        for (int j = 0; j <= l; ++j)
            if (fixed || w.fx()[j]) w.R()[l + j * LD] = (j == l) ? 1.0 : 0.0;
    }
    NTM_WSYNC();
    bool ok = chol_inplace<P>(w.R(), N, 1, LD, l, w.ldi());
    double vfin = 0.0;
    if (ok) {
        double wl = fwd_lanes<P>(w.R(), w.ldi(), N, 1, LD, gl, l);      // w = L^{-1} g
        double tl = -wl;
        if (nS > 0) {
            // E' into Y (= w.J(), row-major N x nS), h_s
            if (l < N) {
                for (int s = 0; s < nS; ++s) {
                    int rid = w.sidx()[s];
                    double nj = -((rows->lin(w, rid, l) * w.D()[l]) / rows->rnorm(w, rid));
                    w.J()[l * LDJ + s] = fixed ? 0.0 : nj;
                }
            }
            double hs = 0.0;
            if (l < nS) {
                int rid = w.sidx()[l];
                double rn = rows->rnorm(w, rid);
                hs = -(rows->bval(w, rid) / rn);
                for (int j = 0; j < N; ++j)
                    if (w.fx()[j]) hs -= (-((rows->lin(w, rid, j) * w.D()[j]) / rn)) * w.Vb()[j];
            }
            if (l < N) w.d()[l] = wl;
            NTM_WSYNC();
            // Y = L^{-1} E' : lane s solves column s in place
            if (l < nS) {
                for (int i = 0; i < N; ++i) {
                    double y = w.J()[i * LDJ + l];
                    for (int k = 0; k < i; ++k) y -= w.R()[i + k * LD] * w.J()[k * LDJ + l];
                    w.J()[i * LDJ + l] = y * w.ldi()[i];
                }
            }
            NTM_WSYNC();
            // K = Y'Y (lower triangle stored transposed in R's strict upper part); rhs = h + Y'w
            double* K = w.R() + LD;
            double rhs = 0.0;
            if (l < nS) {
                for (int c = 0; c <= l; ++c) {
                    double sK = 0.0;
                    for (int i = 0; i < N; ++i) sK += w.J()[i * LDJ + l] * w.J()[i * LDJ + c];
                    K[l * LD + c] = sK;
                }
                rhs = hs;
                for (int i = 0; i < N; ++i) rhs += w.J()[i * LDJ + l] * w.d()[i];
            }
            NTM_WSYNC();
            ok = chol_inplace<P>(K, nS, LD, 1, l, w.kdi());
            if (ok) {
                double t1 = fwd_lanes<P>(K, w.kdi(), nS, LD, 1, rhs, l);
                double mu = bwd_lanes<P>(K, w.kdi(), nS, LD, 1, t1, l);
                if (l < nS) w.np()[l] = mu;
                NTM_WSYNC();
                if (l < N) {
                    double sY = 0.0;
                    for (int a = 0; a < nS; ++a) sY += w.J()[l * LDJ + a] * w.np()[a];
                    tl = sY - wl;
                }
            }
        }
        if (ok) {
            double vl = bwd_lanes<P>(w.R(), w.ldi(), N, 1, LD, tl, l);  // V_F = L^{-T} t
            vfin = fixed ? vb : vl;
        }
    }
    ok = gmaxi<P>(ok ? 0 : 1) == 0;
    if (ok && Gsave) {
        // One step of fixed-precision iterative refinement on the KKT residual with
        // the same factors.  The range-space solve goes through L = chol(G~_FF),
        // which loses digits when G~_FF is nearly singular although the KKT system
        // is well conditioned (input-rate rows holding the last inputs: up to
        // ~1e-8 umax off the exact optimum); the residual of the well-conditioned
        // system, solved again, restores them.  Correction (dV, dmu):
        //   G~_FF dV - E' dmu = -r1,  r1 = G~V + F~ - E'mu (free variables)
        //   E dV = -r2,               r2 = n_s'V - bc_s   (general rows)
        if (l < N) w.V()[l] = vfin;
        NTM_WSYNC();
        double r1 = 0.0, r2 = 0.0;
        if (l < N && !fixed) {
            r1 = w.F()[l];
            for (int j = 0; j < N; ++j) r1 += ((j <= l) ? Gsave[l + j * LD] : Gsave[j + l * LD]) * w.V()[j];
            for (int s = 0; s < nS; ++s) {
                const int rid = w.sidx()[s];
                r1 -= w.np()[s] * (-((rows->lin(w, rid, l) * w.D()[l]) / rows->rnorm(w, rid)));
            }
        }
        if (l < nS) {
            const int rid = w.sidx()[l];
            const double rn = rows->rnorm(w, rid);
            double nv = 0.0;
            for (int j = 0; j < N; ++j) nv += (-((rows->lin(w, rid, j) * w.D()[j]) / rn)) * w.V()[j];
            r2 = nv + rows->bval(w, rid) / rn;
        }
        const double dwl = fwd_lanes<P>(w.R(), w.ldi(), N, 1, LD, r1, l);
        double dt = -dwl;
        if (nS > 0) {
            if (l < N) w.d()[l] = dwl;
            NTM_WSYNC();
            double rhs = 0.0;
            if (l < nS) {
                rhs = -r2;
                for (int i = 0; i < N; ++i) rhs += w.J()[i * LDJ + l] * w.d()[i];
            }
            const double* K = w.R() + LD;
            const double t1 = fwd_lanes<P>(K, w.kdi(), nS, LD, 1, rhs, l);
            const double dmu = bwd_lanes<P>(K, w.kdi(), nS, LD, 1, t1, l);
            NTM_WSYNC();
            if (l < nS) {
                w.d()[l] = dmu;
                w.np()[l] += dmu;
            }
            NTM_WSYNC();
            if (l < N) {
                double sY = 0.0;
                for (int a = 0; a < nS; ++a) sY += w.J()[l * LDJ + a] * w.d()[a];
                dt = sY - dwl;
            }
        }
        const double dv = bwd_lanes<P>(w.R(), w.ldi(), N, 1, LD, dt, l);
        const double vr = fixed ? vb : vfin + dv;
        ok = gmaxi<P>((l < N && !isfinite(vr)) ? 1 : 0) == 0;
        if (ok) vfin = vr;
    }
    if (ok) {
        // ---- KKT certificate ----
        if (l < N) w.V()[l] = vfin;
        NTM_WSYNC();
        double vmax = gmax<P>(l < N ? fabs(vfin) : 0.0);
        Pick vf = rows->template check<P>(w, vfin, l, true, fmax(1.0, vmax));
        ok = vf.p == 0;
        // gradient G~V + F~ (G~ itself is factored now)
        double res = 0.0;
        if (Gsave) {
            if (l < N) {
                res = w.F()[l];
                for (int j = 0; j < N; ++j)
                    res += ((j <= l) ? Gsave[l + j * LD] : Gsave[j + l * LD]) * w.V()[j];
            }
        } else {
            // through Gamma: y = Gamma (D V), grad_j = D_j 2 Gamma_j' Om y + F~_j
            for (int r = l; r < 2 * N; r += P) {
                double y = 0.0;
                for (int j = 0; j <= (r >> 1); ++j) y += w.gt(r, j) * (w.D()[j] * w.V()[j]);
                w.xp()[r] = y;              // scratch: xp is rewritten by the rollout
            }
            NTM_WSYNC();
            if (l < N) {
                double g2 = 0.0;
                for (int i = l; i < N; ++i) {
                    double y0 = w.xp()[2 * i], y1 = w.xp()[2 * i + 1];
                    double o0 = pb.Q[0] * y0 + pb.Q[1] * y1, o1 = pb.Q[2] * y0 + pb.Q[3] * y1;
                    g2 += w.gt(2 * i, l) * o0 + w.gt(2 * i + 1, l) * o1;
                }
                res = w.D()[l] * (2 * g2) + w.F()[l];
            }
        }
        if (l < N) {
            for (int s = 0; s < nS; ++s) {
                int rid = w.sidx()[s];
                res -= w.np()[s] * (-((rows->lin(w, rid, l) * w.D()[l]) / rows->rnorm(w, rid)));
            }
        }
        // multipliers: mu_s (general rows) and res_j / n_j (fixed variables)
        double mval = 0.0;
        bool has = false;
        if (l < nS) { mval = w.np()[l]; has = true; }
        if (fixed) {
            double lam = res / w.hv()[l];
            mval = has ? fmin(mval, lam) : lam;
            has = true;
        }
        double mabs = gmax<P>(has ? fabs(mval) : 0.0);
        double mmin = -gmax<P>(has ? -mval : -kInf);
        ok = ok && !(mmin < -1e-9 * fmax(1.0, mabs));
    }
    if (verify_only && !ok) {
        if (l < N) w.V()[l] = Vgi;
        NTM_WSYNC();
        return false;
    }
    if (l < N) {
        double u;
        if (ok) u = fixed ? w.Uf()[l] : vfin * w.D()[l];
        else u = Vgi * w.D()[l];
        w.U()[l] = u;
        w.V()[l] = ok ? vfin : Vgi;
    }
    NTM_WSYNC();
    return ok;
}

// ---------------------------------------------------------------------------
// Exact re-solve on an active set, compact form for the implicit getWLc rows
// (oracle: polish_active_set).  Used both to VERIFY a warm-start candidate
// (the active set of LPV iteration it-2) and to POLISH the Goldfarb-Idnani
// result.  Single-entry rows fix their variable exactly (U_j = b/Lin_j); the
// nF free variables and the nS general (state) rows form a small KKT system
//   min 1/2 V_F' G~_FF V_F + g_F' V_F  s.t. E V_F = h
// solved in compact nF / nS coordinates: G~_FF from Gamma's free columns
// (bit-identical entries to the full Gram), g_F = D_F 2 Gamma_F' Om (Gamma U_B
// + e - r) by two O(N) passes, Cholesky of G~_FF, Schur complement
// K = E G~_FF^{-1} E'.  Accepted only if the KKT certificate holds (primal
// slack on every row, multiplier signs).  Writes w.U()/w.V() on success or
// when !verify_only (then GI's V is kept); returns success.
// ---------------------------------------------------------------------------
// mult_out (optional, LDS): every active row's multiplier (GI form, n'V >= bc rows),
// by active position, written when the certificate's multipliers are formed.
// dir_p >= 0 (the certified dual path of qp_phase): no solve at all.  The active
// set of q rows must be echelon (sq); the certificate's multiplier pass then runs
// with row dir_p's normal n_p in place of the gradient, i.e. it writes to mult_out
// the r with sum_i r_i n_i = n_p (n_p dependent on the set: Goldfarb-Idnani's
// dual-only step direction).  Returns false for any other set.  V and U are left
// untouched.
template <int P, class W>
__device__ __forceinline__ bool polish_compact(const Prob& pb, const W& w, const StructRows rows, int q, int l, bool verify_only,
                               int* ns_out, int* fail_kind = nullptr, int* fail_pos = nullptr,
                               double* v_out = nullptr, double* mult_out = nullptr, int dir_p = -1) {
    const int N = w.n(), LD = w.ldj(), LDJ = w.ldj();
    const OmQ<qi_on<W>()> om(pb.Q);
    const bool dir = dir_p >= 0;
    const double Vprev = (l < N) ? w.V()[l] : 0.0;
    constexpr int kSplitMask = split_ok<P, W>() ? (W::kFar ? NTM_SPLIT_CERT_FAR : NTM_SPLIT_CERT) : 0;
    constexpr bool kSplitR = (kSplitMask & 1) != 0, kSplitC = (kSplitMask & 2) != 0;
    NTM_T0(tp);
    // --- classify active rows: single-entry rows fix a variable, the rest are general ---
    if (l < N) w.fx()[l] = 0;
    NTM_WSYNC();
    int isgen = 0, fixj = -1, id = -1, srow = 0, constrow = 0;
    double ufix = 0.0, nfix = 0.0, ssign = 0.0;
    if (l < q) {
        id = w.act()[l];
        int kind, j;
        rows.decode(id, N, kind, j);
        if (kind < 2) {                                   // u bound: Lin = -+e_j, b = -umin / umax
            fixj = j;
            double lv = kind == 0 ? -1.0 : 1.0;
            ufix = rows.bval(w, id) / lv;
            nfix = -((lv * w.D()[j]) / w.D()[j]);
        } else if (kind >= 4) {                           // rate row: Lin = sg (e_j - e_{j-1})
            isgen = 1;
            srow = 2 * N + j;                             // general-row code >= 2N: rate row j
            ssign = (kind == 4) ? 1.0 : -1.0;
        } else {                                          // state row r = j: Lin = -+Gamma_r
            const double sg = (kind == 2) ? -1.0 : 1.0;
            // an x_0 row (j < 0) or a state row Gamma doesn't reach has Lin = 0: a
            // constant row is never active (a caller's or a shifted candidate can
            // hold one); the set is rejected like a colliding one
            const int info = (j >= 0) ? w.rinfo()[j] : 0;  // scaling pass: last non-zero column
            const int jj = (info & (kRowMulti - 1)) - 1;
            const int nnz = (info & kRowMulti) ? 2 : (jj >= 0 ? 1 : 0);
            if (nnz == 0) {
                constrow = 1;
            } else if (nnz == 1) {
                double lv = sg * w.gt(j, jj);
                fixj = jj;
                ufix = rows.bval(w, id) / lv;
                nfix = -((lv * w.D()[jj]) * w.irn()[j]);
            } else {
                isgen = 1;
                srow = j;
                ssign = sg;
            }
        }
    }
    NTM_ACC(ST_C_A, tp);
    const int lane = threadIdx.x & 63;
    const unsigned long long gmask = (P == 64) ? ~0ull : (((1ull << P) - 1ull) << (lane & ~(P - 1)));
    const unsigned long long below = (1ull << lane) - 1ull;
    unsigned long long bal = __ballot(isgen) & gmask;
    const int nS = uni<P>((int)__popcll(bal));
    if (ns_out) *ns_out = nS;
    if (l < q) {
        if (isgen) {
            const int k = __popcll(bal & below);
            w.sidx()[k] = l;                              // its position in the active list
            w.srw()[k] = srow;
            w.ssg()[k] = ssign;
        } else if (!constrow) {
            w.fx()[fixj] = (unsigned char)(l + 1);       // tagged by the writing lane
            w.Uf()[fixj] = ufix;
            w.hv()[fixj] = nfix;
        }
    }
    NTM_WSYNC();
    // two active rows fixing one variable (only a caller-supplied candidate can
    // do that; GI never adds a dependent row) cannot be certified: reject; so is a
    // set holding a constant row
    const bool collide =
        gmaxi<P>((l < q && !isgen && (constrow || w.fx()[fixj] != (unsigned char)(l + 1))) ? 1 : 0) != 0;
    const bool fixed = (l < N) && w.fx()[l];
    const double uf = fixed ? w.Uf()[l] : 0.0;
    const double vb = fixed ? uf / w.D()[l] : 0.0;
    if (l < N) {
        w.Vb()[l] = vb;
        w.dr()[l] = uf;                                   // U_B: fixed values, 0 on free variables
    }
    // --- compact map of the free variables ---
    bal = __ballot((l < N) && !fixed) & gmask;
    const int nF = uni<P>((int)__popcll(bal));
    const int fpos = __popcll(bal & below);
    if (l < N && !fixed) w.fidx()[fpos] = l;
    // --- y_B = Gamma U_B (fixed variables only; scratch in w.Phi(), dead until the
    //     next lift) and z = y_B + e - r (scratch in w.xp(), rewritten by the rollout) ---
    NTM_WSYNC();
    NTM_ACC(ST_C_B, tp);
    // Every variable fixed by a bound (no free variable, no general row: the box-only
    // QPs of BASELINE config 2 hold 19.8 of 20 inputs at a bound): Gamma U_B is the
    // certificate's y = Gamma U already, so the pass below writes it where the
    // certificate reads it and the certificate skips its own Gamma U pass (the
    // all-LDS and generic builds; the far N = 20 / 50 kernels keep one code path)
    constexpr bool kFixedY = !W::kFar;
    const bool allfixed = kFixedY && nF == 0 && nS == 0;
    // Long horizons (NTM_CY_LATE): the pass runs after the set's shape is known; an
    // echelon set needs Gamma_r U_B only at its active general rows (h), at most N < P
    // of them, so one trip over those rows replaces two over all 2N (z = y_B + e - r,
    // which only the bordered path's g_F reads, is not formed)
    constexpr bool kLateY = NTM_CY_LATE && W::kNN > 32 && P == 64 && !kSplitR;
    if constexpr (kSplitR) {
        if (!dir) {
            double y[1];
            gamma_rows_split<NTM_CH, 1>(w, {w.dr()}, y, l);
            if (l < 2 * N) {
                w.Phi()[l] = y[0];
                w.xp()[l] = allfixed ? y[0] : y[0] + w.e()[l] - ((l & 1) ? pb.r[1] : pb.r[0]);
            }
        }
    } else if constexpr (!kLateY) {
        for (int r = l; r < 2 * N && !dir; r += P) {
            const double y = gamma_row_dot<NTM_CH>(w, r, w.dr());
            w.Phi()[r] = y;
            w.xp()[r] = allfixed ? y : y + w.e()[r] - ((r & 1) ? pb.r[1] : pb.r[0]);
        }
    }
    NTM_WSYNC();
    NTM_ACC(ST_C_Y, tp);
    // --- square, triangular E (nS == nF, the common "boundary arc": the state held
    //     at its bound by every free input).  The active general rows then pin the
    //     free variables down on their own: sorted by their last free variable they
    //     make E lower triangular with a non-zero diagonal, so V_F follows from
    //     E V_F = h by forward substitution and the multipliers from E' mu = grad_F
    //     by back substitution in the certificate; no Gram of the free columns and
    //     no bordered elimination.  perm[t] = the general row whose last free
    //     variable is the t-th (scratch ints in the R block; E goes to the J block).
    int* const perm = w.permi();                           // sorted row t -> general row
    int* const colrow = perm + (N + 1);                    // compact column -> row ending there
    bool sq = false;                                       // echelon path (k = nF - nS <= 1)
    int nc = -1;                                           // k = 1: the non-pivot compact column
    int nc2 = -1;                                          // k = 1 with one collision: the second hole
    int xb = -1;                                           // one collision: the row left out of the triangle
    int xb2 = -1;                                          // two collisions (k = 0): the second row left out
    int nc3 = -1;                                          // k = 2 with one collision: the third hole
    const int kdim = nF - nS;
#ifdef NTM_STAMPS
    int dg_orph = -1, dg_neg = 0;                          // diagnostic: the shape of a set left to the bordered path
#endif
    // a general row with no non-zero at a free column makes the KKT matrix singular
    // (its row of E is zero): rejected like a colliding set (fail kind 3) instead of
    // running the bordered elimination into a zero pivot (long horizons: N = 50 mode 2
    // met 0.11 such re-solves per MPC step, round 6)
    bool nofree = false;
    // Long horizons with rate rows (config 5) mostly give square sets with ONE
    // collision: two general rows (a rate row and a state row of the same stage)
    // end in the same free column, and one column has no row ending there (83% of
    // the N=50 mode-3 optima, none at N=20 mode 2).  Leaving one of the two rows out
    // makes the rest echelon with k = 1 (the hole as the non-pivot column); the row
    // left out then fixes the step along the null vector instead of the cost.
    constexpr bool kCollision = W::kNN == 0 || W::kNN > 32;
    // Echelon sets with two spare columns (k = 2, round 5; long horizons): the certified
    // dual path passes through them after a drop from a k = 1 set; V = V_0 + w1 Z1 + w2 Z2
    // is minimised over the plane (a 2 x 2 system) instead of the bordered elimination
    constexpr bool kPlane = kCollision && NTM_PLANE;
    constexpr bool kColl2 = kCollision && NTM_COLL2;
    // k = 2 with one collision (round 6): three holes and one row left out; the row
    // left out fixes one of the three spare directions, the cost is minimised over
    // the plane that remains (config 5 mode 3: 0.44 such sets per MPC step took the
    // bordered elimination)
    constexpr bool kColl3 = kPlane && NTM_COLL3;
    if ((kdim == 1 || (kdim == 0 && nS > 0) || (kPlane && kdim == 2 && nS > 0)) && !collide) {
        const unsigned long long fm = bal >> (lane & ~(P - 1));   // bit j: variable j is free
        int lastf = -1;
        if (l < nS) {
            const int r = w.srw()[l];
            int lj = -1;
            if (r >= 2 * N) {                                  // rate row of input i: e_i - e_{i-1}
                const int i = r - 2 * N;
                lj = ((fm >> i) & 1ull) ? i : (((fm >> (i - 1)) & 1ull) ? i - 1 : -1);
            } else {                                           // state row r: from its last non-zero
                lj = (w.rinfo()[r] & (kRowMulti - 1)) - 1;     // column down to the first free one
                while (lj >= 0 && !(((fm >> lj) & 1ull) && w.gt(r, lj) != 0.0)) --lj;
            }
            if (lj >= 0) lastf = __popcll(fm & ((1ull << lj) - 1ull));
        }
        if (l < nF) colrow[l] = -1;
        NTM_WSYNC();
        if (lastf >= 0) colrow[lastf] = l;                     // a repeated last column leaves a hole
        NTM_WSYNC();
        const unsigned long long holes = __ballot(l < nF && colrow[l] < 0) & gmask;
        if constexpr (kCollision) nofree = (__ballot(l < nS && lastf < 0) & gmask) != 0;
#ifdef NTM_STAMPS
        dg_neg = (__ballot(l < nS && lastf < 0) & gmask) != 0;
        dg_orph = (int)__popcll(__ballot(l < nS && lastf >= 0 && colrow[lastf] != l) & gmask);
#endif
        if ((int)__popcll(holes) == kdim) {                    // every row ends in its own column
            sq = true;
            const unsigned long long hg = holes >> (lane & ~(P - 1));
            nc = kdim ? uni<P>((int)__ffsll((long long)hg) - 1) : -1;
            if (kPlane && kdim == 2) nc2 = uni<P>((int)__ffsll((long long)(hg & (hg - 1ull))) - 1);
            if (l < nS) {
                int c = l + ((nc >= 0 && l >= nc) ? 1 : 0);
                if (kPlane && nc2 >= 0 && c >= nc2) ++c;
                perm[l] = colrow[c];
            }
            NTM_WSYNC();
        } else if (kCollision && kdim <= (kColl3 ? 2 : 1) && (int)__popcll(holes) == kdim + 1 &&
                   (__ballot(l < nS && lastf < 0) & gmask) == 0) {
            // one row does not own its last column (the column's owner is the last writer):
            // k = 0 leaves one hole, k = 1 two (the triangle's spare column and the collision's),
            // k = 2 three
            const unsigned long long orph = __ballot(l < nS && colrow[lastf < 0 ? 0 : lastf] != l) & gmask;
            if ((int)__popcll(orph) == 1) {
                sq = true;
                const unsigned long long hg = holes >> (lane & ~(P - 1));
                const unsigned long long hg2 = hg & (hg - 1ull);
                nc = uni<P>((int)__ffsll((long long)hg) - 1);
                if (kdim >= 1) nc2 = uni<P>((int)__ffsll((long long)hg2) - 1);
                if (kColl3 && kdim == 2) nc3 = uni<P>((int)__ffsll((long long)(hg2 & (hg2 - 1ull))) - 1);
                xb = uni<P>((int)__ffsll((long long)(orph >> (lane & ~(P - 1)))) - 1);
                if (l < nS - 1) {
                    int c = l + (l >= nc ? 1 : 0);
                    if (nc2 >= 0 && c >= nc2) ++c;
                    if (kColl3 && nc3 >= 0 && c >= nc3) ++c;
                    perm[l] = colrow[c];
                }
                NTM_WSYNC();
            }
        } else if (kColl2 && kdim <= (kColl3 ? 1 : 0) && (int)__popcll(holes) == kdim + 2 &&
                   (__ballot(l < nS && lastf < 0) & gmask) == 0) {
            // two rows do not own their last columns (square set, two holes): leaving both
            // out leaves an echelon system with two spare columns, and the two rows left out
            // fix the step along the plane instead of the cost (round 5, rate rows at N = 50);
            // k = 1 leaves three holes, and the two rows fix a line (round 6, NTM_COLL3)
            const unsigned long long orph = __ballot(l < nS && colrow[lastf < 0 ? 0 : lastf] != l) & gmask;
            if ((int)__popcll(orph) == 2) {
                sq = true;
                const unsigned long long hg = holes >> (lane & ~(P - 1));
                const unsigned long long hg2 = hg & (hg - 1ull);
                nc = uni<P>((int)__ffsll((long long)hg) - 1);
                nc2 = uni<P>((int)__ffsll((long long)hg2) - 1);
                if (kColl3 && kdim == 1) nc3 = uni<P>((int)__ffsll((long long)(hg2 & (hg2 - 1ull))) - 1);
                const unsigned long long og = orph >> (lane & ~(P - 1));
                xb = uni<P>((int)__ffsll((long long)og) - 1);
                xb2 = uni<P>((int)__ffsll((long long)(og & (og - 1ull))) - 1);
                if (l < nS - 2) {
                    int c = l + (l >= nc ? 1 : 0);
                    if (c >= nc2) ++c;
                    if (kColl3 && nc3 >= 0 && c >= nc3) ++c;
                    perm[l] = colrow[c];
                }
                NTM_WSYNC();
            }
        }
    }
    if constexpr (kLateY) {
        if (!dir) {
            if (sq) {
                if (l < nS) {
                    const int r = w.srw()[l];
                    if (r < 2 * N) w.Phi()[r] = gamma_row_dot<NTM_CH>(w, r, w.dr());
                }
            } else {
                for (int r = l; r < 2 * N; r += P) {
                    const double y = gamma_row_dot<NTM_CH>(w, r, w.dr());
                    w.Phi()[r] = y;
                    w.xp()[r] = allfixed ? y : y + w.e()[r] - ((r & 1) ? pb.r[1] : pb.r[0]);
                }
            }
            NTM_WSYNC();
        }
    }
    NTM_ACC(ST_C_SQ, tp);
    if (dir && !sq) {                                      // the dual path's direction: echelon sets only
        if (fail_kind) *fail_kind = 3;
        return false;
    }
#ifdef NTM_STAMPS
    if (!collide) {                                        // which path the set takes, by spare columns
        if (sq) {
            if (xb >= 0) NTM_CNT(CN_SQ_COLL);
            else if (kdim == 0) NTM_CNT(CN_SQ_K0);
            else if (kdim == 1) NTM_CNT(CN_SQ_K1);
            else NTM_CNT(CN_SQ_K2);
        } else if (kdim <= 0) NTM_CNT(CN_BORD_K0);
        else if (kdim == 1) NTM_CNT(CN_BORD_K1);
        else if (kdim == 2) NTM_CNT(CN_BORD_K2);
        else if (kdim == 3) NTM_CNT(CN_BORD_K3);
        else NTM_CNT(CN_BORD_K4P);
        if (!sq) {
            if (dg_orph < 0) NTM_CNT(CN_BX_NOCLASS);
            else if (dg_neg) NTM_CNT(CN_BX_NEG);
            else if (dg_orph == 1) NTM_CNT(CN_BX_O1);
            else if (dg_orph == 2) NTM_CNT(CN_BX_O2);
            else if (dg_orph >= 3) NTM_CNT(CN_BX_O3P);
        }
    }
#endif
    // --- g_F (lane a = compact index) ---
    double gl = 0.0;
    if (!sq && l < nF) {
        const int ja = w.fidx()[l];
        const double* ca = w.Gt() + w.gidx(2 * ja, ja) - 2 * ja;   // ca[r] = gt(r, ja), r >= 2 ja
        const double g2 = qdot_rows<NTM_CH>(ca, w.xp(), N, ja, om);   // terms i < ja masked
        gl = w.D()[ja] * (2 * g2);
    }
    // Bordered KKT system (fused path): rows 0..nF-1 free variables, nF..nt-1 general
    // rows, nt the right-hand side; kept packed row-major (row r at r(r+1)/2) in the
    // contiguous J/R block.  Falls back to the two-stage Schur solve below when the
    // bordered rows do not fit the group's lanes or the block.
    const int nt = nF + nS;
    // nt <= 2N (nS <= nF); a compile-time horizon whose worst case fits compiles the fused path only
    // Lanes own RPL bordered rows each (row l + r P), enough for the nt + 1 <= 2N + 1 rows
    constexpr int NNc = W::kNN, LDc = NNc | 1;
    constexpr int RPL = NNc > 0 ? (2 * NNc + 1 + P - 1) / P : (2 * NTM_MAX_N + 1 + P - 1) / P;
    constexpr bool kAlwaysFused =
        NNc > 0 && (2 * NNc) * (2 * NNc + 1) / 2 + 2 * NNc <= NNc * LDc + (NNc + 1) * LDc;
    const bool fused = kAlwaysFused || ((nt + 1 <= RPL * P) && (nt * (nt + 1) / 2 + nt <= N * LDJ + (N + 1) * LD));
    double* const Lp = w.J();
    if (!sq && fused && l < nF) Lp[w.brow(nt) + w.bcol(l, nt)] = -gl;
    // --- compact G~_FF: one (a, c) entry per lane (packed rows, or lower col-major in R);
    //     on the matrix cores at long horizons (gram_mfma) ---
    constexpr bool kMfmaGram = NTM_MFMA_FF && W::kNN > 32 && P == 64;
    if constexpr (kMfmaGram) {
        if (!sq)
            gram_mfma<W::kNN>(pb, w, nF, [&](int a) { return w.fidx()[a]; },
                              [&](int a, int c, double sg) {
                                  Lp[w.brow(a) + w.bcol(c, nt)] = (2 * sg) * w.D()[w.fidx()[a]] * w.D()[w.fidx()[c]];
                              },
                              l);
    } else {
        const int npair = sq ? 0 : nF * (nF + 1) / 2;
        for (int idx = l; idx < npair; idx += P) {
            int a = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
            if ((a + 1) * (a + 2) / 2 <= idx) ++a;
            if (a * (a + 1) / 2 > idx) --a;
            const int c = idx - a * (a + 1) / 2;
            const int ja = w.fidx()[a], jc = w.fidx()[c];            // ja >= jc
            const double* ca = w.Gt() + w.gidx(2 * ja, ja) - 2 * ja;
            const double* cc = w.Gt() + w.gidx(2 * jc, jc) - 2 * jc;
            const double sg = qdot_rows<NTM_CH>(ca, cc, N, ja, om);   // terms i < ja masked
            double g2v = 2 * sg;
            if constexpr (ru_on<W>()) g2v = (a == c) ? g2v + 2 * pb.Ru : g2v;      // + 2 Ru I
            const double gv = g2v * w.D()[ja] * w.D()[jc];
            if (fused) Lp[w.brow(a) + w.bcol(c, nt)] = gv;            // row-major: idx == a(a+1)/2 + c
            else w.R()[a + c * LD] = gv;
        }
    }
    NTM_WSYNC();
    // GI normal of general row s at variable j: n = -(Lin_j D_j)/rn, Lin = sg Gamma_r
    auto gen_n = [&](int s2, int j) -> double {
        const int r = w.srw()[s2];
        if (r >= 2 * N) {                                 // rate row i = r - 2N
            const int i = r - 2 * N;
            const double sg = w.ssg()[s2];
            const double lv = (j == i) ? sg : (j == i - 1 ? -sg : 0.0);
            return -((lv * w.D()[j]) * w.idun()[i]);
        }
        return (j <= (r >> 1)) ? -(((w.ssg()[s2] * w.gt(r, j)) * w.D()[j]) * w.irn()[r]) : 0.0;
    };
    // h_s = n_s' V = bc_s - n_s,B' V_B with n_s,B' V_B = -sg irn_r (Gamma_r U_B)
    auto hs_of = [&](int s2) -> double {
        double hs = 0.0;
        if (s2 < nS) {
            const int r = w.srw()[s2];
            const double sg = w.ssg()[s2];
            if (r >= 2 * N) {                             // rate row i: b = du, fixed part sg (U_i - U_{i-1})
                const int i = r - 2 * N;
                const double ir = w.idun()[i];
                const double ui = w.fx()[i] ? w.Uf()[i] : 0.0;
                const double um = w.fx()[i - 1] ? w.Uf()[i - 1] : 0.0;
                hs = -(rows.du * ir) + (sg * (ui - um)) * ir;
            } else {
                const int c = r & 1;
                const double ir = w.irn()[r];
                const double bval = (sg > 0.0) ? (rows.xmax(c) - w.e()[r]) : (-rows.xmin(c) + w.e()[r]);
                hs = -(bval * ir) + (sg * w.Phi()[r]) * ir;
            }
        }
        return hs;
    };
    NTM_ACC(ST_P_GRAM, tp);
    bool ok = !collide && !nofree;
    int fk = ok ? 0 : 3, fpos_out = 0;
    double vfin = 0.0;
    double sq_id = 0.0;                                   // echelon path: 1 / E_p[t][t] on lane t
    bool y_ready = allfixed;                              // k = 1 / all fixed: y = Gamma U already in w.xp()
    if (sq) {
        // Sorted E over the pivot columns (row t = general row perm[t] ends in pivot
        // column pc(t) = t + (t >= nc); lower triangular, n x n row-major at Lp[t LD + u]),
        // the non-pivot column e_c (k = 1) and h
        const int n = nS - (xb >= 0 ? 1 : 0) - (xb2 >= 0 ? 1 : 0);
        auto pc = [&](int u) {                                // pivot column of sorted row u
            int c = u + ((nc >= 0 && u >= nc) ? 1 : 0);
            if (kCollision && nc2 >= 0 && c >= nc2) ++c;
            if (kColl3 && nc3 >= 0 && c >= nc3) ++c;
            return c;
        };
        double* const Ep = w.Ep();
        // long horizons: lane t builds sorted row t (n <= N <= 64 rows).  The row's
        // constants (its general row, sign, norm) are loaded once, and each batch of
        // CH columns costs one LDS round trip: the column index and D_j are the same
        // address on every lane (broadcast reads), only Gamma_rj differs.  The entry-
        // per-lane loop below issues ~5 dependent loads per entry, n^2 / 64 times per
        // lane (n ~ 43 at N = 50).  Entries as gen_n computes them, bit for bit.
        constexpr bool kRowE = W::kNN > 32 || W::kNN == 0 || NTM_ROWE_ALL;
        // (NTM_E_LANEIDX, P = 64) lane u first loads pivot column u's variable and D_j, and
        // each row's loop takes them by readlane: one LDS round trip per batch (Gamma_rj)
        // instead of two (the column index, then Gamma_rj and D_j at it)
        constexpr bool kLaneIdx = NTM_E_LANEIDX && P == 64;
        int jfl = 0;
        double dfl = 0.0;
        if constexpr (kRowE && kLaneIdx) {
            if (l < n) {
                jfl = w.fidx()[pc(l)];
                dfl = w.D()[jfl];
            }
        }
        auto col_of = [&](int u) -> int {                     // pivot column u's variable (u uniform)
            if constexpr (kLaneIdx) return __builtin_amdgcn_readlane(jfl, u);
            else return w.fidx()[pc(u)];
        };
        auto d_of = [&](int u, int j) -> double {             // D at it
            if constexpr (kLaneIdx) return gbcast<P>(dfl, u);
            else return w.D()[j];
        };
        if constexpr (kRowE) {
            if (l < n) {
                const int s2 = perm[l];
                const int r = w.srw()[s2];
                const double sg = w.ssg()[s2];
                double* const erow = Ep + w.eidx(l, 0);
                constexpr int CH = NTM_CH;
                if (r >= 2 * N) {                                  // rate row of input i
                    const int i = r - 2 * N;
                    const double ir = w.idun()[i];
                    for (int u = 0; u <= l; ++u) {
                        const int uu = kLaneIdx ? __builtin_amdgcn_readfirstlane(u) : u;
                        const int j = col_of(uu);
                        const double lv = (j == i) ? sg : (j == i - 1 ? -sg : 0.0);
                        erow[u] = -((lv * d_of(uu, j)) * ir);
                    }
                } else {
                    const double ir = w.irn()[r];
                    const int jm = r >> 1;
                    const double* gr = w.Gt() + r;                 // gt(r, j) = gr[gidx(0, j)]
                    for (int u0 = 0; u0 <= l; u0 += CH) {
                        int jj[CH];
                        double g[CH], d[CH];
                        const int ub = kLaneIdx ? __builtin_amdgcn_readfirstlane(u0) : u0;
#pragma unroll
                        for (int c = 0; c < CH; ++c) {
                            if constexpr (kLaneIdx) jj[c] = col_of((ub + c) & 63);     // lanes >= n hold 0
                            else jj[c] = (u0 + c <= l) ? w.fidx()[pc(u0 + c)] : 0;
                        }
#pragma unroll
                        for (int c = 0; c < CH; ++c) {
                            const bool in = u0 + c <= l && jj[c] <= jm;
                            g[c] = in ? gr[w.gidx(0, jj[c])] : 0.0;
                            if constexpr (kLaneIdx) d[c] = (u0 + c <= l) ? d_of((ub + c) & 63, 0) : 0.0;
                            else d[c] = (u0 + c <= l) ? w.D()[jj[c]] : 0.0;
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int c = 0; c < CH; ++c)
                            if (u0 + c <= l) erow[u0 + c] = (jj[c] <= jm) ? -(((sg * g[c]) * d[c]) * ir) : 0.0;
                    }
                }
                if constexpr (!W::kFar)
                    for (int u = l + 1; u < n; ++u) erow[u] = 0.0;
            }
        } else {
        for (int idx = l; idx < n * n; idx += P) {
            const int t = idx / n, u = idx - t * n;
            if constexpr (W::kFar) {                               // packed: the lower triangle only
                if (u <= t) Ep[w.eidx(t, u)] = gen_n(perm[t], w.fidx()[pc(u)]);
            } else {
                Ep[w.eidx(t, u)] = (u <= t) ? gen_n(perm[t], w.fidx()[pc(u)]) : 0.0;
            }
        }
        }
        double acc = 0.0, acz = 0.0, acz2 = 0.0, acz3 = 0.0;
        if (l < n && !dir) {
            acc = hs_of(perm[l]);
            if (nc >= 0 && nc < pc(l)) acz = -gen_n(perm[l], w.fidx()[nc]);
            if (kCollision && nc2 >= 0 && nc2 < pc(l)) acz2 = -gen_n(perm[l], w.fidx()[nc2]);
            if (kColl3 && nc3 >= 0 && nc3 < pc(l)) acz3 = -gen_n(perm[l], w.fidx()[nc3]);
        }
        const double hxb = (kCollision && xb >= 0 && !dir) ? hs_of(xb) : 0.0;   // before w.Phi() is reused
        const double hxb2 = (kColl2 && xb2 >= 0 && !dir) ? hs_of(xb2) : 0.0;
        NTM_WSYNC();
        if (l < n) sq_id = 1.0 / Ep[w.eidx(l, l)];
        NTM_ACC(ST_S_E, tp);
        if (!dir) {
        // E_p V_p = h and (k = 1) E_p Z_p = -e_c: lane t owns row t; step t broadcasts
        // x_t (z_t) and updates the rows below
        double x = 0.0, zz = 0.0, zz2 = 0.0, zz3 = 0.0;
        // E[l][t] loaded kAhead steps ahead (a register queue; long horizons: NTM_SUB_AHEAD)
        constexpr int kAhead = (W::kNN > 32) ? NTM_SUB_AHEAD : 1;
        double eq[kAhead];
#pragma unroll
        for (int a = 0; a < kAhead; ++a) eq[a] = (a < n && l > a && l < n) ? Ep[w.eidx(l, a)] : 0.0;
        // NTM_SUB_PRESCALE (long horizons): the accumulators carry acc / E[l][l] and the
        // update uses E[l][t] / E[l][l], formed off the chain, so step t's broadcast waits
        // on one operation less (fma -> readlane -> fma)
        constexpr bool kPre = NTM_SUB_PRESCALE && W::kNN > 32;
        if constexpr (kPre) { acc *= sq_id; acz *= sq_id; acz2 *= sq_id; acz3 *= sq_id; }
        for (int t = 0; t < n; ++t) {
            const double et = kPre ? eq[0] * sq_id : eq[0];
#pragma unroll
            for (int a = 0; a + 1 < kAhead; ++a) eq[a] = eq[a + 1];
            {
                const int ta = t + kAhead;
                eq[kAhead - 1] = (ta < n && l > ta && l < n) ? Ep[w.eidx(l, ta)] : 0.0;
            }
            const double xt = gbcast<P>(kPre ? acc : acc * sq_id, t);
            if (l == t) x = xt;
            acc -= et * xt;
            if (nc >= 0) {
                const double zt = gbcast<P>(kPre ? acz : acz * sq_id, t);
                if (l == t) zz = zt;
                acz -= et * zt;
            }
            if (kCollision && nc2 >= 0) {
                const double zt2 = gbcast<P>(kPre ? acz2 : acz2 * sq_id, t);
                if (l == t) zz2 = zt2;
                acz2 -= et * zt2;
            }
            if (kColl3 && nc3 >= 0) {
                const double zt3 = gbcast<P>(kPre ? acz3 : acz3 * sq_id, t);
                if (l == t) zz3 = zt3;
                acz3 -= et * zt3;
            }
        }
        ok = gmaxi<P>((l < n && !(isfinite(x) && isfinite(zz) && isfinite(zz2) && isfinite(zz3))) ? 1 : 0) == 0;
        // V_0 (pivots from E_p V_p = h, fixed values, 0 on the non-pivot columns) and Z
        const bool hole = fpos == nc || (kCollision && nc2 >= 0 && fpos == nc2) || (kColl3 && nc3 >= 0 && fpos == nc3);
        const int rk = hole ? 0
                            : fpos - ((nc >= 0 && fpos > nc) ? 1 : 0) - ((kCollision && nc2 >= 0 && fpos > nc2) ? 1 : 0) -
                                  ((kColl3 && nc3 >= 0 && fpos > nc3) ? 1 : 0);
        const double xs = __shfl(x, (l < N && !fixed) ? rk : 0, P);
        const double zs = __shfl(zz, (l < N && !fixed) ? rk : 0, P);
        const double v0 = fixed ? vb : (hole ? 0.0 : xs);
        vfin = v0;
        // k = 1 with one collision: V = V_0 + w1 Z1 + w2 Z2 (Zi = e_{hole i} + Zi_p); the row
        // left out fixes a1 w1 + a2 w2 = h_B - n_B' V_0 (ai = n_B' Zi), which leaves the line
        // V_p + w Z_d (eliminating the w with the larger |ai|) for the cost to minimise below
        double vline = v0, zline = 0.0;
        bool line = false;
        // k = 2: V = V_0 + w1 Z1 + w2 Z2 (Zi = e_{hole i} + Zi_p); with yi = Gamma D Zi
        // and q = y_0 + e - r the cost is minimised at H w = -g, H_ij = yi' Om yj (+ Ru
        // dUi' dUj), g_i = yi' Om q (+ Ru dUi' U_0): three Gamma passes, five reductions
        auto plane_min = [&](const double v0, const double z1, const double z2) {
            double* const y2s = w.Vb();                       // 2N scratch (Vb, Uf: dead after hs_of)
            if (l < N) {
                w.U()[l] = w.D()[l] * v0;
                w.d()[l] = w.D()[l] * z1;
                w.dr()[l] = w.D()[l] * z2;
            }
            NTM_WSYNC();
            for (int r = l; r < 2 * N; r += P) {
                double ya, yb;
                gamma_row_dot2<NTM_CH>(w, r, w.U(), w.d(), ya, yb);
                w.xp()[r] = ya;
                w.Phi()[r] = yb;
                y2s[r] = gamma_row_dot<NTM_CH>(w, r, w.dr());
            }
            NTM_WSYNC();
            double g1 = 0.0, g2 = 0.0, h11 = 0.0, h12 = 0.0, h22 = 0.0;
            if (l < N) {
                const double qa = w.xp()[2 * l] + w.e()[2 * l] - pb.r[0];
                const double qb = w.xp()[2 * l + 1] + w.e()[2 * l + 1] - pb.r[1];
                const double aa = w.Phi()[2 * l], ab = w.Phi()[2 * l + 1];
                const double ca = y2s[2 * l], cb = y2s[2 * l + 1];
                const double oa = om.o0(aa, ab), ob = om.o1(aa, ab);      // Om y1
                const double oc = om.o0(ca, cb), od = om.o1(ca, cb);      // Om y2
                g1 = oa * qa + ob * qb;
                g2 = oc * qa + od * qb;
                h11 = oa * aa + ob * ab;
                h12 = oa * ca + ob * cb;
                h22 = oc * ca + od * cb;
                if constexpr (ru_on<W>()) {
                    const double u0 = w.U()[l], d1 = w.d()[l], d2 = w.dr()[l];
                    g1 += pb.Ru * (d1 * u0);
                    g2 += pb.Ru * (d2 * u0);
                    h11 += pb.Ru * (d1 * d1);
                    h12 += pb.Ru * (d1 * d2);
                    h22 += pb.Ru * (d2 * d2);
                }
            }
            g1 = gsum<P>(g1);
            g2 = gsum<P>(g2);
            h11 = gsum<P>(h11);
            h12 = gsum<P>(h12);
            h22 = gsum<P>(h22);
            const double det = h11 * h22 - h12 * h12;
            ok = det > 0.0 && h11 > 0.0 && det < kInf && isfinite(g1) && isfinite(g2);
            const double w1 = ok ? -((h22 * g1 - h12 * g2) / det) : 0.0;
            const double w2 = ok ? -((h11 * g2 - h12 * g1) / det) : 0.0;
            vfin = v0 + w1 * z1 + w2 * z2;
            for (int r = l; r < 2 * N; r += P) w.xp()[r] += w1 * w.Phi()[r] + w2 * y2s[r];   // y
            y_ready = true;
        };
        if (kColl3 && ok && xb2 >= 0 && nc3 >= 0) {
            // k = 1 with two collisions: V = V_0 + w1 Z1 + w2 Z2 + w3 Z3 and the two rows left
            // out fix A w = r (A 2 x 3, A_ij = n_Bi' Zj, r_i = h_Bi - n_Bi' V_0): a particular
            // solution from the best-conditioned 2 x 2 minor plus t times the null vector
            // (the rows' cross product) leaves the line V_p + t Z_n for the cost to minimise
            const double zs2 = __shfl(zz2, (l < N && !fixed) ? rk : 0, P);
            const double zs3 = __shfl(zz3, (l < N && !fixed) ? rk : 0, P);
            const double z1 = fixed ? 0.0 : ((fpos == nc) ? 1.0 : (hole ? 0.0 : zs));
            const double z2 = fixed ? 0.0 : ((fpos == nc2) ? 1.0 : (hole ? 0.0 : zs2));
            const double z3 = fixed ? 0.0 : ((fpos == nc3) ? 1.0 : (hole ? 0.0 : zs3));
            const double nb1 = (l < N && !fixed) ? gen_n(xb, l) : 0.0;
            const double nb2 = (l < N && !fixed) ? gen_n(xb2, l) : 0.0;
            const double b10 = gsum<P>(nb1 * v0), a11 = gsum<P>(nb1 * z1), a12 = gsum<P>(nb1 * z2), a13 = gsum<P>(nb1 * z3);
            const double b20 = gsum<P>(nb2 * v0), a21 = gsum<P>(nb2 * z1), a22 = gsum<P>(nb2 * z2), a23 = gsum<P>(nb2 * z3);
            const double r1 = hxb - b10, r2 = hxb2 - b20;
            const double d12 = a11 * a22 - a12 * a21, d13 = a11 * a23 - a13 * a21, d23 = a12 * a23 - a13 * a22;
            const double scl = fmax(fmax(fmax(fabs(a11), fabs(a12)), fabs(a13)), fmax(fmax(fabs(a21), fabs(a22)), fabs(a23)));
            const int im = (fabs(d12) >= fabs(d13) && fabs(d12) >= fabs(d23)) ? 0 : (fabs(d13) >= fabs(d23) ? 1 : 2);
            const double dm = im == 0 ? d12 : (im == 1 ? d13 : d23);
            ok = isfinite(dm) && fabs(dm) > 1e-14 * scl * scl && isfinite(b10) && isfinite(b20);
            double w1 = 0.0, w2 = 0.0, w3 = 0.0;
            if (ok) {
                if (im == 0) { w1 = (a22 * r1 - a12 * r2) / dm; w2 = (a11 * r2 - a21 * r1) / dm; }
                else if (im == 1) { w1 = (a23 * r1 - a13 * r2) / dm; w3 = (a11 * r2 - a21 * r1) / dm; }
                else { w2 = (a23 * r1 - a13 * r2) / dm; w3 = (a12 * r2 - a22 * r1) / dm; }
            }
            vline = ok ? v0 + w1 * z1 + w2 * z2 + w3 * z3 : v0;
            zline = ok ? (d23 / dm) * z1 - (d13 / dm) * z2 + (d12 / dm) * z3 : 0.0;
            line = ok;
        } else if (kColl3 && ok && xb >= 0 && nc3 >= 0) {
            // k = 2 with one collision: V = V_0 + w1 Z1 + w2 Z2 + w3 Z3; the row left out
            // fixes a1 w1 + a2 w2 + a3 w3 = h_B - n_B' V_0 (ai = n_B' Zi): eliminating the w
            // with the largest |ai| leaves the plane V_p + wa Za + wb Zb for the cost below
            const double zs2 = __shfl(zz2, (l < N && !fixed) ? rk : 0, P);
            const double zs3 = __shfl(zz3, (l < N && !fixed) ? rk : 0, P);
            const double z1 = fixed ? 0.0 : ((fpos == nc) ? 1.0 : (hole ? 0.0 : zs));
            const double z2 = fixed ? 0.0 : ((fpos == nc2) ? 1.0 : (hole ? 0.0 : zs2));
            const double z3 = fixed ? 0.0 : ((fpos == nc3) ? 1.0 : (hole ? 0.0 : zs3));
            const double nb = (l < N && !fixed) ? gen_n(xb, l) : 0.0;
            const double b0 = gsum<P>(nb * v0), a1 = gsum<P>(nb * z1), a2 = gsum<P>(nb * z2), a3 = gsum<P>(nb * z3);
            const int ip = (fabs(a3) > fabs(a2)) ? ((fabs(a3) > fabs(a1)) ? 3 : 1) : ((fabs(a2) >= fabs(a1)) ? 2 : 1);
            const double ap = ip == 1 ? a1 : (ip == 2 ? a2 : a3);
            const double aa = ip == 1 ? a2 : a1, ab = ip == 3 ? a2 : a3;
            const double zp = ip == 1 ? z1 : (ip == 2 ? z2 : z3);
            const double za = ip == 1 ? z2 : z1, zb = ip == 3 ? z2 : z3;
            ok = ap != 0.0 && isfinite(ap) && isfinite(aa) && isfinite(ab) && isfinite(b0);
            if (ok) plane_min(v0 + ((hxb - b0) / ap) * zp, za - (aa / ap) * zp, zb - (ab / ap) * zp);
        } else if (kColl2 && ok && xb2 >= 0) {
            // two collisions: V = V_0 + w1 Z1 + w2 Z2 with the rows left out fixing
            // [n_B1'Z1 n_B1'Z2; n_B2'Z1 n_B2'Z2] w = [h_B1 - n_B1'V_0; h_B2 - n_B2'V_0]
            const double zs2 = __shfl(zz2, (l < N && !fixed) ? rk : 0, P);
            const double z1 = fixed ? 0.0 : ((fpos == nc) ? 1.0 : (hole ? 0.0 : zs));
            const double z2 = fixed ? 0.0 : ((fpos == nc2) ? 1.0 : (hole ? 0.0 : zs2));
            const double nb1 = (l < N && !fixed) ? gen_n(xb, l) : 0.0;
            const double nb2 = (l < N && !fixed) ? gen_n(xb2, l) : 0.0;
            const double b10 = gsum<P>(nb1 * v0), a11 = gsum<P>(nb1 * z1), a12 = gsum<P>(nb1 * z2);
            const double b20 = gsum<P>(nb2 * v0), a21 = gsum<P>(nb2 * z1), a22 = gsum<P>(nb2 * z2);
            const double det = a11 * a22 - a12 * a21;
            const double scl = fmax(fmax(fabs(a11), fabs(a12)), fmax(fabs(a21), fabs(a22)));
            ok = isfinite(det) && fabs(det) > 1e-14 * scl * scl && isfinite(b10) && isfinite(b20);
            const double r1 = hxb - b10, r2 = hxb2 - b20;
            const double w1 = ok ? (a22 * r1 - a12 * r2) / det : 0.0;
            const double w2 = ok ? (a11 * r2 - a21 * r1) / det : 0.0;
            vfin = v0 + w1 * z1 + w2 * z2;
        } else if (kCollision && ok && xb >= 0 && nc2 >= 0) {
            const double zs2 = __shfl(zz2, (l < N && !fixed) ? rk : 0, P);
            const double z1 = fixed ? 0.0 : ((fpos == nc) ? 1.0 : (hole ? 0.0 : zs));
            const double z2 = fixed ? 0.0 : ((fpos == nc2) ? 1.0 : (hole ? 0.0 : zs2));
            const double nb = (l < N && !fixed) ? gen_n(xb, l) : 0.0;
            const double b0 = gsum<P>(nb * v0), a1 = gsum<P>(nb * z1), a2 = gsum<P>(nb * z2);
            const bool use2 = fabs(a2) >= fabs(a1);
            const double ap = use2 ? a2 : a1, ao = use2 ? a1 : a2;
            ok = ap != 0.0 && isfinite(ap) && isfinite(ao) && isfinite(b0);
            const double zp = use2 ? z2 : z1, zo = use2 ? z1 : z2;
            vline = ok ? v0 + ((hxb - b0) / ap) * zp : v0;
            zline = ok ? zo - (ao / ap) * zp : 0.0;
            line = ok;
        } else if (kCollision && ok && xb >= 0) {
            // the row left out fixes the step along Z: n_B' (V_0 + w Z) = h_B
            const double zv = fixed ? 0.0 : ((fpos == nc) ? 1.0 : zs);
            const double nb = (l < N && !fixed) ? gen_n(xb, l) : 0.0;
            const double b0 = gsum<P>(nb * v0), b1 = gsum<P>(nb * zv);
            ok = b1 != 0.0 && isfinite(b1) && isfinite(b0);
            const double wv = ok ? (hxb - b0) / b1 : 0.0;
            vfin = v0 + wv * zv;
        } else if (kPlane && ok && nc2 >= 0) {
            const double zs2 = __shfl(zz2, (l < N && !fixed) ? rk : 0, P);
            const double z1 = fixed ? 0.0 : ((fpos == nc) ? 1.0 : (hole ? 0.0 : zs));
            const double z2 = fixed ? 0.0 : ((fpos == nc2) ? 1.0 : (hole ? 0.0 : zs2));
            plane_min(v0, z1, z2);
        } else if (ok && nc >= 0) {
            zline = fixed ? 0.0 : ((fpos == nc) ? 1.0 : zs);
            line = true;
        }
        if (line) {
            // k = 1: the minimum along V_0 + w Z, Z = e_c + Z_p:
            //   w = -(2 yz' Om (y0 + e - r)) / (2 yz' Om yz), y0 = Gamma D V_0, yz = Gamma D Z
            const double v0 = vline, zv = zline;
            if (l < N) {
                w.U()[l] = w.D()[l] * v0;
                w.d()[l] = w.D()[l] * zv;
            }
            NTM_WSYNC();
            if constexpr (kSplitR) {
                double yy[2];
                gamma_rows_split<NTM_CH, 2>(w, {w.U(), w.d()}, yy, l);
                if (l < 2 * N) {
                    w.xp()[l] = yy[0];
                    w.Phi()[l] = yy[1];                          // scratch (hs_of is done with it)
                }
            } else {
                for (int r = l; r < 2 * N; r += P) {
                    double ya, yb;
                    gamma_row_dot2<NTM_CH>(w, r, w.U(), w.d(), ya, yb);
                    w.xp()[r] = ya;
                    w.Phi()[r] = yb;                             // scratch (hs_of is done with it)
                }
            }
            NTM_WSYNC();
            double num = 0.0, den = 0.0;
            if (l < N) {
                const double y0a = w.xp()[2 * l] + w.e()[2 * l] - pb.r[0];
                const double y0b = w.xp()[2 * l + 1] + w.e()[2 * l + 1] - pb.r[1];
                const double za = w.Phi()[2 * l], zb = w.Phi()[2 * l + 1];
                const double oa = om.o0(za, zb), ob = om.o1(za, zb);
                num = oa * y0a + ob * y0b;
                den = oa * za + ob * zb;
                if constexpr (ru_on<W>()) {               // Ru (dU' U_0, dU' dU): w.U() = D V_0, w.d() = D Z
                    const double ua = w.U()[l], da = w.d()[l];
                    num += pb.Ru * (da * ua);
                    den += pb.Ru * (da * da);
                }
            }
            num = gsum<P>(num);
            den = gsum<P>(den);
            ok = den > 0.0 && den < kInf && isfinite(num);
            const double wv = ok ? -(num / den) : 0.0;
            vfin = v0 + wv * zv;
            for (int r = l; r < 2 * N; r += P) w.xp()[r] += wv * w.Phi()[r];   // y = y0 + w yz
            y_ready = true;
        }
        }   // !dir
        if (!ok) fk = 3;
        NTM_ACC(ST_S_Y, tp);
    } else if (fused) {
        // E rows over the free variables (one entry per lane) and h; the trailing
        // block of A is zero and is never stored (the elimination starts it at 0)
        for (int idx = l; idx < nF * nS; idx += P) {
            const int s2 = idx / nF, a = idx - s2 * nF;
            Lp[w.brow(nF + s2) + w.bcol(a, nt)] = gen_n(s2, w.fidx()[a]);
        }
        if (l < nS) Lp[w.brow(nt) + w.bcol(nF + l, nt)] = hs_of(l);
        NTM_WSYNC();
        NTM_ACC(ST_S_E, tp);
        // Left-looking elimination of A = [[G~_FF, E'], [E, 0]] = L_A diag(I, -I) L_A'
        // over its nt columns: L_A = [[L, 0], [Y', L_K]] with L L' = G~_FF,
        // Y = L^{-1} E', L_K L_K' = K = Y'Y (the Schur complement), in one pass
        // whose right-hand-side row carries the forward substitution
        // z = L_A^{-1} [-g_F; h].  Lane r owns row r.
        // Lane l owns rows l + r P (r < RPL); a group-uniform row index k lives on
        // lane k % P in slot k / P.
        auto slot_of = [&](const double* v, int k) -> double {   // v[k / P] (k uniform)
            double o = v[0];
#pragma unroll
            for (int r = 1; r < RPL; ++r) o = (k / P == r) ? v[r] : o;
            return o;
        };
        double* myrow[RPL];
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            const int lr = l + r * P;
            myrow[r] = Lp + w.brow(lr);
        }
        if (ok) {
            // blocks of KB columns: one pass of loads over the finished columns j < k
            // serves all KB pivot rows, then the block's own triangle is finished in
            // registers (L[k+b, k+c] broadcast from the lane of row k+b).  Each column
            // still accumulates its terms in column order, as the unblocked elimination.
            constexpr int KB = 4;
            for (int k = 0; k < nt; k += KB) {
                const int kb = (nt - k < KB) ? nt - k : KB;
                double sacc[RPL][KB];
                bool live[RPL];
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    const int lr = l + r * P;
                    live[r] = lr >= k && lr <= nt;
#pragma unroll
                    for (int b2 = 0; b2 < KB; ++b2) {
                        const int col = k + b2;
                        sacc[r][b2] = (b2 < kb && live[r] && lr >= col) ? ((col >= nF && lr < nt) ? 0.0 : myrow[r][w.bcol(col, nt)])
                                                                        : 0.0;
                    }
                }
                const int kf = k < nF ? k : nF;
                // unconditional loads (no branch per load): j + 1 <= k stays inside each
                // live row (>= k) and pivot row k+b2; pivot rows past the block clamp to row nt
                const double* prb[KB];
#pragma unroll
                for (int b2 = 0; b2 < KB; ++b2) {
                    const int rr = (k + b2 < nt) ? k + b2 : nt;
                    prb[b2] = Lp + w.brow(rr);
                }
                if constexpr (W::kFar && NTM_FAR_JB > 0) {
                    // far block (HBM): JB columns per trip for all of the lane's rows and
                    // the KB pivot rows, every load issued before the first use (one
                    // memory round trip per trip instead of one per column pair); the
                    // column index is clamped to k (inside every live row and pivot row),
                    // the terms past k are skipped, so each sum keeps its column order
                    constexpr int JB = NTM_FAR_JB > 0 ? NTM_FAR_JB : 1;
                    for (int j = 0; j < k; j += JB) {
                        int cj[JB];
#pragma unroll
                        for (int u = 0; u < JB; ++u) cj[u] = w.bcol((j + u < k) ? j + u : k, nt);
                        double av[RPL][JB], pv[KB][JB];
#pragma unroll
                        for (int r = 0; r < RPL; ++r)
#pragma unroll
                            for (int u = 0; u < JB; ++u) av[r][u] = live[r] ? myrow[r][cj[u]] : 0.0;
#pragma unroll
                        for (int b2 = 0; b2 < KB; ++b2)
#pragma unroll
                            for (int u = 0; u < JB; ++u) pv[b2][u] = prb[b2][cj[u]];
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int u = 0; u < JB; ++u) {
                            if (j + u >= k) break;
                            const double su = (j + u < kf) ? -1.0 : 1.0;
#pragma unroll
                            for (int r = 0; r < RPL; ++r)
                                if (live[r])
#pragma unroll
                                    for (int b2 = 0; b2 < KB; ++b2) sacc[r][b2] += (su * av[r][u]) * pv[b2][u];
                        }
                    }
                } else {
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    if (!live[r]) continue;
                    for (int j = 0; j < k; j += 2) {
                        const bool in1 = j + 1 < k;
                        const int cj0 = w.bcol(j, nt), cj1 = w.bcol(j + 1, nt);
                        const double a0 = myrow[r][cj0], a1 = myrow[r][cj1];
                        double p0[KB], p1[KB];
#pragma unroll
                        for (int b2 = 0; b2 < KB; ++b2) {
                            p0[b2] = prb[b2][cj0];
                            p1[b2] = prb[b2][cj1];
                        }
                        const double s0 = (j < kf) ? -1.0 : 1.0, s1 = (j + 1 < kf) ? -1.0 : 1.0;
#pragma unroll
                        for (int b2 = 0; b2 < KB; ++b2) {
                            sacc[r][b2] += (s0 * a0) * p0[b2];
                            sacc[r][b2] += in1 ? (s1 * a1) * p1[b2] : 0.0;
                        }
                    }
                }
                }
                double Lc[RPL][KB];
#pragma unroll
                for (int b2 = 0; b2 < KB; ++b2) {
#pragma unroll
                    for (int r = 0; r < RPL; ++r) Lc[r][b2] = 0.0;
                    if (b2 < kb) {
                        const int col = k + b2, cl = col % P;
#pragma unroll
                        for (int c = 0; c < b2; ++c) {           // block columns k..col-1, in order
                            double lcc[RPL];
#pragma unroll
                            for (int r = 0; r < RPL; ++r) lcc[r] = Lc[r][c];
                            const double lkc = gbcast<P>(slot_of(lcc, col), cl);   // L[col, k+c]
                            const double sc = (k + c < nF) ? -1.0 : 1.0;
#pragma unroll
                            for (int r = 0; r < RPL; ++r) sacc[r][b2] += (sc * Lc[r][c]) * lkc;
                        }
                        double skr[RPL];
#pragma unroll
                        for (int r = 0; r < RPL; ++r) skr[r] = (col < nF) ? sacc[r][b2] : -sacc[r][b2];
                        const double dk = gbcast<P>(slot_of(skr, col), cl);
                        if (!(dk > 0.0) || !(dk < kInf)) { ok = false; fk = 3; }
                        else {
                            const double il = rsqrt_nr(dk);
#pragma unroll
                            for (int r = 0; r < RPL; ++r) {
                                const int lr = l + r * P;
                                Lc[r][b2] = (lr == col) ? dk * il : skr[r] * il;
                                if (lr == col) w.ldi()[col] = il;   // ldi/kdi: 2N contiguous
                            }
                        }
                    }
                }
                if (!ok) break;
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    const int lr = l + r * P;
#pragma unroll
                    for (int b2 = 0; b2 < KB; ++b2)
                        if (b2 < kb && lr >= k + b2 && lr <= nt) myrow[r][w.bcol(k + b2, nt)] = Lc[r][b2];
                }
                NTM_WSYNC();
            }
        }
        NTM_ACC(ST_S_CHOL, tp);
        if (ok) {
            // L_A' x = diag(I, -I) z: x = [V_F; -mu], one backward sweep.  The
            // right-hand-side row holds sigma_k z_k (sigma = +1 free, -1 general
            // columns), which is exactly diag(I, -I) z
            double acc[RPL], x[RPL];
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
                const int lr = l + r * P;
                acc[r] = (lr < nt) ? Lp[w.brow(nt) + w.bcol(lr, nt)] : 0.0;
                x[r] = 0.0;
            }
            // the loads of column k-1 are issued before the broadcast of x_k (one-deep pipeline)
            double lkn[RPL], dkn = 0.0;
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
                const int lr = l + r * P;
                lkn[r] = (nt > 0 && lr < nt - 1) ? Lp[w.brow(nt - 1) + w.bcol(lr, nt)] : 0.0;
            }
            if (nt > 0) dkn = w.ldi()[nt - 1];
            for (int k = nt - 1; k >= 0; --k) {
                double lk[RPL];
#pragma unroll
                for (int r = 0; r < RPL; ++r) lk[r] = lkn[r];
                const double dk = dkn;
                if (k > 0) {
#pragma unroll
                    for (int r = 0; r < RPL; ++r) {
                        const int lr = l + r * P;
                        lkn[r] = (lr < k - 1) ? Lp[w.brow(k - 1) + w.bcol(lr, nt)] : 0.0;
                    }
                    dkn = w.ldi()[k - 1];
                }
                const double xk = gbcast<P>(slot_of(acc, k), k % P) * dk;
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    const int lr = l + r * P;
                    if (lr == k) x[r] = xk;
                    if (lr < k) acc[r] -= lk[r] * xk;
                }
            }
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
                const int lr = l + r * P;
                if (lr >= nF && lr < nt) w.np()[lr - nF] = -x[r];
            }
            NTM_WSYNC();
            // V_F sits in rows < nF <= N <= P: slot 0
            const double vsc = __shfl(x[0], (l < N && !fixed) ? fpos : 0, P);
            vfin = fixed ? vb : vsc;
        }
        NTM_ACC(ST_S_SOLVE, tp);
    } else if constexpr (!kAlwaysFused) {
    ok = !collide && chol_inplace<P>(w.R(), nF, 1, LD, l, w.ldi());
    fk = ok ? 0 : 3;
    if (ok) {
        const double wl = fwd_lanes<P>(w.R(), w.ldi(), nF, 1, LD, gl, l);    // L^{-1} g_F
        double tl = -wl;
        NTM_ACC(ST_P_CHOL, tp);
        if (nS > 0) {
            // E' (compact rows) into Y = w.J() (row-major nF x nS), one entry per lane
            for (int idx = l; idx < nF * nS; idx += P) {
                const int a = idx / nS, s2 = idx - a * nS;
                w.J()[a * LDJ + s2] = gen_n(s2, w.fidx()[a]);
            }
            if (l < nF) w.d()[l] = wl;
            const double hs = hs_of(l);
            NTM_WSYNC();
            NTM_ACC(ST_S_E, tp);
            if (l < nS) {                          // Y = L^{-1} E': lane s solves column s
                for (int i = 0; i < nF; ++i) {
                    double y = w.J()[i * LDJ + l];
                    for (int k = 0; k < i; ++k) y -= w.R()[i + k * LD] * w.J()[k * LDJ + l];
                    w.J()[i * LDJ + l] = y * w.ldi()[i];
                }
            }
            NTM_WSYNC();
            NTM_ACC(ST_S_Y, tp);
            double* K = w.R() + LD;                // K(a, c), a >= c, at R[c + (a+1) LD]
            double rhs = 0.0;
            {
                const int npair = nS * (nS + 1) / 2;
                for (int idx = l; idx < npair; idx += P) {
                    int a = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
                    if ((a + 1) * (a + 2) / 2 <= idx) ++a;
                    if (a * (a + 1) / 2 > idx) --a;
                    const int c = idx - a * (a + 1) / 2;
                    double sK = 0.0;
                    for (int i = 0; i < nF; ++i) sK += w.J()[i * LDJ + a] * w.J()[i * LDJ + c];
                    K[a * LD + c] = sK;
                }
            }
            if (l < nS) {
                rhs = hs;
                for (int i = 0; i < nF; ++i) rhs += w.J()[i * LDJ + l] * w.d()[i];
            }
            NTM_WSYNC();
            NTM_ACC(ST_S_K, tp);
            ok = chol_inplace<P>(K, nS, LD, 1, l, w.kdi());
            NTM_ACC(ST_S_CHOL, tp);
            if (!ok) fk = 3;
            if (ok) {
                double t1 = fwd_lanes<P>(K, w.kdi(), nS, LD, 1, rhs, l);
                double mu = bwd_lanes<P>(K, w.kdi(), nS, LD, 1, t1, l);
                if (l < nS) w.np()[l] = mu;
                NTM_WSYNC();
                if (l < nF) {
                    double sY = 0.0;
                    for (int a = 0; a < nS; ++a) sY += w.J()[l * LDJ + a] * w.np()[a];
                    tl = sY - wl;
                }
                NTM_ACC(ST_S_SOLVE, tp);
            }
        }
        NTM_ACC(ST_P_SCHUR, tp);
        if (ok) {
            const double vF = bwd_lanes<P>(w.R(), w.ldi(), nF, 1, LD, tl, l);   // compact V_F
            const double vsc = __shfl(vF, (l < N && !fixed) ? fpos : 0, P);
            vfin = fixed ? vb : vsc;
        }
    }
    }
    NTM_ACC(ST_P_BWD, tp);
    // Generic kernels: one step of fixed-precision iterative refinement after the
    // bordered elimination.  Its range-space factor goes through L L' = G~_FF, which
    // loses digits when G~_FF is nearly singular although the KKT system is well
    // conditioned (input-rate rows holding the last inputs, N = 20 mode 3, which
    // runs here: ~1e-9 umax off the exact optimum).  Pass 0 of the certificate
    // loop computes the KKT residual [r1; r2] (r1 = G~V + F~ - E'mu on the free
    // variables, r2 = n_s'V - bc_s on the general rows), solves A [dV; -dmu] =
    // -[r1; r2] with the same factor (forward and backward sweeps), and pass 1
    // certifies the corrected point.  The specialised N = 20 / 50 kernels keep the
    // single pass (their register allocation decides their speed).
    constexpr bool kRefine = W::kNN == 0;
    bool refine = kRefine && ok && !sq && fused;
    double r2 = 0.0;
    for (int pass = 0; ok; ++pass) {
        // ---- KKT certificate ----
        const bool resid = refine && pass == 0;
        if (!dir) {
        if (l < N) { w.V()[l] = vfin; w.U()[l] = w.D()[l] * vfin; }
        NTM_WSYNC();
        // y = Gamma U once, for the primal check (state rows) and the gradient
        if (!y_ready) {
            if constexpr (kSplitR) {
                double y[1];
                gamma_rows_split<NTM_CH, 1>(w, {w.U()}, y, l);
                if (l < 2 * N) w.xp()[l] = y[0];
            } else {
                for (int r = l; r < 2 * N; r += P) w.xp()[r] = gamma_row_dot<NTM_CH>(w, r, w.U());
            }
            NTM_WSYNC();
        }
        }
        NTM_ACC(ST_K_Y, tp);
        Pick vf{};
        if (dir) {
        } else if (resid) {
            if (l < nS) {                                  // primal residual of general row l
                const int r = w.srw()[l];
                const double sg = w.ssg()[l];
                if (r >= 2 * N) {
                    const int i = r - 2 * N;
                    r2 = w.idun()[i] * (rows.du - sg * (w.U()[i] - w.U()[i - 1]));
                } else {
                    const int c = r & 1;
                    const double bval = (sg > 0.0) ? (rows.xmax(c) - w.e()[r]) : (-rows.xmin(c) + w.e()[r]);
                    r2 = w.irn()[r] * (bval - sg * w.xp()[r]);
                }
            }
        } else {
            double vmax = gmax<P>(l < N ? fabs(vfin) : 0.0);
            vf = rows.template check<P>(w, vfin, l, true, fmax(1.0, vmax), w.xp());
            ok = vf.p == 0;
        }
        NTM_ACC(ST_K_CHK, tp);
        // gradient G~V + F~ = D (2 Gamma' Om y) + F~, with Om y once per stage into
        // scratch (w.Phi() + 2N: Phi is dead until the next lift; the sparse pass
        // below uses its first nS entries, the refinement its first nt <= 2N): y
        // itself stays in w.xp(), where the rollout of a certified U reads it
        // (kSlim: Om = I, so Om y is y itself, read from w.xp())
        constexpr bool kOmyX = W::kSlim && qi_on<W>();     // Om y = y: read w.xp()
        double* const omy = kOmyX ? w.xp() : (W::kSlim ? w.Phi() : w.Phi() + 2 * N);
        double res = 0.0;
        if (dir) {                                         // n_p in place of the gradient
            if (l < N) res = -((rows.lin(w, dir_p, l) * w.D()[l]) / rows.rnorm(w, dir_p));
        } else {
        if (l < N && !kOmyX) {
            const double y0 = w.xp()[2 * l], y1 = w.xp()[2 * l + 1];
            omy[2 * l] = om.o0(y0, y1);
            omy[2 * l + 1] = om.o1(y0, y1);
        }
        NTM_WSYNC();
        double g2c = 0.0;
        if constexpr (kSplitC) g2c = gamma_col_split<NTM_CH>(w, omy, l);
        if (l < N) {
            const double* cl = w.Gt() + w.gidx(2 * l, l) - 2 * l;
            const double g2 = kSplitC ? g2c : dot_rows2<NTM_CH>(cl, omy, N, l);      // terms i < l masked
            double gu = 2 * g2;
            if constexpr (ru_on<W>()) gu = gu + 2 * pb.Ru * w.U()[l];  // + 2 Ru U_l
            res = w.D()[l] * gu + w.F()[l];
        }
        }
        NTM_ACC(ST_K_GRAD, tp);
        if (sq) {
            // square path: the multipliers from E' mu = grad_F (E upper triangular in
            // sorted order), back substitution; lane t owns row t and grad at f_t
            if (l < N && !fixed) w.d()[fpos] = res;
            NTM_WSYNC();
            const int n = nS - (xb >= 0 ? 1 : 0) - (xb2 >= 0 ? 1 : 0);
            int pl = l + ((nc >= 0 && l >= nc) ? 1 : 0);             // lane t's pivot column
            if (kCollision && nc2 >= 0 && pl >= nc2) ++pl;
            if (kColl3 && nc3 >= 0 && pl >= nc3) ++pl;
            double acc = (l < n) ? w.d()[pl] : 0.0, mu = 0.0;
            // one collision: a second right-hand side, the left-out row B at the pivot columns
            double acb = (kCollision && xb >= 0 && l < n) ? gen_n(xb, w.fidx()[pl]) : 0.0, mb = 0.0;
            double acb2 = (kColl2 && xb2 >= 0 && l < n) ? gen_n(xb2, w.fidx()[pl]) : 0.0, mb2 = 0.0;
            // E[u][l] loaded kAheadB steps ahead (long horizons: NTM_MU_AHEAD; a register queue)
            constexpr int kAheadB = (W::kNN > 32) ? NTM_MU_AHEAD : 0;
            double bq[kAheadB > 0 ? kAheadB : 1];
#pragma unroll
            for (int a = 0; a < kAheadB; ++a) {
                const int ua = n - 1 - a;
                bq[a] = (ua >= 0 && l < ua) ? w.Ep()[w.eidx(ua, l)] : 0.0;
            }
            constexpr bool kPreB = NTM_SUB_PRESCALE && W::kNN > 32;   // as the forward substitution
            if constexpr (kPreB) { acc *= sq_id; acb *= sq_id; acb2 *= sq_id; }
            for (int u = n - 1; u >= 0; --u) {
                double eu;
                if constexpr (kAheadB > 0) {
                    eu = bq[0];
#pragma unroll
                    for (int a = 0; a + 1 < kAheadB; ++a) bq[a] = bq[a + 1];
                    const int ua = u - kAheadB;
                    bq[kAheadB - 1] = (ua >= 0 && l < ua) ? w.Ep()[w.eidx(ua, l)] : 0.0;
                } else {
                    eu = (l < u) ? w.Ep()[w.eidx(u, l)] : 0.0;
                }
                if constexpr (kPreB) eu *= sq_id;
                const double mu_u = gbcast<P>(kPreB ? acc : acc * sq_id, u);
                if (l == u) mu = mu_u;
                acc -= eu * mu_u;
                if (kCollision && xb >= 0) {
                    const double mb_u = gbcast<P>(kPreB ? acb : acb * sq_id, u);
                    if (l == u) mb = mb_u;
                    acb -= eu * mb_u;
                }
                if (kColl2 && xb2 >= 0) {
                    const double mb2_u = gbcast<P>(kPreB ? acb2 : acb2 * sq_id, u);
                    if (l == u) mb2 = mb2_u;
                    acb2 -= eu * mb2_u;
                }
            }
            if (kColl2 && xb2 >= 0) {
                // mu = a - mu_1 b1 - mu_2 b2; the two hole columns' equations give mu_1, mu_2:
                // mu_1 (n_B1[h] - E_h' b1) + mu_2 (n_B2[h] - E_h' b2) = grad[h] - E_h' a
                const double e1 = (l < n && nc < pl) ? gen_n(perm[l], w.fidx()[nc]) : 0.0;
                const double e2 = (l < n && nc2 < pl) ? gen_n(perm[l], w.fidx()[nc2]) : 0.0;
                const double sa1 = gsum<P>(e1 * mu), s11 = gsum<P>(e1 * mb), s12 = gsum<P>(e1 * mb2);
                const double sa2 = gsum<P>(e2 * mu), s21 = gsum<P>(e2 * mb), s22 = gsum<P>(e2 * mb2);
                double m11 = gen_n(xb, w.fidx()[nc]) - s11, m12 = gen_n(xb2, w.fidx()[nc]) - s12;
                double m21 = gen_n(xb, w.fidx()[nc2]) - s21, m22 = gen_n(xb2, w.fidx()[nc2]) - s22;
                double q1 = w.d()[nc] - sa1, q2 = w.d()[nc2] - sa2;
                double det = m11 * m22 - m12 * m21;
                if (kColl3 && nc3 >= 0) {
                    // k = 1: three hole equations, two unknowns; the best-conditioned pair
                    const double e3 = (l < n && nc3 < pl) ? gen_n(perm[l], w.fidx()[nc3]) : 0.0;
                    const double sa3 = gsum<P>(e3 * mu), s31 = gsum<P>(e3 * mb), s32 = gsum<P>(e3 * mb2);
                    const double m31 = gen_n(xb, w.fidx()[nc3]) - s31, m32 = gen_n(xb2, w.fidx()[nc3]) - s32;
                    const double q3 = w.d()[nc3] - sa3;
                    const double det13 = m11 * m32 - m12 * m31, det23 = m21 * m32 - m22 * m31;
                    if (fabs(det13) > fabs(det) && fabs(det13) >= fabs(det23)) {
                        m21 = m31; m22 = m32; q2 = q3; det = det13;
                    } else if (fabs(det23) > fabs(det)) {
                        m11 = m31; m12 = m32; q1 = q3; det = -det23;   // rows (3, 2): det = m31 m22 - m32 m21
                    }
                }
                const double mu1 = (m22 * q1 - m12 * q2) / det, mu2 = (m11 * q2 - m21 * q1) / det;
                mu -= mu1 * mb + mu2 * mb2;
                if (l == 0) { w.np()[xb] = mu1; w.np()[xb2] = mu2; }
            } else if (kCollision && xb >= 0) {
                // mu = a - mu_B b; a hole column's equation gives mu_B (with two holes,
                // k = 1, the one with the larger pivot; the other holds at the optimum)
                const double eh = (l < n && nc < pl) ? gen_n(perm[l], w.fidx()[nc]) : 0.0;
                const double sa = gsum<P>(eh * mu), sb = gsum<P>(eh * mb);
                double den = gen_n(xb, w.fidx()[nc]) - sb;
                double muB = (w.d()[nc] - sa) / den;
                if (nc2 >= 0) {
                    const double eh2 = (l < n && nc2 < pl) ? gen_n(perm[l], w.fidx()[nc2]) : 0.0;
                    const double sa2 = gsum<P>(eh2 * mu), sb2 = gsum<P>(eh2 * mb);
                    const double den2 = gen_n(xb, w.fidx()[nc2]) - sb2;
                    if (fabs(den2) > fabs(den)) { den = den2; muB = (w.d()[nc2] - sa2) / den2; }
                }
                if (kColl3 && nc3 >= 0) {                  // k = 2: a third hole
                    const double eh3 = (l < n && nc3 < pl) ? gen_n(perm[l], w.fidx()[nc3]) : 0.0;
                    const double sa3 = gsum<P>(eh3 * mu), sb3 = gsum<P>(eh3 * mb);
                    const double den3 = gen_n(xb, w.fidx()[nc3]) - sb3;
                    if (fabs(den3) > fabs(den)) { den = den3; muB = (w.d()[nc3] - sa3) / den3; }
                }
                mu -= muB * mb;
                if (l == 0) w.np()[xb] = muB;
            }
            if (l < n) w.np()[perm[l]] = mu;
            NTM_WSYNC();
        }
        NTM_ACC(ST_K_MU, tp);
        // - sum_s mu_s n_s[l]: for state rows n_s[l] = -ssg_s Gamma_{r_s l} D_l irn_{r_s},
        // i.e. + D_l sum_s Gamma_{r_s l} z_s with z_s = mu_s ssg_s irn_{r_s}: a sparse
        // pass over the nS active general rows only (z_s scratch in w.Phi(), dead
        // until the next lift; rows r_s >= 2N are rate rows, handled directly)
        double* const z = w.Phi();
        // (NTM_SUB_LANEIDX, long horizons) row s's index and z_s stay on lane s and the
        // column loop takes them by readlane: one LDS round trip per batch instead of two
        constexpr bool kSubLane = NTM_SUB_LANEIDX && P == 64 && (W::kNN > 32 || W::kNN == 0);
        int rsl = 0;
        double zsl = 0.0;
        if (l < nS) {
            const int r = w.srw()[l];
            const double zl = (r < 2 * N) ? (w.np()[l] * w.ssg()[l]) * w.irn()[r] : 0.0;
            if constexpr (kSubLane) { rsl = r; zsl = zl; }
            else z[l] = zl;
        }
        if constexpr (!kSubLane) NTM_WSYNC();
        if (l < N) {
            const double* cl = w.Gt() + w.gidx(2 * l, l) - 2 * l;   // cl[r] = gt(r, l), r >= 2l
            double sub = 0.0;
            constexpr int CH = NTM_CH;
            NTM_CHUNK_PRAGMA
            for (int s0 = 0; s0 < nS; s0 += CH) {
                int rr[CH];
                double zv[CH], gv[CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const bool in = s0 + u < nS;
                    if constexpr (kSubLane) {
                        const int src = __builtin_amdgcn_readfirstlane(s0 + u) & 63;
                        rr[u] = in ? __builtin_amdgcn_readlane(rsl, src) : 0;
                        zv[u] = in ? gbcast<P>(zsl, src) : 0.0;
                    } else {
                        rr[u] = in ? w.srw()[s0 + u] : 0;
                        zv[u] = in ? z[s0 + u] : 0.0;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const bool on = s0 + u < nS && rr[u] < 2 * N && (rr[u] >> 1) >= l;
                    gv[u] = on ? cl[rr[u]] : 0.0;
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < CH; ++u) sub += gv[u] * zv[u];
            }
            res += w.D()[l] * sub;
        }
        if (W::kNN != 20 && rows.has_rate()) {            // (N = 20 with rate rows runs on the generic kernels)
            // active rate rows (mode 3): row s of input i has normal entries at i and i-1
            // only, so each scatters mu_s n_s into two per-input slots (scratch: w.Vb() and
            // w.d(), dead here) and lane l takes its two; one active rate row per input at
            // most (both directions of one input active is singular, rejected above).
            // Replaces an nS-long loop per lane (config 5 mode 3: k_sub 235K cycles per
            // wave-step)
            double* const rhi = w.Vb();
            double* const rlo = w.d();
            if (l < N) { rhi[l] = 0.0; rlo[l] = 0.0; }
            NTM_WSYNC();
            if (l < nS && w.srw()[l] >= 2 * N) {
                const int i = w.srw()[l] - 2 * N;
                const double m = w.np()[l];
                rhi[i] = m * gen_n(l, i);
                rlo[i - 1] = m * gen_n(l, i - 1);
            }
            NTM_WSYNC();
            if (l < N) res -= rhi[l] + rlo[l];
        }
        NTM_ACC(ST_K_SUB, tp);
        if constexpr (kRefine) {
            if (resid) {
                // right-hand side -[r1; r2] in bordered-row order (scratch: w.Phi(), dead
                // after the sparse pass above), then L_A z = b, L_A' x = diag(I, -I) z
                NTM_WSYNC();
                if (l < N && !fixed) z[fpos] = -res;
                if (l < nS) z[nF + l] = -r2;
                NTM_WSYNC();
                auto slot_of = [&](const double* v, int k) -> double {   // v[k / P] (k uniform)
                    double o = v[0];
#pragma unroll
                    for (int r = 1; r < RPL; ++r) o = (k / P == r) ? v[r] : o;
                    return o;
                };
                double acc[RPL], xr[RPL];
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    const int lr = l + r * P;
                    acc[r] = (lr < nt) ? z[lr] : 0.0;
                    xr[r] = 0.0;
                }
                for (int k = 0; k < nt; ++k) {             // forward: L_A z = b
                    const double zk = gbcast<P>(slot_of(acc, k), k % P) * w.ldi()[k];
#pragma unroll
                    for (int r = 0; r < RPL; ++r) {
                        const int lr = l + r * P;
                        if (lr == k) xr[r] = zk;
                        if (lr > k && lr < nt) acc[r] -= Lp[w.brow(lr) + w.bcol(k, nt)] * zk;
                    }
                }
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    const int lr = l + r * P;
                    acc[r] = (lr < nF) ? xr[r] : -xr[r];
                    xr[r] = 0.0;
                }
                for (int k = nt - 1; k >= 0; --k) {        // backward: L_A' x = diag(I, -I) z
                    const double xk = gbcast<P>(slot_of(acc, k), k % P) * w.ldi()[k];
#pragma unroll
                    for (int r = 0; r < RPL; ++r) {
                        const int lr = l + r * P;
                        if (lr == k) xr[r] = xk;
                        if (lr < k) acc[r] -= Lp[w.brow(k) + w.bcol(lr, nt)] * xk;
                    }
                }
                // x = [dV_F; -dmu]: V_F in rows < nF <= N <= P (slot 0)
                const double dvs = __shfl(xr[0], (l < N && !fixed) ? fpos : 0, P);
                const double vr = fixed ? vfin : vfin + dvs;
                bool good = !(l < N) || isfinite(vr);
                NTM_WSYNC();
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    const int lr = l + r * P;
                    if (lr >= nF && lr < nt) good = good && isfinite(w.np()[lr - nF] - xr[r]);
                }
                good = gmaxi<P>(good ? 0 : 1) == 0;
                if (good) {
                    vfin = vr;
#pragma unroll
                    for (int r = 0; r < RPL; ++r) {
                        const int lr = l + r * P;
                        if (lr >= nF && lr < nt) w.np()[lr - nF] -= xr[r];
                    }
                }
                NTM_WSYNC();
                refine = false;
                y_ready = false;                           // V moved: y again
                continue;
            }
        }
        if (mult_out) {                                    // by active position
            if (l < nS) mult_out[w.sidx()[l]] = w.np()[l];
            if (fixed) mult_out[w.fx()[l] - 1] = res / w.hv()[l];
        }
#ifdef NTM_STAMPS
        if (!dir) {                                        // non-finite multipliers, by re-solve path
            const int nanm = gmaxi<P>(((l < nS && !isfinite(w.np()[l])) || (fixed && !isfinite(res / w.hv()[l]))) ? 1 : 0);
            const int nanv = gmaxi<P>((l < N && !isfinite(vfin)) ? 1 : 0);
            if (nanm) {
                if (!sq) NTM_CNT(CN_NAN_BORD);
                else if (xb2 >= 0) NTM_CNT(CN_NAN_COLL2);
                else if (xb >= 0) NTM_CNT(CN_NAN_COLL);
                else if (kdim == 0) NTM_CNT(CN_NAN_K0);
                else if (kdim == 1) NTM_CNT(CN_NAN_K1);
                else NTM_CNT(CN_NAN_K2);
                if (!ok) NTM_CNT(CN_NAN_PRIMFAIL);
                if (nanv) NTM_CNT(CN_NAN_V);
            }
        }
#endif
        if (dir) {
            ok = gmaxi<P>(((l < nS && !isfinite(w.np()[l])) || (fixed && !isfinite(res / w.hv()[l]))) ? 1 : 0) == 0;
            fk = ok ? 0 : 3;
            break;
        }
        // multipliers: general row s on lane s, fixed variable j on lane j; each
        // lane keeps its most negative one and that row's active-list position
        double mval = 0.0;
        int mpos = 0x7fffffff;
        bool has = false;
        if (l < nS) { mval = w.np()[l]; mpos = w.sidx()[l]; has = true; }
        if (!(fabs(mval) < kInf)) mval = -1e300;         // a non-finite multiplier fails the dual check
        if (fixed) {
            double lam = res / w.hv()[l];
            if (!(fabs(lam) < kInf)) lam = -1e300;
            if (!has || lam < mval) { mval = lam; mpos = w.fx()[l] - 1; }
            has = true;
        }
        double mabs = gmax<P>(has ? fabs(mval) : 0.0);
        double mkey = has ? mval : kInf;
        gargmin<P>(mkey, mpos);
        const bool dual_ok = !(mkey < -1e-9 * fmax(1.0, mabs));
        fk = !ok ? (dual_ok ? 2 : 4) : (!dual_ok ? 1 : 0);
        fpos_out = mpos;
        ok = ok && dual_ok;
        break;
    }
    ok = gmaxi<P>(ok ? 0 : 1) == 0;
    NTM_ACC(ST_P_KKT, tp);
    if (fail_kind) *fail_kind = uni<P>(fk);
    if (fail_pos) *fail_pos = uni<P>(fpos_out);
    if (v_out) *v_out = vfin;
    if (dir) {
        NTM_WSYNC();
        return ok;
    }
    if (verify_only && !ok) {
        if (l < N) w.V()[l] = Vprev;
        NTM_WSYNC();
        return false;
    }
    if (l < N) {
        w.U()[l] = ok ? (fixed ? uf : vfin * w.D()[l]) : Vprev * w.D()[l];
        w.V()[l] = ok ? vfin : Vprev;
    }
    NTM_WSYNC();
    return ok;
}

// ---------------------------------------------------------------------------
// rollout + scheduling update + convergence (NTM_MPC_Sim.m:110-117, 123-127)
// Returns (group-uniform) whether sum|Uold - U| < eps; updates Uold.
// ---------------------------------------------------------------------------
// With y_valid (the QP's U was certified by polish_compact, which leaves y = Gamma U
// in w.xp()) the rollout is the lifted prediction itself: x^_{i+1} = e_i + (Gamma U)_i
// with e = Phi x_k + Lambda, one row per lane.  That is the rollout identity the
// oracle tests pin (CANON D4/D6: Phi x_0 + Gamma U + Lambda == the recursion of
// NTM_MPC_Sim.m:113 with this iteration's rho), evaluated in another order: the
// same states to rounding, without the N-step serial recursion.  Otherwise (GI's
// uncertified result, a non-optimal flag, the literal D4/D6 lifts, for which the
// identity does not hold) the recursion runs on lane 0 as the reference writes it.
template <int P, class W>
__device__ __forceinline__ bool rollout_phase(const Prob& pb, const W& w, double x0, double x1, int l,
                                              bool y_valid = false) {
    const int N = w.n();
    const Coef k = scn_coef(pb, w);
    if constexpr (W::kNN == 0) {
        if (pb.flags & (NTM_LITERAL_PHI_RIGHTMUL | NTM_LITERAL_GAMMA_INDEX)) y_valid = false;
    }
    constexpr int RR = W::kNN > 0 ? (2 * W::kNN + P - 1) / P : 2;   // rows per lane (2N <= 2P)
    if (y_valid) {
        double v[RR];
#pragma unroll
        for (int t = 0; t < RR; ++t) {
            const int r = l + t * P;
            v[t] = (r < 2 * N) ? w.e()[r] + w.xp()[r] : 0.0;
        }
        NTM_WSYNC();
#pragma unroll
        for (int t = 0; t < RR; ++t) {
            const int r = l + t * P;
            if (r < 2 * N) w.xp()[r + 2] = v[t];
        }
        if (l == 0) {
            w.xp()[0] = x0;
            w.xp()[1] = x1;
        }
    } else if (l == 0) {
        double y0 = x0, y1 = x1;
        w.xp()[0] = y0;
        w.xp()[1] = y1;
        constexpr int CH = NTM_CH;                   // the loads of CH steps ahead of their stores
        NTM_CHUNK_PRAGMA
        for (int i0 = 0; i0 < N; i0 += CH) {
            double ca[CH], cb[CH], cc[CH], cu[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = i0 + u;
                if constexpr (W::kSlim) {           // the lift's coefficients, from this iteration's rho
                    ca[u] = i < N ? coef_a11(k, w.rho()[3 * i]) : 0.0;
                    cb[u] = i < N ? coef_b(k, w.rho()[3 * i + 2]) : 0.0;
                    cc[u] = i < N ? coef_a21(k, w.rho()[3 * i + 1]) : 0.0;
                } else {
                    ca[u] = i < N ? w.a11()[i] : 0.0;
                    cb[u] = i < N ? w.bb()[i] : 0.0;
                    cc[u] = i < N ? w.a21()[i] : 0.0;
                }
                cu[u] = i < N ? w.U()[i] : 0.0;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = i0 + u;
                if (i < N) {
                    const double n0 = (ca[u] * y0 + cb[u] * cu[u]) + k.C1;
                    const double n1 = (cc[u] * y0 + k.a22 * y1) + k.C2;
                    y0 = n0;
                    y1 = n1;
                    w.xp()[2 * i + 2] = y0;
                    w.xp()[2 * i + 3] = y1;
                }
            }
        }
    }
    NTM_WSYNC();
    double dsum = 0.0, u = 0.0;
    if (l < N) {
        double r1, r2, r3;
        rho_eval(k, w.xp()[2 * l], w.xp()[2 * l + 1], r1, r2, r3);
        w.rho()[3 * l] = r1;
        w.rho()[3 * l + 1] = r2;
        w.rho()[3 * l + 2] = r3;
        u = w.U()[l];
        dsum = fabs(w.Uold()[l] - u);
    }
    const bool conv = gsum<P>(dsum) < pb.eps;      // :123
    if (!conv && l < N) w.Uold()[l] = u;           // :127; the break at :125 skips it
    NTM_WSYNC();
    return conv;
}

// plant step NTM_MPC_Sim.m:130 (CANON D13: plant = prediction model, + C), plus
// the scenario's disturbance realisation at time index kt (ntm_ctx_set_scenarios;
// the model the controller predicts with does not know it)
template <bool GEN = false>
__device__ __forceinline__ void plant_step(const Prob& pb, const Coef& k, double x0, double x1, double u,
                                           double& n0, double& n1, int64_t gid = 0, int kt = 0) {
    double r1, r2, r3;
    rho_eval(k, x0, x1, r1, r2, r3);
    double a11 = coef_a11(k, r1), a21 = coef_a21(k, r2), b = coef_b(k, r3);
    n0 = a11 * x0 + b * u;
    n1 = a21 * x0 + k.a22 * x1;
    if (!(pb.flags & NTM_LITERAL_PLANT_NO_C)) { n0 += k.C1; n1 += k.C2; }
    if (GEN && gen_dist(pb)) {
        if (pb.g.sw != 0.0) n0 += pb.g.sw * gen_normal(pb.g.seed, gid, (uint32_t)kt, 0);
        if (pb.g.so != 0.0) n1 += pb.g.so * gen_normal(pb.g.seed, gid, (uint32_t)kt, 1);
    }
}

// ---------------------------------------------------------------------------
// Receding-horizon shift of a carried warm-start set, into w.act() (returns
// the shifted count).  The previous step planned stages k..k+N-1; this step
// plans k+1..k+N, so a row of stage i >= 1 moves to stage i-1, stage-0 rows
// are dropped, and the bound rows of the old last input and the terminal state
// rows are kept for the new last stage as well.  It is the SECOND candidate of inner iteration 2, after
// the unshifted set: in the closed loop's steady state the LPV iteration
// 2-cycles through the same pair of active sets every step (the odd and even
// iterations), so the previous step's set hits unshifted (70% at iteration 2
// over steps 5-20, against 7% shifted; 36% vs 31% over steps 1-4, where the
// plan still moves in time).  Only a hint: every candidate is re-solved
// exactly and KKT-certified.
// ---------------------------------------------------------------------------
template <int P, class W>
__device__ __forceinline__ int shifted_into_act(const Prob& pb, const W& w, const int* c, int l, bool hint_only = false) {
    const int N = w.n();
    const int lane = threadIdx.x & 63;
    const unsigned long long gmask = (P == 64) ? ~0ull : (((1ull << P) - 1ull) << (lane & ~(P - 1)));
    const unsigned long long below = (1ull << lane) - 1ull;
    const int q = uni<P>(c[N]);
    int nid = -1, dup = -1;
    if (l < q) {
        const int id = c[l];
        if (pb.mode == NTM_MODE_BOX) {
            const int j = id < N ? id : id - N;
            if (j >= 1) nid = id - 1;
            if (j == N - 1) dup = id;
        } else if (id >= 6 * N + 4) {                    // rate row of input j
            const int j = ((id - (6 * N + 4)) >> 1) + 1;
            if (j >= 2) nid = id - 2;
            if (j == N - 1) dup = id;
        } else if (id >= 6 * N) {                        // terminal state row -> stage N-1, and kept
            nid = 6 * (N - 1) + 2 + (id - 6 * N);
            dup = id;
        } else {
            const int blk = id / 6, rr = id - 6 * blk;
            if (blk >= 2 || (blk == 1 && rr < 2)) nid = id - 6;   // x_1's state rows would become
            if (blk == N - 1 && rr < 2) dup = id;                  // x_0 rows (constant): dropped
        }
    }
    if (hint_only) {                                     // flag the shifted rows (kCandRow) instead
        if (nid >= 0) w.aflag()[nid] = kCandRow;
        if (dup >= 0) w.aflag()[dup] = kCandRow;
        NTM_WSYNC();
        return 0;
    }
    const unsigned long long bk = __ballot(nid >= 0) & gmask;
    const unsigned long long bd = __ballot(dup >= 0) & gmask;
    const int nk = uni<P>((int)__popcll(bk)), nd = uni<P>((int)__popcll(bd));
    const bool with_dup = nk + nd <= N;
    if (nid >= 0) w.act()[__popcll(bk & below)] = nid;
    if (with_dup && dup >= 0) w.act()[nk + __popcll(bd & below)] = dup;
    NTM_WSYNC();
    return nk + (with_dup ? nd : 0);
}

// ---------------------------------------------------------------------------
// qp_phase's Goldfarb-Idnani fallback (the full G~, GI warm-started from the
// failed candidate, then its certified polish; ~2.5% of the QPs at N = 20).
// NTM_GI_OUTLINE=1 makes it a real call, so that its register allocation is its
// own instead of the step kernel's (the caller's live registers are saved around
// the call); 0 inlines it like every other phase.
// ---------------------------------------------------------------------------
#ifndef NTM_GI_DEFER_PROBE
#define NTM_GI_DEFER_PROBE 0   // timing probe only: GI compiled out of qp_phase
#endif
#ifndef NTM_GI_OUTLINE
#define NTM_GI_OUTLINE 0
#endif
#if NTM_GI_OUTLINE
#define NTM_GI_ATTR __attribute__((noinline))
#else
#define NTM_GI_ATTR __forceinline__
#endif
template <int P, class W>
__device__ NTM_GI_ATTR int gi_fallback(const Prob& pb, const W w, const StructRows rows, int nrows, int l, int nwarm,
                                       int it, int* qp_iters, int* q_out, int* ns_out, bool* yv_out) {
    NTM_T0(tq);
    int flag, q = 0, ns = 0;
    bool yv = false;
    if (!full_gram<P>(pb, w, l)) {
        flag = NTM_EXIT_NONFINITE;
    } else {
        NTM_ACC(ST_REGRAM, tq);
        NTM_CNT(CN_GIRUN);
        if (it == 1) NTM_CNT(CN_GI_IT1); else if (it == 2) NTM_CNT(CN_GI_IT2); else NTM_CNT(CN_GI_LATE);
        // warm from the failed candidate; if its multipliers are not all >= 0, warm
        // again from the rows whose multipliers were; then cold
        for (int pass = 0;; ++pass) {
            flag = gi_solve<P, StructRows, W>(w, rows, pb.mode != NTM_MODE_NONE, nrows, l, qp_iters, &q,
                                              pass < 2 ? nwarm : 0);
            if (flag != kGiWarmRejected) break;
            nwarm = (pass == 0) ? q : 0;
            q = 0;
            if (!full_gram<P>(pb, w, l)) { flag = NTM_EXIT_NONFINITE; break; }
        }
        NTM_ACC(ST_GI, tq);
        if (flag == NTM_EXIT_OPTIMAL) {
            const bool okp = polish_compact<P>(pb, w, rows, q, l, false, &ns);
            NTM_TRACE("QP GI flag %d q %d polish %d\n", flag, q, (int)okp);
            yv = okp;
        }
        NTM_ACC(ST_POLISH, tq);
    }
    *q_out = q;
    *ns_out = ns;
    *yv_out = yv;
    return flag;
}

// ---------------------------------------------------------------------------
// one inner iteration's QP: build -> scale -> GI -> polish -> w.U()
// ---------------------------------------------------------------------------
template <int P, class W>
__device__ __forceinline__ int qp_phase(const Prob& pb, const W& w, double x0, double x1, int l, int* qp_iters,
                        int* q_out, int* ns_out, int slot, int* n_try = nullptr, int* n_girun = nullptr,
                        int it = 0, bool* y_valid = nullptr) {
    const int N = w.n();
    bool yv = false;                                     // w.xp() holds Gamma U of the final U
    NTM_T0(tq);
    ColSums colsum;
    lift_phase<P>(pb, w, l, x0, x1, &colsum);
    NTM_ACC(ST_LIFT, tq);
    free_response<P>(w, x0, x1, l, &pb);     // F is formed with the Jacobi scaling below
    NTM_ACC(ST_COST, tq);
    const bool full = pb.mode >= NTM_MODE_FULL;        // state rows present
    int flag, q = 0, ns = 0;
    *qp_iters = 0;
    StructRows rows(pb);
    int* cand = w.cand() + slot * (N + 1);               // this QP's active set is stored here
    const int scode = diag_scale_phase<P>(pb, w, l, full, x0, x1, &colsum);
    if (scode >= 2) {
        flag = NTM_EXIT_NONFINITE;
    } else {
        const int nrows = (pb.mode == NTM_MODE_NONE) ? 0 : rows.rows();
        if (pb.mode != NTM_MODE_NONE) {
            for (int i = l; i < nrows; i += P) w.aflag()[i] = 0;
            NTM_WSYNC();
        }
        bool infeasible;                                   // a constant row violated (D15, D22)
        if constexpr (fold_const<W>()) infeasible = pb.mode != NTM_MODE_NONE && scode == 1;
        else infeasible = pb.mode != NTM_MODE_NONE && !rows.template feasible_const<P>(w, x0, x1, l);
        if (infeasible) {
            flag = NTM_EXIT_INFEASIBLE;
        } else {
            NTM_ACC(ST_SCALE, tq);
            bool done = false;
            int nwarm = 0;
            // warm start: the LPV loop alternates between two QPs (a 2-cycle),
            // so the active set of iteration it-2 is tried first; it is taken
            // only if the exact active-set solve passes the KKT certificate
            // (the optimum of this strictly convex QP is unique).
            const int cq0 = uni<P>(cand[N]);
            if (cq0 >= 0) {
                NTM_CNT(CN_CAND);
                int cq = cq0;
                // long horizons shift the carried set first at iteration 2: offline
                // (NumPy oracle, steps 5-12) the receding-horizon shift of the previous
                // step's last even set is iteration 2's optimum for 75% of the N = 50
                // scenario-steps (mode 2; 72% in mode 3) and the unshifted set for 19%;
                // at N = 20 the unshifted set wins (55% against 18%)
                const bool shift_first = (W::kNN > 32 || (W::kNN == 0 && N > 32)) && it == 2 &&
                                         pb.mode != NTM_MODE_NONE;
                if (shift_first) {
                    cq = shifted_into_act<P>(pb, w, cand, l);
                } else {
                    if (l < cq) w.act()[l] = cand[l];
                    NTM_WSYNC();
                }
#ifdef NTM_DEBUG_SCEN
                NTM_TRACE("SET it %d cand %d:", it, cq);
                for (int i = 0; i < cq; ++i) NTM_TRACE(" %d", w.act()[i]);
                NTM_TRACE("\n");
#endif
#if NTM_CDP
                // Certified dual path (round 5).  The candidate's re-solve either
                // certifies, or it gives the set's equality-constrained optimum and
                // multipliers.  A set whose multipliers are not all >= 0 first drops
                // its most negative one, re-solving each time, until it is dual
                // feasible.  From there Goldfarb & Idnani's dual method runs with
                // certified re-solves as its linear algebra: the most violated row p
                // is added; the re-solve on A + {p} is the end point of GI's (linear)
                // step, so a multiplier of A that is negative there is dropped at the
                // fraction of the step where it reaches zero (V and the multipliers
                // interpolated), and A - {i} + {p} is re-solved; a row p dependent on
                // A (a full set: q = N) takes GI's dual-only step, with r from the
                // certificate's multiplier pass on n_p (polish_compact, dir_p).  The
                // last re-solve of a full step that passes the KKT certificate is
                // the answer.  Offline (tools/repair_study.py, N = 20 mode 2, steps
                // 6-25): every iteration-2 QP certifies, 3.2 re-solves on average,
                // where the single-row repairs left 16% to Goldfarb-Idnani.  GI itself
                // (warm from the current set) is the fallback when the budget runs
                // out or the set degenerates.
                // Iteration 2: a singular carried set is replaced by the other form
                // (shifted or unshifted) of the previous step's last even set.
                bool alt = it == 2 && pb.mode != NTM_MODE_NONE;
                const int budget = N + kCdpExtra;
                // drop position `pos` of the active list (and of the lane-per-position u)
                auto drop_at = [&](int pos, double& u) {
                    int an = 0;
                    if (l >= pos && l + 1 < cq) an = w.act()[l + 1];
                    const double un = __shfl(u, (l + 1) & (P - 1), P);
                    NTM_WSYNC();
                    if (l >= pos && l + 1 < cq) w.act()[l] = an;
                    if (l >= pos) u = (l + 1 < cq) ? un : 0.0;
                    --cq;
                    NTM_WSYNC();
                };
                // One polish_compact call site (the kernel inlines it): each trip re-solves
                // qs rows (A, or A + {p} at position cq) or, with dirp >= 0, takes the
                // dual-only direction of row dirp on A.  stage 0: the carried set;
                // 1: dropping negative multipliers; 2: A + {p}; 3: the direction of p
                int stage = 0, qs = cq, dirp = -1, p = -1, nres = 0, fk = 0, fp = 0;
                // Long horizons: an A + {p} whose end point has a non-finite multiplier (p
                // (nearly) depends on A) leaves p out (kSkipRow) and adds another violated row
                // instead, as the dual method may add any violated row; p is eligible again
                // once A changes.  Before round 6 these QPs went to GI (N = 50 mode 2: 0.1 per
                // MPC step, 7% of the cycles)
                constexpr bool kSkipNan = NTM_CDP_SKIP && (W::kNN > 32 || W::kNN == 0);
                constexpr bool kSkipDir = kSkipNan && NTM_CDP_SKIPDIR;
                int nskip = 0;
                bool fresh_y = false;                      // the pick recomputes y = Gamma U at V0
                auto clear_skips = [&]() {
                    if (kSkipNan && nskip > 0) {
                        for (int i = l; i < nrows; i += P) w.aflag()[i] &= (unsigned char)~kSkipRow;
                        NTM_WSYNC();
                        nskip = 0;
                    }
                };
                // iteration 2 at N <= 32 starts from the unshifted carried set; the dual
                // path then adds violated rows of its receding-horizon shift first
                // (StructRows::check prefers kCandRow rows).  Offline (tools/repair_study.py,
                // N = 20 mode 2): 2.67 -> 2.50 re-solves per iteration-2 QP; on the device
                // 6.45 -> 6.36 ms per step-batch (A/B on one box).  Not for box-only QPs
                // (their single-row exchanges: config 2 0.206 -> 0.214 ms with it)
                if (NTM_CDP_HINT && alt && !shift_first && pb.mode != NTM_MODE_BOX)
                    (void)shifted_into_act<P>(pb, w, cand, l, true);
                double vf = 0.0, V0 = 0.0, u0 = 0.0;   // V0: lane = variable; u0: lane = active position
                bool okc = false;
                for (;;) {
                    if (n_try && dirp < 0) ++*n_try;
                    const bool oks = polish_compact<P>(pb, w, rows, qs, l, true, &ns, &fk, &fp, &vf, w.uu(), dirp);
                    NTM_TRACE("QP cdp stage %d qs %d dir %d ok %d fk %d fp %d\n", stage, qs, dirp, (int)oks, fk, fp);
                    ++nres;
                    bool pick = false;
                    if (stage == 0) {
                        if (it <= 2) NTM_CNT(CN_TRY_EARLY);
                        if (!oks) { if (it <= 2) NTM_CNT(CN_FAIL_EARLY); else NTM_CNT(CN_FAIL_LATE); }
                        if (it <= 2 && !oks) {
                            if (fk == 1) NTM_CNT(CN_FK_DUAL);
                            else if (fk == 2) NTM_CNT(CN_FK_PRIMAL);
                            else if (fk == 3) NTM_CNT(CN_FK_SING);
                            else NTM_CNT(CN_FK_BOTH);
                        }
                        if (it == 1) { NTM_CNT(CN_TRY_IT1); if (!oks) NTM_CNT(CN_FAIL_IT1); }
                        if (it == 2) { NTM_CNT(CN_TRY_IT2); if (!oks) NTM_CNT(CN_FAIL_IT2); }
                        if (oks) { okc = true; break; }
                        if (fk == 3) {                     // singular: the other form of the carried set
                            if (!alt) { NTM_CNT(CN_CDPX_SING0); break; }
                            alt = false;
                            NTM_CNT(CN_ALT_TRY);
                            if (shift_first) {
                                cq = cq0;
                                if (l < cq) w.act()[l] = cand[l];
                                NTM_WSYNC();
                            } else {
                                cq = shifted_into_act<P>(pb, w, cand, l);
                            }
                            qs = cq;
                            continue;
                        }
                        stage = pb.mode == NTM_MODE_BOX ? 4 : 1;
                    }
                    if (stage == 4) {
                        // Box-only QPs (BASELINE config 2): single-row exchanges, as before round
                        // 5.  A violated bound joins (with a negative multiplier too, that row
                        // leaves in the same exchange; in a full set it takes the place of the
                        // smallest multiplier); a negative multiplier alone leaves.  Measured on
                        // the all-LDS build at B = 1024 (one wave per SIMD: the longest scenario
                        // decides): 0.281 ms per step with the dual path, 0.262 with 8 exchanges,
                        // 0.224 with 16 (A/B on one box)
                        if (oks) { okc = true; break; }
                        if (fk == 3 || nres > kBoxRepairs) { NTM_CNT(CN_CDPX_BUDGET); break; }
                        if (fk == 1) {
                            double ud = 0.0;
                            drop_at(fp, ud);
                        } else {
                            if (l < cq) w.aflag()[w.act()[l]] = kActiveRow;
                            NTM_WSYNC();
                            const double vmx = fmax(1.0, gmax<P>(l < N ? fabs(vf) : 0.0));
                            const Pick pk = rows.template check<P>(w, vf, l, false, vmx, w.xp());
                            NTM_WSYNC();
                            if (l < cq) w.aflag()[w.act()[l]] = 0;
                            NTM_WSYNC();
                            if (pk.p < 0) break;
                            const int lane = threadIdx.x & 63;
                            const unsigned long long gm = (P == 64) ? ~0ull : (((1ull << P) - 1ull) << (lane & ~(P - 1)));
                            const bool keep = l < cq && !(fk == 4 && l == fp);
                            const unsigned long long km = __ballot(keep) & gm;
                            const int nkeep = uni<P>((int)__popcll(km));
                            const int my = (l < cq) ? w.act()[l] : 0;
                            NTM_WSYNC();
                            if (nkeep < N) {
                                if (keep) w.act()[__popcll(km & ((1ull << lane) - 1ull))] = my;
                                if (l == 0) w.act()[nkeep] = pk.p;
                                cq = nkeep + 1;
                            } else if (l == 0) {
                                w.act()[fp] = pk.p;
                            }
                            NTM_WSYNC();
                        }
                        qs = cq;
                        NTM_CNT(CN_CDP_DROP);
                        continue;
                    }
                    if (stage == 1) {                      // dual feasibility first
                        if (oks) { okc = true; break; }
                        if (fk == 1 || fk == 4) {
                            if (nres >= budget) { NTM_CNT(CN_CDPX_BUDGET); break; }
                            double ud = 0.0;
                            drop_at(fp, ud);
                            qs = cq;
                            NTM_CNT(CN_CDP_DROP);
                            continue;
                        }
                        if (fk != 2) { NTM_CNT(CN_CDPX_SING1); break; }
                        V0 = vf;
                        u0 = (l < cq) ? w.uu()[l] : 0.0;
                        pick = true;
                    } else if (stage == 2) {               // the end point of adding p
                        NTM_CNT(CN_CDP_RES);
                        if (oks) { ++cq; okc = true; break; }
                        if (fk == 3) {                     // A + {p} singular: p depends on A
                            dirp = p;
                            qs = cq;
                            stage = 3;
                            continue;
                        }
                        const double u1 = (l <= cq) ? w.uu()[l] : 0.0;
                        double th = (l < cq && u1 < 0.0) ? u0 / (u0 - u1) : kInf;
                        // a non-finite end-point multiplier (A's or p's own) makes the step
                        // meaningless: th = -1 (a real fraction is in [0, 1)) hands the QP to
                        // GI below instead of reading it as a negative multiplier
                        if (l <= cq && !isfinite(u1)) th = -1.0;
                        int li = l;
                        gargmin<P>(th, li);
                        if (th < 0.0) {
                            NTM_CNT(CN_CDPX_NAN);
                            if (!kSkipNan || nres >= budget) break;
                            if (l == 0) w.aflag()[p] |= kSkipRow;
                            if (l < N) w.U()[l] = w.D()[l] * V0;   // the pick's y at V0, not the end point's
                            NTM_WSYNC();
                            ++nskip;
                            NTM_CNT(CN_CDP_SKIP);
                            pick = true;
                            fresh_y = true;
                        } else if (!(th < kInf)) {         // full step: p joins A
                            if (fk != 2) {
                                // p's own multiplier < 0 at the end point (A's are all >= 0): p
                                // (nearly) depends on A, an ill-conditioned step at long horizons.
                                // GI would take its dual-only step there; so does the path (A, V0
                                // and u0 unchanged).  Dropping that multiplier and continuing
                                // instead measured slower (config 5 mode 2: 112 -> 156 ms)
                                NTM_CNT(CN_CDPX_FULLDUAL);
                                dirp = p;
                                qs = cq;
                                stage = 3;
                                continue;
                            }
                            ++cq;
                            u0 = (l < cq) ? u1 : 0.0;
                            V0 = vf;
                            pick = true;
                            clear_skips();
                        } else {                           // partial step: row li reaches u = 0 and leaves
                            V0 += th * (vf - V0);
                            u0 += th * (u1 - u0);
                            drop_at(li, u0);
                            NTM_CNT(CN_CDP_PART);
                            clear_skips();
                        }
                    } else {                               // dual-only step: n_p = sum_i r_i n_i over A
                        NTM_CNT(CN_CDP_DIR);
                        dirp = -1;
                        if (!oks) { NTM_CNT(CN_CDPX_DIR); break; }
                        const double r = (l < cq) ? w.uu()[l] : 0.0;
                        double tt = (l < cq && r > 0.0) ? u0 / r : kInf;
                        int li = l;
                        gargmin<P>(tt, li);
                        if (!(tt < kInf)) { NTM_CNT(CN_CDPX_TINF); break; }   // no row can leave: GI decides (infeasible)
                        u0 -= tt * r;
                        drop_at(li, u0);
                        clear_skips();
                    }
                    if (pick) {                            // the most violated row at V0 (y of the last re-solve in w.xp())
                        if (l < cq) w.aflag()[w.act()[l]] = kActiveRow;
                        NTM_WSYNC();
                        const double vmx = fmax(1.0, gmax<P>(l < N ? fabs(V0) : 0.0));
                        const Pick pk = rows.template check<P>(w, V0, l, false, vmx, fresh_y ? nullptr : w.xp());
                        fresh_y = false;
                        NTM_WSYNC();
                        if (l < cq) w.aflag()[w.act()[l]] = 0;
                        NTM_WSYNC();
                        if (pk.p < 0 || !(pk.s < -1e-9 * fmax(vmx, fabs(pk.bc)))) {
                            // the only violated rows left are skipped ones (A + {p} had a
                            // non-finite end point: p nearly depends on A): GI's step for a
                            // dependent row, the dual-only direction of the last skipped row p
                            // (round 6, NTM_CDP_SKIPDIR), instead of handing the QP to GI
                            if (kSkipDir && nskip > 0 && p >= 0 && nres < budget) {
                                NTM_CNT(CN_CDP_SKIPDIR);
                                dirp = p;
                                qs = cq;
                                stage = 3;
                                continue;
                            }
                            NTM_CNT(CN_CDPX_NOVIOL);
                            break;
                        }
                        p = pk.p;
                    }
                    if (nres >= budget) { NTM_CNT(CN_CDPX_BUDGET); break; }   // add p: A + {p}, or its direction when A is full
                    if (cq >= N) {
                        dirp = p;
                        qs = cq;
                        stage = 3;
                    } else {
                        if (l == 0) w.act()[cq] = p;
                        NTM_WSYNC();
                        qs = cq + 1;
                        stage = 2;
                    }
                }
                if (okc) {
                    flag = NTM_EXIT_OPTIMAL;
                    q = cq;
                    done = true;
                    yv = true;
                    NTM_CNT(CN_HIT);
                    if (nres > 1) NTM_CNT(CN_REPAIR);
                } else {
                    NTM_CNT(CN_CDP_GI);
                    clear_skips();
                    // GI warm from the current set (dual feasible on the primal phase)
                    if (l < cq) {
                        w.aflag()[w.act()[l]] = kCandRow;
                        w.sidx()[l] = w.act()[l];
                    }
                    nwarm = cq;
                    NTM_WSYNC();
                }
#else
                // iteration 2: the carried set is the previous step's (slot 1 is only
                // written at even iterations); when its repairs fail, its
                // receding-horizon shift is tried before GI (it hits in the
                // transient of the first steps, where the plan moves in time)
                bool alt = it == 2 && pb.mode != NTM_MODE_NONE;
                int keep_id = -1, keep_q = -1;     // the repaired set (lane l: entry l) while the shift is tried
                // certified re-solve of the candidate; on failure, up to kRepairs
                // single-row repairs (add the most violated row and/or drop the row
                // with the most negative multiplier) before falling back to GI.
                // Only a set that passes the KKT certificate is ever accepted.
                for (int rep = 0;; ++rep) {
                    if (n_try) ++*n_try;
                    int fk = 0, fp = 0;
                    double vf = 0.0;
                    const bool okc = polish_compact<P>(pb, w, rows, cq, l, true, &ns, &fk, &fp, &vf);
                    NTM_TRACE("QP cand rep %d cq %d ok %d fk %d fp %d\n", rep, cq, (int)okc, fk, fp);
                    if (rep == 0) {
                        if (it <= 2) NTM_CNT(CN_TRY_EARLY);
                        if (!okc) { if (it <= 2) NTM_CNT(CN_FAIL_EARLY); else NTM_CNT(CN_FAIL_LATE); }
                        if (it <= 2 && !okc) {
                            if (fk == 1) NTM_CNT(CN_FK_DUAL);
                            else if (fk == 2) NTM_CNT(CN_FK_PRIMAL);
                            else if (fk == 3) NTM_CNT(CN_FK_SING);
                            else NTM_CNT(CN_FK_BOTH);
                        }
                        if (it == 1) { NTM_CNT(CN_TRY_IT1); if (!okc) NTM_CNT(CN_FAIL_IT1); }
                        if (it == 2) { NTM_CNT(CN_TRY_IT2); if (!okc) NTM_CNT(CN_FAIL_IT2); }
                    }
                    if (rep < 0 && okc) NTM_CNT(CN_ALT_HIT);
                    if (okc) {
                        flag = NTM_EXIT_OPTIMAL;
                        q = cq;
                        done = true;
                        yv = true;
                        NTM_CNT(CN_HIT);
                        if (rep > 0) NTM_CNT(CN_REPAIR);
                        break;
                    }
                    bool stop = rep >= kRepairs || rep < 0 || fk == 3;   // rep < 0: the shifted set failed
                    if (!stop && (fk == 2 || fk == 4)) {   // primal: add the most violated row
                        if (l < cq) w.aflag()[w.act()[l]] = kActiveRow;
                        NTM_WSYNC();
                        const double vmx = gmax<P>(l < N ? fabs(vf) : 0.0);
                        const Pick pk = rows.template check<P>(w, vf, l, false, fmax(1.0, vmx));
                        NTM_WSYNC();
                        if (l < cq) w.aflag()[w.act()[l]] = 0;
                        NTM_WSYNC();
                        if (pk.p < 0) {
                            stop = true;
                        } else {
                            // A state or rate row whose last variable is held by a bound row
                            // takes that bound row's place (adding it next to the bound would
                            // leave it no free variable: a singular system).  This is how a
                            // boundary arc moves by one stage from step to step.  With a
                            // negative multiplier too (fk 4) that row goes as well.
                            int kind, jr, jl = -1;
                            rows.decode(pk.p, N, kind, jr);
                            if ((kind == 2 || kind == 3) && jr >= 0) jl = (w.rinfo()[jr] & (kRowMulti - 1)) - 1;
                            else if (kind >= 4) jl = jr;
                            int my = -1;
                            bool drop_me = false, rate_hold = false;
                            // rate rows (long horizons and the generic kernels): a u bound on
                            // input jb entering a full set replaces the one active rate row that
                            // holds jb (U_i - U_{i-1} with i or i-1 = jb), and a rate row entering
                            // one replaces the bound on its earlier input.  With rate rows the
                            // odd LPV iterations can alternate between two sets that differ in
                            // exactly that pair (a period-4 cycle), and the
                            // smallest-multiplier swap below would pick another row
                            constexpr bool kRateSwap = W::kNN > 32 || W::kNN == 0;
                            const int jb = (kRateSwap && kind < 2) ? jr : -1;
                            if (l < cq) {
                                my = w.act()[l];
                                int k2, j2;
                                rows.decode(my, N, k2, j2);
                                drop_me = (jl >= 0 && k2 < 2 && j2 == jl) || (fk == 4 && l == fp);
                                rate_hold = jb >= 0 && k2 >= 4 && (j2 == jb || j2 - 1 == jb);
                                // and a rate row of input jr entering a full set replaces the
                                // u bound on input jr - 1 (the one on jr is dropped above)
                                if (kRateSwap && kind >= 4 && k2 < 2 && j2 == jr - 1) rate_hold = true;
                            }
                            const int lane = threadIdx.x & 63;
                            const unsigned long long gm =
                                (P == 64) ? ~0ull : (((1ull << P) - 1ull) << (lane & ~(P - 1)));
                            const unsigned long long keepm = __ballot(l < cq && !drop_me) & gm;
                            const int nkeep = uni<P>((int)__popcll(keepm));
                            const unsigned long long rhm = kRateSwap ? (__ballot(rate_hold) & gm) : 0ull;
                            NTM_WSYNC();
                            if (nkeep < N) {
                                if (l < cq && !drop_me) w.act()[__popcll(keepm & ((1ull << lane) - 1ull))] = my;
                                if (l == 0) w.act()[nkeep] = pk.p;
                                cq = nkeep + 1;
                            } else if (kRateSwap && __popcll(rhm) == 1) {   // a full set: the rate row holding jb
                                if (rate_hold) w.act()[l] = pk.p;
                            } else if (l == 0) {           // a full set: swap out the smallest multiplier
                                w.act()[fp] = pk.p;
                            }
                        }
                    } else if (!stop) {                    // dual: drop position fp
                        int an = 0;
                        if (l >= fp && l + 1 < cq) an = w.act()[l + 1];
                        NTM_WSYNC();
                        if (l >= fp && l + 1 < cq) w.act()[l] = an;
                        --cq;
                    }
                    if (stop) {
                        if (!alt) break;
                        alt = false;                       // last try: the other form of the carried set
                        NTM_CNT(CN_ALT_TRY);
                        keep_id = (l < cq) ? w.act()[l] : -1;   // the repaired set, for GI's warm start
                        keep_q = cq;
                        NTM_WSYNC();
                        if (shift_first) {                 // the unshifted carried set
                            cq = cq0;
                            if (l < cq) w.act()[l] = cand[l];
                            NTM_WSYNC();
                        } else {                           // the shifted carried set
                            cq = shifted_into_act<P>(pb, w, cand, l);
                        }
                        rep = -2;                          // counted as neither a first try nor a repair
                    }
                    NTM_WSYNC();
                }
                if (!done) {
                    if (keep_q >= 0) {                     // back to the repaired set
                        cq = keep_q;
                        if (l < cq) w.act()[l] = keep_id;
                        NTM_WSYNC();
                    }
                    // the repaired set steers GI's add order (StructRows::check) and,
                    // is GI's warm-start set (gi_solve)
                    if (l < cq) {
                        w.aflag()[w.act()[l]] = kCandRow;
                        w.sidx()[l] = w.act()[l];
                    }
                    nwarm = cq;
                    NTM_WSYNC();
                }
#endif
                NTM_ACC(ST_CAND, tq);
            }
            if (!done) {
                if (n_girun) ++*n_girun;
#if NTM_GI_DEFER_PROBE
                // timing probe only: the set at hand is taken as if certified (wrong
                // values for these ~1% of QPs; the other 99% run exactly as built)
                flag = NTM_EXIT_OPTIMAL;
                q = nwarm;
#else
                flag = gi_fallback<P, W>(pb, w, rows, nrows, l, nwarm, it, qp_iters, &q, &ns, &yv);
#endif
            }
        }
    }
    if (flag != NTM_EXIT_OPTIMAL) {
        if (l < N) w.U()[l] = (flag == NTM_EXIT_MAXITER) ? w.V()[l] * w.D()[l] : 0.0;
        if (l == 0) cand[N] = -1;
    } else {
        if (l < q) cand[l] = w.act()[l];
        if (l == 0) cand[N] = q;
    }
    NTM_WSYNC();
#ifdef NTM_DEBUG_SCEN
    NTM_TRACE("SET it %d final %d flag %d:", it, flag == NTM_EXIT_OPTIMAL ? q : -1, flag);
    for (int i = 0; flag == NTM_EXIT_OPTIMAL && i < q; ++i) NTM_TRACE(" %d", cand[i]);
    NTM_TRACE("\n");
#endif
    if (q_out) *q_out = q;
    if (ns_out) *ns_out = ns;
    if (y_valid) *y_valid = yv && flag == NTM_EXIT_OPTIMAL;
    return flag;
}

}  // namespace ntm

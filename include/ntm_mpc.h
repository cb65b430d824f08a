/*
 * ntm_mpc.h — C-ABI of the MI355X-native batched LPV-MPC hot path.
 *
 * Drop-in boundary for the receding-horizon loop of the MATLAB reference
 * IsaacSavona/MPC-NTM-Control (NTM_MPC_Sim.m:93-131).  The reference has no
 * FFI of its own: its hot path is a set of MATLAB functions resolved by name
 * (rho1.m, rho2.m, rho3.m, A.m, B.m, Rho_to_PhiGammaLambda.m, getWLc.m and
 * MathWorks quadprog).  Function-handle arguments cannot cross a C ABI, so the
 * boundary sits at the time-step level (one MEX call replaces lines 94-130 for
 * a whole batch of scenarios) plus one entry point per reference function for
 * per-function parity.  See INTEGRATION.md for the MEX / ctypes bindings.
 *
 * Conventions
 *  - fp64 everywhere; all per-scenario matrices are MATLAB column-major.
 *  - Batched arrays are scenario-major: a per-scenario record of E elements
 *    is contiguous, element e of scenario s at [s*E + e].  In MATLAB this is
 *    an E-by-B array with one column per scenario (x0 is 2-by-B, U is N-by-B,
 *    rho is 3N-by-B), and a contiguous range of scenarios (one GPU's shard) is
 *    a contiguous block of memory.  The time histories of ntm_mpc_run are
 *    E-by-k_sim-by-B.  (ABI v2 was scenario-minor, [e*B + s].)
 *    Exception: the optional instrumentation counters (ntm_ctx_set_stats).
 *  - Host-pointer entry points (no suffix) stage through the device and are
 *    synchronous.  *_device entry points take device pointers and a
 *    hipStream_t (as void*), enqueue only, and never synchronise.
 *  - Return value: NTM_OK (0) or a negative NTM_E_* code; the message is in
 *    ntm_last_error(ctx).  Per-scenario solver outcomes are NOT errors: they
 *    are reported in exitflag[] with quadprog's codes (NTM_MPC_Sim.m:98-103).
 *  - Caller owns every array; the library never retains a pointer past the
 *    call.  One call at a time per ntm_ctx.
 */
#ifndef NTM_MPC_H
#define NTM_MPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NTM_MPC_ABI_VERSION 5   /* v5: ntm_config.Ru (input weight); v4: ntm_scenario_gen */
#define NTM_MAX_N 64

/* Physics constants, NTM_MPC_Sim.m:5-22 (same names and units). */
typedef struct {
    double j_BS, w_dep, w_marg, w_sat, tau_r, rs, a, eta_CD, tau_E0, tau_E,
           mu0, Lq, B_pol, m, Cw, tau_A0, tau_w, omega0;
} ntm_physics;

/* Constraint modes. */
enum { NTM_MODE_NONE = 0,   /* unconstrained LQ (BASELINE config 1)       */
       NTM_MODE_BOX = 1,    /* u in [umin, umax] only (config 2)          */
       NTM_MODE_FULL = 2,   /* full getWLc.m polyhedron, m = 6N+4 (cfg 3) */
       NTM_MODE_FULL_DU = 3 }; /* getWLc rows + input-rate rows
                                *   |U_i - U_{i-1}| <= du_max, i = 1..N-1,
                                * m = 8N+2 (BASELINE config 5; an extension
                                * of getWLc.m's row structure, not in the
                                * reference) */

/* Literal-reference switches; 0 = canonical semantics. */
enum { NTM_LITERAL_PHI_RIGHTMUL = 1 << 0,  /* D4  Rho_to_PhiGammaLambda.m:21 */
       NTM_LITERAL_GAMMA_INDEX = 1 << 1,   /* D6  Rho_to_PhiGammaLambda.m:32 */
       NTM_LITERAL_PLANT_NO_C = 1 << 2,    /* D13 NTM_MPC_Sim.m:130          */
       NTM_RHO1_SQUARED = 1 << 3 };        /* D18 rhos.m:18                  */

/* Controller configuration, NTM_MPC_Sim.m:30-60, 80-88. */
typedef struct {
    int32_t N;          /* :30 prediction horizon, 1..NTM_MAX_N            */
    int32_t i_sim;      /* :81 max LPV scheduling iterations               */
    int32_t mode;       /* NTM_MODE_*                                      */
    int32_t flags;      /* NTM_LITERAL_* / NTM_RHO1_SQUARED                */
    double Ts;          /* :31                                             */
    double xmin[2];     /* :44                                             */
    double xmax[2];     /* :45                                             */
    double umin, umax;  /* :49-50                                          */
    double Q[4];        /* :59 state weight, row-major 2x2, symmetric PSD  */
    double r[2];        /* :60 reference state                             */
    double epsilon;     /* :87 convergence threshold on sum|U - Uold|      */
    double du_max;      /* NTM_MODE_FULL_DU only: input-rate bound (W/step) */
    double Ru;          /* input weight R_u >= 0: the cost of
                         * NTM_MPC_Sim.m:71-73,120 becomes G = 2 Gamma' Om Gamma
                         * + 2 Ru I (F unchanged).  The reference has none: 0,
                         * its default, is the reference's cost (ABI v5).  A
                         * non-zero Ru runs on the generic (runtime-N) kernels. */
} ntm_config;

/* Return codes. */
enum { NTM_OK = 0, NTM_E_INVALID = -1, NTM_E_DEVICE = -2, NTM_E_NOMEM = -3,
       NTM_E_UNSUPPORTED = -4 };

/* Per-scenario QP exit flags (quadprog convention, NTM_MPC_Sim.m:98-103). */
enum { NTM_EXIT_OPTIMAL = 1, NTM_EXIT_MAXITER = 0, NTM_EXIT_INFEASIBLE = -2,
       NTM_EXIT_NONFINITE = -7 };

/* Defaults = the reference's hard-coded literals (NTM_MPC_Sim.m:5-88). */
void ntm_physics_default(ntm_physics* p);
void ntm_config_default(ntm_config* c, int32_t N);
int32_t ntm_abi_version(void);

typedef struct ntm_ctx ntm_ctx;
int ntm_ctx_create(ntm_ctx** out, int32_t device);
void ntm_ctx_destroy(ntm_ctx* ctx);
const char* ntm_last_error(const ntm_ctx* ctx);
/* Optional instrumentation: device array of NTM_STATS_ROWS*B int32 (SoA, row
 * k of scenario s at [k*B + s]) that subsequent step/run launches ACCUMULATE
 * into: 0 QP solves, 1 Goldfarb-Idnani iterations, 2 final active rows,
 * 3 general (state) active rows, 4 warm-start candidate verifications,
 * 5 full Goldfarb-Idnani solves.  NULL disables. */
#define NTM_STATS_ROWS 6
int ntm_ctx_set_stats(ntm_ctx* ctx, int32_t* dev_stats);
/* Workspace layout of the N = 20 step/run kernels by batch size: batches of at
 * most max_scenarios run on the all-LDS build (2 waves per SIMD), larger ones on
 * the far-workspace build (4 waves per SIMD, GI factors in a per-scenario HBM
 * block).  Default (and max_scenarios < 0): 8 x the device's compute units, the
 * measured crossover (2048 on an MI355X); 0 = always the far build.  Results of
 * the two builds agree to the parity tolerances, not bit for bit; within one
 * build a scenario's results do not depend on the batch around it. */
int ntm_ctx_set_small_batch(ntm_ctx* ctx, int64_t max_scenarios);
/* Among the all-LDS N = 20 batches, those of at most max_scenarios run with a
 * one-wave-per-SIMD register budget (round 6): default (and < 0) 4 x the compute
 * units (1024 on an MI355X: one wave per SIMD), 0 = never.  Bit-identical
 * results to the two-wave budget; only the speed differs. */
int ntm_ctx_set_one_wave_batch(ntm_ctx* ctx, int64_t max_scenarios);
/* The build a step/run launch of B scenarios with cfg takes on this context:
 * *build = 0 far workspace, 1 all-LDS, 2 all-LDS with the one-wave budget. */
int ntm_ctx_step_build(const ntm_ctx* ctx, const ntm_config* cfg, int64_t B, int32_t* build);
/* Which build a step/run launch of B scenarios at horizon N takes on this
 * context: *far = 1 for the far-workspace build, 0 for an all-LDS one. */
int ntm_ctx_step_layout(const ntm_ctx* ctx, int32_t N, int64_t B, int32_t* far);
/* The same for a full config, as the step/run launch of B scenarios would take it
 * (flags included: the literal D4/D6 switches run on the generic kernels) and
 * the launch shape of that kernel: lanes per scenario and the compile-time
 * horizon (0 = generic).  ntm_ctx_step_layout is this with the default config. */
int ntm_ctx_step_layout_cfg(const ntm_ctx* ctx, const ntm_config* cfg, int64_t B, int32_t* far, int32_t* lanes,
                            int32_t* horizon_template);
/* Diagnostic builds only: per-phase s_memtime cycle totals and counters (104 entries);
 * NTM_E_UNSUPPORTED in production builds. */
int ntm_debug_stamps(unsigned long long* out32, int reset);
/* Launch shape the step/run kernels use for horizon N: lanes per scenario
 * (16/32/64) and the compile-time horizon of the specialisation (0 = generic). */
int ntm_step_launch_info(int32_t N, int32_t* lanes, int32_t* horizon_template);

/* ---- time-step level: the drop-in for NTM_MPC_Sim.m:94-130 ------------ */
/* Initial LPV state for x0[2]: rho[3N] = repmat(rho(x0), 1, N)
 * (NTM_MPC_Sim.m:63-65) and U_old[N] = +Inf (the first convergence test never
 * passes, D14; the literal Uold = ones(...) at :86 is an implicit-expansion
 * defect). */
int ntm_mpc_init(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                 int64_t B, const double* x0, double* rho, double* U_old);
int ntm_mpc_init_device(ntm_ctx* ctx, const ntm_physics* phys,
                        const ntm_config* cfg, int64_t B, const double* x0,
                        double* rho, double* U_old, void* stream);
/* One MPC step for B scenarios.  In/out state per scenario:
 *   x_k[2], rho[3N] (3xN col-major: rows rho1,rho2,rho3; carried unshifted,
 *   D20), U_old[N] (persists across steps, D14; +inf on the first step).
 * Outputs: U[N] (last QP solve), x_pred[2(N+1)] (2x(N+1) rollout x_0..x_N),
 *   x_next[2] (plant step :130), exitflag (last QP), inner_iters (QP solves). */
int ntm_mpc_step(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                 int64_t B, const double* x_k, double* rho, double* U_old,
                 double* U, double* x_pred, double* x_next,
                 int32_t* exitflag, int32_t* inner_iters);
int ntm_mpc_step_device(ntm_ctx* ctx, const ntm_physics* phys,
                        const ntm_config* cfg, int64_t B, const double* x_k,
                        double* rho, double* U_old, double* U, double* x_pred,
                        double* x_next, int32_t* exitflag, int32_t* inner_iters,
                        void* stream);

/* Same, with an optional warm-start workspace carried from step to step:
 * active_ws[2(N+1)] int32 per scenario (in/out; initialise every entry to -1;
 * NULL = none) holds the active sets of the previous step's last two QPs.
 * They are tried first and taken only when the exact re-solve passes the KKT
 * certificate, so the result is the QP optimum either way;
 * entries that are not a valid active set are ignored.  ntm_mpc_run keeps
 * this state on chip by itself. */
int ntm_mpc_step_ws(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                    int64_t B, const double* x_k, double* rho, double* U_old,
                    double* U, double* x_pred, double* x_next,
                    int32_t* exitflag, int32_t* inner_iters, int32_t* active_ws);
int ntm_mpc_step_ws_device(ntm_ctx* ctx, const ntm_physics* phys,
                           const ntm_config* cfg, int64_t B, const double* x_k,
                           double* rho, double* U_old, double* U, double* x_pred,
                           double* x_next, int32_t* exitflag, int32_t* inner_iters,
                           int32_t* active_ws, void* stream);

/* Closed loop NTM_MPC_Sim.m:80-131 over k_sim steps, device-resident.
 * Per scenario: x0[2]; outputs xk[2(k_sim+1)] (2x(k_sim+1)), uk[k_sim],
 * Uk[N k_sim] (N x k_sim), wpred[(N+1) k_sim] ((N+1) x k_sim, predicted island
 * width per step), exitflag[k_sim], inner_iters[k_sim].  Any output pointer
 * may be NULL. */
int ntm_mpc_run(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                int64_t B, int32_t k_sim, const double* x0, double* xk,
                double* uk, double* Uk, double* wpred, int32_t* exitflag,
                int32_t* inner_iters);
int ntm_mpc_run_device(ntm_ctx* ctx, const ntm_physics* phys,
                       const ntm_config* cfg, int64_t B, int32_t k_sim,
                       const double* x0, double* xk, double* uk, double* Uk,
                       double* wpred, int32_t* exitflag, int32_t* inner_iters,
                       void* stream);

/* ---- function level: one entry per reference function (device ptrs) --- */
/* rho1.m / rho2.m / rho3.m at x[2] -> rho[3]. */
int ntm_rho_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                   int64_t B, const double* x, double* rho, void* stream);
/* A.m / B.m at rho[3] -> A[4] (2x2 col-major), Bv[2] (2x1 column, D5). */
int ntm_AB_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                  int64_t B, const double* rho, double* A, double* Bv,
                  void* stream);
/* Rho_to_PhiGammaLambda.m: rho[3N] -> Phi[2N*2], Gamma[2N*N], Lambda[2N]. */
int ntm_lift_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                    int64_t B, const double* rho, double* Phi, double* Gamma,
                    double* Lambda, void* stream);
/* NTM_MPC_Sim.m:120-121: (rho, x_k) -> G[N*N], F[N]. */
int ntm_cost_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg,
                    int64_t B, const double* rho, const double* x_k, double* G,
                    double* F, void* stream);
/* getWLc.m: rho -> W[m*2], L[m*N], c[m], m = 6N+4. */
int ntm_getwlc_device(ntm_ctx* ctx, const ntm_physics* phys,
                      const ntm_config* cfg, int64_t B, const double* rho,
                      double* W, double* L, double* c, void* stream);
/* quadprog stand-in (NTM_MPC_Sim.m:97): min 1/2 U'GU + F'U s.t. Lin U <= b,
 * G[N*N], F[N], Lin[m*N], b[m] per scenario -> U[N], exitflag. */
int ntm_qp_device(ntm_ctx* ctx, int64_t B, int32_t N, int32_t m,
                  const double* G, const double* F, const double* Lin,
                  const double* b, double* U, int32_t* exitflag,
                  int32_t* iters, void* stream);

/* Mixed precision (BASELINE config 5's "fp32 vs fp64" leg; NOT the fp64 product
 * path): the same QP as ntm_qp_device solved by Goldfarb-Idnani entirely in
 * fp32 on fp32-rounded data -> U32[N] (widened), then that active set re-solved
 * exactly in fp64 with the KKT certificate -> U[N]; if it does not certify, the
 * fp64 solve takes over.  info: bit 0 the fp32 active set certified, bit 1 fp64
 * fallback, bit 2 the fp32 solve itself was not optimal.  iters32: fp32 GI
 * iterations.  N <= 64, m <= 8N+4 rows within the 160 KiB LDS of one CU. */
int ntm_qp_mixed_device(ntm_ctx* ctx, int64_t B, int32_t N, int32_t m,
                        const double* G, const double* F, const double* Lin,
                        const double* b, double* U, double* U32, int32_t* exitflag,
                        int32_t* info, int32_t* iters32, void* stream);

/* Synthetic scenarios, counter-based and shard-invariant:
 * x0 for global scenario ids first_id .. first_id+B-1 (host array, 2 per scenario). */
void ntm_scenarios_x0(uint64_t seed, int64_t first_id, int64_t B, double* x0);

/* ---- scenario generator: plasma scenarios and disturbance realisations --- */
/* North_star's "independent plasma scenarios / disturbance realisations"
 * (SURVEY.md §8d): per-scenario plasma parameters j_BS and w_dep (NTM_MPC_Sim.m:5-6,
 * which enter C at :37, B.m:2 and rho3.m:2) and an additive disturbance on the
 * plant step (NTM_MPC_Sim.m:130).  The controller's model is the scenario's own
 * plasma (plant = model, D13); the disturbance is the plant's alone.
 * Counter-based: every value is a function of (seed, global scenario id, time
 * index) only, so any sharding or batching reproduces the same realisations.
 *   u(seed, id, k, ch) = splitmix64^3 chain >> 11, times 2^-53 (uniform [0,1));
 *   n(seed, id, k, c)  = (sum of u at ch = 4c..4c+3 - 2) * sqrt(3): unit variance,
 *                        zero mean, bounded at +-2 sqrt(3) (Irwin-Hall; + and *
 *                        only, so host, device and oracles agree bit for bit);
 *   scenario id: j_BS * (1 + jbs_spread (2 u(id, 0xFFFFFFFF, 0) - 1)),
 *                w_dep * (1 + wdep_spread (2 u(id, 0xFFFFFFFF, 1) - 1));
 *   plant step k: x_{k+1} += [sigma_w n(id, k, 0); sigma_omega n(id, k, 1)]. */
typedef struct {
    uint64_t seed;
    int64_t first_id;    /* global id of the batch's scenario 0 (a shard's offset)   */
    int32_t k0;          /* time index of the next launch's first plant step: the one
                            plant step of ntm_mpc_step*, k0 .. k0+k_sim-1 in ntm_mpc_run* */
    int32_t reserved;    /* must be 0                                                */
    double sigma_w;      /* additive w disturbance per plant step [m], >= 0          */
    double sigma_omega;  /* additive omega disturbance per plant step [rad/s], >= 0  */
    double jbs_spread;   /* relative j_BS spread over scenarios, in [0, 1)           */
    double wdep_spread;  /* relative w_dep spread over scenarios, in [0, 1)          */
} ntm_scenario_gen;
/* Attach a generator to the context (copied): subsequent ntm_mpc_init*,
 * ntm_mpc_step* and ntm_mpc_run* launches use it.  NULL restores the nominal,
 * disturbance-free plant (the reference's own deterministic loop).  The
 * function-level entry points (rho, A/B, lift, cost, getWLc, QP) stay nominal. */
int ntm_ctx_set_scenarios(ntm_ctx* ctx, const ntm_scenario_gen* gen);
/* Host-side samples of the same generator (no GPU): per scenario
 * first_id .. first_id+B-1, out4[4s..4s+3] = (j_BS factor, w_dep factor,
 * n(id, k, 0), n(id, k, 1)). */
void ntm_scenario_sample(const ntm_scenario_gen* gen, int64_t B, int32_t k, double* out4);

#ifdef __cplusplus
}
#endif
#endif /* NTM_MPC_H */

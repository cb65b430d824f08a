// ntm_kernels.hip — HIP kernels (gfx950) and the C-ABI of include/ntm_mpc.h.
//
// Hot path: k_mpc_step / k_mpc_run — one fused launch per MPC time step (or
// per closed loop) for the whole scenario batch.  Each group of P lanes runs
// the complete NTM_MPC_Sim.m:94-130 body for one scenario out of LDS:
// lift -> cost -> Jacobi scaling -> Goldfarb-Idnani QP -> rollout / rho update
// -> convergence test, i_sim times, then the plant step.  Nothing but the
// per-scenario state (x_k, rho, U_old) and the outputs touches HBM.
//
// The remaining kernels are the function-level entry points (one per MATLAB
// function) used by the per-function parity tests; they reuse the very same
// device phases.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "ntm_device.h"
#include "ntm_mixed.h"
#include "ntm_step.h"

using namespace ntm;

#ifdef NTM_STAMPS
__device__ unsigned long long ntm::ntm_stamps[NTM_NSTAMPS];
#endif

namespace {

// ---------------------------------------------------------------- building blocks
__global__ void k_rho(Prob pb, int64_t B, const double* x, double* rho) {
    int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    double r1, r2, r3;
    rho_eval(pb.k, x[2 * s], x[2 * s + 1], r1, r2, r3);
    rho[3 * s] = r1;
    rho[3 * s + 1] = r2;
    rho[3 * s + 2] = r3;
}

// initial LPV state: Rho = repmat(rho(x0), 1, N) (NTM_MPC_Sim.m:63-65), Uold = +Inf (D14)
__global__ void k_init_state(Prob pb, int64_t B, const double* x, double* rho, double* U_old) {
    int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    Prob pbs = pb;                                     // scenario's w_dep (rho3.m:2)
    if (pb.g.phys_on) gen_apply_physics(pbs, pb.g.first_id + s);
    double r1, r2, r3;
    rho_eval(pbs.k, x[2 * s], x[2 * s + 1], r1, r2, r3);
    double* rs = rho + s * (3 * pb.N);
    for (int i = 0; i < pb.N; ++i) {
        rs[3 * i] = r1;
        rs[3 * i + 1] = r2;
        rs[3 * i + 2] = r3;
        U_old[s * pb.N + i] = __builtin_inf();
    }
}

__global__ void k_AB(Prob pb, int64_t B, const double* rho, double* A, double* Bv) {
    int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    double a11 = coef_a11(pb.k, rho[3 * s]), a21 = coef_a21(pb.k, rho[3 * s + 1]), b = coef_b(pb.k, rho[3 * s + 2]);
    A[4 * s] = a11;
    A[4 * s + 1] = a21;
    A[4 * s + 2] = 0.0;
    A[4 * s + 3] = pb.k.a22;
    Bv[2 * s] = b;
    Bv[2 * s + 1] = 0.0;
}

template <int P, int NN>
__global__ __launch_bounds__(64) void k_lift(Prob pb, int64_t B, const double* rho, double* Phi, double* Gam,
                                             double* Lam) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int G = 64 / P;
    const int g = threadIdx.x / P, l = threadIdx.x % P;
    const int64_t s = (int64_t)blockIdx.x * G + g;
    const int N = pb.N, R = 2 * N;
    if (s >= B) return;
    auto w = ws_carve<NN>(smem + g * ws_bytes(N), N);
    for (int e = l; e < 3 * N; e += P) w.rho()[e] = rho[s * (3 * N) + e];
    NTM_WSYNC();
    lift_phase<P>(pb, w, l);
    double* Phs = Phi + s * (4 * N);
    double* Las = Lam + s * R;
    for (int i = l; i < N; i += P) {
        const double* Ph = w.Phi() + 4 * i;
        Phs[2 * i] = Ph[0];
        Phs[2 * i + 1] = Ph[1];
        Phs[R + 2 * i] = Ph[2];
        Phs[R + 2 * i + 1] = Ph[3];
        Las[2 * i] = w.Lam()[2 * i];
        Las[2 * i + 1] = w.Lam()[2 * i + 1];
    }
    double* Gs = Gam + s * (R * N);
    for (int e = l; e < R * N; e += P) {
        int r = e % R, j = e / R;
        Gs[e] = (r >= 2 * j) ? w.gt(r, j) : 0.0;
    }
}

template <int P, int NN>
__global__ __launch_bounds__(64) void k_cost(Prob pb, int64_t B, const double* rho, const double* x,
                                             double* G_out, double* F_out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int G = 64 / P;
    const int g = threadIdx.x / P, l = threadIdx.x % P;
    const int64_t s = (int64_t)blockIdx.x * G + g;
    const int N = NN > 0 ? NN : pb.N;
    if (s >= B) return;
    auto w = ws_carve<NN>(smem + g * ws_bytes(N), N);
    for (int e = l; e < 3 * N; e += P) w.rho()[e] = rho[s * (3 * N) + e];
    NTM_WSYNC();
    lift_phase<P>(pb, w, l);
    free_response<P>(w, x[2 * s], x[2 * s + 1], l);
    cost_phase<P>(pb, w, l);
    if (l < N) {
        double* Gs = G_out + s * (N * N);
        for (int kk = 0; kk <= l; ++kk) {
            double v = w.R()[l + kk * w.ldj()];
            Gs[l + kk * N] = v;
            Gs[kk + l * N] = v;
        }
        F_out[s * N + l] = w.F()[l];
    }
}

// getWLc.m:9-59 materialised (for parity only; the hot path never builds it)
template <int P, int NN>
__global__ __launch_bounds__(64) void k_getwlc(Prob pb, int64_t B, const double* rho, double* W, double* L,
                                               double* c) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int G = 64 / P;
    const int g = threadIdx.x / P, l = threadIdx.x % P;
    const int64_t s = (int64_t)blockIdx.x * G + g;
    const int N = pb.N, m = 6 * N + 4;
    if (s >= B) return;
    auto w = ws_carve<NN>(smem + g * ws_bytes(N), N);
    for (int e = l; e < 3 * N; e += P) w.rho()[e] = rho[s * (3 * N) + e];
    NTM_WSYNC();
    lift_phase<P>(pb, w, l);
    L += s * ((int64_t)m * N);
    W += s * (2 * m);
    c += s * m;
    for (int row = l; row < m; row += P) {
        int blk = row / 6, rr = row - 6 * blk;
        double Wr0 = 0.0, Wr1 = 0.0, cr = 0.0;
        for (int j = 0; j < N; ++j) L[row + j * m] = 0.0;
        bool urow = blk < N && rr < 2;
        if (urow) {
            L[row + blk * m] = (rr == 0) ? -1.0 : 1.0;
            cr = (rr == 0) ? -pb.umin : pb.umax;
        } else {
            int i, cc;
            bool upper;
            if (blk < N) { i = blk; cc = (rr - 2) & 1; upper = rr >= 4; }
            else { i = N; cc = rr & 1; upper = rr >= 2; }
            double sg = upper ? 1.0 : -1.0;
            cr = upper ? pb.xmax[cc] : -pb.xmin[cc];
            if (i == 0) {                     // Dcal rows: W = -Mi
                if (cc == 0) Wr0 = -sg; else Wr1 = -sg;
            } else {
                int r = 2 * (i - 1) + cc;
                for (int j = 0; j < N; ++j) L[row + j * m] = sg * ((r >= 2 * j) ? w.gt(r, j) : 0.0);
                Wr0 = -sg * w.Phi()[4 * (i - 1) + cc];
                Wr1 = -sg * w.Phi()[4 * (i - 1) + 2 + cc];
                cr -= sg * w.Lam()[r];
            }
        }
        W[row] = Wr0;
        W[m + row] = Wr1;
        c[row] = cr;
    }
}

// quadprog stand-in on explicit data (dense rows)
template <int P, int NN>
__global__ __launch_bounds__(64) void k_qp(int64_t B, int N, int m, const double* G_in, const double* F_in,
                                           const double* Lin, const double* b, double* U, int32_t* exitflag,
                                           int32_t* iters) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int G = 64 / P;
    const int g = threadIdx.x / P, l = threadIdx.x % P;
    const int64_t s = (int64_t)blockIdx.x * G + g;
    if (s >= B) return;
    const int wsm = ws_bytes_rows(N, m);        // active-row flags sized for all m rows
    const int wsb = wsm + ((m * 8 + 15) & ~15) + N * ldj_of(N) * 8;
    char* base = smem + g * wsb;
    auto w = ws_carve<NN>(base, N);
    double* rnrm = reinterpret_cast<double*>(base + wsm);
    double* gsave = rnrm + ((m + 1) & ~1);     // copy of G~ for the polish (N x LDJ)
    if (l < N) {
        for (int kk = 0; kk <= l; ++kk) w.R()[l + kk * w.ldj()] = G_in[s * (N * N) + l + kk * N];
        w.F()[l] = F_in[s * N + l];
    }
    for (int i = l; i < m; i += P) w.aflag()[i] = 0;
    NTM_WSYNC();
    int flag, its = 0, q = 0;
    DenseRows rows{Lin, b, rnrm, (int64_t)N, s, m};
    if (!scale_phase<P>(w, l, false)) {
        flag = NTM_EXIT_NONFINITE;
    } else {
        int code = rows.template prepare_code<P>(w, l);
        if (code & 1) flag = NTM_EXIT_NONFINITE;
        else if (code & 2) flag = NTM_EXIT_INFEASIBLE;
        else {
            // keep G~ for the polish (w.Gt() is unused without a lifted model)
            if (l < N) for (int j = 0; j <= l; ++j) gsave[l + j * w.ldj()] = w.R()[l + j * w.ldj()];
            NTM_WSYNC();
            flag = gi_solve<P, DenseRows, decltype(w)>(w, rows, m > 0, m, l, &its, &q);
        }
    }
    if (flag == NTM_EXIT_OPTIMAL) {
        (void)polish_phase<P, DenseRows, decltype(w)>(Prob{}, w, &rows, q, l, gsave, false, false, nullptr);
    } else if (l < N) {
        w.U()[l] = (flag == NTM_EXIT_MAXITER) ? w.V()[l] * w.D()[l] : 0.0;
    }
    NTM_WSYNC();
    if (l < N) U[s * N + l] = w.U()[l];
    if (l == 0) {
        exitflag[s] = flag;
        if (iters) iters[s] = its;
    }
}

// Mixed precision (BASELINE config 5's fp32 leg; not the fp64 product path):
// the QP solved by Goldfarb-Idnani in fp32 on fp32-rounded data (ntm_mixed.h),
// then its active set re-solved exactly in fp64 and KKT-certified (the fp64
// path's polish); when the fp32 set does not certify, the fp64 GI solves it.
// info bits: 1 = the fp32 active set certified in fp64, 2 = fp64 GI fallback,
// 4 = the fp32 solve itself ended non-optimal.
template <int P>
__global__ __launch_bounds__(64) void k_qp_mixed(int64_t B, int N, int m, const double* G_in, const double* F_in,
                                                 const double* Lin, const double* b, double* U, double* U32,
                                                 int32_t* exitflag, int32_t* info, int32_t* iters32) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int l = threadIdx.x;
    const int64_t s = blockIdx.x;
    if (s >= B) return;
    const int wsm = ws_bytes_rows(N, m);
    char* base = smem;
    auto w = ws_carve<0>(base, N);
    double* rnrm = reinterpret_cast<double*>(base + wsm);
    double* gsave = rnrm + ((m + 1) & ~1);
    char* b32 = reinterpret_cast<char*>(gsave + N * ldj_of(N));
    GI32 g;
    g.carve(b32, N, m);
    // ---- fp32 stage
    int q32 = 0, it32 = 0;
    const Dense32 r32{Lin, b, s, N, m};
    const int f32 = gi32_solve<P>(g, G_in, F_in, r32, s, l, &q32, &it32);
    // ---- fp64 data (as k_qp)
    if (l < N) {
        for (int kk = 0; kk <= l; ++kk) w.R()[l + kk * w.ldj()] = G_in[s * (N * N) + l + kk * N];
        w.F()[l] = F_in[s * N + l];
    }
    for (int i = l; i < m; i += P) w.aflag()[i] = 0;
    NTM_WSYNC();
    int flag, its = 0, q = 0, inf = (f32 != NTM_EXIT_OPTIMAL) ? 4 : 0;
    DenseRows rows{Lin, b, rnrm, (int64_t)N, s, m};
    if (!scale_phase<P>(w, l, false)) {
        flag = NTM_EXIT_NONFINITE;
    } else {
        const int code = rows.template prepare_code<P>(w, l);
        if (code & 1) flag = NTM_EXIT_NONFINITE;
        else if (code & 2) flag = NTM_EXIT_INFEASIBLE;
        else {
            if (l < N) for (int j = 0; j <= l; ++j) gsave[l + j * w.ldj()] = w.R()[l + j * w.ldj()];
            NTM_WSYNC();
            bool ok = false;
            if (f32 == NTM_EXIT_OPTIMAL) {
                // ---- fp64 refinement on the fp32 active set
                if (l < q32) w.act()[l] = g.act[l];
                if (l < N) w.V()[l] = (double)g.U[l] / w.D()[l];
                NTM_WSYNC();
                ok = polish_phase<P, DenseRows, decltype(w)>(Prob{}, w, &rows, q32, l, gsave, false, false, nullptr);
                NTM_WSYNC();
            }
            if (ok) {
                flag = NTM_EXIT_OPTIMAL;
                inf |= 1;
            } else {
                // ---- fp64 Goldfarb-Idnani fallback (G~ restored from the saved copy)
                inf |= 2;
                if (l < N) for (int j = 0; j <= l; ++j) w.R()[l + j * w.ldj()] = gsave[l + j * w.ldj()];
                for (int i = l; i < m; i += P) w.aflag()[i] = 0;
                NTM_WSYNC();
                flag = gi_solve<P, DenseRows, decltype(w)>(w, rows, m > 0, m, l, &its, &q);
                if (flag == NTM_EXIT_OPTIMAL)
                    (void)polish_phase<P, DenseRows, decltype(w)>(Prob{}, w, &rows, q, l, gsave, false, false,
                                                                  nullptr);
            }
        }
    }
    if (flag != NTM_EXIT_OPTIMAL && l < N) w.U()[l] = (flag == NTM_EXIT_MAXITER) ? w.V()[l] * w.D()[l] : 0.0;
    NTM_WSYNC();
    if (l < N) {
        U[s * N + l] = w.U()[l];
        U32[s * N + l] = (double)g.U[l];
    }
    if (l == 0) {
        exitflag[s] = flag;
        info[s] = inf;
        iters32[s] = it32;
    }
}

// ------------------------------------------------------------------ host helpers
// NTM_MPC_Sim.m:24 (same expression as oracle/ntm_oracle.c orc_coeffs)
double kappa_of(const ntm_physics* p) {
    const double pi = 3.14159265358979323846;
    return 16 * p->mu0 * p->Lq * (p->rs * p->rs) / (0.82 * p->tau_r * p->B_pol * pi);
}

Prob make_prob(const ntm_physics* p, const ntm_config* c) {
    // identical expressions to oracle/ntm_oracle.c orc_coeffs (NTM_MPC_Sim.m:24-25, 37; A.m; B.m)
    double kappa = kappa_of(p);
    double zeta = p->m * p->Cw * (p->tau_A0 * p->tau_A0) * p->tau_w * (p->a * p->a * p->a);
    Prob pb;
    std::memset(&pb, 0, sizeof(pb));
    double Ts = c->Ts;
    pb.k.a11c = (4.0 / 3.0) * (kappa * p->rs / (0.82 * p->tau_r)) * Ts;
    pb.k.za3 = zeta * (p->a * p->a * p->a);
    pb.k.a22 = 1 - Ts / p->tau_E;
    pb.k.bc = (kappa * Ts * p->eta_CD / p->w_dep);
    pb.k.C1 = -4.0 / 3.0 * (kappa * Ts * p->j_BS * p->w_sat) / (p->w_sat * p->w_sat + p->w_marg * p->w_marg);
    pb.k.C2 = Ts * p->omega0 / p->tau_E0;
    pb.k.wmarg2 = p->w_marg * p->w_marg;
    pb.k.wdep = p->w_dep;
    pb.k.Ts = Ts;
    pb.k.rho1_sq = (c->flags & NTM_RHO1_SQUARED) != 0;
    pb.N = c->N;
    pb.i_sim = c->i_sim;
    pb.mode = c->mode;
    pb.flags = c->flags;
    pb.du = c->du_max;
    pb.Ru = c->Ru;
    for (int i = 0; i < 2; ++i) {
        pb.xmin[i] = c->xmin[i];
        pb.xmax[i] = c->xmax[i];
        pb.r[i] = c->r[i];
    }
    pb.umin = c->umin;
    pb.umax = c->umax;
    for (int i = 0; i < 4; ++i) pb.Q[i] = c->Q[i];
    pb.eps = c->epsilon;
    return pb;
}

// a scenario generator into pb.g (the time-step entry points); the pieces of
// C1 (NTM_MPC_Sim.m:37) and of the B.m:2 gain that gen_apply_physics rebuilds
// per scenario, in make_prob's expression order
void attach_gen(const ntm_scenario_gen& g, const ntm_physics* p, const ntm_config* c, Prob& pb) {
    pb.g.seed = g.seed;
    pb.g.first_id = g.first_id;
    pb.g.k0 = g.k0;
    pb.g.sw = g.sigma_w;
    pb.g.so = g.sigma_omega;
    pb.g.dist_on = (g.sigma_w != 0.0 || g.sigma_omega != 0.0) ? 1 : 0;
    pb.g.sj = g.jbs_spread;
    pb.g.sd = g.wdep_spread;
    pb.g.phys_on = (g.jbs_spread != 0.0 || g.wdep_spread != 0.0) ? 1 : 0;
    pb.g.kTs = kappa_of(p) * c->Ts;
    pb.g.wsat = p->w_sat;
    pb.g.den = p->w_sat * p->w_sat + p->w_marg * p->w_marg;
    pb.g.jbs = p->j_BS;
    pb.g.kte = pb.g.kTs * p->eta_CD;
    pb.g.wdep = p->w_dep;
}

int lanes_for(int N) {
    // lanes per scenario: the smallest power of two >= N (NTM_LANES=64 forces one scenario per wave)
    static int forced = [] {
        const char* e = std::getenv("NTM_LANES");
        return e ? std::atoi(e) : 0;
    }();
    // measured on MI355X (N=20): one scenario per wave (P = 64) beats two per wave
    // (P = 32): every group decision becomes wave-uniform (scalar branches)
    int p = N <= 16 ? 16 : 64;
    if (forced == 16 || forced == 32 || forced == 64) p = forced < N ? 64 : forced;
    return p;
}

}  // namespace

// =========================================================================
// C-ABI
// =========================================================================
struct ntm_ctx {
    int device = 0;
    int32_t* stats = nullptr;   // optional device counters (ntm_ctx_set_stats)
    bool gen_on = false;        // scenario generator attached (ntm_ctx_set_scenarios)
    ntm_scenario_gen gen{};
    std::string err;
    void* dbuf = nullptr;
    size_t dbuf_bytes = 0;
    void* fbuf = nullptr;       // far workspaces of the long-horizon kernels (ws_far)
    size_t fbuf_bytes = 0;
    hipEvent_t fbuf_done = nullptr;   // recorded after the last launch that used fbuf
    int cus = 256;                    // compute units of the device (small_batch)
    int64_t near_max = -1;            // ntm_ctx_set_small_batch (< 0: 8 x cus)
    int64_t near1_max = -1;           // ntm_ctx_set_one_wave_batch (< 0: 4 x cus)
    hipStream_t stream = nullptr;
};

namespace {

// Makes ctx->device current for the duration of an entry point and restores the
// caller's device on exit: hipMalloc, hipFuncSetAttribute (the > 64 KiB LDS
// opt-in) and the launches all act on the current device.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(const ntm_ctx* ctx) {
        int cur = -1;
        if (ctx && hipGetDevice(&cur) == hipSuccess && cur != ctx->device && hipSetDevice(ctx->device) == hipSuccess)
            prev = cur;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

int fail(ntm_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int check_hip(ntm_ctx* ctx, hipError_t e, const char* what) {
    if (e == hipSuccess) return NTM_OK;
    return fail(ctx, NTM_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int kKnownFlags =
    NTM_LITERAL_PHI_RIGHTMUL | NTM_LITERAL_GAMMA_INDEX | NTM_LITERAL_PLANT_NO_C | NTM_RHO1_SQUARED;
// D4 / D6 are compiled into the generic (runtime-N) kernels only
constexpr int kGenericOnlyFlags = NTM_LITERAL_PHI_RIGHTMUL | NTM_LITERAL_GAMMA_INDEX;

int validate(ntm_ctx* ctx, const ntm_physics* p, const ntm_config* c, int64_t B) {
    if (!ctx) return NTM_E_INVALID;
    if (!p || !c) return fail(ctx, NTM_E_INVALID, "null physics/config");
    if (c->N < 1 || c->N > NTM_MAX_N) return fail(ctx, NTM_E_INVALID, "N out of range [1, 64]");
    if (c->i_sim < 1) return fail(ctx, NTM_E_INVALID, "i_sim must be >= 1");
    if (c->flags & ~kKnownFlags) return fail(ctx, NTM_E_UNSUPPORTED, "unknown flag bits");
    if (c->mode < NTM_MODE_NONE || c->mode > NTM_MODE_FULL_DU) return fail(ctx, NTM_E_INVALID, "bad mode");
    if (c->mode == NTM_MODE_FULL_DU && !(std::isfinite(c->du_max)))
        return fail(ctx, NTM_E_INVALID, "du_max must be finite");
    if (!(std::isfinite(c->Ru) && c->Ru >= 0.0)) return fail(ctx, NTM_E_INVALID, "Ru must be finite and >= 0");
    if (B < 0) return fail(ctx, NTM_E_INVALID, "negative batch");
    return NTM_OK;
}

template <typename K>
int set_lds(ntm_ctx* ctx, K kern, size_t lds) {
    if (lds > 160 * 1024) return fail(ctx, NTM_E_UNSUPPORTED, "LDS workspace exceeds 160 KiB");
    if (lds > 64 * 1024)
        return check_hip(ctx,
                         hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                         "hipFuncSetAttribute");
    return NTM_OK;
}

// the far workspace (J/R in HBM, far_doubles(N) per scenario) of a kernel whose WS
// keeps it out of LDS; grown on demand, one per context.  Calls return before
// their kernels finish and may come on different streams (a caller's stream, the
// context's own for host buffers), so the block is stream-ordered: a launch that
// uses it waits for the previous one (fbuf_done, recorded by far_release)
template <int NN>
int attach_far(ntm_ctx* ctx, Prob& pb, int64_t B, hipStream_t st) {
    if constexpr (!ws_far(NN)) {
        return NTM_OK;
    } else {
        const size_t bytes = (size_t)B * far_doubles(pb.N) * sizeof(double);
        int rc;
        if (!ctx->fbuf_done &&
            (rc = check_hip(ctx, hipEventCreateWithFlags(&ctx->fbuf_done, hipEventDisableTiming), "hipEventCreate")))
            return rc;
        if (ctx->fbuf_bytes < bytes) {
            // hipFree waits for the device, so no launch still reads the old block
            if (ctx->fbuf) (void)hipFree(ctx->fbuf);
            ctx->fbuf = nullptr;
            ctx->fbuf_bytes = 0;
            rc = check_hip(ctx, hipMalloc(&ctx->fbuf, bytes), "hipMalloc (far workspace)");
            if (rc) return fail(ctx, NTM_E_NOMEM, ctx->err);
            ctx->fbuf_bytes = bytes;
        }
        if ((rc = check_hip(ctx, hipStreamWaitEvent(st, ctx->fbuf_done, 0), "hipStreamWaitEvent"))) return rc;
        pb.far = static_cast<double*>(ctx->fbuf);
        return NTM_OK;
    }
}
template <int NN>
int far_release(ntm_ctx* ctx, int rc, hipStream_t st) {
    if constexpr (ws_far(NN)) {
        if (rc == NTM_OK) rc = check_hip(ctx, hipEventRecord(ctx->fbuf_done, st), "hipEventRecord");
    }
    return rc;
}


// N = 20 batches up to 8 scenarios per CU (one round of the all-LDS 2-wave build,
// which holds 8 per CU at once) run on that build: each of its waves is faster
// than the far build's, whose occupancy such a batch cannot use.  Round 5 (the
// slim far build at 4 waves per SIMD, 16 per CU; steps 6-25, mode 2, ms per
// step-batch, all-LDS / far): B = 2048 0.563 / 0.637, 4096 0.772 / 0.708, 8192
// 1.157 / 0.990, 16384 1.900 / 1.484; BASELINE config 2 (mode 1, B = 1024) 0.279 /
// 0.319.  (Round 3, the far build at 3 waves: up to 32 per CU, B = 8192 1.49 vs 1.51.)
// ntm_ctx_set_small_batch overrides the threshold (0: always the far build).
template <int NN>
bool small_batch(const ntm_ctx* ctx, int64_t B) {
    if constexpr (NN != 20 || !ws_far(NN)) {
        return false;
    } else {
        const int64_t lim = ctx->near_max >= 0 ? ctx->near_max : 8LL * ctx->cus;
        return B <= lim;
    }
}
// Among those, batches of at most 4 per CU (one wave per SIMD) take the one-wave
// register budget of the same build (ntm_n20near1w.hip, bit-identical results)
template <int NN>
bool one_wave_batch(const ntm_ctx* ctx, int64_t B) {
    if (!small_batch<NN>(ctx, B)) return false;
    const int64_t lim = ctx->near1_max >= 0 ? ctx->near1_max : 4LL * ctx->cus;
    return B <= lim;
}

template <int P, int NN>
int launch_step(ntm_ctx* ctx, Prob pb, int64_t B, const double* x_k, double* rho, double* U_old,
                double* U, double* x_pred, double* x_next, int32_t* exitflag, int32_t* inner_iters,
                int32_t* active_ws, hipStream_t st) {
    constexpr int G = 64 / P;
#ifndef NTM_SINGLE_TU
    if constexpr (P == 64 && (NN == 20 || NN == 50)) {   // ntm_n20.hip, ntm_n50.hip
        const bool near = small_batch<NN>(ctx, B);
        size_t lds = (size_t)G * ws_bytes(pb.N, ws_far(NN) && !near);
#ifdef NTM_LDS_PAD
        lds += NTM_LDS_PAD;   // occupancy study only (tools/occupancy_study.sh): fewer scenarios per CU
#endif
        if (lds > 160 * 1024) return fail(ctx, NTM_E_UNSUPPORTED, "LDS workspace exceeds 160 KiB");
        if (!near)
            if (int rc = attach_far<NN>(ctx, pb, B, st)) return rc;
        const hipError_t e =
            NN == 50 ? (pb.mode == NTM_MODE_FULL_DU
                            ? ntm_launch_step_n50m3(pb, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters,
                                                    active_ws, lds, st)
                            : ntm_launch_step_n50(pb, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters,
                                                  active_ws, lds, st))
            : near   ? (one_wave_batch<NN>(ctx, B)
                            ? ntm_launch_step_n20near1w(pb, B, x_k, rho, U_old, U, x_pred, x_next, exitflag,
                                                        inner_iters, active_ws, lds, st)
                            : ntm_launch_step_n20near(pb, B, x_k, rho, U_old, U, x_pred, x_next, exitflag,
                                                      inner_iters, active_ws, lds, st))
                     : ntm_launch_step_n20(pb, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters, active_ws,
                                           lds, st);
        const int rc = check_hip(ctx, e, "k_mpc_step<64,NN> launch");
        return near ? rc : far_release<NN>(ctx, rc, st);
    } else
#endif
    {
    size_t lds = (size_t)G * ws_bytes(pb.N, ws_far(NN));
    if (int rc = attach_far<NN>(ctx, pb, B, st)) return rc;
#ifdef NTM_LDS_PAD
    lds += NTM_LDS_PAD;
#endif
    const bool gen = pb.g.phys_on || pb.g.dist_on;     // the generator's build only when it is used
    if (static_lds<P, NN>()) lds = 0;                  // the workspace is the kernel's static LDS
    int rc = gen ? set_lds(ctx, k_mpc_step<P, NN, true>, lds) : set_lds(ctx, k_mpc_step<P, NN, false>, lds);
    if (rc) return rc;
    int64_t blocks = (B + G - 1) / G;
    if (blocks == 0) return NTM_OK;
    if (gen)
        hipLaunchKernelGGL((k_mpc_step<P, NN, true>), dim3((unsigned)blocks), dim3(64), lds, st, pb, B, x_k, rho,
                           U_old, U, x_pred, x_next, exitflag, inner_iters, active_ws);
    else
        hipLaunchKernelGGL((k_mpc_step<P, NN, false>), dim3((unsigned)blocks), dim3(64), lds, st, pb, B, x_k, rho,
                           U_old, U, x_pred, x_next, exitflag, inner_iters, active_ws);
    return far_release<NN>(ctx, check_hip(ctx, hipGetLastError(), "k_mpc_step launch"), st);
    }
}

template <int P, int NN>
int launch_run(ntm_ctx* ctx, Prob pb, int64_t B, int k_sim, const double* x0, double* xk, double* uk,
               double* Uk, double* wpred, int32_t* exitflag, int32_t* inner_iters, hipStream_t st) {
    constexpr int G = 64 / P;
#ifndef NTM_SINGLE_TU
    if constexpr (P == 64 && (NN == 20 || NN == 50)) {   // ntm_n20.hip, ntm_n50.hip
        const bool near = small_batch<NN>(ctx, B);
        const size_t lds = (size_t)G * ws_bytes(pb.N, ws_far(NN) && !near);
        if (lds > 160 * 1024) return fail(ctx, NTM_E_UNSUPPORTED, "LDS workspace exceeds 160 KiB");
        if (!near)
            if (int rc = attach_far<NN>(ctx, pb, B, st)) return rc;
        const hipError_t e =
            NN == 50 ? (pb.mode == NTM_MODE_FULL_DU
                            ? ntm_launch_run_n50m3(pb, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, lds, st)
                            : ntm_launch_run_n50(pb, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, lds, st))
            : near   ? (one_wave_batch<NN>(ctx, B)
                            ? ntm_launch_run_n20near1w(pb, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, lds,
                                                       st)
                            : ntm_launch_run_n20near(pb, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, lds,
                                                     st))
                     : ntm_launch_run_n20(pb, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, lds, st);
        const int rc = check_hip(ctx, e, "k_mpc_run<64,NN> launch");
        return near ? rc : far_release<NN>(ctx, rc, st);
    } else
#endif
    {
    const size_t lds = static_lds<P, NN>() ? 0 : (size_t)G * ws_bytes(pb.N, ws_far(NN));
    if (int rc = attach_far<NN>(ctx, pb, B, st)) return rc;
    int rc = set_lds(ctx, k_mpc_run<P, NN>, lds);
    if (rc) return rc;
    int64_t blocks = (B + G - 1) / G;
    if (blocks == 0) return NTM_OK;
    hipLaunchKernelGGL((k_mpc_run<P, NN>), dim3((unsigned)blocks), dim3(64), lds, st, pb, B, k_sim, x0, xk, uk, Uk,
                       wpred, exitflag, inner_iters);
    return far_release<NN>(ctx, check_hip(ctx, hipGetLastError(), "k_mpc_run launch"), st);
    }
}

// hot-path dispatch: compile-time horizons for the BASELINE configs (N = 10,
// 20, 50), a runtime-N kernel for every other horizon
bool force_generic() {
    static bool g = std::getenv("NTM_GENERIC") != nullptr;
    return g;
}
// The generic kernels also take N = 20 with input-rate rows (mode 3, an extension
// no BASELINE config runs at N = 20): they compile the one-collision re-solve
// paths (polish_compact kCollision), whose null-space solve stays accurate where
// two general rows end in the same free column.  The bordered elimination the
// N = 20 kernel would take there factors a nearly singular G~_FF (the last inputs
// act almost alike) and sat up to ~1e-8 umax off the exact optimum; compiled into
// the N = 20 kernel the paths cost mode 2 ~1% through register allocation.
// The input weight Ru (ABI v5) is compiled into the generic kernels only (ru_on in
// ntm_device.h), like D4 / D6: the reference's cost has none (Ru = 0).  So is a
// stage weight other than the reference's Q = I (NTM_MPC_Sim.m:59; qi_on): the
// specialised kernels up to NTM_QI_MAXN (N = 10, 20) take the identity for Om; the
// N = 50 kernel keeps a general Om and runs any Q itself.
bool q_is_identity(const ntm_config* c) { return c->Q[0] == 1.0 && c->Q[1] == 0.0 && c->Q[2] == 0.0 && c->Q[3] == 1.0; }
bool use_generic(const ntm_config* c) {
    return force_generic() || (c->flags & kGenericOnlyFlags) != 0 || (c->N == 20 && c->mode == NTM_MODE_FULL_DU) ||
           c->Ru != 0.0 || (c->N <= NTM_QI_MAXN && !q_is_identity(c));
}
#ifdef NTM_RU_ONLY20
// resource-usage check of the N=20 hot kernel alone (make ru20): every horizon
// goes to it; the library built this way is not for use
#define NTM_DISPATCH_P(N, GEN, CALL) CALL(64, 20)
#else
#ifdef NTM_EXP_P32
// experiment: N = 20 with two scenarios per wave on the far layout
#define NTM_N20_CALL(CALL) CALL(32, 20)
#else
#define NTM_N20_CALL(CALL) CALL(64, 20)
#endif
#define NTM_DISPATCH_P(N, GEN, CALL)                                                \
    ((GEN) ? (lanes_for(N) == 16 ? CALL(16, 0) : (lanes_for(N) == 32 ? CALL(32, 0) : CALL(64, 0))) \
    : lanes_for(N) == 16 ? ((N) == 10 ? CALL(16, 10) : CALL(16, 0))                  \
                        : (lanes_for(N) == 32 ? CALL(32, 0)                          \
                                              : ((N) == 20 ? NTM_N20_CALL(CALL)      \
                                                           : ((N) == 50 ? CALL(64, 50) : CALL(64, 0)))))
#endif

struct DevBuf {
    ntm_ctx* ctx;
    char* cur;
    char* end;
};

int ensure_buf(ntm_ctx* ctx, size_t bytes) {
    if (ctx->dbuf_bytes >= bytes) return NTM_OK;
    if (ctx->dbuf) (void)hipFree(ctx->dbuf);
    ctx->dbuf = nullptr;
    ctx->dbuf_bytes = 0;
    int rc = check_hip(ctx, hipMalloc(&ctx->dbuf, bytes), "hipMalloc");
    if (rc) return fail(ctx, NTM_E_NOMEM, ctx->err);
    ctx->dbuf_bytes = bytes;
    return NTM_OK;
}

size_t al(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

void ntm_physics_default(ntm_physics* p) {
    // NTM_MPC_Sim.m:5-22
    p->j_BS = 73e3;
    p->w_dep = 0.024;
    p->w_marg = 0.02;
    p->w_sat = 0.32;
    p->tau_r = 293;
    p->rs = 1.55;
    p->a = 2.0;
    p->eta_CD = 0.9;
    p->tau_E0 = 3.7;
    p->tau_E = p->tau_E0;
    p->mu0 = 4e-7 * 3.14159265358979323846;
    p->Lq = 0.87;
    p->B_pol = 0.97;
    p->m = 2;
    p->Cw = 1;
    p->tau_A0 = 3e-6;
    p->tau_w = 0.188;
    p->omega0 = 2 * 3.14159265358979323846 * 420;
}

void ntm_config_default(ntm_config* c, int32_t N) {
    // NTM_MPC_Sim.m:30-60, 80-88
    const double pi = 3.14159265358979323846;
    std::memset(c, 0, sizeof(*c));
    c->N = N;
    c->i_sim = 10;
    c->mode = NTM_MODE_FULL;
    c->flags = 0;
    c->Ts = 0.1;
    c->xmin[0] = 0.06;
    c->xmin[1] = 100 * 2 * pi;
    c->xmax[0] = 0.15;
    c->xmax[1] = 5000 * 2 * pi;
    c->umin = 0;
    c->umax = 2e6;
    c->Q[0] = 1; c->Q[1] = 0; c->Q[2] = 0; c->Q[3] = 1;
    c->r[0] = 0;
    c->r[1] = 1000 * 2 * pi;
    c->epsilon = 1e-14;
    c->du_max = 5e5;   // config 5 only (not in the reference): a quarter of the input range per step
}

int32_t ntm_abi_version(void) { return NTM_MPC_ABI_VERSION; }

int ntm_ctx_create(ntm_ctx** out, int32_t device) {
    if (!out) return NTM_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return NTM_E_DEVICE;
    if (device < 0 || device >= n) return NTM_E_INVALID;
    ntm_ctx* c = new ntm_ctx();
    c->device = device;
    int rc = NTM_OK;
    {
        // the stream is created on ctx->device; the guard restores the caller's
        // current device on every path out of this block
        DeviceGuard dg(c);
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess || cur != device ||
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
            rc = NTM_E_DEVICE;
        int cus = 0;
        if (rc == NTM_OK && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
            cus > 0)
            c->cus = cus;
    }
    if (rc != NTM_OK) {
        delete c;
        return rc;
    }
    *out = c;
    return NTM_OK;
}

void ntm_ctx_destroy(ntm_ctx* ctx) {
    if (!ctx) return;
    DeviceGuard dg(ctx);
    if (ctx->fbuf) (void)hipFree(ctx->fbuf);
    if (ctx->fbuf_done) (void)hipEventDestroy(ctx->fbuf_done);
    if (ctx->dbuf) (void)hipFree(ctx->dbuf);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* ntm_last_error(const ntm_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// Diagnostic builds (-DNTM_STAMPS) only: copy (and optionally reset) the
// per-phase cycle totals; returns NTM_E_UNSUPPORTED in production builds.
int ntm_debug_stamps(unsigned long long* out32, int reset) {
#ifdef NTM_STAMPS
    if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(ntm::ntm_stamps), NTM_NSTAMPS * sizeof(unsigned long long)) != hipSuccess)
        return NTM_E_DEVICE;
    if (reset) {
        unsigned long long z[NTM_NSTAMPS] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(ntm::ntm_stamps), z, sizeof z) != hipSuccess) return NTM_E_DEVICE;
    }
    return NTM_OK;
#else
    (void)out32;
    (void)reset;
    return NTM_E_UNSUPPORTED;
#endif
}

int ntm_ctx_set_stats(ntm_ctx* ctx, int32_t* dev_stats) {
    if (!ctx) return NTM_E_INVALID;
    ctx->stats = dev_stats;
    return NTM_OK;
}

int ntm_ctx_set_small_batch(ntm_ctx* ctx, int64_t max_scenarios) {
    if (!ctx) return NTM_E_INVALID;
    ctx->near_max = max_scenarios < 0 ? -1 : max_scenarios;
    return NTM_OK;
}

int ntm_ctx_set_one_wave_batch(ntm_ctx* ctx, int64_t max_scenarios) {
    if (!ctx) return NTM_E_INVALID;
    ctx->near1_max = max_scenarios < 0 ? -1 : max_scenarios;
    return NTM_OK;
}

int ntm_ctx_step_build(const ntm_ctx* ctx, const ntm_config* cfg, int64_t B, int32_t* build) {
    if (!build) return NTM_E_INVALID;
    int32_t far = 0, lanes = 0, nn = 0;
    if (int rc = ntm_ctx_step_layout_cfg(ctx, cfg, B, &far, &lanes, &nn)) return rc;
#ifndef NTM_SINGLE_TU
    *build = far ? 0 : ((lanes == 64 && nn == 20 && one_wave_batch<20>(ctx, B)) ? 2 : 1);
#else
    *build = far ? 0 : 1;
#endif
    return NTM_OK;
}

int ntm_ctx_step_layout(const ntm_ctx* ctx, int32_t N, int64_t B, int32_t* far) {
    if (!ctx || !far || N < 1 || N > NTM_MAX_N || B < 0) return NTM_E_INVALID;
    ntm_config c;
    ntm_config_default(&c, N);
    int32_t lanes = 0, nn = 0;
    return ntm_ctx_step_layout_cfg(ctx, &c, B, far, &lanes, &nn);
}

int ntm_ctx_step_layout_cfg(const ntm_ctx* ctx, const ntm_config* cfg, int64_t B, int32_t* far, int32_t* lanes,
                            int32_t* horizon_template) {
    if (!ctx || !cfg || !far || !lanes || !horizon_template || cfg->N < 1 || cfg->N > NTM_MAX_N || B < 0)
        return NTM_E_INVALID;
    // the same decisions launch_step makes: the dispatch (generic kernels for the
    // literal D4/D6 flags), then the N = 20 build by batch size, which only the
    // multi-TU library has (single-TU builds run the ws_far(20) layout throughout)
#define INFO(P_, NN_) (*lanes = (P_), *horizon_template = (NN_), 0)
    (void)NTM_DISPATCH_P(cfg->N, use_generic(cfg), INFO);
#undef INFO
    const bool n20 = *lanes == 64 && *horizon_template == 20;
    const bool n50 = *lanes == 64 && *horizon_template == 50;
#ifndef NTM_SINGLE_TU
    *far = n20 ? (small_batch<20>(ctx, B) ? 0 : (ws_far(20) ? 1 : 0)) : (n50 && ws_far(50) ? 1 : 0);
#else
    *far = n20 ? (ws_far(20) ? 1 : 0) : (n50 && ws_far(50) ? 1 : 0);
#endif
    return NTM_OK;
}

int ntm_ctx_set_scenarios(ntm_ctx* ctx, const ntm_scenario_gen* gen) {
    if (!ctx) return NTM_E_INVALID;
    if (!gen) {
        ctx->gen_on = false;
        return NTM_OK;
    }
    const double v[4] = {gen->sigma_w, gen->sigma_omega, gen->jbs_spread, gen->wdep_spread};
    for (double x : v)
        if (!std::isfinite(x) || x < 0.0) return fail(ctx, NTM_E_INVALID, "generator parameters must be finite and >= 0");
    if (gen->jbs_spread >= 1.0 || gen->wdep_spread >= 1.0)
        return fail(ctx, NTM_E_INVALID, "parameter spreads must be < 1");
    if (gen->reserved != 0) return fail(ctx, NTM_E_INVALID, "reserved must be 0");
    if (gen->k0 < 0) return fail(ctx, NTM_E_INVALID, "negative k0");
    ctx->gen = *gen;
    ctx->gen_on = true;
    return NTM_OK;
}

void ntm_scenario_sample(const ntm_scenario_gen* gen, int64_t B, int32_t k, double* out4) {
    // the device's own generator code (ntm_device.h), compiled for the host
    for (int64_t s = 0; s < B; ++s) {
        const int64_t id = gen->first_id + s;
        out4[4 * s] = gen_factor(gen->seed, id, 0, gen->jbs_spread);
        out4[4 * s + 1] = gen_factor(gen->seed, id, 1, gen->wdep_spread);
        out4[4 * s + 2] = gen_normal(gen->seed, id, (uint32_t)k, 0);
        out4[4 * s + 3] = gen_normal(gen->seed, id, (uint32_t)k, 1);
    }
}

int ntm_mpc_step_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B,
                        const double* x_k, double* rho, double* U_old, double* U, double* x_pred, double* x_next,
                        int32_t* exitflag, int32_t* inner_iters, void* stream) {
    return ntm_mpc_step_ws_device(ctx, phys, cfg, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters,
                                  nullptr, stream);
}

int ntm_mpc_step_ws_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B,
                           const double* x_k, double* rho, double* U_old, double* U, double* x_pred, double* x_next,
                           int32_t* exitflag, int32_t* inner_iters, int32_t* active_ws, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc) return rc;
    if (B == 0) return NTM_OK;
    if (!x_k || !rho || !U_old || !U || !x_pred || !x_next || !exitflag || !inner_iters)
        return fail(ctx, NTM_E_INVALID, "null array");
    Prob pb = make_prob(phys, cfg);
    pb.stats = ctx->stats;
    if (ctx->gen_on) attach_gen(ctx->gen, phys, cfg, pb);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define CALL(P, NN) \
    launch_step<P, NN>(ctx, pb, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters, active_ws, st)
    return NTM_DISPATCH_P(cfg->N, use_generic(cfg), CALL);
#undef CALL
}

int ntm_step_launch_info(int32_t N, int32_t* lanes, int32_t* horizon_template) {
    if (N < 1 || N > NTM_MAX_N || !lanes || !horizon_template) return NTM_E_INVALID;
#define INFO(P_, NN_) (*lanes = (P_), *horizon_template = (NN_), 0)
    return NTM_DISPATCH_P(N, force_generic(), INFO);
#undef INFO
}

int ntm_mpc_step(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* x_k,
                 double* rho, double* U_old, double* U, double* x_pred, double* x_next, int32_t* exitflag,
                 int32_t* inner_iters) {
    return ntm_mpc_step_ws(ctx, phys, cfg, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters, nullptr);
}

int ntm_mpc_step_ws(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* x_k,
                    double* rho, double* U_old, double* U, double* x_pred, double* x_next, int32_t* exitflag,
                    int32_t* inner_iters, int32_t* active_ws) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc) return rc;
    if (B == 0) return NTM_OK;
    if (!x_k || !rho || !U_old || !U || !x_pred || !x_next || !exitflag || !inner_iters)
        return fail(ctx, NTM_E_INVALID, "null array");
    const int N = cfg->N;
    size_t bx = al(2 * B * 8), brho = al(3 * N * B * 8), bu = al(N * B * 8), bxp = al(2 * (N + 1) * B * 8),
           bi = al(B * 4), bws = active_ws ? al(2 * (N + 1) * B * 4) : 0;
    rc = ensure_buf(ctx, bx * 2 + brho + bu * 2 + bxp + bi * 2 + bws);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->dbuf);
    double* dx = (double*)p; p += bx;
    double* drho = (double*)p; p += brho;
    double* duo = (double*)p; p += bu;
    double* dU = (double*)p; p += bu;
    double* dxp = (double*)p; p += bxp;
    double* dxn = (double*)p; p += bx;
    int32_t* dfl = (int32_t*)p; p += bi;
    int32_t* dit = (int32_t*)p; p += bi;
    int32_t* dws = active_ws ? (int32_t*)p : nullptr;
    hipStream_t st = ctx->stream;
    const size_t wsb = 2 * (size_t)(N + 1) * B * 4;
    if ((rc = check_hip(ctx, hipMemcpyAsync(dx, x_k, 2 * B * 8, hipMemcpyHostToDevice, st), "H2D"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(drho, rho, 3 * N * B * 8, hipMemcpyHostToDevice, st), "H2D"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(duo, U_old, N * B * 8, hipMemcpyHostToDevice, st), "H2D"))) return rc;
    if (dws && (rc = check_hip(ctx, hipMemcpyAsync(dws, active_ws, wsb, hipMemcpyHostToDevice, st), "H2D")))
        return rc;
    rc = ntm_mpc_step_ws_device(ctx, phys, cfg, B, dx, drho, duo, dU, dxp, dxn, dfl, dit, dws, st);
    if (rc) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(rho, drho, 3 * N * B * 8, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(U_old, duo, N * B * 8, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(U, dU, N * B * 8, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(x_pred, dxp, 2 * (N + 1) * B * 8, hipMemcpyDeviceToHost, st), "D2H")))
        return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(x_next, dxn, 2 * B * 8, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(exitflag, dfl, B * 4, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(inner_iters, dit, B * 4, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    if (dws && (rc = check_hip(ctx, hipMemcpyAsync(active_ws, dws, wsb, hipMemcpyDeviceToHost, st), "D2H")))
        return rc;
    return check_hip(ctx, hipStreamSynchronize(st), "sync");
}

int ntm_mpc_run_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, int32_t k_sim,
                       const double* x0, double* xk, double* uk, double* Uk, double* wpred, int32_t* exitflag,
                       int32_t* inner_iters, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc) return rc;
    if (k_sim < 0) return fail(ctx, NTM_E_INVALID, "negative k_sim");
    if (B == 0) return NTM_OK;
    if (!x0) return fail(ctx, NTM_E_INVALID, "null x0");
    Prob pb = make_prob(phys, cfg);
    pb.stats = ctx->stats;
    if (ctx->gen_on) attach_gen(ctx->gen, phys, cfg, pb);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define CALL(P, NN) launch_run<P, NN>(ctx, pb, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, st)
    return NTM_DISPATCH_P(cfg->N, use_generic(cfg), CALL);
#undef CALL
}

int ntm_mpc_run(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, int32_t k_sim,
                const double* x0, double* xk, double* uk, double* Uk, double* wpred, int32_t* exitflag,
                int32_t* inner_iters) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc) return rc;
    if (k_sim < 0) return fail(ctx, NTM_E_INVALID, "negative k_sim");
    if (B == 0) return NTM_OK;
    const int N = cfg->N;
    size_t b0 = al(2 * B * 8), bxk = al(2 * (size_t)(k_sim + 1) * B * 8), buk = al((size_t)k_sim * B * 8),
           bUk = al((size_t)N * k_sim * B * 8), bwp = al((size_t)(N + 1) * k_sim * B * 8),
           bi = al((size_t)k_sim * B * 4);
    rc = ensure_buf(ctx, b0 + bxk + buk + bUk + bwp + 2 * bi);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->dbuf);
    double* d0 = (double*)p; p += b0;
    double* dxk = (double*)p; p += bxk;
    double* duk = (double*)p; p += buk;
    double* dUk = (double*)p; p += bUk;
    double* dwp = (double*)p; p += bwp;
    int32_t* dfl = (int32_t*)p; p += bi;
    int32_t* dit = (int32_t*)p;
    hipStream_t st = ctx->stream;
    if ((rc = check_hip(ctx, hipMemcpyAsync(d0, x0, 2 * B * 8, hipMemcpyHostToDevice, st), "H2D"))) return rc;
    rc = ntm_mpc_run_device(ctx, phys, cfg, B, k_sim, d0, xk ? dxk : nullptr, uk ? duk : nullptr,
                            Uk ? dUk : nullptr, wpred ? dwp : nullptr, exitflag ? dfl : nullptr,
                            inner_iters ? dit : nullptr, st);
    if (rc) return rc;
    struct { void* h; void* d; size_t n; } outs[] = {
        {xk, dxk, 2 * (size_t)(k_sim + 1) * B * 8}, {uk, duk, (size_t)k_sim * B * 8},
        {Uk, dUk, (size_t)N * k_sim * B * 8},        {wpred, dwp, (size_t)(N + 1) * k_sim * B * 8},
        {exitflag, dfl, (size_t)k_sim * B * 4},      {inner_iters, dit, (size_t)k_sim * B * 4}};
    for (auto& o : outs)
        if (o.h && (rc = check_hip(ctx, hipMemcpyAsync(o.h, o.d, o.n, hipMemcpyDeviceToHost, st), "D2H")))
            return rc;
    return check_hip(ctx, hipStreamSynchronize(st), "sync");
}

int ntm_rho_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* x,
                   double* rho, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc || B == 0) return rc;
    Prob pb = make_prob(phys, cfg);
    hipLaunchKernelGGL(k_rho, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, pb, B, x, rho);
    return check_hip(ctx, hipGetLastError(), "k_rho");
}

int ntm_mpc_init_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* x0,
                        double* rho, double* U_old, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc || B == 0) return rc;
    if (!x0 || !rho || !U_old) return fail(ctx, NTM_E_INVALID, "null array");
    Prob pb = make_prob(phys, cfg);
    if (ctx->gen_on) attach_gen(ctx->gen, phys, cfg, pb);
    hipLaunchKernelGGL(k_init_state, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, pb, B,
                       x0, rho, U_old);
    return check_hip(ctx, hipGetLastError(), "k_init_state");
}

int ntm_mpc_init(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* x0,
                 double* rho, double* U_old) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc || B == 0) return rc;
    if (!x0 || !rho || !U_old) return fail(ctx, NTM_E_INVALID, "null array");
    const int N = cfg->N;
    size_t bx = al(2 * B * 8), brho = al(3 * N * B * 8), bu = al(N * B * 8);
    if ((rc = ensure_buf(ctx, bx + brho + bu))) return rc;
    char* p = static_cast<char*>(ctx->dbuf);
    double* dx = (double*)p; p += bx;
    double* drho = (double*)p; p += brho;
    double* duo = (double*)p;
    hipStream_t st = ctx->stream;
    if ((rc = check_hip(ctx, hipMemcpyAsync(dx, x0, 2 * B * 8, hipMemcpyHostToDevice, st), "H2D"))) return rc;
    if ((rc = ntm_mpc_init_device(ctx, phys, cfg, B, dx, drho, duo, st))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(rho, drho, 3 * N * B * 8, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    if ((rc = check_hip(ctx, hipMemcpyAsync(U_old, duo, N * B * 8, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
    return check_hip(ctx, hipStreamSynchronize(st), "sync");
}

int ntm_AB_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* rho,
                  double* A, double* Bv, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc || B == 0) return rc;
    Prob pb = make_prob(phys, cfg);
    hipLaunchKernelGGL(k_AB, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, pb, B, rho, A,
                       Bv);
    return check_hip(ctx, hipGetLastError(), "k_AB");
}

#define NTM_GROUP_LAUNCH(KERN, N, B, st, ...)                                                        \
    do {                                                                                            \
        int P_ = lanes_for(N);                                                                      \
        int G_ = 64 / P_;                                                                           \
        size_t lds_ = (size_t)G_ * ws_bytes(N);                                                     \
        unsigned blocks_ = (unsigned)(((B) + G_ - 1) / G_);                                         \
        if (P_ == 16) {                                                                             \
            if ((rc = set_lds(ctx, KERN<16, 0>, lds_))) return rc;                                     \
            hipLaunchKernelGGL((KERN<16, 0>), dim3(blocks_), dim3(64), lds_, st, __VA_ARGS__);           \
        } else if (P_ == 32) {                                                                      \
            if ((rc = set_lds(ctx, KERN<32, 0>, lds_))) return rc;                                     \
            hipLaunchKernelGGL((KERN<32, 0>), dim3(blocks_), dim3(64), lds_, st, __VA_ARGS__);           \
        } else {                                                                                    \
            if ((rc = set_lds(ctx, KERN<64, 0>, lds_))) return rc;                                     \
            hipLaunchKernelGGL((KERN<64, 0>), dim3(blocks_), dim3(64), lds_, st, __VA_ARGS__);           \
        }                                                                                           \
    } while (0)

int ntm_lift_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* rho,
                    double* Phi, double* Gamma, double* Lambda, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc || B == 0) return rc;
    Prob pb = make_prob(phys, cfg);
    NTM_GROUP_LAUNCH(k_lift, cfg->N, B, (hipStream_t)stream, pb, B, rho, Phi, Gamma, Lambda);
    return check_hip(ctx, hipGetLastError(), "k_lift");
}

int ntm_cost_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* rho,
                    const double* x_k, double* G, double* F, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc || B == 0) return rc;
    Prob pb = make_prob(phys, cfg);
    NTM_GROUP_LAUNCH(k_cost, cfg->N, B, (hipStream_t)stream, pb, B, rho, x_k, G, F);
    return check_hip(ctx, hipGetLastError(), "k_cost");
}

int ntm_getwlc_device(ntm_ctx* ctx, const ntm_physics* phys, const ntm_config* cfg, int64_t B, const double* rho,
                      double* W, double* L, double* c, void* stream) {
    DeviceGuard dg(ctx);
    int rc = validate(ctx, phys, cfg, B);
    if (rc || B == 0) return rc;
    Prob pb = make_prob(phys, cfg);
    NTM_GROUP_LAUNCH(k_getwlc, cfg->N, B, (hipStream_t)stream, pb, B, rho, W, L, c);
    return check_hip(ctx, hipGetLastError(), "k_getwlc");
}

int ntm_qp_device(ntm_ctx* ctx, int64_t B, int32_t N, int32_t m, const double* G, const double* F,
                  const double* Lin, const double* b, double* U, int32_t* exitflag, int32_t* iters, void* stream) {
    DeviceGuard dg(ctx);
    if (!ctx) return NTM_E_INVALID;
    if (N < 1 || N > NTM_MAX_N) return fail(ctx, NTM_E_INVALID, "N out of range [1, 64]");
    if (m < 0 || m > 8 * NTM_MAX_N + 4) return fail(ctx, NTM_E_INVALID, "m out of range");
    if (B < 0) return fail(ctx, NTM_E_INVALID, "negative batch");
    if (B == 0) return NTM_OK;
    if (!G || !F || !U || !exitflag) return fail(ctx, NTM_E_INVALID, "null array");
    if (m > 0 && (!Lin || !b)) return fail(ctx, NTM_E_INVALID, "m > 0 needs Lin and b");
    int P = lanes_for(N), Gs = 64 / P;
    size_t per = (size_t)ws_bytes_rows(N, m) + ((m * 8 + 15) & ~15) + (size_t)N * ldj_of(N) * 8;
    size_t lds = Gs * per;
    unsigned blocks = (unsigned)((B + Gs - 1) / Gs);
    hipStream_t st = (hipStream_t)stream;
    int rc;
    if (P == 16) {
        if ((rc = set_lds(ctx, k_qp<16, 0>, lds))) return rc;
        hipLaunchKernelGGL((k_qp<16, 0>), dim3(blocks), dim3(64), lds, st, B, N, m, G, F, Lin, b, U, exitflag, iters);
    } else if (P == 32) {
        if ((rc = set_lds(ctx, k_qp<32, 0>, lds))) return rc;
        hipLaunchKernelGGL((k_qp<32, 0>), dim3(blocks), dim3(64), lds, st, B, N, m, G, F, Lin, b, U, exitflag, iters);
    } else {
        if ((rc = set_lds(ctx, k_qp<64, 0>, lds))) return rc;
        hipLaunchKernelGGL((k_qp<64, 0>), dim3(blocks), dim3(64), lds, st, B, N, m, G, F, Lin, b, U, exitflag, iters);
    }
    return check_hip(ctx, hipGetLastError(), "k_qp");
}

int ntm_qp_mixed_device(ntm_ctx* ctx, int64_t B, int32_t N, int32_t m, const double* G, const double* F,
                        const double* Lin, const double* b, double* U, double* U32, int32_t* exitflag,
                        int32_t* info, int32_t* iters32, void* stream) {
    DeviceGuard dg(ctx);
    if (!ctx) return NTM_E_INVALID;
    if (N < 1 || N > NTM_MAX_N) return fail(ctx, NTM_E_INVALID, "N out of range [1, 64]");
    if (m < 0 || m > 8 * NTM_MAX_N + 4) return fail(ctx, NTM_E_INVALID, "m out of range");
    if (B < 0) return fail(ctx, NTM_E_INVALID, "negative batch");
    if (B == 0) return NTM_OK;
    if (!G || !F || !U || !U32 || !exitflag || !info || !iters32) return fail(ctx, NTM_E_INVALID, "null array");
    if (m > 0 && (!Lin || !b)) return fail(ctx, NTM_E_INVALID, "m > 0 needs Lin and b");
    size_t lds = (size_t)ws_bytes_rows(N, m) + ((m * 8 + 15) & ~15) + (size_t)N * ldj_of(N) * 8 + GI32::bytes(N, m);
    int rc;
    if ((rc = set_lds(ctx, k_qp_mixed<64>, lds))) return rc;
    hipLaunchKernelGGL((k_qp_mixed<64>), dim3((unsigned)B), dim3(64), lds, (hipStream_t)stream, B, N, m, G, F, Lin, b,
                       U, U32, exitflag, info, iters32);
    return check_hip(ctx, hipGetLastError(), "k_qp_mixed");
}

// splitmix64-based counter generator (identical to oracle/ntm_oracle.py scenario_x0)
void ntm_scenarios_x0(uint64_t seed, int64_t first_id, int64_t B, double* x0) {
    const double pi = 3.14159265358979323846;
    for (int64_t k = 0; k < B; ++k) {
        uint64_t sid = (uint64_t)(first_id + k);
        uint64_t base = seed * 0x100000001B3ull + sid * 2;
        double u0 = (double)(splitmix64(base) >> 11) * (1.0 / 9007199254740992.0);
        double u1 = (double)(splitmix64(base + 1) >> 11) * (1.0 / 9007199254740992.0);
        x0[2 * k] = 0.07 + 0.07 * u0;
        x0[2 * k + 1] = (0.8 + 0.4 * u1) * 2000 * pi;
    }
}

}  // extern "C"

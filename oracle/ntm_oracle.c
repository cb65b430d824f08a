/*
 * ntm_oracle.c — C restatement of the CPU oracle.  TEST INFRASTRUCTURE ONLY.
 *
 * The checker, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load liboracle (oracle/libntm_oracle.so).  It is
 * the C twin of oracle/ntm_oracle.py (same CANON semantics, SURVEY.md §2.1,
 * same Goldfarb-Idnani QP) and is itself pinned against the Python oracle by
 * tests/test_oracle_c.py; the Python oracle is pinned by the reference-derived
 * invariants and 50-digit KKT certificates (see its header).  It is also the
 * CPU baseline timed by bench.py ("kind": "port": the reference is MATLAB and
 * cannot run here).  OpenMP parallelism is over independent scenarios.
 *
 * Reference citations (file:line of /root/reference):
 *   rho1.m:2, rho2.m:2, rho3.m:2-3         -> orc_rho
 *   A.m:2, B.m:2, NTM_MPC_Sim.m:24-25,37   -> orc_coeffs / orc_A / orc_B
 *   Rho_to_PhiGammaLambda.m:17-52          -> orc_lift   (CANON D4, D6)
 *   NTM_MPC_Sim.m:67-73,120-121            -> orc_cost   (CANON D8, D12)
 *   getWLc.m:9-59                          -> orc_getwlc (CANON D10)
 *   NTM_MPC_Sim.m:97 (quadprog)            -> orc_qp     (Goldfarb-Idnani)
 *   NTM_MPC_Sim.m:110-117,123-127,130      -> orc_step
 *   NTM_MPC_Sim.m:80-131                   -> ntm_oracle_run
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/ntm_mpc.h"

#define NMAX NTM_MAX_N
#define MMAX (8 * NMAX + 4)   /* getWLc rows + rate rows (NTM_MODE_FULL_DU) */
/* constant-row violation tolerance (D22; oracle/ntm_oracle.py CONST_ROW_TOL) */
#define CONST_ROW_TOL 1e-9

typedef struct {
    double a11c, a21num_den, a22, bc, C1, C2, wmarg2, wdep;
    int rho1_sq;
} orc_coef;

/* NTM_MPC_Sim.m:24-25 (kappa, zeta), A.m:2, B.m:2, :37 (C). */
static void orc_coeffs(const ntm_physics* p, const ntm_config* c, orc_coef* k) {
    const double pi = 3.14159265358979323846;
    double kappa = 16 * p->mu0 * p->Lq * (p->rs * p->rs) / (0.82 * p->tau_r * p->B_pol * pi);
    double zeta = p->m * p->Cw * (p->tau_A0 * p->tau_A0) * p->tau_w * (p->a * p->a * p->a);
    double Ts = c->Ts;
    k->a11c = (4.0 / 3.0) * (kappa * p->rs / (0.82 * p->tau_r)) * Ts;
    k->a21num_den = zeta * (p->a * p->a * p->a);      /* (rho2*Ts)/(zeta*a^3), D19 */
    k->a22 = 1 - Ts / p->tau_E;
    k->bc = (kappa * Ts * p->eta_CD / p->w_dep);
    k->C1 = -4.0 / 3.0 * (kappa * Ts * p->j_BS * p->w_sat) / (p->w_sat * p->w_sat + p->w_marg * p->w_marg);
    k->C2 = Ts * p->omega0 / p->tau_E0;
    k->wmarg2 = p->w_marg * p->w_marg;
    k->wdep = p->w_dep;
    k->rho1_sq = (c->flags & NTM_RHO1_SQUARED) != 0;
}

/* rho1.m:2, rho2.m:2, rho3.m:2-3 */
static void orc_rho(const orc_coef* k, const double* x, double* r) {
    double w = x[0];
    r[0] = 1.0 / ((k->rho1_sq ? w * w : w) + k->wmarg2);
    r[1] = (w * w) / x[1];
    double ws = w / k->wdep;
    r[2] = (0.25 + 0.24 * ws) / (1 + 1.5 * ws + 0.43 * (ws * ws) + 0.64 * (ws * ws * ws));
}

/* A.m:2 -> a11, a21 (a12 = 0, a22 constant) ; B.m:2 -> b (column [b;0], D5) */
static inline double orc_a11(const orc_coef* k, double r1) { return k->a11c * r1 + 1; }
static inline double orc_a21(const orc_coef* k, double r2, double Ts) { return (r2 * Ts) / k->a21num_den; }
static inline double orc_b(const orc_coef* k, double r3) { return k->bc * r3; }

/* ------------------------------------------------------------------ */
/* Scenario generator (include/ntm_mpc.h ntm_scenario_gen): per-scenario */
/* plasma (j_BS, w_dep; NTM_MPC_Sim.m:5-6) and plant disturbances (:130) */
/* ------------------------------------------------------------------ */
static uint64_t o_splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double o_u01(uint64_t seed, int64_t id, uint32_t k, uint32_t ch) {
    uint64_t h = o_splitmix64(seed ^ 0xD1B54A32D192ED03ull);
    h = o_splitmix64(h ^ (uint64_t)id);
    h = o_splitmix64(h ^ (((uint64_t)k << 8) | ch));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}
static double o_normal(uint64_t seed, int64_t id, uint32_t k, uint32_t c) {   /* Irwin-Hall(4), unit variance */
    double s = o_u01(seed, id, k, 4 * c);
    s = s + o_u01(seed, id, k, 4 * c + 1);
    s = s + o_u01(seed, id, k, 4 * c + 2);
    s = s + o_u01(seed, id, k, 4 * c + 3);
    return (s - 2.0) * 1.7320508075688772;
}
static double o_factor(uint64_t seed, int64_t id, uint32_t c, double spread) {
    return fma(spread, 2.0 * o_u01(seed, id, 0xFFFFFFFFu, c) - 1.0, 1.0);   /* one rounding, as the device */
}
/* scenario id's physics: j_BS and w_dep scaled (the rest nominal) */
static void orc_scn_physics(const ntm_physics* p, const ntm_scenario_gen* g, int64_t id, ntm_physics* ps) {
    *ps = *p;
    if (!g) return;
    ps->j_BS = p->j_BS * o_factor(g->seed, id, 0, g->jbs_spread);
    ps->w_dep = p->w_dep * o_factor(g->seed, id, 1, g->wdep_spread);
}
/* additive plant disturbance of scenario id at time index k */
static void orc_disturbance(const ntm_scenario_gen* g, int64_t id, int32_t k, double* d) {
    d[0] = (g && g->sigma_w != 0.0) ? g->sigma_w * o_normal(g->seed, id, (uint32_t)k, 0) : 0.0;
    d[1] = (g && g->sigma_omega != 0.0) ? g->sigma_omega * o_normal(g->seed, id, (uint32_t)k, 1) : 0.0;
}

/* Rho_to_PhiGammaLambda.m:1-54 (CANON D3-D6).  rho: 3xN col-major.
 * Phi 2N x 2, Gamma 2N x N, Lambda 2N, all column-major. */
static void orc_lift(const orc_coef* k, const ntm_config* c, const double* rho,
                     double* Phi, double* Gam, double* Lam) {
    int N = c->N, R = 2 * N;
    double a11[NMAX], a21[NMAX], b[NMAX];
    for (int i = 0; i < N; ++i) {
        a11[i] = orc_a11(k, rho[3 * i]);
        a21[i] = orc_a21(k, rho[3 * i + 1], c->Ts);
        b[i] = orc_b(k, rho[3 * i + 2]);
    }
    double a22 = k->a22;
    /* Phi (:17-23) */
    Phi[0] = a11[0]; Phi[1] = a21[0]; Phi[R + 0] = 0.0; Phi[R + 1] = a22;
    for (int j = 1; j < N; ++j) {
        double p00 = Phi[2 * j - 2], p10 = Phi[2 * j - 1];
        double p01 = Phi[R + 2 * j - 2], p11 = Phi[R + 2 * j - 1];
        if (c->flags & NTM_LITERAL_PHI_RIGHTMUL) {        /* D4 literal: Phi_{j-1} A_j */
            Phi[2 * j] = p00 * a11[j] + p01 * a21[j];
            Phi[R + 2 * j] = p01 * a22;
            Phi[2 * j + 1] = p10 * a11[j] + p11 * a21[j];
            Phi[R + 2 * j + 1] = p11 * a22;
        } else {                                         /* CANON: A_j Phi_{j-1} */
            Phi[2 * j] = a11[j] * p00;
            Phi[R + 2 * j] = a11[j] * p01;
            Phi[2 * j + 1] = a21[j] * p00 + a22 * p10;
            Phi[R + 2 * j + 1] = a21[j] * p01 + a22 * p11;
        }
    }
    /* Gamma (:26-40) */
    memset(Gam, 0, sizeof(double) * (size_t)R * N);
    for (int j = 0; j < N; ++j) {
        Gam[(size_t)j * R + 2 * j] = b[j];
        Gam[(size_t)j * R + 2 * j + 1] = 0.0;
    }
    for (int i = 1; i < N; ++i) {
        for (int j = 0; j < i; ++j) {
            int ai = (c->flags & NTM_LITERAL_GAMMA_INDEX) ? (i - j - 1) : i;   /* D6 */
            double g0 = Gam[(size_t)j * R + 2 * i - 2], g1 = Gam[(size_t)j * R + 2 * i - 1];
            Gam[(size_t)j * R + 2 * i] = a11[ai] * g0;
            Gam[(size_t)j * R + 2 * i + 1] = a21[ai] * g0 + a22 * g1;
        }
    }
    /* Lambda (:47-52) */
    Lam[0] = k->C1; Lam[1] = k->C2;
    for (int i = 1; i < N; ++i) {
        double l0 = Lam[2 * i - 2], l1 = Lam[2 * i - 1];
        Lam[2 * i] = a11[i] * l0 + k->C1;
        Lam[2 * i + 1] = (a21[i] * l0 + a22 * l1) + k->C2;
    }
}

/* NTM_MPC_Sim.m:71-73,120-121: G = 2 Gam' Om Gam (+ 2 Ru I), F = 2 Gam' Om (Phi x + Lam - R). */
static void orc_cost(const ntm_config* c, const double* Phi, const double* Gam,
                     const double* Lam, const double* x, double* G, double* F) {
    int N = c->N, R = 2 * N;
    double q00 = c->Q[0], q01 = c->Q[1], q10 = c->Q[2], q11 = c->Q[3];
    double OG[2 * NMAX * NMAX];  /* Om*Gam (2N x N) */
    for (int j = 0; j < N; ++j)
        for (int i = 0; i < N; ++i) {
            double g0 = Gam[(size_t)j * R + 2 * i], g1 = Gam[(size_t)j * R + 2 * i + 1];
            OG[(size_t)j * R + 2 * i] = q00 * g0 + q01 * g1;
            OG[(size_t)j * R + 2 * i + 1] = q10 * g0 + q11 * g1;
        }
    for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b) {
            double s = 0.0;
            for (int r = 0; r < R; ++r) s += Gam[(size_t)a * R + r] * OG[(size_t)b * R + r];
            G[(size_t)b * N + a] = 2 * s;
        }
    /* input weight (ABI v5): G += 2 Ru I; the reference has Ru = 0 */
    if (c->Ru != 0.0)
        for (int a = 0; a < N; ++a) G[(size_t)a * N + a] = G[(size_t)a * N + a] + 2 * c->Ru;
    double e[2 * NMAX];
    for (int i = 0; i < N; ++i) {
        e[2 * i] = (Phi[2 * i] * x[0] + Phi[R + 2 * i] * x[1]) + Lam[2 * i] - c->r[0];
        e[2 * i + 1] = (Phi[2 * i + 1] * x[0] + Phi[R + 2 * i + 1] * x[1]) + Lam[2 * i + 1] - c->r[1];
    }
    for (int a = 0; a < N; ++a) {
        double s = 0.0;
        for (int i = 0; i < N; ++i) {
            double oe0 = q00 * e[2 * i] + q01 * e[2 * i + 1];
            double oe1 = q10 * e[2 * i] + q11 * e[2 * i + 1];
            s += Gam[(size_t)a * R + 2 * i] * oe0 + Gam[(size_t)a * R + 2 * i + 1] * oe1;
        }
        F[a] = 2 * s;
    }
}

/* getWLc.m:9-59 (D10 fix).  Row order per block i=0..N-1:
 * [-u_i; u_i; -w_i; -om_i; w_i; om_i], terminal [-w_N; -om_N; w_N; om_N].
 * W m x 2, L m x N, c m (column-major). */
static void orc_getwlc(const ntm_config* c, const double* Phi, const double* Gam,
                       const double* Lam, double* W, double* L, double* cv) {
    int N = c->N, R = 2 * N, m = 6 * N + 4;
    memset(W, 0, sizeof(double) * (size_t)m * 2);
    memset(L, 0, sizeof(double) * (size_t)m * N);
    for (int i = 0; i <= N; ++i) {
        int base = 6 * i;
        int xr = base + (i < N ? 2 : 0);   /* first state row of this block */
        if (i < N) {
            L[(size_t)i * m + base] = -1.0;            /* Ecal: -u_i */
            L[(size_t)i * m + base + 1] = 1.0;         /*        u_i */
            cv[base] = -c->umin;
            cv[base + 1] = c->umax;
        }
        cv[xr] = -c->xmin[0]; cv[xr + 1] = -c->xmin[1];
        cv[xr + 2] = c->xmax[0]; cv[xr + 3] = c->xmax[1];
        if (i == 0) {                                   /* Dcal: W = -Mi */
            W[xr] = 1.0; W[m + xr + 1] = 1.0;
            W[xr + 2] = -1.0; W[m + xr + 3] = -1.0;
            continue;
        }
        int sr = 2 * (i - 1);                           /* x_i rows of Phi/Gam/Lam */
        for (int s = 0; s < 2; ++s) {
            double sg = (s == 0) ? -1.0 : 1.0;          /* -x (min) then +x (max) */
            for (int comp = 0; comp < 2; ++comp) {
                int row = xr + 2 * s + comp;
                for (int j = 0; j < N; ++j) L[(size_t)j * m + row] = sg * Gam[(size_t)j * R + sr + comp];
                W[row] = -sg * Phi[sr + comp];
                W[m + row] = -sg * Phi[R + sr + comp];
                cv[row] -= sg * Lam[sr + comp];
            }
        }
    }
}

static double gi_dep_tol = 1e-8;
static int gi_polish = 1;
__attribute__((visibility("default"))) void ntm_oracle_set_polish(int on) { gi_polish = on; }
__attribute__((visibility("default"))) void ntm_oracle_set_dep_tol(double t) { gi_dep_tol = t; }

/* ------------------------------------------------------------------ */
/* Goldfarb-Idnani dual active set: min 1/2 U'GU + F'U  s.t. Lin U <= b. */
/* ------------------------------------------------------------------ */
static void givens(double a, double b, double* cc, double* ss, double* h) {
    double hh = hypot(a, b);
    if (hh == 0.0) { *cc = 1.0; *ss = 0.0; *h = 0.0; return; }
    *cc = a / hh; *ss = b / hh; *h = hh;
}

static int orc_gi(int n, int m, const double* G, const double* F, const double* Lin,
                  const double* b, double* U, int* iters_out, int* act_out, int* q_out) {
    double J[NMAX * NMAX], Rm[NMAX * NMAX], Lc[NMAX * NMAX];
    double up[NMAX + 1], d[NMAX], z[NMAX], r[NMAX];
    static const int max_extra = 50;
    int act[NMAX + 1];
    int q = 0, it = 0, max_iter = 10 * (n + m) + max_extra;
    *iters_out = 0;
    for (int i = 0; i < n; ++i) U[i] = 0.0;
    for (int i = 0; i < n * n; ++i) if (!isfinite(G[i])) return NTM_EXIT_NONFINITE;
    for (int i = 0; i < n; ++i) if (!isfinite(F[i])) return NTM_EXIT_NONFINITE;
    for (int i = 0; i < m * n; ++i) if (!isfinite(Lin[i])) return NTM_EXIT_NONFINITE;
    for (int i = 0; i < m; ++i) if (!isfinite(b[i])) return NTM_EXIT_NONFINITE;
    /* GI form n_i'U >= bc_i with n_i = -Lin_i, bc_i = -b_i; constant rows (D15). */
    double nrm[MMAX];
    unsigned char nz[MMAX];
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += Lin[(size_t)j * m + i] * Lin[(size_t)j * m + i];
        nrm[i] = sqrt(s);
        nz[i] = s > 0.0;
        if (!nz[i] && -b[i] > CONST_ROW_TOL) return NTM_EXIT_INFEASIBLE;   /* D15, D22 */
    }
    /* Cholesky G = Lc Lc' (lower, row-major Lc[i*n+j]) */
    for (int j = 0; j < n; ++j) {
        double s = G[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) s -= Lc[j * n + k] * Lc[j * n + k];
        if (!(s > 0.0)) return NTM_EXIT_NONFINITE;
        double l = sqrt(s);
        Lc[j * n + j] = l;
        for (int i = j + 1; i < n; ++i) {
            double t = G[(size_t)j * n + i];
            for (int k = 0; k < j; ++k) t -= Lc[i * n + k] * Lc[j * n + k];
            Lc[i * n + j] = t / l;
        }
        for (int i = 0; i < j; ++i) Lc[i * n + j] = 0.0;
    }
    /* J = Lc^{-T}: solve Lc X = I (X = Lc^{-1}, lower), J = X' (row-major J[i*n+k]) */
    for (int col = 0; col < n; ++col) {
        double x[NMAX];
        for (int i = 0; i < n; ++i) {
            double s = (i == col) ? 1.0 : 0.0;
            for (int k = 0; k < i; ++k) s -= Lc[i * n + k] * x[k];
            x[i] = s / Lc[i * n + i];
        }
        for (int i = 0; i < n; ++i) J[col * n + i] = x[i];   /* J[col][i] = X[i][col] */
    }
    memset(Rm, 0, sizeof(double) * (size_t)n * n);
    /* U = -J J' F */
    {
        double t[NMAX];
        for (int k = 0; k < n; ++k) { double s = 0.0; for (int i = 0; i < n; ++i) s += J[i * n + k] * F[i]; t[k] = s; }
        for (int i = 0; i < n; ++i) { double s = 0.0; for (int k = 0; k < n; ++k) s += J[i * n + k] * t[k]; U[i] = -s; }
    }
    for (;;) {
        /* choose the most violated (normalised) inactive row */
        int p = -1; double best = 0.0, sp_best = 0.0;
        double umax_abs = 1.0;
        for (int j = 0; j < n; ++j) if (fabs(U[j]) > umax_abs) umax_abs = fabs(U[j]);
        for (int i = 0; i < m; ++i) {
            if (!nz[i]) continue;
            int isact = 0;
            for (int a = 0; a < q; ++a) if (act[a] == i) { isact = 1; break; }
            if (isact) continue;
            double s = 0.0;
            for (int j = 0; j < n; ++j) s -= Lin[(size_t)j * m + i] * U[j];
            s += b[i];                                    /* s = n_i'U - bc_i */
            double v = s / nrm[i];
            if (p < 0 || v < best) { best = v; p = i; sp_best = s; }
        }
        if (p < 0 || sp_best >= -1e-12 * fmax(nrm[p] * umax_abs, fabs(b[p]))) {
            *iters_out = it;
            if (act_out) { for (int a = 0; a < q; ++a) act_out[a] = act[a]; *q_out = q; }
            return NTM_EXIT_OPTIMAL;
        }
        double np_[NMAX];
        for (int j = 0; j < n; ++j) np_[j] = -Lin[(size_t)j * m + p];
        up[q] = 0.0;
        for (;;) {
            if (++it > max_iter) { *iters_out = it; return NTM_EXIT_MAXITER; }
            for (int k = 0; k < n; ++k) { double s = 0.0; for (int i = 0; i < n; ++i) s += J[i * n + k] * np_[i]; d[k] = s; }
            double znrm = 0.0, dnrm = 0.0;
            for (int i = 0; i < n; ++i) {
                double s = 0.0;
                for (int k = q; k < n; ++k) s += J[i * n + k] * d[k];
                z[i] = s; znrm += s * s;
            }
            for (int k = 0; k < n; ++k) dnrm += d[k] * d[k];
            for (int a = q - 1; a >= 0; --a) {            /* r = R^{-1} d[0:q] */
                double s = d[a];
                for (int bb = a + 1; bb < q; ++bb) s -= Rm[a * n + bb] * r[bb];
                r[a] = s / Rm[a * n + a];
            }
            double t1 = INFINITY; int l = -1;
            for (int a = 0; a < q; ++a)
                if (r[a] > 0.0) { double ta = up[a] / r[a]; if (ta < t1) { t1 = ta; l = a; } }
            /* z'n_p = |d2|^2 exactly (z = J2 d2): computed that way it can never
             * be negative; n_p is treated as dependent on the active rows when
             * |d2| <= GI_DEP_TOL |d| (consecutive w-rows plus a u-bound are
             * dependent up to a11 - 1 ~ 5e-10). */
            double zn = 0.0, sp = b[p];                   /* sp = n_p'U - bc_p */
            for (int kk = q; kk < n; ++kk) zn += d[kk] * d[kk];
            for (int j = 0; j < n; ++j) sp += np_[j] * U[j];
            double t2 = (zn <= 1e-300 || sqrt(zn) <= gi_dep_tol * sqrt(dnrm)) ? INFINITY : -sp / zn;
            double t = t1 < t2 ? t1 : t2;
            if (t == INFINITY) { for (int j = 0; j < n; ++j) U[j] = 0.0; *iters_out = it; return NTM_EXIT_INFEASIBLE; }
            if (t2 == INFINITY) {
                for (int a = 0; a < q; ++a) up[a] = fmax(0.0, up[a] - t * r[a]);
                up[q] += t;
            } else {
                for (int j = 0; j < n; ++j) U[j] += t * z[j];
                for (int a = 0; a < q; ++a) up[a] = fmax(0.0, up[a] - t * r[a]);
                up[q] += t;
                if (t == t2) {                                 /* add constraint p */
                    for (int kk = n - 1; kk > q; --kk) {
                        double cc, ss, h;
                        givens(d[kk - 1], d[kk], &cc, &ss, &h);
                        d[kk - 1] = h; d[kk] = 0.0;
                        for (int i = 0; i < n; ++i) {
                            double j1 = J[i * n + kk - 1], j2 = J[i * n + kk];
                            J[i * n + kk - 1] = cc * j1 + ss * j2;
                            J[i * n + kk] = -ss * j1 + cc * j2;
                        }
                    }
                    for (int a = 0; a <= q; ++a) Rm[a * n + q] = d[a];
                    act[q] = p;
                    ++q;
                    break;
                }
            }
            /* drop constraint l (partial step, or dual-only step) */
            for (int a = 0; a < n; ++a)
                for (int bb = l; bb < q - 1; ++bb) Rm[a * n + bb] = Rm[a * n + bb + 1];
            for (int a = 0; a < n; ++a) Rm[a * n + q - 1] = 0.0;
            for (int jj = l; jj < q - 1; ++jj) {
                double cc, ss, h;
                givens(Rm[jj * n + jj], Rm[(jj + 1) * n + jj], &cc, &ss, &h);
                for (int bb = jj; bb < n; ++bb) {
                    double r1 = Rm[jj * n + bb], r2 = Rm[(jj + 1) * n + bb];
                    Rm[jj * n + bb] = cc * r1 + ss * r2;
                    Rm[(jj + 1) * n + bb] = -ss * r1 + cc * r2;
                }
                Rm[(jj + 1) * n + jj] = 0.0;
                for (int i = 0; i < n; ++i) {
                    double j1 = J[i * n + jj], j2 = J[i * n + jj + 1];
                    J[i * n + jj] = cc * j1 + ss * j2;
                    J[i * n + jj + 1] = -ss * j1 + cc * j2;
                }
            }
            for (int a = l; a < q; ++a) { act[a] = act[a + 1]; up[a] = up[a + 1]; }
            --q;
        }
    }
}

/* left-looking Cholesky of the n x n (row-major) A into L (row-major lower); 0 if not PD */
static int chol_rm(int n, const double* A, double* L) {
    for (int k = 0; k < n; ++k) {
        for (int i = k; i < n; ++i) {
            double s = A[i * n + k];
            for (int j = 0; j < k; ++j) s -= L[i * n + j] * L[k * n + j];
            if (i == k) {
                if (!(s > 0.0)) return 0;
                L[k * n + k] = sqrt(s);
            } else {
                L[i * n + k] = s / L[k * n + k];
            }
        }
        for (int j = k + 1; j < n; ++j) L[k * n + j] = 0.0;
    }
    return 1;
}
static void fwd_rm(int n, const double* L, const double* b, double* x) {
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * x[k];
        x[i] = s / L[i * n + i];
    }
}
static void bwd_rm(int n, const double* L, const double* b, double* x) {   /* L' x = b */
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * x[k];
        x[i] = s / L[i * n + i];
    }
}

/* Exact re-solve on GI's final active set (see oracle/ntm_oracle.py
 * polish_active_set).  Gs/Ls/bs: scaled, normalised data
 * (Lin U <= b form); Lin/b: unscaled.  Writes U and returns 1 when the KKT
 * certificate holds. */
static int orc_polish(int n, int m, const double* Gs, const double* Fs, const double* Ls,
                      const double* bs, const double* Lin, const double* b, const double* D,
                      const int* act, int q, double* U) {
    static __thread double Gm[NMAX * NMAX], Lc[NMAX * NMAX], Y[NMAX * NMAX], K[NMAX * NMAX], Lk[NMAX * NMAX];
    double Vb[NMAX], Ufix[NMAX], g[NMAX], w[NMAX], V[NMAX], mu[NMAX], tmp[NMAX], h[NMAX];
    unsigned char fixed[NMAX];
    int S[NMAX], nS = 0;
    memset(fixed, 0, sizeof fixed);
    for (int j = 0; j < n; ++j) Vb[j] = 0.0;
    for (int a = 0; a < q; ++a) {
        int row = act[a], nzc = 0, jj = -1;
        for (int j = 0; j < n; ++j) if (Lin[(size_t)j * m + row] != 0.0) { ++nzc; jj = j; }
        if (nzc == 1) {
            Ufix[jj] = b[row] / Lin[(size_t)jj * m + row];
            Vb[jj] = Ufix[jj] / D[jj];
            fixed[jj] = 1;
        } else {
            S[nS++] = row;
        }
    }
    /* Square, triangular E (nS == number of free variables; the GPU's
     * polish_compact square path): the active general rows alone determine the
     * free variables.  Sorted by their last free column, E is lower triangular:
     * V_F by forward substitution, the multipliers by back substitution on
     * E' mu = grad_F below (same order of operations as the device). */
    int nF = 0, fidx[NMAX], perm[NMAX], sq = 0;
    static __thread double Eq[NMAX * NMAX];
    double sqid[NMAX];
    for (int j = 0; j < n; ++j) if (!fixed[j]) fidx[nF++] = j;
    if (nS == nF && nS > 0) {
        sq = 1;
        for (int t = 0; t < nS; ++t) perm[t] = -1;
        for (int k = 0; k < nS && sq; ++k) {
            int last = -1;
            for (int a = 0; a < nF; ++a) if (Ls[(size_t)fidx[a] * m + S[k]] != 0.0) last = a;
            if (last < 0 || perm[last] >= 0) sq = 0;
            else perm[last] = k;
        }
    }
    if (sq) {
        double acc[NMAX];
        for (int t = 0; t < nS; ++t) {
            const int row = S[perm[t]];
            double hk = -bs[row];
            for (int j = 0; j < n; ++j) if (fixed[j]) hk -= (-Ls[(size_t)j * m + row]) * Vb[j];
            acc[t] = hk;
            for (int a = 0; a < nS; ++a) Eq[t * NMAX + a] = (a <= t) ? -Ls[(size_t)fidx[a] * m + row] : 0.0;
            sqid[t] = 1.0 / Eq[t * NMAX + t];
        }
        for (int t = 0; t < nS; ++t) {
            const double xt = acc[t] * sqid[t];
            V[fidx[t]] = xt;
            for (int u = t + 1; u < nS; ++u) acc[u] -= Eq[u * NMAX + t] * xt;
        }
    } else {
    for (int i = 0; i < n; ++i) {
        double s = Fs[i];
        for (int j = 0; j < n; ++j) if (fixed[j]) s += Gs[(size_t)j * n + i] * Vb[j];
        g[i] = fixed[i] ? 0.0 : s;
        for (int j = 0; j < n; ++j)
            Gm[i * n + j] = (fixed[i] || fixed[j]) ? (i == j ? 1.0 : 0.0) : Gs[(size_t)j * n + i];
    }
    if (!chol_rm(n, Gm, Lc)) return 0;
    fwd_rm(n, Lc, g, w);
    if (nS > 0) {
        for (int k = 0; k < nS; ++k) {
            double e[NMAX], y[NMAX], hk = -bs[S[k]];           /* bc = -bs, n = -Ls */
            for (int j = 0; j < n; ++j) {
                double nj = -Ls[(size_t)j * m + S[k]];
                if (fixed[j]) { hk -= nj * Vb[j]; e[j] = 0.0; } else e[j] = nj;
            }
            h[k] = hk;
            fwd_rm(n, Lc, e, y);
            for (int i = 0; i < n; ++i) Y[i * NMAX + k] = y[i];
        }
        for (int a = 0; a < nS; ++a)
            for (int c2 = 0; c2 < nS; ++c2) {
                double s = 0.0;
                for (int i = 0; i < n; ++i) s += Y[i * NMAX + a] * Y[i * NMAX + c2];
                K[a * nS + c2] = s;
            }
        if (!chol_rm(nS, K, Lk)) return 0;
        for (int a = 0; a < nS; ++a) {
            double s = h[a];
            for (int i = 0; i < n; ++i) s += Y[i * NMAX + a] * w[i];
            tmp[a] = s;
        }
        double t2[NMAX];
        fwd_rm(nS, Lk, tmp, t2);
        bwd_rm(nS, Lk, t2, mu);
        for (int i = 0; i < n; ++i) {
            double s = -w[i];
            for (int a = 0; a < nS; ++a) s += Y[i * NMAX + a] * mu[a];
            tmp[i] = s;
        }
        bwd_rm(n, Lc, tmp, V);
    } else {
        for (int i = 0; i < n; ++i) tmp[i] = -w[i];
        bwd_rm(n, Lc, tmp, V);
    }
    }
    for (int j = 0; j < n; ++j) if (fixed[j]) V[j] = Vb[j];
    /* KKT certificate: primal slack on every non-constant row, multiplier signs */
    double vmax = 1.0;
    for (int j = 0; j < n; ++j) if (fabs(V[j]) > vmax) vmax = fabs(V[j]);
    for (int i = 0; i < m; ++i) {
        double s = bs[i], nz2 = 0.0;
        for (int j = 0; j < n; ++j) { double l = Ls[(size_t)j * m + i]; s -= l * V[j]; nz2 += l * l; }
        if (nz2 > 0.0 && s < -1e-9 * fmax(vmax, fabs(bs[i]))) return 0;
    }
    double res[NMAX], mults[2 * NMAX], mscale = 1.0;
    int nm = 0;
    for (int i = 0; i < n; ++i) {
        double s = Fs[i];
        for (int j = 0; j < n; ++j) s += Gs[(size_t)j * n + i] * V[j];
        res[i] = s;
    }
    if (sq) {                                   /* E' mu = grad_F, back substitution */
        double acc[NMAX];
        for (int t = 0; t < nS; ++t) acc[t] = res[fidx[t]];
        for (int u = nS - 1; u >= 0; --u) {
            const double mu_u = acc[u] * sqid[u];
            mu[perm[u]] = mu_u;
            for (int t = 0; t < u; ++t) acc[t] -= Eq[u * NMAX + t] * mu_u;
        }
    }
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < nS; ++k) res[i] -= mu[k] * (-Ls[(size_t)i * m + S[k]]);
    for (int k = 0; k < nS; ++k) mults[nm++] = mu[k];
    for (int a = 0; a < q; ++a) {
        int row = act[a], isS = 0;
        for (int k = 0; k < nS; ++k) if (S[k] == row) isS = 1;
        if (isS) continue;
        for (int j = 0; j < n; ++j)
            if (Lin[(size_t)j * m + row] != 0.0) { mults[nm++] = res[j] / (-Ls[(size_t)j * m + row]); break; }
    }
    double mmin = 0.0;
    for (int k = 0; k < nm; ++k) { if (fabs(mults[k]) > mscale) mscale = fabs(mults[k]); if (mults[k] < mmin) mmin = mults[k]; }
    if (mmin < -1e-9 * mscale) return 0;
    for (int j = 0; j < n; ++j) U[j] = fixed[j] ? Ufix[j] : V[j] * D[j];
    return 1;
}

/* Partial-pivoting Gaussian elimination of the dense n x n row-major A (long
 * double, destroyed) with right-hand side x (overwritten by the solution);
 * 0 when a pivot vanishes. */
static int ge_solve_ld(int n, long double* A, long double* x) {
    for (int k = 0; k < n; ++k) {
        int p = k;
        for (int i = k + 1; i < n; ++i) if (fabsl(A[i * n + k]) > fabsl(A[p * n + k])) p = i;
        if (!(A[p * n + k] != 0.0L)) return 0;
        if (p != k) {
            for (int j = 0; j < n; ++j) { long double t = A[k * n + j]; A[k * n + j] = A[p * n + j]; A[p * n + j] = t; }
            long double t = x[k]; x[k] = x[p]; x[p] = t;
        }
        for (int i = k + 1; i < n; ++i) {
            const long double f = A[i * n + k] / A[k * n + k];
            for (int j = k; j < n; ++j) A[i * n + j] -= f * A[k * n + j];
            x[i] -= f * x[k];
        }
    }
    for (int k = n - 1; k >= 0; --k) {
        long double s = x[k];
        for (int j = k + 1; j < n; ++j) s -= A[k * n + j] * x[j];
        x[k] = s / A[k * n + k];
    }
    return 1;
}

/* Accurate value on the final active set (oracle/ntm_oracle.py accurate_resolve,
 * DESIGN.md §3): the KKT system of the free variables,
 *   [G~_FF  N_SF'; N_SF  0] [V_F; -mu] = [-(F~_F + G~_FB V_B); bc_S - N_SB V_B],
 * formed from the fp64 data in long double (Jacobi-scaled variables, unit-norm
 * rows) and solved by partial-pivoting elimination plus one refinement step.
 * The fp64 Cholesky / Schur re-solve loses digits when G~_FF is nearly singular
 * (input-rate rows: ~6e-9 umax) although the KKT system is well conditioned.
 * Variables fixed by single-entry rows keep U_j = b_a / Lin_aj.  U is left
 * unchanged when the system is singular. */
static void orc_accurate(int n, int m, const double* G, const double* F, const double* Lin, const double* b,
                         const int* act, int q, double* U) {
    static __thread long double M[4 * NMAX * NMAX], M2[4 * NMAX * NMAX], Ns[NMAX * NMAX];
    long double D[NMAX], Vb[NMAX], g[NMAX], rhs[2 * NMAX], sol[2 * NMAX], res[2 * NMAX];
    double Ufix[NMAX];
    unsigned char fixed[NMAX];
    int S[NMAX + 1], nS = 0, fidx[NMAX], nF = 0;
    if (q <= 0) return;
    memset(fixed, 0, sizeof fixed);
    for (int j = 0; j < n; ++j) {
        const double gj = G[(size_t)j * n + j];
        D[j] = (gj > 0.0) ? (long double)(1.0 / sqrt(gj)) : 1.0L;   /* the fp64 Jacobi factors */
        Vb[j] = 0.0L;
    }
    for (int a = 0; a < q; ++a) {
        int row = act[a], nzc = 0, jj = -1;
        for (int j = 0; j < n; ++j) if (Lin[(size_t)j * m + row] != 0.0) { ++nzc; jj = j; }
        if (nzc == 1) {
            Ufix[jj] = b[row] / Lin[(size_t)jj * m + row];
            fixed[jj] = 1;
            Vb[jj] = (long double)Ufix[jj] / D[jj];
        } else if (nzc > 1) {
            S[nS++] = row;
        }
    }
    for (int j = 0; j < n; ++j) if (!fixed[j]) fidx[nF++] = j;
    if (nF == 0) { for (int j = 0; j < n; ++j) U[j] = Ufix[j]; return; }
    const int nt = nF + nS;
    for (int i = 0; i < n; ++i) {
        long double s = (long double)F[i] * D[i];
        for (int j = 0; j < n; ++j) if (fixed[j]) s += ((long double)G[(size_t)j * n + i] * D[i] * D[j]) * Vb[j];
        g[i] = s;
    }
    for (int a = 0; a < nF; ++a) {
        for (int c = 0; c < nF; ++c)
            M[a * nt + c] = (long double)G[(size_t)fidx[c] * n + fidx[a]] * D[fidx[a]] * D[fidx[c]];
        rhs[a] = -g[fidx[a]];
    }
    for (int k = 0; k < nS; ++k) {
        long double s2 = 0.0L;
        for (int j = 0; j < n; ++j) { const long double v = (long double)Lin[(size_t)j * m + S[k]] * D[j]; Ns[k * NMAX + j] = v; s2 += v * v; }
        const long double rn = sqrtl(s2);
        long double h = (long double)b[S[k]] / rn;
        for (int j = 0; j < n; ++j) {
            Ns[k * NMAX + j] /= rn;
            if (fixed[j]) h -= Ns[k * NMAX + j] * Vb[j];
        }
        for (int a = 0; a < nF; ++a) {
            M[(nF + k) * nt + a] = Ns[k * NMAX + fidx[a]];
            M[a * nt + nF + k] = Ns[k * NMAX + fidx[a]];
        }
        for (int c = 0; c < nS; ++c) M[(nF + k) * nt + nF + c] = 0.0L;
        rhs[nF + k] = h;
    }
    memcpy(M2, M, sizeof(long double) * (size_t)nt * nt);
    for (int i = 0; i < nt; ++i) sol[i] = rhs[i];
    if (!ge_solve_ld(nt, M2, sol)) return;
    for (int i = 0; i < nt; ++i) {                          /* one refinement step */
        long double s = rhs[i];
        for (int j = 0; j < nt; ++j) s -= M[i * nt + j] * sol[j];
        res[i] = s;
    }
    memcpy(M2, M, sizeof(long double) * (size_t)nt * nt);
    if (ge_solve_ld(nt, M2, res))
        for (int i = 0; i < nt; ++i) sol[i] += res[i];
    double Uo[NMAX];
    for (int j = 0; j < n; ++j) Uo[j] = fixed[j] ? Ufix[j] : 0.0;
    for (int a = 0; a < nF; ++a) Uo[fidx[a]] = (double)(sol[a] * D[fidx[a]]);
    for (int j = 0; j < n; ++j) if (!isfinite(Uo[j])) return;
    for (int j = 0; j < n; ++j) U[j] = Uo[j];
}

/* quadprog stand-in: Jacobi variable scaling U = D V (diag(DGD) = 1) and
 * unit-norm constraint rows, then Goldfarb-Idnani on the scaled problem
 * (cond(G) ~1e9-1e11 drops to ~1e6; see oracle/ntm_oracle.py qp_solve). */
static int orc_qp(int n, int m, const double* G, const double* F, const double* Lin,
                  const double* b, double* U, int* iters_out) {
    static __thread double Gs[NMAX * NMAX], Ls[MMAX * NMAX];
    double D[NMAX], Fs[NMAX] = {0}, bs[MMAX] = {0}, V[NMAX];
    for (int j = 0; j < n; ++j) {
        double g = G[(size_t)j * n + j];
        D[j] = (g > 0.0) ? 1.0 / sqrt(g) : 1.0;
    }
    for (int j = 0; j < n; ++j) {
        for (int i = 0; i < n; ++i) Gs[(size_t)j * n + i] = G[(size_t)j * n + i] * D[i] * D[j];
        Fs[j] = F[j] * D[j];
    }
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) { double v = Lin[(size_t)j * m + i] * D[j]; Ls[(size_t)j * m + i] = v; s += v * v; }
        double rn = s > 0.0 ? sqrt(s) : 1.0;
        for (int j = 0; j < n; ++j) Ls[(size_t)j * m + i] /= rn;
        bs[i] = b[i] / rn;
    }
    int act[NMAX + 1], q = 0;
    int flag = orc_gi(n, m, Gs, Fs, Ls, bs, V, iters_out, act, &q);
    for (int j = 0; j < n; ++j) U[j] = V[j] * D[j];
    if (flag == NTM_EXIT_OPTIMAL && gi_polish) {
        (void)orc_polish(n, m, Gs, Fs, Ls, bs, Lin, b, D, act, q, U);
        orc_accurate(n, m, G, F, Lin, b, act, q, U);
    }
    return flag;
}

/* Solve the configured QP for one scenario; returns exitflag. */
static int orc_solve(const orc_coef* k, const ntm_config* c, const double* rho,
                     const double* x, double* U, int* qp_iters) {
    int N = c->N, R = 2 * N;
    double Phi[2 * NMAX * 2], Gam[2 * NMAX * NMAX], Lam[2 * NMAX];
    double G[NMAX * NMAX], F[NMAX];
    (void)R;
    orc_lift(k, c, rho, Phi, Gam, Lam);
    orc_cost(c, Phi, Gam, Lam, x, G, F);
    *qp_iters = 0;
    if (c->mode == NTM_MODE_NONE) {
        int flag = orc_qp(N, 0, G, F, NULL, NULL, U, qp_iters);
        return flag;
    }
    if (c->mode == NTM_MODE_BOX) {
        double Lin[2 * NMAX * NMAX], bb[2 * NMAX];
        memset(Lin, 0, sizeof(double) * (size_t)2 * N * N);
        for (int j = 0; j < N; ++j) {
            Lin[(size_t)j * 2 * N + j] = -1.0;
            Lin[(size_t)j * 2 * N + N + j] = 1.0;
            bb[j] = -c->umin;
            bb[N + j] = c->umax;
        }
        return orc_qp(N, 2 * N, G, F, Lin, bb, U, qp_iters);
    }
    int m = 6 * N + 4;
    double W[MMAX * 2], L[MMAX * NMAX], cv[MMAX];
    orc_getwlc(c, Phi, Gam, Lam, W, L, cv);
    for (int i = 0; i < m; ++i) cv[i] += W[i] * x[0] + W[m + i] * x[1];   /* c + W x_k (:97) */
    if (c->mode == NTM_MODE_FULL_DU) {
        /* config 5 (extension): rate rows after the getWLc rows; L is col-major m x N,
         * so re-stride it to mm = m + 2(N-1) rows */
        int mm = m + 2 * (N - 1);
        double L2[MMAX * NMAX];
        memset(L2, 0, sizeof(double) * (size_t)mm * N);
        for (int j = 0; j < N; ++j)
            for (int i = 0; i < m; ++i) L2[(size_t)j * mm + i] = L[(size_t)j * m + i];
        for (int i = 1; i < N; ++i) {
            int r = m + 2 * (i - 1);
            L2[(size_t)i * mm + r] = 1.0;       L2[(size_t)(i - 1) * mm + r] = -1.0;
            L2[(size_t)i * mm + r + 1] = -1.0;  L2[(size_t)(i - 1) * mm + r + 1] = 1.0;
            cv[r] = c->du_max;
            cv[r + 1] = c->du_max;
        }
        return orc_qp(N, mm, G, F, L2, cv, U, qp_iters);
    }
    return orc_qp(N, m, G, F, L, cv, U, qp_iters);
}

/* One MPC step, NTM_MPC_Sim.m:94-130 (CANON ordering). */
static void orc_step(const orc_coef* k, const ntm_config* c, const double* x,
                     double* rho, double* Uold, double* U, double* xpred,
                     double* xnext, int* flag_out, int* iters_out, const double* dist) {
    int N = c->N;
    int flag = NTM_EXIT_OPTIMAL, it = 0;
    for (it = 1; it <= c->i_sim; ++it) {
        int qi;
        flag = orc_solve(k, c, rho, x, U, &qi);
        /* rollout + rho update (:110-117) */
        double x0 = x[0], x1 = x[1];
        xpred[0] = x0; xpred[1] = x1;
        for (int i = 0; i < N; ++i) {
            double a11 = orc_a11(k, rho[3 * i]);
            double a21 = orc_a21(k, rho[3 * i + 1], c->Ts);
            double b = orc_b(k, rho[3 * i + 2]);
            double n0 = (a11 * x0 + b * U[i]) + k->C1;
            double n1 = (a21 * x0 + k->a22 * x1) + k->C2;
            double xi[2] = {x0, x1};
            orc_rho(k, xi, &rho[3 * i]);
            x0 = n0; x1 = n1;
            xpred[2 * i + 2] = x0; xpred[2 * i + 3] = x1;
        }
        double s = 0.0;                                      /* :123 */
        for (int j = 0; j < N; ++j) s += fabs(Uold[j] - U[j]);
        if (s < c->epsilon) break;                           /* :125, before :127 */
        for (int j = 0; j < N; ++j) Uold[j] = U[j];          /* :127 (skipped on break) */
    }
    if (it > c->i_sim) it = c->i_sim;
    /* plant step (:130, D13) */
    double r[3];
    orc_rho(k, x, r);
    double a11 = orc_a11(k, r[0]), a21 = orc_a21(k, r[1], c->Ts), b = orc_b(k, r[2]);
    xnext[0] = a11 * x[0] + b * U[0];
    xnext[1] = a21 * x[0] + k->a22 * x[1];
    if (!(c->flags & NTM_LITERAL_PLANT_NO_C)) { xnext[0] += k->C1; xnext[1] += k->C2; }
    if (dist) {                                              /* scenario generator */
        if (dist[0] != 0.0) xnext[0] += dist[0];
        if (dist[1] != 0.0) xnext[1] += dist[1];
    }
    *flag_out = flag;
    *iters_out = it;
}

/* ------------------------------------------------------------------ */
/* exported (ctypes) entry points                                     */
/* ------------------------------------------------------------------ */
#define EXPORT __attribute__((visibility("default")))

static int valid(const ntm_config* c) {
    return c && c->N >= 1 && c->N <= NMAX && c->i_sim >= 1 && c->mode >= 0 && c->mode <= 3;
}

EXPORT int ntm_oracle_rho(const ntm_physics* p, const ntm_config* c, const double* x, double* rho3) {
    orc_coef k; orc_coeffs(p, c, &k); orc_rho(&k, x, rho3); return 0;
}

EXPORT int ntm_oracle_lift(const ntm_physics* p, const ntm_config* c, const double* rho,
                           double* Phi, double* Gam, double* Lam) {
    if (!valid(c)) return NTM_E_INVALID;
    orc_coef k; orc_coeffs(p, c, &k); orc_lift(&k, c, rho, Phi, Gam, Lam); return 0;
}

EXPORT int ntm_oracle_cost(const ntm_physics* p, const ntm_config* c, const double* rho,
                           const double* x, double* G, double* F) {
    if (!valid(c)) return NTM_E_INVALID;
    orc_coef k; orc_coeffs(p, c, &k);
    double Phi[2 * NMAX * 2], Gam[2 * NMAX * NMAX], Lam[2 * NMAX];
    orc_lift(&k, c, rho, Phi, Gam, Lam); orc_cost(c, Phi, Gam, Lam, x, G, F); return 0;
}

EXPORT int ntm_oracle_getwlc(const ntm_physics* p, const ntm_config* c, const double* rho,
                             double* W, double* L, double* cv) {
    if (!valid(c)) return NTM_E_INVALID;
    orc_coef k; orc_coeffs(p, c, &k);
    double Phi[2 * NMAX * 2], Gam[2 * NMAX * NMAX], Lam[2 * NMAX];
    orc_lift(&k, c, rho, Phi, Gam, Lam); orc_getwlc(c, Phi, Gam, Lam, W, L, cv); return 0;
}

EXPORT int ntm_oracle_qp(int n, int m, const double* G, const double* F, const double* Lin,
                         const double* b, double* U, int* iters) {
    if (n < 1 || n > NMAX || m < 0 || m > MMAX) return NTM_E_INVALID;
    return orc_qp(n, m, G, F, Lin, b, U, iters);
}

/* Per-scenario coefficients: nominal, or scenario (first_id + s)'s plasma. */
static void orc_scn_coeffs(const ntm_physics* p, const ntm_config* c, const ntm_scenario_gen* g,
                           int64_t s, const orc_coef* nominal, orc_coef* k) {
    if (!g || (g->jbs_spread == 0.0 && g->wdep_spread == 0.0)) { *k = *nominal; return; }
    ntm_physics ps;
    orc_scn_physics(p, g, g->first_id + s, &ps);
    orc_coeffs(&ps, c, k);
}

/* Initial LPV state (NTM_MPC_Sim.m:63-65, D14), SoA scenario-minor layout. */
EXPORT int ntm_oracle_init_gen(const ntm_physics* p, const ntm_config* c, const ntm_scenario_gen* gen,
                               int64_t B, const double* x0, double* rho, double* U_old) {
    if (!valid(c) || B < 0) return NTM_E_INVALID;
    orc_coef k0; orc_coeffs(p, c, &k0);
    int N = c->N;
    for (int64_t s = 0; s < B; ++s) {
        orc_coef k; orc_scn_coeffs(p, c, gen, s, &k0, &k);
        double x[2] = {x0[s], x0[B + s]}, r[3];
        orc_rho(&k, x, r);
        for (int i = 0; i < N; ++i)
            for (int e = 0; e < 3; ++e) rho[(int64_t)(3 * i + e) * B + s] = r[e];
        for (int j = 0; j < N; ++j) U_old[(int64_t)j * B + s] = INFINITY;
    }
    return 0;
}

/* Batched MPC step, SoA scenario-minor layout (see include/ntm_mpc.h); gen may be
 * NULL (nominal plant), its k0 is the plant step's time index. */
EXPORT int ntm_oracle_step_gen(const ntm_physics* p, const ntm_config* c, const ntm_scenario_gen* gen,
                               int64_t B, const double* x_k, double* rho, double* U_old, double* U,
                               double* x_pred, double* x_next, int32_t* exitflag,
                               int32_t* inner_iters, int nthreads) {
    if (!valid(c) || B < 0) return NTM_E_INVALID;
    orc_coef k0; orc_coeffs(p, c, &k0);
    int N = c->N;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int64_t s = 0; s < B; ++s) {
        double x[2], rh[3 * NMAX], uo[NMAX], u[NMAX], xp[2 * (NMAX + 1)], xn[2], d[2];
        int fl, its;
        orc_coef k; orc_scn_coeffs(p, c, gen, s, &k0, &k);
        if (gen) orc_disturbance(gen, gen->first_id + s, gen->k0, d);
        for (int e = 0; e < 2; ++e) x[e] = x_k[e * B + s];
        for (int e = 0; e < 3 * N; ++e) rh[e] = rho[e * B + s];
        for (int e = 0; e < N; ++e) uo[e] = U_old[e * B + s];
        orc_step(&k, c, x, rh, uo, u, xp, xn, &fl, &its, gen ? d : NULL);
        for (int e = 0; e < 3 * N; ++e) rho[e * B + s] = rh[e];
        for (int e = 0; e < N; ++e) { U_old[e * B + s] = uo[e]; U[e * B + s] = u[e]; }
        for (int e = 0; e < 2 * (N + 1); ++e) x_pred[e * B + s] = xp[e];
        for (int e = 0; e < 2; ++e) x_next[e * B + s] = xn[e];
        exitflag[s] = fl;
        inner_iters[s] = its;
    }
    return 0;
}

EXPORT int ntm_oracle_step(const ntm_physics* p, const ntm_config* c, int64_t B,
                           const double* x_k, double* rho, double* U_old, double* U,
                           double* x_pred, double* x_next, int32_t* exitflag,
                           int32_t* inner_iters, int nthreads) {
    return ntm_oracle_step_gen(p, c, NULL, B, x_k, rho, U_old, U, x_pred, x_next, exitflag, inner_iters,
                               nthreads);
}

/* Batched closed loop NTM_MPC_Sim.m:80-131.  Output layouts as ntm_mpc_run;
 * gen may be NULL, plant step kk uses time index gen->k0 + kk. */
EXPORT int ntm_oracle_run_gen(const ntm_physics* p, const ntm_config* c, const ntm_scenario_gen* gen,
                              int64_t B, int32_t k_sim, const double* x0, double* xk, double* uk, double* Uk,
                              double* wpred, int32_t* exitflag, int32_t* inner_iters, int nthreads) {
    if (!valid(c) || B < 0 || k_sim < 0) return NTM_E_INVALID;
    orc_coef k0; orc_coeffs(p, c, &k0);
    int N = c->N;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int64_t s = 0; s < B; ++s) {
        double x[2], rh[3 * NMAX], uo[NMAX], u[NMAX], xp[2 * (NMAX + 1)], xn[2], d[2];
        orc_coef k; orc_scn_coeffs(p, c, gen, s, &k0, &k);
        x[0] = x0[s]; x[1] = x0[B + s];
        orc_rho(&k, x, rh);
        for (int i = 1; i < N; ++i) for (int e = 0; e < 3; ++e) rh[3 * i + e] = rh[e];
        for (int j = 0; j < N; ++j) uo[j] = INFINITY;
        if (xk) { xk[s] = x[0]; xk[B + s] = x[1]; }
        for (int kk = 0; kk < k_sim; ++kk) {
            int fl, its;
            if (gen) orc_disturbance(gen, gen->first_id + s, gen->k0 + kk, d);
            orc_step(&k, c, x, rh, uo, u, xp, xn, &fl, &its, gen ? d : NULL);
            if (uk) uk[(int64_t)kk * B + s] = u[0];
            if (Uk) for (int j = 0; j < N; ++j) Uk[((int64_t)kk * N + j) * B + s] = u[j];
            if (wpred) for (int i = 0; i <= N; ++i) wpred[((int64_t)kk * (N + 1) + i) * B + s] = xp[2 * i];
            if (exitflag) exitflag[(int64_t)kk * B + s] = fl;
            if (inner_iters) inner_iters[(int64_t)kk * B + s] = its;
            x[0] = xn[0]; x[1] = xn[1];
            if (xk) { xk[(int64_t)(2 * (kk + 1)) * B + s] = x[0]; xk[(int64_t)(2 * (kk + 1) + 1) * B + s] = x[1]; }
        }
    }
    return 0;
}

EXPORT int ntm_oracle_run(const ntm_physics* p, const ntm_config* c, int64_t B, int32_t k_sim,
                          const double* x0, double* xk, double* uk, double* Uk, double* wpred,
                          int32_t* exitflag, int32_t* inner_iters, int nthreads) {
    return ntm_oracle_run_gen(p, c, NULL, B, k_sim, x0, xk, uk, Uk, wpred, exitflag, inner_iters, nthreads);
}

/* The generator's samples (same layout as the library's ntm_scenario_sample). */
EXPORT void ntm_oracle_scenario_sample(const ntm_scenario_gen* g, int64_t B, int32_t k, double* out4) {
    for (int64_t s = 0; s < B; ++s) {
        int64_t id = g->first_id + s;
        out4[4 * s] = o_factor(g->seed, id, 0, g->jbs_spread);
        out4[4 * s + 1] = o_factor(g->seed, id, 1, g->wdep_spread);
        out4[4 * s + 2] = o_normal(g->seed, id, (uint32_t)k, 0);
        out4[4 * s + 3] = o_normal(g->seed, id, (uint32_t)k, 1);
    }
}

/*
 * sanitize_main.c — TEST INFRASTRUCTURE ONLY: drives the C oracle
 * (oracle/ntm_oracle.c) through every exported entry point under
 * AddressSanitizer + UndefinedBehaviorSanitizer (make -C oracle sanitize,
 * tests/test_oracle_c.py::test_c_oracle_under_asan_ubsan).  Covers every
 * constraint mode, the horizon extremes (N = 1 and NTM_MAX_N), the literal
 * switches, the scenario generator, the infeasible reference x0 and non-finite
 * data.  Exits non-zero on any sanitizer report (halt_on_error) or failed check.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ntm_mpc.h"

int ntm_oracle_run_gen(const ntm_physics*, const ntm_config*, const ntm_scenario_gen*, int64_t, int32_t,
                       const double*, double*, double*, double*, double*, int32_t*, int32_t*, int);
int ntm_oracle_step_gen(const ntm_physics*, const ntm_config*, const ntm_scenario_gen*, int64_t, const double*,
                        double*, double*, double*, double*, double*, int32_t*, int32_t*, int);
int ntm_oracle_init_gen(const ntm_physics*, const ntm_config*, const ntm_scenario_gen*, int64_t, const double*,
                        double*, double*);
int ntm_oracle_lift(const ntm_physics*, const ntm_config*, const double*, double*, double*, double*);
int ntm_oracle_cost(const ntm_physics*, const ntm_config*, const double*, const double*, double*, double*);
int ntm_oracle_getwlc(const ntm_physics*, const ntm_config*, const double*, double*, double*, double*);
int ntm_oracle_qp(int, int, const double*, const double*, const double*, const double*, double*, int*);
void ntm_oracle_scenario_sample(const ntm_scenario_gen*, int64_t, int32_t, double*);

static ntm_physics phys(void) {
    ntm_physics p = {73e3, 0.024, 0.02, 0.32, 293, 1.55, 2.0, 0.9, 3.7, 3.7, 4e-7 * M_PI, 0.87, 0.97, 2, 1,
                     3e-6, 0.188, 2 * M_PI * 420};
    return p;
}
static ntm_config cfg(int N, int mode, int flags) {
    ntm_config c;
    memset(&c, 0, sizeof c);
    c.N = N; c.i_sim = 10; c.mode = mode; c.flags = flags; c.Ts = 0.1;
    c.xmin[0] = 0.06; c.xmin[1] = 200 * M_PI; c.xmax[0] = 0.15; c.xmax[1] = 10000 * M_PI;
    c.umin = 0; c.umax = 2e6; c.Q[0] = 1; c.Q[3] = 1; c.r[1] = 2000 * M_PI; c.epsilon = 1e-14; c.du_max = 5e5;
    return c;
}

static int fails = 0;
#define CHECK(x) do { if (!(x)) { fprintf(stderr, "check failed: %s (line %d)\n", #x, __LINE__); ++fails; } } while (0)

static void closed_loop(int N, int mode, int flags, const ntm_scenario_gen* g, int B, int k_sim) {
    ntm_physics p = phys();
    ntm_config c = cfg(N, mode, flags);
    double* x0 = malloc(sizeof(double) * 2 * B);
    for (int s = 0; s < B; ++s) { x0[s] = 0.07 + 0.07 * s / (B + 1.0); x0[B + s] = (0.8 + 0.4 * s / (B + 1.0)) * 2000 * M_PI; }
    double* xk = malloc(sizeof(double) * 2 * (k_sim + 1) * B);
    double* uk = malloc(sizeof(double) * k_sim * B);
    double* Uk = malloc(sizeof(double) * N * k_sim * B);
    double* wp = malloc(sizeof(double) * (N + 1) * k_sim * B);
    int32_t* fl = malloc(sizeof(int32_t) * k_sim * B);
    int32_t* it = malloc(sizeof(int32_t) * k_sim * B);
    CHECK(ntm_oracle_run_gen(&p, &c, g, B, k_sim, x0, xk, uk, Uk, wp, fl, it, 1) == 0);
    for (int i = 0; i < k_sim * B; ++i) CHECK(fl[i] == 1 || fl[i] == -2 || fl[i] == 0 || fl[i] == -7);
    /* the step entry point from the same start */
    double* rho = malloc(sizeof(double) * 3 * N * B);
    double* uo = malloc(sizeof(double) * N * B);
    double* U = malloc(sizeof(double) * N * B);
    double* xp = malloc(sizeof(double) * 2 * (N + 1) * B);
    double* xn = malloc(sizeof(double) * 2 * B);
    CHECK(ntm_oracle_init_gen(&p, &c, g, B, x0, rho, uo) == 0);
    CHECK(ntm_oracle_step_gen(&p, &c, g, B, x0, rho, uo, U, xp, xn, fl, it, 1) == 0);
    free(x0); free(xk); free(uk); free(Uk); free(wp); free(fl); free(it);
    free(rho); free(uo); free(U); free(xp); free(xn);
}

int main(void) {
    ntm_scenario_gen g = {20241220, 0, 0, 0, 1e-3, 10.0, 0.1, 0.1};
    const int modes[] = {NTM_MODE_NONE, NTM_MODE_BOX, NTM_MODE_FULL, NTM_MODE_FULL_DU};
    for (int m = 0; m < 4; ++m) {
        closed_loop(1, modes[m], 0, NULL, 3, 4);
        closed_loop(3, modes[m], 0, NULL, 5, 6);
        closed_loop(20, modes[m], 0, &g, 4, 3);
    }
    closed_loop(NTM_MAX_N, NTM_MODE_FULL, 0, NULL, 2, 2);
    closed_loop(NTM_MAX_N, NTM_MODE_FULL_DU, 0, NULL, 1, 2);
    for (int f = 1; f <= 15; ++f) closed_loop(6, NTM_MODE_FULL, f, NULL, 3, 3);
    {   /* infeasible reference x0 (NTM_MPC_Sim.m:34) and non-finite data */
        ntm_physics p = phys();
        ntm_config c = cfg(3, NTM_MODE_FULL, 0);
        double x[4] = {0.0, 0.1, 2000 * M_PI, NAN};
        double rho[18], uo[6], U[6], xp[16], xn[4];
        int32_t fl[2], it[2];
        CHECK(ntm_oracle_init_gen(&p, &c, NULL, 2, x, rho, uo) == 0);
        CHECK(ntm_oracle_step_gen(&p, &c, NULL, 2, x, rho, uo, U, xp, xn, fl, it, 1) == 0);
        CHECK(fl[0] == -2 && fl[1] == -7);
    }
    {   /* function-level entries and the dense QP at N = 20 */
        ntm_physics p = phys();
        ntm_config c = cfg(20, NTM_MODE_FULL, 0);
        double rho[60], x[2] = {0.1, 2000 * M_PI}, Phi[80], Gam[800], Lam[40], G[400], F[20];
        double W[248], L[124 * 20], cv[124], U[20];
        for (int i = 0; i < 20; ++i) { rho[3 * i] = 9.9; rho[3 * i + 1] = 1.6e-6; rho[3 * i + 2] = 0.02; }
        CHECK(ntm_oracle_lift(&p, &c, rho, Phi, Gam, Lam) == 0);
        CHECK(ntm_oracle_cost(&p, &c, rho, x, G, F) == 0);
        CHECK(ntm_oracle_getwlc(&p, &c, rho, W, L, cv) == 0);
        for (int i = 0; i < 124; ++i) cv[i] += W[i] * x[0] + W[124 + i] * x[1];
        int its = 0;
        CHECK(ntm_oracle_qp(20, 124, G, F, L, cv, U, &its) == 1);
        CHECK(ntm_oracle_qp(20, 0, G, F, NULL, NULL, U, &its) == 1);
        c.N = 0;
        CHECK(ntm_oracle_lift(&p, &c, rho, Phi, Gam, Lam) != 0);
    }
    {
        double out[4 * 64];
        ntm_oracle_scenario_sample(&g, 64, 7, out);
        for (int i = 0; i < 64; ++i) CHECK(fabs(out[4 * i + 2]) <= 2 * sqrt(3.0));
    }
    if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
    printf("oracle sanitizer run: ok\n");
    return 0;
}

/*
 * ntm_mpc_mex.c — MATLAB MEX gateway over the C-ABI in include/ntm_mpc.h.
 *
 * Replaces, for a batch of B scenarios, the body of the receding-horizon loop
 * of NTM_MPC_Sim.m (lines 94-130: the LPV iteration, quadprog call and plant
 * step) or the whole closed loop (lines 80-131).  Build, where MATLAB exists:
 *
 *   mex -R2018a -I../../include ntm_mpc_mex.c \
 *       -L../../mpc-ntm-control_amd/lib -lntm_mpc
 *
 * Calls (every batched array is E-by-B: one column per scenario, which is the
 * ABI's scenario-major layout [s*E + e] in MATLAB's column-major storage, so
 * arrays pass through without copies):
 *
 *   [U, x_pred, x_next, exitflag, iters, rho, Uold, ws] = ...
 *       ntm_mpc_mex('step', x_k, rho, Uold, cfg[, ws])
 *         x_k  2-by-B        current state [w; omega]           (xk(:,k))
 *         rho  3N-by-B       Rho(:) per scenario                (:63-65,116)
 *         Uold N-by-B        +Inf on the first step (D14)
 *         ws   2(N+1)-by-B   optional int32 warm-start workspace (start with
 *                            -1 everywhere; pass the returned one back next step)
 *       outputs: U N-by-B, x_pred 2(N+1)-by-B, x_next 2-by-B, exitflag and
 *       iters 1-by-B
 *   [rho, Uold] = ntm_mpc_mex('init', x0, cfg)                 (:63-65, :86)
 *   [xk, uk, Uk, wpred, exitflag, iters] = ntm_mpc_mex('run', x0, k_sim, cfg)
 *       outputs 2(k_sim+1)-by-B, k_sim-by-B, N k_sim-by-B, (N+1) k_sim-by-B,
 *       k_sim-by-B, k_sim-by-B (per scenario column: xk(:), uk, Uk(:), ...)
 *   ntm_mpc_mex('scenarios', gen)                               
 *       gen struct with any of seed, first_id, k0, sigma_w, sigma_omega,
 *       jbs_spread, wdep_spread (ntm_scenario_gen): per-scenario plasma and
 *       plant disturbances for the following init/step/run calls; [] = off.
 *       With 'step', set k0 to the step's time index before each call.
 *   ntm_mpc_mex('close')
 *
 * cfg is an optional struct with any of the fields N, i_sim, mode, flags, Ts,
 * xmin, xmax, umin, umax, Q (2x2), r, epsilon, du_max, Ru (input weight, ABI v5);
 * missing fields take the
 * reference literals (ntm_config_default).  Library errors become MATLAB
 * errors (ntm:...); solver outcomes are returned in exitflag (quadprog codes,
 * NTM_MPC_Sim.m:98-103), never raised.
 */
#include <string.h>

#include "mex.h"
#include "ntm_mpc.h"

static ntm_ctx* g_ctx = NULL;

static void release(void) {
    if (g_ctx) {
        ntm_ctx_destroy(g_ctx);
        g_ctx = NULL;
    }
}

static void check(int rc, const char* what) {
    if (rc != NTM_OK) {
        mexErrMsgIdAndTxt("ntm:library", "%s failed (%d): %s", what, rc, g_ctx ? ntm_last_error(g_ctx) : "no context");
    }
}

static ntm_ctx* ctx(void) {
    if (!g_ctx) {
        check(ntm_ctx_create(&g_ctx, 0), "ntm_ctx_create");
        mexAtExit(release);
    }
    return g_ctx;
}

static double scalar_field(const mxArray* s, const char* name, double dflt) {
    const mxArray* f = s ? mxGetField(s, 0, name) : NULL;
    return (f && mxIsDouble(f) && mxGetNumberOfElements(f) >= 1) ? mxGetDoubles(f)[0] : dflt;
}

static void vec_field(const mxArray* s, const char* name, double* dst, size_t n) {
    const mxArray* f = s ? mxGetField(s, 0, name) : NULL;
    if (!f) return;
    if (!mxIsDouble(f) || mxGetNumberOfElements(f) != n) mexErrMsgIdAndTxt("ntm:cfg", "cfg.%s must have %d doubles", name, (int)n);
    memcpy(dst, mxGetDoubles(f), n * sizeof(double));
}

static ntm_config read_cfg(const mxArray* s) {
    ntm_config c;
    if (s && !mxIsStruct(s)) mexErrMsgIdAndTxt("ntm:cfg", "cfg must be a struct");
    ntm_config_default(&c, (int32_t)scalar_field(s, "N", 20));
    c.i_sim = (int32_t)scalar_field(s, "i_sim", c.i_sim);
    c.mode = (int32_t)scalar_field(s, "mode", c.mode);
    c.flags = (int32_t)scalar_field(s, "flags", c.flags);
    c.Ts = scalar_field(s, "Ts", c.Ts);
    c.umin = scalar_field(s, "umin", c.umin);
    c.umax = scalar_field(s, "umax", c.umax);
    c.epsilon = scalar_field(s, "epsilon", c.epsilon);
    c.du_max = scalar_field(s, "du_max", c.du_max);
    c.Ru = scalar_field(s, "Ru", c.Ru);
    vec_field(s, "xmin", c.xmin, 2);
    vec_field(s, "xmax", c.xmax, 2);
    vec_field(s, "r", c.r, 2);
    if (s && mxGetField(s, 0, "Q")) {   /* MATLAB 2x2 is column-major; the ABI's Q is row-major */
        double q[4];
        vec_field(s, "Q", q, 4);
        c.Q[0] = q[0]; c.Q[1] = q[2]; c.Q[2] = q[1]; c.Q[3] = q[3];
    }
    return c;
}

static const double* in_matrix(const mxArray* a, size_t rows, size_t cols, const char* name) {
    if (!mxIsDouble(a) || mxIsComplex(a) || mxGetM(a) != rows || mxGetN(a) != cols)
        mexErrMsgIdAndTxt("ntm:arg", "%s must be a real %d-by-%d double array", name, (int)rows, (int)cols);
    return mxGetDoubles(a);
}

static void do_step(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 4) mexErrMsgIdAndTxt("ntm:arg", "usage: ntm_mpc_mex('step', x_k, rho, Uold[, cfg[, ws]])");
    const ntm_config c = read_cfg(nrhs > 4 ? prhs[4] : NULL);
    ntm_physics p;
    ntm_physics_default(&p);
    const size_t B = mxGetN(prhs[1]), N = (size_t)c.N;
    const double* x = in_matrix(prhs[1], 2, B, "x_k");
    in_matrix(prhs[2], 3 * N, B, "rho");
    in_matrix(prhs[3], N, B, "Uold");
    /* value semantics: rho / Uold are updated in copies returned as outputs 6-7 */
    mxArray* rho = mxDuplicateArray(prhs[2]);
    mxArray* uold = mxDuplicateArray(prhs[3]);
    mxArray* U = mxCreateDoubleMatrix(N, B, mxREAL);
    mxArray* xp = mxCreateDoubleMatrix(2 * (N + 1), B, mxREAL);
    mxArray* xn = mxCreateDoubleMatrix(2, B, mxREAL);
    mxArray* fl = mxCreateNumericMatrix(1, B, mxINT32_CLASS, mxREAL);
    mxArray* it = mxCreateNumericMatrix(1, B, mxINT32_CLASS, mxREAL);
    mxArray* ws = NULL;
    if (nrhs > 5) {
        const mxArray* w = prhs[5];
        if (!mxIsInt32(w) || mxGetM(w) != 2 * (N + 1) || mxGetN(w) != B)
            mexErrMsgIdAndTxt("ntm:arg", "ws must be an int32 %d-by-%d array", (int)(2 * (N + 1)), (int)B);
        ws = mxDuplicateArray(w);
    } else {
        ws = mxCreateNumericMatrix(2 * (N + 1), B, mxINT32_CLASS, mxREAL);
        int32_t* wp = mxGetInt32s(ws);
        for (size_t i = 0; i < B * 2 * (N + 1); ++i) wp[i] = -1;
    }
    check(ntm_mpc_step_ws(ctx(), &p, &c, (int64_t)B, x, mxGetDoubles(rho), mxGetDoubles(uold), mxGetDoubles(U),
                          mxGetDoubles(xp), mxGetDoubles(xn), mxGetInt32s(fl), mxGetInt32s(it), mxGetInt32s(ws)),
          "ntm_mpc_step_ws");
    mxArray* outs[8] = {U, xp, xn, fl, it, rho, uold, ws};
    for (int i = 0; i < 8; ++i) {
        if (i < (nlhs > 0 ? nlhs : 1)) plhs[i] = outs[i];
        else mxDestroyArray(outs[i]);
    }
}

static void do_init(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 2) mexErrMsgIdAndTxt("ntm:arg", "usage: ntm_mpc_mex('init', x0[, cfg])");
    const ntm_config c = read_cfg(nrhs > 2 ? prhs[2] : NULL);
    ntm_physics p;
    ntm_physics_default(&p);
    const size_t B = mxGetN(prhs[1]), N = (size_t)c.N;
    const double* x0 = in_matrix(prhs[1], 2, B, "x0");
    mxArray* rho = mxCreateDoubleMatrix(3 * N, B, mxREAL);
    mxArray* uold = mxCreateDoubleMatrix(N, B, mxREAL);
    check(ntm_mpc_init(ctx(), &p, &c, (int64_t)B, x0, mxGetDoubles(rho), mxGetDoubles(uold)), "ntm_mpc_init");
    plhs[0] = rho;
    if (nlhs > 1) plhs[1] = uold;
    else mxDestroyArray(uold);
}

static void do_run(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 3) mexErrMsgIdAndTxt("ntm:arg", "usage: ntm_mpc_mex('run', x0, k_sim[, cfg])");
    const ntm_config c = read_cfg(nrhs > 3 ? prhs[3] : NULL);
    ntm_physics p;
    ntm_physics_default(&p);
    const size_t B = mxGetN(prhs[1]), N = (size_t)c.N;
    const double* x0 = in_matrix(prhs[1], 2, B, "x0");
    const int k = (int)mxGetScalar(prhs[2]);
    if (k < 1) mexErrMsgIdAndTxt("ntm:arg", "k_sim must be >= 1");
    mxArray* xk = mxCreateDoubleMatrix(2 * (size_t)(k + 1), B, mxREAL);
    mxArray* uk = mxCreateDoubleMatrix((size_t)k, B, mxREAL);
    mxArray* Uk = mxCreateDoubleMatrix(N * (size_t)k, B, mxREAL);
    mxArray* wp = mxCreateDoubleMatrix((N + 1) * (size_t)k, B, mxREAL);
    mxArray* fl = mxCreateNumericMatrix((size_t)k, B, mxINT32_CLASS, mxREAL);
    mxArray* it = mxCreateNumericMatrix((size_t)k, B, mxINT32_CLASS, mxREAL);
    check(ntm_mpc_run(ctx(), &p, &c, (int64_t)B, k, x0, mxGetDoubles(xk), mxGetDoubles(uk), mxGetDoubles(Uk),
                      mxGetDoubles(wp), mxGetInt32s(fl), mxGetInt32s(it)),
          "ntm_mpc_run");
    mxArray* outs[6] = {xk, uk, Uk, wp, fl, it};
    for (int i = 0; i < 6; ++i) {
        if (i < (nlhs > 0 ? nlhs : 1)) plhs[i] = outs[i];
        else mxDestroyArray(outs[i]);
    }
}

static void do_scenarios(int nrhs, const mxArray* prhs[]) {
    if (nrhs < 2 || (mxIsDouble(prhs[1]) && mxGetNumberOfElements(prhs[1]) == 0)) {
        check(ntm_ctx_set_scenarios(ctx(), NULL), "ntm_ctx_set_scenarios");
        return;
    }
    const mxArray* s = prhs[1];
    if (!mxIsStruct(s)) mexErrMsgIdAndTxt("ntm:arg", "gen must be a struct or []");
    ntm_scenario_gen g;
    memset(&g, 0, sizeof g);
    g.seed = (uint64_t)scalar_field(s, "seed", 20241220);
    g.first_id = (int64_t)scalar_field(s, "first_id", 0);
    g.k0 = (int32_t)scalar_field(s, "k0", 0);
    g.sigma_w = scalar_field(s, "sigma_w", 0.0);
    g.sigma_omega = scalar_field(s, "sigma_omega", 0.0);
    g.jbs_spread = scalar_field(s, "jbs_spread", 0.0);
    g.wdep_spread = scalar_field(s, "wdep_spread", 0.0);
    check(ntm_ctx_set_scenarios(ctx(), &g), "ntm_ctx_set_scenarios");
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 1 || !mxIsChar(prhs[0]))
        mexErrMsgIdAndTxt("ntm:arg", "first argument: 'init', 'step', 'run', 'scenarios' or 'close'");
    char cmd[16];
    mxGetString(prhs[0], cmd, sizeof cmd);
    if (!strcmp(cmd, "step")) do_step(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "init")) do_init(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "run")) do_run(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "scenarios")) do_scenarios(nrhs, prhs);
    else if (!strcmp(cmd, "close")) release();
    else mexErrMsgIdAndTxt("ntm:arg", "unknown command '%s'", cmd);
}

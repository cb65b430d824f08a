"""Algorithmic fp64 flop count of one MPC step of THIS build.

SURVEY.md §8(d) prices an interior-point path (F_kkt per IPM iteration).  This
build solves each QP on one of two paths, and is priced against its own count,
which stays far below the survey's (a GI iteration is O(N^2), an IPM
iteration O(N^3)):

* warm-start verify: the active set of LPV iteration it-2 is re-solved exactly
  (compact KKT system on the free variables) and certified;
* full solve: Gram + Cholesky, Goldfarb-Idnani dual active set, exact polish.

Every QP also pays the common build (lift, free response, F, Jacobi scaling).
Counts are the useful flops of the formulas as implemented (an FMA = 2; no
padding lanes, masked terms or recomputation counted), driven by the per-step
counters the kernel records (include/ntm_mpc.h ntm_ctx_set_stats):
qps = QP solves, tries = warm-start verifications, giruns = full GI solves,
K = GI iterations (all per MPC step), q / s = final active rows / general
(state) active rows per QP.
"""
from __future__ import annotations

MODE_NONE, MODE_BOX, MODE_FULL, MODE_FULL_DU = 0, 1, 2, 3


def common_build(N: int, mode: int) -> float:
    """Per QP: lift (Rho_to_PhiGammaLambda.m), free response, F, Jacobi scaling."""
    f = 20 * N + 2 * N * (N - 1)                      # A/B coefficients, Phi, Lambda, Gamma blocks
    f += 8 * N                                        # e = Phi x_k + Lambda
    f += 10 * N + 2 * N * (N + 1)                     # F~ = D 2 Gamma' Om (e - r)
    f += 5 * N * (N + 1) + 4 * N                      # diag(G~) -> D, scaled bounds
    if mode >= MODE_FULL:
        f += 3 * N * (N + 1) + 2 * N                  # state-row norms |Gamma_r D|
    if mode == MODE_FULL_DU:
        f += 4 * (N - 1)                              # rate-row norms
    return f


def check(N: int, mode: int) -> float:
    """One most-violated-row search (or KKT primal verification)."""
    if mode == MODE_NONE:
        return 0.0
    f = 2 * N                                         # u bounds
    if mode >= MODE_FULL:
        f += 2 * N * (N + 1) + 8 * N                  # x^ = Gamma U + e, two slacks per state row
    if mode == MODE_FULL_DU:
        f += 5 * (N - 1)                              # U_i - U_{i-1}, two slacks per rate pair
    return f


def gi_setup(N: int) -> float:
    """Full Gram of G~ (lower), scaling, Cholesky, J = L^-T, unconstrained V."""
    return 10 * N * (N + 1) * (N + 2) / 6 + N * (N + 1) + N ** 3 / 3 + N ** 3 / 3 + 4 * N * N


def gi_iteration(N: int, qbar: float, state_frac: float) -> float:
    """Direction (d, z, r), step lengths, update, and the add/drop factor update."""
    free = max(N - qbar, 0.0)
    f = 2 * N * N * state_frac                        # d = J' n_p (u rows: a signed row of J)
    f += 2 * N * free + qbar * (qbar + 1) + qbar      # z = J2 d2, r = T d1, ratios
    f += 2 * free + 4 * N + 7 * N + 2 * qbar          # |d2|^2, n'V, |d|^2, V/U/u updates
    f += 4 * N * free                                 # Householder add (drop: Givens, fewer)
    return f


def polish(N: int, mode: int, q: float, s: float) -> float:
    """Exact active-set solve on the compact free variables + KKT certificate."""
    nF = max(N - (q - s), 0.0)
    f = N * (N + 1)                                   # Gamma U_B + e - r
    f += 5 * nF * N + 2.5 * nF * (nF + 1) * N         # g_F, G~_FF
    f += nF ** 3 / 3 + 2 * nF * nF                    # Cholesky, two triangular solves
    f += s * nF * nF + s * (s + 1) * nF + 4 * s * nF  # Y = L^-1 E', K = Y'Y, rhs, V_F update
    f += s ** 3 / 3 + 2 * s * s                       # Schur Cholesky + solves
    f += check(N, mode) + 2 * N * (N + 1) + 5 * N * (N + 1) + 2 * s * N   # certificate: slacks, gradient
    return f


def rollout(N: int) -> float:
    """Rollout, scheduling update (rho1/2/3) and convergence test."""
    return 10 * N + 20 * N + 3 * N


def per_step(N: int, mode: int, qps: float, tries: float, giruns: float, K: float, q: float,
             s: float) -> float:
    """Useful fp64 flops of one MPC step (one scenario k -> k+1)."""
    qbar = q / 2.0
    state_frac = (s / q) if (mode >= MODE_FULL and q > 0) else 0.0
    f = qps * (common_build(N, mode) + rollout(N))
    f += (tries + giruns) * polish(N, mode, q, s)
    f += giruns * (gi_setup(N) + check(N, mode))
    f += K * (gi_iteration(N, qbar, state_frac) + check(N, mode))
    return f + 30.0                                   # plant step


def hbm_bytes_per_step(N: int, workspace: bool = False) -> int:
    """Algorithmic HBM bytes of one MPC step (state in/out + outputs), SURVEY §8(d):
    x_k (2), rho in/out (2*3N), U_old in/out (2N), U (N), x_pred (2(N+1)),
    x_next (2) doubles + exitflag, inner_iters (int32); with ``workspace`` also
    the warm-start active sets in and out (2 x 2(N+1) int32, ntm_mpc_step_ws)."""
    ws = 2 * 4 * 2 * (N + 1) if workspace else 0
    return 8 * (2 + 6 * N + 2 * N + N + 2 * (N + 1) + 2) + 8 + ws

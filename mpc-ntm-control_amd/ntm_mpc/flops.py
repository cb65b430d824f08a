"""Algorithmic fp64 flop count of one MPC step of THIS build.

SURVEY.md §8(d) prices an IPM-based path (F_kkt per IPM iteration); this build
solves each QP with a Jacobi-scaled Goldfarb-Idnani dual active-set method
followed by an exact active-set polish, so it reports against its own count,
which is far below the survey's (a GI iteration costs O(N^2), an IPM iteration
O(N^3)).  Counts are the useful flops of the formulas as implemented (no
padding lanes, no masked work), from measured per-QP averages:
K = GI iterations, q = final active rows, s = general (state) active rows.
"""
from __future__ import annotations


def per_qp(N: int, mode: int, K: float, q: float, s: float) -> float:
    full = mode == 2
    f = 0.0
    f += 3 * N + 2 * N * (N - 1) + 12 * N                    # lift: A/B coefficients, Gamma, Phi/Lambda
    f += 8 * N                                               # free response e = Phi x + Lambda
    gram = 10 * N * (N + 1) * (N + 2) / 6                    # G = 2 Gamma' Om Gamma (lower)
    f += gram + 12 * N * (N + 1) / 2                         # + F
    f += N * (N + 1) + N + (3 * N * (N + 1) if full else 0)  # Jacobi scaling, state-row norms
    f += N ** 3 / 3 + N ** 3 / 3 + 4 * N * N                 # Cholesky, J = L^-T, unconstrained V
    if mode != 0:
        qbar = q / 2.0
        check = 2 * N + ((3 * N * (N + 1) + 12 * N) if full else 0)
        it = check + 2 * N * N + 6 * N * max(N - qbar, 0.0) + qbar * qbar + 8 * N
        f += K * it
    nF = max(N - (q - s), 0.0)
    f += gram + nF ** 3 / 3 + 4 * N * N                      # polish: G~ again, masked Cholesky, solves
    f += s * nF * nF + s * s * nF + s ** 3 / 3 + 4 * s * N    # Schur complement on the state rows
    f += 2 * N * N + (3 * N * (N + 1) if full else 2 * N)     # KKT certificate
    f += 8 * N + 20 * N                                      # rollout + rho update
    return f


def per_step(N: int, mode: int, qps: float, K: float, q: float, s: float) -> float:
    """qps = QP solves (inner iterations) per MPC step; K, q, s per QP."""
    return qps * per_qp(N, mode, K, q, s) + 30.0             # + plant step


def hbm_bytes_per_step(N: int) -> int:
    """Algorithmic HBM bytes of one MPC step (state in/out + outputs), SURVEY §8(d):
    x_k (2), rho in/out (2*3N), U_old in/out (2N), U (N), x_pred (2(N+1)),
    x_next (2) doubles + exitflag, inner_iters (int32)."""
    return 8 * (2 + 6 * N + 2 * N + N + 2 * (N + 1) + 2) + 8

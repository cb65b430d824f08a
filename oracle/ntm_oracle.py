"""CPU ORACLE for the batched LPV-MPC hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``mpc-ntm-control_amd/``) never routes through here and
fails loudly when its HIP library is missing.

It restates, in plain NumPy (plus mpmath for the exact QP polish), the
canonical ("CANON") semantics of the reference's receding-horizon loop
``NTM_MPC_Sim.m:93-131`` as repaired in SURVEY.md §2.1 (defects D1-D21).  Every
function cites the reference file:line it follows.  ``LITERAL_*`` switches
reproduce the literal reference behaviour where it is computable (D4, D6, D13,
D18) so the divergence can be quantified.

Parity pinning: the reference is MATLAB; MATLAB/Octave
are absent from this image, so the reference can be neither run nor imported
(absence, not a denial) and it ships no tests, fixtures or golden vectors.
``quadprog`` (MathWorks, closed source, no pinned version) cannot be run
either.  The oracle is therefore pinned by reference-derived invariants
(tests/test_oracle.py): the rollout identity Phi x0 + Gamma U + Lambda ==
rollout of NTM_MPC_Sim.m:113, LTI closed forms, the getWLc <-> per-step
constraint identity, the infeasible-x0 known answer (NTM_MPC_Sim.m:34 vs
:40-50), QP KKT certificates checked in 50-digit arithmetic, brute-force
active-set enumeration at small N, and the unconstrained LQ against an mpmath
solve.  The QP itself is "parity unpinned" against quadprog; it is pinned
against the exact (50-digit) KKT solution instead.
"""
from __future__ import annotations

import dataclasses
import math
from fractions import Fraction
from dataclasses import dataclass, field

import numpy as np

# --------------------------------------------------------------------------
# Physics / configuration  (NTM_MPC_Sim.m:5-60, 80-88)
# --------------------------------------------------------------------------


@dataclass
class Physics:
    """Physics constants, NTM_MPC_Sim.m:5-22 (same names, same units)."""

    j_BS: float = 73e3          # :5  [A/m^2]
    w_dep: float = 0.024        # :6  [m]
    w_marg: float = 0.02        # :7  [m]
    w_sat: float = 0.32         # :8  [m]
    tau_r: float = 293.0        # :9  [s]
    rs: float = 1.55            # :10 [m]
    a: float = 2.0              # :11 [m]
    eta_CD: float = 0.9         # :12
    tau_E0: float = 3.7         # :13 [s]
    tau_E: float = 3.7          # :14 (= tau_E0)
    mu0: float = 4e-7 * math.pi  # :15
    Lq: float = 0.87            # :16 [m]
    B_pol: float = 0.97         # :17 [T]
    m: float = 2.0              # :18
    Cw: float = 1.0             # :19
    tau_A0: float = 3e-6        # :20 [s]
    tau_w: float = 0.188        # :21 [s]
    omega0: float = 2 * math.pi * 420  # :22 [rad/s]

    def kappa(self) -> float:
        """NTM_MPC_Sim.m:24  kappa = 16*mu0*Lq*rs^2/(0.82*tau_r*B_pol*pi)."""
        return 16 * self.mu0 * self.Lq * self.rs ** 2 / (0.82 * self.tau_r * self.B_pol * math.pi)

    def zeta(self) -> float:
        """NTM_MPC_Sim.m:25  zeta = m*Cw*tau_A0^2*tau_w*a^3."""
        return self.m * self.Cw * self.tau_A0 ** 2 * self.tau_w * self.a ** 3


# constraint modes
MODE_NONE = 0   # unconstrained LQ (BASELINE config 1)
MODE_BOX = 1    # u in [umin, umax] only (BASELINE config 2)
MODE_FULL = 2   # full getWLc.m polyhedron (BASELINE config 3/4)
MODE_FULL_DU = 3  # getWLc rows + input-rate rows |U_i - U_{i-1}| <= du_max (BASELINE
                  # config 5; an extension of getWLc.m's row structure, not in the
                  # reference: parity for this mode is pinned only by this oracle)

# flags
LITERAL_PHI_RIGHTMUL = 1 << 0    # D4: Phi_j = Phi_{j-1} * A_j
LITERAL_GAMMA_INDEX = 1 << 1     # D6: Gamma_ij = A(rho_{i-j}) Gamma_{i-1,j}
LITERAL_PLANT_NO_C = 1 << 2      # D13: plant step without +C
RHO1_SQUARED = 1 << 3            # D18: rho1 = 1/(w^2 + w_marg^2) (rhos.m:18)


@dataclass
class Config:
    """Model / controller configuration, NTM_MPC_Sim.m:30-60, 80-88."""

    N: int = 3                                   # :30 prediction horizon
    Ts: float = 0.1                              # :31 sampling time
    xmin: tuple = (0.06, 100 * 2 * math.pi)      # :40,42,44
    xmax: tuple = (0.15, 5000 * 2 * math.pi)     # :41,43,45
    umin: float = 0.0                            # :47,49
    umax: float = 2e6                            # :48,50
    Q: tuple = (1.0, 0.0, 0.0, 1.0)              # :59 (row-major 2x2)
    r: tuple = (0.0, 1000 * 2 * math.pi)         # :60 reference state
    i_sim: int = 10                              # :81
    epsilon: float = 1e-14                       # :87
    mode: int = MODE_FULL
    flags: int = 0
    du_max: float = 5e5                          # MODE_FULL_DU only (W per step)
    Ru: float = 0.0                              # input weight (ABI v5); the reference: 0

    @property
    def m_rows(self) -> int:
        return constraint_rows(self.N, self.mode)


def constraint_rows(N: int, mode: int) -> int:
    if mode == MODE_NONE:
        return 0
    if mode == MODE_BOX:
        return 2 * N
    if mode == MODE_FULL_DU:
        return 8 * N + 2                          # getWLc rows + 2(N-1) rate rows
    return 6 * N + 4                              # getWLc.m:30-44


REFERENCE_X0 = np.array([0.0, 1000 * 2 * math.pi])   # NTM_MPC_Sim.m:34

# --------------------------------------------------------------------------
# L0: scheduling functions  (rho1.m, rho2.m, rho3.m)
# --------------------------------------------------------------------------


def rho1(x, w_marg, squared=False):
    """rho1.m:2  rho1 = 1/(x(1) + wmarg^2)   (D18: rhos.m:18 squares x(1))."""
    w = x[0]
    return 1.0 / ((w * w if squared else w) + w_marg ** 2)


def rho2(x):
    """rho2.m:2  rho2 = x(1)^2/x(2)."""
    return x[0] ** 2 / x[1]


def rho3(x, w_dep):
    """rho3.m:2-3  wstar = x(1)/w_dep; rational ECCD-efficiency fit."""
    ws = x[0] / w_dep
    return (0.25 + 0.24 * ws) / (1 + 1.5 * ws + 0.43 * ws ** 2 + 0.64 * ws ** 3)


def rho_all(x, phys: Physics, cfg: Config):
    """(rho1, rho2, rho3) at state x — NTM_MPC_Sim.m:63-65 / :114-116 (D1 repaired)."""
    return np.array([rho1(x, phys.w_marg, bool(cfg.flags & RHO1_SQUARED)),
                     rho2(x), rho3(x, phys.w_dep)])

# --------------------------------------------------------------------------
# L1: LPV matrices  (A.m, B.m, NTM_MPC_Sim.m:37)
# --------------------------------------------------------------------------


def A_mat(r1, r2, phys: Physics, Ts: float):
    """A.m:2  [[(4/3)(kappa rs/(0.82 taur)) Ts rho1 + 1, 0], [(rho2 Ts)/(zeta a^3), 1 - Ts/TE]]."""
    kappa, zeta = phys.kappa(), phys.zeta()
    a11 = (4 / 3) * (kappa * phys.rs / (0.82 * phys.tau_r)) * Ts * r1 + 1
    a21 = (r2 * Ts) / (zeta * phys.a ** 3)          # D19: zeta already holds a^3; kept
    a22 = 1 - Ts / phys.tau_E
    return np.array([[a11, 0.0], [a21, a22]])


def B_mat(r3, phys: Physics, Ts: float):
    """B.m:2  (kappa Ts etaCD / wdep) rho3, as the 2x1 column [b; 0] (D5)."""
    b = (phys.kappa() * Ts * phys.eta_CD / phys.w_dep) * r3
    return np.array([b, 0.0])


def C_vec(phys: Physics, Ts: float):
    """NTM_MPC_Sim.m:37  C = [-4/3 (kappa Ts j_BS w_sat)/(w_sat^2 + w_marg^2); Ts omega0/tau_E0]."""
    kappa = phys.kappa()
    c1 = -4 / 3 * (kappa * Ts * phys.j_BS * phys.w_sat) / (phys.w_sat ** 2 + phys.w_marg ** 2)
    c2 = Ts * phys.omega0 / phys.tau_E0
    return np.array([c1, c2])

# --------------------------------------------------------------------------
# L2: lifted prediction  (Rho_to_PhiGammaLambda.m)
# --------------------------------------------------------------------------


def lift(Rho, phys: Physics, cfg: Config):
    """Rho_to_PhiGammaLambda.m:1-54 under CANON D3-D6.

    Rho is 3xN (rows rho1, rho2, rho3; column i = predicted step i+1).
    Returns Phi (2N x 2), Gamma (2N x N), Lambda (2N,) with
    X = [x_1; ...; x_N] = Phi x0 + Gamma U + Lambda.
      Phi_1 = A_1,  Phi_i = A_i Phi_{i-1}               (:17-23, D4 left-multiply)
      Gamma_ii = B_i, Gamma_ij = A_i Gamma_{i-1,j}, j<i (:26-40, D6 index i)
      Lambda_1 = C,  Lambda_i = A_i Lambda_{i-1} + C    (:47-52)
    """
    N = Rho.shape[1]
    Ts = cfg.Ts
    C = C_vec(phys, Ts)
    As = [A_mat(Rho[0, i], Rho[1, i], phys, Ts) for i in range(N)]
    Bs = [B_mat(Rho[2, i], phys, Ts) for i in range(N)]
    Phi = np.zeros((2 * N, 2))
    Gamma = np.zeros((2 * N, N))
    Lam = np.zeros(2 * N)
    Phi[0:2] = As[0]
    for j in range(1, N):
        if cfg.flags & LITERAL_PHI_RIGHTMUL:
            Phi[2 * j:2 * j + 2] = Phi[2 * j - 2:2 * j] @ As[j]
        else:
            Phi[2 * j:2 * j + 2] = As[j] @ Phi[2 * j - 2:2 * j]
    Gamma[0:2, 0] = Bs[0]
    for i in range(1, N):
        for j in range(i + 1):
            if i != j:
                Ai = As[i - j - 1] if cfg.flags & LITERAL_GAMMA_INDEX else As[i]
                Gamma[2 * i:2 * i + 2, j] = Ai @ Gamma[2 * i - 2:2 * i, j]
            else:
                Gamma[2 * i:2 * i + 2, j] = Bs[j]
    Lam[0:2] = C
    for i in range(1, N):
        Lam[2 * i:2 * i + 2] = As[i] @ Lam[2 * i - 2:2 * i] + C
    return Phi, Gamma, Lam


def omega_blk(cfg: Config):
    """NTM_MPC_Sim.m:67-70  Omega = blkdiag(Q, ..., Q)."""
    Q = np.array(cfg.Q, dtype=float).reshape(2, 2)
    return np.kron(np.eye(cfg.N), Q)


def cost(Phi, Gamma, Lam, xk, cfg: Config):
    """NTM_MPC_Sim.m:71-73 / :120-121:  G = 2 Gamma' Omega Gamma,
    F = 2 Gamma' Omega (Phi x_k + Lambda - R), R = [r; ...; r] (D8), x_k not x0 (D12).
    With an input weight R_u (D17, "Q, R_u exposed in config"; the reference has none,
    NTM_MPC_Sim.m:59,72) the cost sum x'Qx + R_u u^2 adds 2 R_u I to G; F is unchanged."""
    Om = omega_blk(cfg)
    R = np.tile(np.array(cfg.r, dtype=float), cfg.N)
    G = 2 * Gamma.T @ Om @ Gamma
    if cfg.Ru != 0.0:
        G = G + 2 * cfg.Ru * np.eye(cfg.N)
    F = 2 * Gamma.T @ Om @ (Phi @ xk + Lam - R)
    return G, F

# --------------------------------------------------------------------------
# L2': constraint lifting  (getWLc.m)
# --------------------------------------------------------------------------


def getWLc(xmax, xmin, umax, umin, Gamma, Phi, Lam):
    """getWLc.m:1-63 (7-arg semantics, D9) with the Ccal fix D10.

    Constraint L U <= c + W x_k with m = 6N+4 rows: per step i = 0..N-1 the
    block [-u_i <= -umin; u_i <= umax; -x_i <= -xmin; x_i <= xmax] and the
    terminal block [-x_N <= -xmin; x_N <= xmax].
    """
    xmax = np.atleast_1d(np.asarray(xmax, dtype=float))
    xmin = np.atleast_1d(np.asarray(xmin, dtype=float))
    umax = np.atleast_1d(np.asarray(umax, dtype=float))
    umin = np.atleast_1d(np.asarray(umin, dtype=float))
    nu, nx = umin.shape[0], xmin.shape[0]
    N = Phi.shape[0] // nx
    Mi = np.vstack([np.zeros((nu, nx)), np.zeros((nu, nx)), -np.eye(nx), np.eye(nx)])   # :9-12
    Ei = np.vstack([-np.eye(nu), np.eye(nu), np.zeros((nx, nu)), np.zeros((nx, nu))])   # :14-17
    bi = np.concatenate([-umin, umax, -xmin, xmax])                                     # :20-23
    MN = np.vstack([-np.eye(nx), np.eye(nx)])                                           # :25
    bN = np.concatenate([-xmin, xmax])                                                  # :26
    ri, rN = Mi.shape[0], MN.shape[0]
    m = ri * N + rN
    Dcal = np.zeros((m, nx))                                                            # :30
    Dcal[:ri] = Mi
    Mcal = np.zeros((m, nx * N))                                                        # :33-37
    for i in range(1, N):
        Mcal[ri * i:ri * (i + 1), nx * (i - 1):nx * i] = Mi
    Mcal[ri * N:, nx * (N - 1):] = MN
    Ecal = np.zeros((m, nu * N))                                                        # :40-44
    for i in range(N):
        Ecal[ri * i:ri * (i + 1), nu * i:nu * (i + 1)] = Ei
    Ccal = np.concatenate([np.tile(bi, N), bN])                                         # :51-55 (D10)
    L = Mcal @ Gamma + Ecal                                                             # :57
    W = -Dcal - Mcal @ Phi                                                              # :58
    c = Ccal - Mcal @ Lam                                                               # :59
    return W, L, c


def constraints(Phi, Gamma, Lam, xk, cfg: Config):
    """The QP's inequality system Lin U <= b for the configured mode."""
    N = cfg.N
    if cfg.mode == MODE_NONE:
        return np.zeros((0, N)), np.zeros(0)
    if cfg.mode == MODE_BOX:
        Lin = np.vstack([-np.eye(N), np.eye(N)])
        b = np.concatenate([np.full(N, -cfg.umin), np.full(N, cfg.umax)])
        return Lin, b
    W, L, c = getWLc(cfg.xmax, cfg.xmin, cfg.umax, cfg.umin, Gamma, Phi, Lam)
    Lin, b = L, c + W @ xk                                                              # NTM_MPC_Sim.m:97
    if cfg.mode == MODE_FULL_DU:
        Lin, b = np.vstack([Lin, rate_rows(N)]), np.concatenate([b, np.full(2 * (N - 1), cfg.du_max)])
    return Lin, b


def rate_rows(N):
    """Input-rate rows appended after getWLc's 6N+4 (config 5): for i = 1..N-1,
    row 2(i-1):  U_i - U_{i-1} <= du_max;  row 2(i-1)+1:  U_{i-1} - U_i <= du_max."""
    R = np.zeros((2 * (N - 1), N))
    for i in range(1, N):
        R[2 * (i - 1), i], R[2 * (i - 1), i - 1] = 1.0, -1.0
        R[2 * (i - 1) + 1, i], R[2 * (i - 1) + 1, i - 1] = -1.0, 1.0
    return R

# --------------------------------------------------------------------------
# L2'': QP  (quadprog call site NTM_MPC_Sim.m:97; exitflag :98-103)
# --------------------------------------------------------------------------

EXIT_OK, EXIT_MAXIT, EXIT_INFEASIBLE, EXIT_NONFINITE = 1, 0, -2, -7
GI_DEP_TOL = 1e-8
# A constant row (Lin_i == 0) is violated when b_i < -CONST_ROW_TOL (DESIGN.md
# D22): quadprog judges feasibility to a tolerance, and the closed loop's plant
# step can leave x_{k+1} one ulp outside a bound the plan held it at.
CONST_ROW_TOL = 1e-9


def _givens(a, b):
    h = math.hypot(a, b)
    if h == 0.0:
        return 1.0, 0.0, 0.0
    return a / h, b / h, h


def qp_dual_active_set(G, F, Lin, b, max_iter=None):
    """Goldfarb-Idnani dual active-set method (own restatement of the 1983
    algorithm) for  min 1/2 U'GU + F'U  s.t.  Lin U <= b.

    This is the oracle's stand-in for MathWorks ``quadprog`` (NTM_MPC_Sim.m:97),
    which is closed source and absent.  Returns (U, exitflag, active_rows,
    multipliers, iterations).  Constant rows (Lin_i == 0, e.g. the x_0 rows of
    getWLc) are checked directly: 0 <= b_i (to CONST_ROW_TOL) or the problem is
    infeasible (D15, D22).
    """
    n = G.shape[0]
    m = Lin.shape[0]
    if max_iter is None:
        max_iter = 10 * (n + m) + 50
    if not (np.all(np.isfinite(G)) and np.all(np.isfinite(F)) and np.all(np.isfinite(Lin))
            and np.all(np.isfinite(b))):
        return np.zeros(n), EXIT_NONFINITE, [], np.zeros(0), 0
    # GI form: n_i' U >= b_i   with n_i = -Lin_i, b_i = -b
    Nc = -Lin
    bc = -b
    nonzero = np.any(Nc != 0.0, axis=1)
    if np.any((~nonzero) & (bc > CONST_ROW_TOL)):   # 0 >= bc violated  -> infeasible (D15, D22)
        return np.zeros(n), EXIT_INFEASIBLE, [], np.zeros(0), 0
    nrm = np.linalg.norm(Nc, axis=1)
    try:
        Lc = np.linalg.cholesky(G)
    except np.linalg.LinAlgError:
        return np.zeros(n), EXIT_NONFINITE, [], np.zeros(0), 0
    J = np.linalg.inv(Lc).T                      # G^{-1} = J J'
    U = -(J @ (J.T @ F))
    R = np.zeros((n, n))
    act: list[int] = []
    u = np.zeros(0)
    it = 0
    while True:
        s = Nc @ U - bc
        # constant rows were checked above (never candidates), active rows are held
        viol = np.where(nonzero, s / np.where(nrm > 0, nrm, 1.0), np.inf)
        if act:
            viol[act] = np.inf
        p = int(np.argmin(viol))
        # stop when the worst row is satisfied to 1e-12 of its own scale
        if viol[p] == np.inf or s[p] >= -1e-12 * max(nrm[p] * np.max(np.abs(U), initial=1.0), abs(bc[p])):
            return U, EXIT_OK, act, u, it
        up = np.append(u, 0.0)
        while True:
            it += 1
            if it > max_iter:
                return U, EXIT_MAXIT, act, up[:len(act)], it
            q = len(act)
            d = J.T @ Nc[p]
            z = J[:, q:] @ d[q:]
            r = np.linalg.solve(np.triu(R[:q, :q]), d[:q]) if q else np.zeros(0)
            t1, l = math.inf, -1
            for j in range(q):
                if r[j] > 0.0:
                    tj = up[j] / r[j]
                    if tj < t1:
                        t1, l = tj, j
            # z'n_p = |d2|^2 (z = J2 d2): never negative; n_p counts as dependent
            # on the active rows when |d2| <= GI_DEP_TOL |d|
            zn = float(d[q:] @ d[q:])
            sp = float(Nc[p] @ U - bc[p])
            t2 = math.inf if zn <= 1e-300 or math.sqrt(zn) <= GI_DEP_TOL * np.linalg.norm(d) else -sp / zn
            t = min(t1, t2)
            if t == math.inf:
                return np.zeros(n), EXIT_INFEASIBLE, act, up[:q], it
            if t2 == math.inf:
                up[:q] = np.maximum(0.0, up[:q] - t * r)
                up[q] += t
                J, R = _drop(J, R, q, l)
                act.pop(l)
                up = np.delete(up, l)
                continue
            U = U + t * z
            up[:q] = np.maximum(0.0, up[:q] - t * r)
            up[q] += t
            if t == t2:
                J, R = _add(J, R, q, d)
                act.append(p)
                u = up
                break
            J, R = _drop(J, R, q, l)
            act.pop(l)
            up = np.delete(up, l)


def _add(J, R, q, d):
    n = J.shape[0]
    J = J.copy()
    R = R.copy()
    d = d.copy()
    for k in range(n - 1, q, -1):
        c, s, h = _givens(d[k - 1], d[k])
        d[k - 1], d[k] = h, 0.0
        jk1, jk = J[:, k - 1].copy(), J[:, k].copy()
        J[:, k - 1] = c * jk1 + s * jk
        J[:, k] = -s * jk1 + c * jk
    R[:q + 1, q] = d[:q + 1]
    return J, R


def _drop(J, R, q, l):
    J = J.copy()
    R = R.copy()
    R[:, l:q - 1] = R[:, l + 1:q]
    R[:, q - 1] = 0.0
    for j in range(l, q - 1):
        c, s, h = _givens(R[j, j], R[j + 1, j])
        rj, rj1 = R[j, j:].copy(), R[j + 1, j:].copy()
        R[j, j:] = c * rj + s * rj1
        R[j + 1, j:] = -s * rj + c * rj1
        R[j + 1, j] = 0.0
        jj, jj1 = J[:, j].copy(), J[:, j + 1].copy()
        J[:, j] = c * jj + s * jj1
        J[:, j + 1] = -s * jj + c * jj1
    return J, R


def kkt_polish(G, F, Lin, b, act, dps=50):
    """Exact solve of the equality-constrained QP on the active rows in
    ``dps``-digit arithmetic (mpmath): [G  Lin_A'; Lin_A 0][U; lam] = [-F; b_A].
    The fp64 data are taken as exact binary fractions, so the result is the
    exact KKT point of the fp64 QP (rounded once to fp64).  Returns (U, lam,
    certificate dict with max primal violation and min multiplier)."""
    import mpmath as mp
    n = G.shape[0]
    q = len(act)
    with mp.workdps(dps):
        K = mp.zeros(n + q, n + q)
        rhs = mp.zeros(n + q, 1)
        for i in range(n):
            for j in range(n):
                K[i, j] = mp.mpf(float(G[i, j]))
            rhs[i] = -mp.mpf(float(F[i]))
        for a_, row in enumerate(act):
            for j in range(n):
                v = mp.mpf(float(Lin[row, j]))
                K[n + a_, j] = v
                K[j, n + a_] = v
            rhs[n + a_] = mp.mpf(float(b[row]))
        sol = mp.lu_solve(K, rhs)
        Um = [sol[i] for i in range(n)]
        lam = [sol[n + a_] for a_ in range(q)]
        viol = mp.mpf(0)
        for i in range(Lin.shape[0]):
            srow = mp.fsum(mp.mpf(float(Lin[i, j])) * Um[j] for j in range(n)) - mp.mpf(float(b[i]))
            scale = max(mp.mpf(1), abs(mp.mpf(float(b[i]))))
            viol = max(viol, srow / scale)
        lam_min = min(lam) if q else mp.mpf(0)
        U = np.array([float(v) for v in Um])
        return U, np.array([float(v) for v in lam]), {"max_violation": float(viol),
                                                      "min_multiplier": float(lam_min)}


def _chol_lower(A):
    """Left-looking Cholesky (the order the GPU and the C oracle use); None if not PD."""
    n = A.shape[0]
    L = np.zeros_like(A)
    for k in range(n):
        s = A[k:, k] - L[k:, :k] @ L[k, :k]
        if not s[0] > 0.0:
            return None
        lk = math.sqrt(s[0])
        L[k, k] = lk
        L[k + 1:, k] = s[1:] / lk
    return L


def _fwd(L, b):
    x = np.zeros_like(b, dtype=float)
    for i in range(L.shape[0]):
        x[i] = (b[i] - L[i, :i] @ x[:i]) / L[i, i]
    return x


def _bwd(L, b):
    """Solve L' x = b (L lower)."""
    n = L.shape[0]
    x = np.zeros_like(b, dtype=float)
    for i in range(n - 1, -1, -1):
        x[i] = (b[i] - L[i + 1:, i] @ x[i + 1:]) / L[i, i]
    return x


POLISH_PRIMAL_TOL = 1e-9
POLISH_DUAL_TOL = 1e-9


def polish_active_set(Gs, Fs, Ns, bcs, act, Lin, b, Dv):
    """Exact re-solve of the scaled QP on GI's final active set.

    Rows with a single non-zero (u bounds, and the w-rows of x_1 which only
    see u_0) fix their variable: U_j = b_a / Lin_aj exactly.  The remaining
    active rows S are equality constraints on the free variables F:
        min 1/2 V_F' G~_FF V_F + g_F' V_F  s.t.  E V_F = h
    solved with a fresh Cholesky of G~_FF (B rows/cols masked to identity)
    and of the Schur complement K = E G~_FF^{-1} E'.  The result is accepted
    only if it passes the KKT check (primal slack, multiplier signs); returns
    (V, U, ok)."""
    n = Gs.shape[0]
    fixed = np.zeros(n, dtype=bool)
    Vb = np.zeros(n)
    Ufix = np.zeros(n)
    S = []
    for a in act:
        nz = np.flatnonzero(Lin[a])
        if len(nz) == 1:
            j = nz[0]
            Ufix[j] = b[a] / Lin[a, j]
            Vb[j] = Ufix[j] / Dv[j]
            fixed[j] = True
        else:
            S.append(a)
    free = np.flatnonzero(~fixed)
    if S and len(S) == len(free):
        # Square, triangular E (the device's polish_compact square path): the
        # active general rows alone determine the free variables.  Sorted by their
        # last free column E is lower triangular: V_F by forward substitution, the
        # multipliers by back substitution on E' mu = grad_F (same order of
        # operations as the device and oracle/ntm_oracle.c).
        nS = len(S)
        perm = [-1] * nS
        for k, a in enumerate(S):
            nzf = np.flatnonzero(Ns[a, free] != 0.0)
            last = int(nzf[-1]) if len(nzf) else -1
            if last < 0 or perm[last] >= 0:
                perm = None
                break
            perm[last] = k
        if perm is not None:
            rows = [S[k] for k in perm]
            E = np.array([[Ns[r, free[c]] if c <= t else 0.0 for c in range(nS)] for t, r in enumerate(rows)])
            acc = np.array([bcs[r] - Ns[r, fixed] @ Vb[fixed] for r in rows])
            sqid = 1.0 / np.diag(E)
            V = Vb.copy()
            for t in range(nS):
                xt = acc[t] * sqid[t]
                V[free[t]] = xt
                acc[t + 1:] -= E[t + 1:, t] * xt
            grad = Gs @ V + Fs
            acc = grad[free].copy()
            mu = np.zeros(nS)
            for u in range(nS - 1, -1, -1):
                mu_u = acc[u] * sqid[u]
                mu[perm[u]] = mu_u
                acc[:u] -= E[u, :u] * mu_u
            return _polish_certify(Gs, Fs, Ns, bcs, act, Lin, Dv, S, fixed, Ufix, V, mu)
    g = Fs + Gs[:, fixed] @ Vb[fixed]
    Gm = Gs.copy()
    Gm[fixed, :] = 0.0
    Gm[:, fixed] = 0.0
    Gm[fixed, fixed] = 1.0
    gm = np.where(fixed, 0.0, g)
    Lc = _chol_lower(Gm)
    if Lc is None:
        return None, None, False
    w = _fwd(Lc, gm)
    mu = np.zeros(0)
    if S:
        E = Ns[S].copy()
        h = bcs[S] - E[:, fixed] @ Vb[fixed]
        E[:, fixed] = 0.0
        Y = np.stack([_fwd(Lc, E[k]) for k in range(len(S))], axis=1)     # n x nS
        K = Y.T @ Y
        Lk = _chol_lower(K)
        if Lk is None:
            return None, None, False
        mu = _bwd(Lk, _fwd(Lk, h + Y.T @ w))
        V = _bwd(Lc, Y @ mu - w)
    else:
        V = _bwd(Lc, -w)
    V = np.where(fixed, Vb, V)
    return _polish_certify(Gs, Fs, Ns, bcs, act, Lin, Dv, S, fixed, Ufix, V, mu)


def _polish_certify(Gs, Fs, Ns, bcs, act, Lin, Dv, S, fixed, Ufix, V, mu):
    """KKT certificate of an active-set re-solve: primal slack on every
    non-constant row, multiplier signs.  Returns (V, U, ok)."""
    U = np.where(fixed, Ufix, V * Dv)
    nzr = np.any(Ns != 0.0, axis=1)
    slack = Ns @ V - bcs
    vmax = max(1.0, float(np.max(np.abs(V))))
    if np.any(nzr & (slack < -POLISH_PRIMAL_TOL * np.maximum(vmax, np.abs(bcs)))):
        return V, U, False
    grad = Gs @ V + Fs
    res = grad - (Ns[S].T @ mu if S else 0.0)
    lam = []
    for a in act:
        if a in S:
            continue
        j = np.flatnonzero(Lin[a])[0]
        lam.append(res[j] / Ns[a, j])
    mults = np.concatenate([mu, np.asarray(lam)])
    scale = max(1.0, float(np.max(np.abs(mults))) if len(mults) else 1.0)
    if len(mults) and np.min(mults) < -POLISH_DUAL_TOL * scale:
        return V, U, False
    return V, U, True


def _ge_solve_ld(M, rhs):
    """Gaussian elimination with partial pivoting in extended precision
    (np.longdouble: the x87 80-bit format, 64-bit significand, on x86-64, the
    same type as the C oracle's ``long double``).  None when a pivot vanishes."""
    A = np.array(M, dtype=np.longdouble)
    x = np.array(rhs, dtype=np.longdouble)
    n = A.shape[0]
    for k in range(n):
        p = k + int(np.argmax(np.abs(A[k:, k])))
        if not A[p, k] != 0:
            return None
        if p != k:
            A[[k, p]] = A[[p, k]]
            x[[k, p]] = x[[p, k]]
        f = A[k + 1:, k] / A[k, k]
        A[k + 1:, k:] -= f[:, None] * A[k, k:][None, :]
        x[k + 1:] -= f * x[k]
    for k in range(n - 1, -1, -1):
        x[k] = (x[k] - A[k, k + 1:] @ x[k + 1:]) / A[k, k]
    return x


def accurate_resolve(G, F, Lin, b, act, U):
    """Accurate equality-constrained re-solve on a final active set.

    The fp64 re-solves (polish_active_set) factor G~_FF by Cholesky and form the
    Schur complement, which loses digits when G~_FF is nearly singular although
    the KKT system itself is well conditioned (with input-rate rows the last two
    inputs act almost alike: cond(G) ~1e11, re-solve errors up to ~6e-9 umax while
    a one-ulp perturbation of the data moves the exact optimum by ~1e-16 umax).
    This solves the KKT system of the free variables directly,
        [G~_FF  N_SF'] [V_F ]   [-(F~_F + G~_FB V_B)]
        [N_SF   0    ] [-mu ] = [  bc_S - N_SB V_B  ]
    (Jacobi-scaled variables, unit-norm rows, all formed from the fp64 data in
    long double), by partial-pivoting elimination in long double plus one
    refinement step.  Variables fixed by single-entry rows keep U_j = b_a / Lin_aj
    exactly.  Returns U (fp64), or the given U if the system is singular."""
    n = G.shape[0]
    act = [int(a) for a in act]
    if not act:
        return U
    LD = np.longdouble
    Dv = jacobi_scale(G).astype(LD)
    fixed = np.zeros(n, dtype=bool)
    Ufix = np.zeros(n)
    S = []
    for a in act:
        nz = np.flatnonzero(Lin[a])
        if len(nz) == 1:
            j = nz[0]
            Ufix[j] = b[a] / Lin[a, j]
            fixed[j] = True
        elif len(nz) > 1:
            S.append(a)
    free = np.flatnonzero(~fixed)
    nF, nS = len(free), len(S)
    if nF == 0:
        return np.where(fixed, Ufix, U)
    Gs = G.astype(LD) * Dv[:, None] * Dv[None, :]
    Vb = np.where(fixed, Ufix.astype(LD) / Dv, LD(0))
    g = F.astype(LD) * Dv + Gs[:, fixed] @ Vb[fixed]
    M = np.zeros((nF + nS, nF + nS), dtype=LD)
    rhs = np.zeros(nF + nS, dtype=LD)
    M[:nF, :nF] = Gs[np.ix_(free, free)]
    rhs[:nF] = -g[free]
    if nS:
        Ls = Lin[S].astype(LD) * Dv[None, :]
        rn = np.sqrt(np.sum(Ls * Ls, axis=1))
        Ns = Ls / rn[:, None]
        bs = b[S].astype(LD) / rn
        M[nF:, :nF] = Ns[:, free]
        M[:nF, nF:] = Ns[:, free].T
        rhs[nF:] = bs - Ns[:, fixed] @ Vb[fixed]
    sol = _ge_solve_ld(M, rhs)
    if sol is None:
        return U
    res = rhs - M @ sol
    corr = _ge_solve_ld(M, res)
    if corr is not None:
        sol = sol + corr
    Uo = np.where(fixed, Ufix, 0.0)
    Uo[free] = np.asarray(sol[:nF] * Dv[free], dtype=np.float64)
    if not np.all(np.isfinite(Uo)):
        return U
    return Uo


def jacobi_scale(G):
    """D = diag(1/sqrt(G_jj)) (1 where G_jj <= 0)."""
    dg = np.diag(G)
    return np.where(dg > 0.0, 1.0 / np.sqrt(np.where(dg > 0.0, dg, 1.0)), 1.0)


def qp_solve(G, F, Lin, b, polish=False):
    """quadprog stand-in (NTM_MPC_Sim.m:97) -> (U, exitflag, info).

    exitflag follows quadprog: 1 optimal, 0 max iterations, -2 infeasible
    (U returned as zeros, D16), -7 non-finite data (build-specific)."""
    n = G.shape[0]
    if Lin.shape[0] == 0:
        try:
            U = np.linalg.solve(G, -F)
        except np.linalg.LinAlgError:
            return np.zeros(n), EXIT_NONFINITE, {}
        flag = EXIT_OK if np.all(np.isfinite(U)) else EXIT_NONFINITE
        if polish and flag == EXIT_OK:
            U, _, cert = kkt_polish(G, F, Lin, b, [])
            return U, flag, {"active": [], "cert": cert}
        return (U if flag == EXIT_OK else np.zeros(n)), flag, {"active": []}
    # Jacobi variable scaling U = D V (diag(D G D) = 1) and unit-norm rows:
    # cond(G) ~ 1e9-1e11 drops to ~1e6, which keeps the dual active set
    # method stable at the near-degenerate vertices this problem produces.
    Dv = jacobi_scale(G)
    Gs = G * Dv[:, None] * Dv[None, :]
    Ls = Lin * Dv[None, :]
    rn = np.linalg.norm(Ls, axis=1)
    rn = np.where(rn > 0.0, rn, 1.0)
    Ns, bcs, Fs = -(Ls / rn[:, None]), -(b / rn), F * Dv
    V, flag, act, lam, its = qp_dual_active_set(Gs, Fs, -Ns, -bcs)
    U = V * Dv
    polished = False
    if flag == EXIT_OK:
        Vp, Up, ok = polish_active_set(Gs, Fs, Ns, bcs, act, Lin, b, Dv)
        if ok:
            U, polished = Up, True
        # the value on the final active set, accurate to the fp64 data
        U = accurate_resolve(G, F, Lin, b, act, U)
    lam = np.asarray(lam) / rn[act] if len(act) else np.asarray(lam)
    info = {"active": list(act), "iters": its, "multipliers": lam, "polished": polished}
    if flag == EXIT_OK and polish:
        U, lam, cert = kkt_polish(G, F, Lin, b, act)
        info["multipliers"] = lam
        info["cert"] = cert
    if flag != EXIT_OK:
        U = np.zeros(n) if flag in (EXIT_INFEASIBLE, EXIT_NONFINITE) else U
    return U, flag, info

# --------------------------------------------------------------------------
# L3: rollout, inner iteration, closed loop  (NTM_MPC_Sim.m:93-131)
# --------------------------------------------------------------------------


def rollout(xk, Rho, U, phys: Physics, cfg: Config):
    """NTM_MPC_Sim.m:110-117: x_0 = x_k; x_i = A(rho_i) x_{i-1} + B(rho_i) U_i + C,
    then rho_i <- rho(x_{i-1}).  Returns (xpred 2x(N+1), Rho_new 3xN)."""
    N = cfg.N
    C = C_vec(phys, cfg.Ts)
    xp = np.zeros((2, N + 1))
    xp[:, 0] = xk
    Rn = Rho.copy()
    for i in range(N):
        xp[:, i + 1] = (A_mat(Rn[0, i], Rn[1, i], phys, cfg.Ts) @ xp[:, i]
                        + B_mat(Rn[2, i], phys, cfg.Ts) * U[i] + C)
        Rn[:, i] = rho_all(xp[:, i], phys, cfg)
    return xp, Rn


def plant_step(xk, uk, phys: Physics, cfg: Config):
    """NTM_MPC_Sim.m:130 (D13): x_{k+1} = A(rho(x_k)) x_k + B(rho(x_k)) u_k + C."""
    rr = rho_all(xk, phys, cfg)
    xn = A_mat(rr[0], rr[1], phys, cfg.Ts) @ xk + B_mat(rr[2], phys, cfg.Ts) * uk
    if not (cfg.flags & LITERAL_PLANT_NO_C):
        xn = xn + C_vec(phys, cfg.Ts)
    return xn


def initial_rho(x0, phys: Physics, cfg: Config):
    """NTM_MPC_Sim.m:63-65: Rho = repmat(rho(x0), 1, N)."""
    return np.tile(rho_all(np.asarray(x0, dtype=float), phys, cfg)[:, None], (1, cfg.N))


def mpc_step(xk, Rho, Uold, phys: Physics, cfg: Config, polish=False, dist=None):
    """One MPC time step for one scenario: NTM_MPC_Sim.m:94-130 (CANON ordering
    per SURVEY.md §2.1: build -> QP -> rollout -> rho update -> convergence).

    Returns dict: U (N), u (scalar U(1)), xpred (2x(N+1)), xnext (2), Rho (3xN,
    carried unshifted, D20), Uold (N, persists across k, D14), exitflag,
    inner_iters."""
    xk = np.asarray(xk, dtype=float)
    Rho = np.array(Rho, dtype=float)
    Uold = np.array(Uold, dtype=float)
    U = np.zeros(cfg.N)
    flag = EXIT_OK
    xp = None
    it = 0
    for it in range(1, cfg.i_sim + 1):
        Phi, Gam, Lam = lift(Rho, phys, cfg)
        G, F = cost(Phi, Gam, Lam, xk, cfg)
        Lin, bvec = constraints(Phi, Gam, Lam, xk, cfg)
        U, flag, _ = qp_solve(G, F, Lin, bvec, polish=polish)
        xp, Rho = rollout(xk, Rho, U, phys, cfg)
        if np.sum(np.abs(Uold - U)) < cfg.epsilon:           # :123
            break                                            # :125, before :127
        Uold = U.copy()                                      # :127 (skipped on break)
    xn = plant_step(xk, U[0], phys, cfg)
    if dist is not None:                                     # scenario generator (plant only)
        xn = np.array([xn[0] + dist[0] if dist[0] != 0.0 else xn[0],
                       xn[1] + dist[1] if dist[1] != 0.0 else xn[1]])
    return {"U": U, "u": U[0], "xpred": xp, "xnext": xn, "Rho": Rho, "Uold": Uold,
            "exitflag": flag, "inner_iters": it}


def closed_loop(x0, phys: Physics, cfg: Config, k_sim=20, polish=False, gen=None, sid=0):
    """NTM_MPC_Sim.m:80-131 for one scenario.  Returns the workspace
    variables xk (2 x k_sim+1), uk (k_sim), Uk (N x k_sim) plus per-step
    exitflag / inner iteration counts and the last predicted trajectories.
    ``gen`` (ScenarioGen) makes it global scenario ``gen.first_id + sid``:
    its own plasma (scenario_physics) and plant disturbances at time indices
    gen.k0 + k."""
    N = cfg.N
    if gen is not None:
        phys = scenario_physics(phys, gen, gen.first_id + sid)
    xk = np.zeros((2, k_sim + 1))
    xk[:, 0] = x0
    uk = np.zeros(k_sim)
    Uk = np.zeros((N, k_sim))
    xpred = np.zeros((k_sim, 2, N + 1))
    flags = np.zeros(k_sim, dtype=np.int32)
    iters = np.zeros(k_sim, dtype=np.int32)
    Rho = initial_rho(x0, phys, cfg)
    Uold = np.full(N, np.inf)                                 # D14
    for k in range(k_sim):
        d = None if gen is None else disturbance(gen, gen.first_id + sid, gen.k0 + k)
        out = mpc_step(xk[:, k], Rho, Uold, phys, cfg, polish=polish, dist=d)
        Rho, Uold = out["Rho"], out["Uold"]
        Uk[:, k] = out["U"]
        uk[k] = out["u"]
        xpred[k] = out["xpred"]
        flags[k] = out["exitflag"]
        iters[k] = out["inner_iters"]
        xk[:, k + 1] = out["xnext"]
    return {"xk": xk, "uk": uk, "Uk": Uk, "xpred": xpred, "exitflag": flags,
            "inner_iters": iters, "Rho": Rho, "Uold": Uold}

# --------------------------------------------------------------------------
# Synthetic scenario generator: counter-based, shard-invariant
# --------------------------------------------------------------------------


def _splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def scenario_x0(ids, seed=20241220):
    """Initial states for global scenario ids: w0 ~ U[0.07, 0.14] m,
    omega0 ~ U[0.8, 1.2] * 2000 pi rad/s.  Counter-based (splitmix64 of
    seed, id, stream) so any shard reproduces the same scenario; the same
    generator is implemented in the C-ABI (ntm_scenarios_x0)."""
    ids = np.asarray(ids, dtype=np.uint64)
    out = np.zeros((ids.shape[0], 2))
    for k, s in enumerate(ids.tolist()):
        base = (seed * 0x100000001B3 + s * 2) & 0xFFFFFFFFFFFFFFFF
        r0 = _splitmix64(base) >> 11
        r1 = _splitmix64((base + 1) & 0xFFFFFFFFFFFFFFFF) >> 11
        u0 = r0 * (1.0 / 9007199254740992.0)
        u1 = r1 * (1.0 / 9007199254740992.0)
        out[k, 0] = 0.07 + 0.07 * u0
        out[k, 1] = (0.8 + 0.4 * u1) * 2000 * math.pi
    return out


# --------------------------------------------------------------------------
# Scenario generator (include/ntm_mpc.h ntm_scenario_gen): independent plasma
# scenarios (j_BS, w_dep of NTM_MPC_Sim.m:5-6) and plant disturbance
# realisations (added to the plant step NTM_MPC_Sim.m:130), counter-based on
# (seed, global scenario id, time index)
# --------------------------------------------------------------------------
_M64 = 0xFFFFFFFFFFFFFFFF
GEN_PARAM_K = 0xFFFFFFFF


@dataclass
class ScenarioGen:
    seed: int = 20241220
    first_id: int = 0
    k0: int = 0
    sigma_w: float = 0.0          # [m] per plant step
    sigma_omega: float = 0.0      # [rad/s] per plant step
    jbs_spread: float = 0.0       # j_BS (1 + spread (2u - 1))
    wdep_spread: float = 0.0      # w_dep (1 + spread (2u - 1))


def gen_u01(seed, sid, k, ch):
    """Uniform [0, 1): splitmix64 chain over (seed, id, k, ch)."""
    h = _splitmix64((seed ^ 0xD1B54A32D192ED03) & _M64)
    h = _splitmix64(h ^ (sid & _M64))
    h = _splitmix64(h ^ ((((k & 0xFFFFFFFF) << 8) | ch) & _M64))
    return (h >> 11) * (1.0 / 9007199254740992.0)


def gen_normal(seed, sid, k, c):
    """Irwin-Hall(4) unit-variance sample, channel c (sub-channels 4c..4c+3)."""
    s = gen_u01(seed, sid, k, 4 * c)
    s = s + gen_u01(seed, sid, k, 4 * c + 1)
    s = s + gen_u01(seed, sid, k, 4 * c + 2)
    s = s + gen_u01(seed, sid, k, 4 * c + 3)
    return (s - 2.0) * 1.7320508075688772


def gen_factor(seed, sid, c, spread):
    """1 + spread (2u - 1) with ONE rounding (a fused multiply-add, as the C-ABI and the
    device compute it): exact rational arithmetic, then one correctly rounded float()."""
    t = 2.0 * gen_u01(seed, sid, GEN_PARAM_K, c) - 1.0          # exact
    return float(Fraction(spread) * Fraction(t) + 1)


def scenario_physics(phys: Physics, gen: ScenarioGen, sid: int) -> Physics:
    """Global scenario sid's plasma: j_BS and w_dep scaled by their factors."""
    return dataclasses.replace(phys, j_BS=phys.j_BS * gen_factor(gen.seed, sid, 0, gen.jbs_spread),
                               w_dep=phys.w_dep * gen_factor(gen.seed, sid, 1, gen.wdep_spread))


def disturbance(gen: ScenarioGen, sid: int, k: int):
    """Additive plant disturbance [d_w, d_omega] of scenario sid at time index k."""
    dw = gen.sigma_w * gen_normal(gen.seed, sid, k, 0) if gen.sigma_w != 0.0 else 0.0
    do = gen.sigma_omega * gen_normal(gen.seed, sid, k, 1) if gen.sigma_omega != 0.0 else 0.0
    return np.array([dw, do])

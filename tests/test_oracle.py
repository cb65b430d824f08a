"""Pin the CPU oracle (oracle/ntm_oracle.py) to the reference.

The MATLAB reference cannot run here and ships no tests or golden vectors
(SURVEY.md §4), so the oracle is pinned by invariants derived from the
reference's own code, each test citing the lines it follows, plus
50-digit KKT certificates for the QP (quadprog itself is unavailable:
"parity unpinned" against quadprog, pinned against the exact optimum).
"""
import itertools
import math
from pathlib import Path

import numpy as np
import pytest

from oracle import cbind
from oracle import ntm_oracle as O

GOLD = Path(__file__).resolve().parent / "golden"
PH = O.Physics()


def cfg(N=3, mode=O.MODE_FULL, **kw):
    return O.Config(N=N, mode=mode, **kw)


def rand_rho(N, seed=0):
    rng = np.random.default_rng(seed)
    c = cfg(N)
    xs = np.stack([rng.uniform(0.06, 0.15, N), rng.uniform(0.8, 1.2, N) * 2000 * math.pi])
    return np.stack([O.rho_all(xs[:, i], PH, c) for i in range(N)], axis=1)


# ------------------------------------------------------------------ constants
def test_derived_constants():
    """NTM_MPC_Sim.m:24-25, 37 (values quoted in SURVEY.md App. A)."""
    assert PH.kappa() == pytest.approx(5.7400e-8, rel=1e-3)
    assert PH.zeta() == pytest.approx(2.7072e-11, rel=1e-4)
    C = O.C_vec(PH, 0.1)
    assert C[0] == pytest.approx(-1.7391e-3, rel=1e-4)
    assert C[1] == pytest.approx(71.3226, rel=1e-5)
    A = O.A_mat(*O.rho_all(np.array([0.1, 2000 * math.pi]), PH, cfg())[:2], PH, 0.1)
    assert A[1, 0] == pytest.approx(734.9, rel=1e-3)
    assert A[1, 1] == pytest.approx(1 - 0.1 / 3.7)


def test_rho_functions_match_reference_formulas():
    """rho1.m:2 (unsquared w, D18), rho2.m:2, rho3.m:2-3."""
    x = np.array([0.1, 5000.0])
    assert O.rho1(x, 0.02) == 1 / (0.1 + 0.02 ** 2)
    assert O.rho1(x, 0.02, squared=True) == 1 / (0.1 ** 2 + 0.02 ** 2)
    assert O.rho2(x) == 0.1 ** 2 / 5000.0
    ws = 0.1 / 0.024
    assert O.rho3(x, 0.024) == pytest.approx((0.25 + 0.24 * ws) / (1 + 1.5 * ws + 0.43 * ws ** 2 + 0.64 * ws ** 3),
                                             rel=1e-15)


# ------------------------------------------------------------------ lift
@pytest.mark.parametrize("N", [1, 2, 5, 20])
def test_rollout_identity(N):
    """CANON D4/D6: X = Phi x0 + Gamma U + Lambda equals the step-by-step model of
    NTM_MPC_Sim.m:113 (x_{i} = A_i x_{i-1} + B_i u_i + C) for any U."""
    c = cfg(N)
    Rho = rand_rho(N, N)
    Phi, Gam, Lam = O.lift(Rho, PH, c)
    rng = np.random.default_rng(7)
    x0 = np.array([0.1, 6000.0])
    U = rng.uniform(0, 2e6, N)
    X = Phi @ x0 + Gam @ U + Lam
    x = x0.copy()
    Cv = O.C_vec(PH, c.Ts)
    for i in range(N):
        x = O.A_mat(Rho[0, i], Rho[1, i], PH, c.Ts) @ x + O.B_mat(Rho[2, i], PH, c.Ts) * U[i] + Cv
        np.testing.assert_allclose(X[2 * i:2 * i + 2], x, rtol=1e-13)


def test_lti_closed_forms():
    """Constant rho: Phi_i = A^i, Gamma_ij = A^(i-j) B, Lambda_i = sum_{k<i} A^k C."""
    N = 6
    c = cfg(N)
    r = O.rho_all(np.array([0.1, 6000.0]), PH, c)
    Rho = np.tile(r[:, None], (1, N))
    Phi, Gam, Lam = O.lift(Rho, PH, c)
    A = O.A_mat(r[0], r[1], PH, c.Ts)
    B = O.B_mat(r[2], PH, c.Ts)
    Cv = O.C_vec(PH, c.Ts)
    for i in range(1, N + 1):
        np.testing.assert_allclose(Phi[2 * i - 2:2 * i], np.linalg.matrix_power(A, i), rtol=1e-13)
        np.testing.assert_allclose(Lam[2 * i - 2:2 * i], sum(np.linalg.matrix_power(A, k) @ Cv for k in range(i)),
                                   rtol=1e-13)
        for j in range(1, i + 1):
            np.testing.assert_allclose(Gam[2 * i - 2:2 * i, j - 1], np.linalg.matrix_power(A, i - j) @ B, rtol=1e-13)


def test_literal_switches_agree_for_lti_only():
    """D4 / D6: the literal index/product order equals CANON for constant rho
     and differs once rho varies."""
    N = 5
    r = O.rho_all(np.array([0.1, 6000.0]), PH, cfg(N))
    Rho = np.tile(r[:, None], (1, N))
    lit = cfg(N, flags=O.LITERAL_GAMMA_INDEX)
    _, G1, _ = O.lift(Rho, PH, cfg(N))
    _, G2, _ = O.lift(Rho, PH, lit)
    np.testing.assert_allclose(G1, G2, rtol=1e-14)
    Rv = rand_rho(N, 3)
    _, G1, _ = O.lift(Rv, PH, cfg(N))
    _, G2, _ = O.lift(Rv, PH, lit)
    assert np.max(np.abs(G1 - G2)) > 0


# ------------------------------------------------------------------ getWLc
@pytest.mark.parametrize("N", [1, 3, 8])
def test_getwlc_equals_per_step_constraints(N):
    """getWLc.m:9-26: L U <= c + W x0 row by row equals the per-step box
    constraints u_i in [umin, umax] (i=0..N-1), x_i in [xmin, xmax] (i=0..N)."""
    c = cfg(N)
    Rho = rand_rho(N, 11)
    Phi, Gam, Lam = O.lift(Rho, PH, c)
    W, L, cv = O.getWLc(c.xmax, c.xmin, c.umax, c.umin, Gam, Phi, Lam)
    assert L.shape == (6 * N + 4, N) and W.shape == (6 * N + 4, 2)
    rng = np.random.default_rng(5)
    x0 = np.array([0.1, 6000.0])
    U = rng.uniform(-1e6, 3e6, N)
    lhs = L @ U - (cv + W @ x0)
    X = np.concatenate([x0, Phi @ x0 + Gam @ U + Lam])
    expect = []
    for i in range(N + 1):
        xi = X[2 * i:2 * i + 2]
        if i < N:
            expect += [-U[i] + c.umin, U[i] - c.umax]
        expect += [-xi[0] + c.xmin[0], -xi[1] + c.xmin[1], xi[0] - c.xmax[0], xi[1] - c.xmax[1]]
    np.testing.assert_allclose(lhs, np.array(expect), rtol=1e-10, atol=1e-9)


def test_reference_x0_is_infeasible():
    """Known answer (D15): x0 = [0; 2000 pi] (NTM_MPC_Sim.m:34) violates w >= 0.06
    (:40): the constant k=0 row reads 0 <= -0.06, so quadprog returns -2 (:100)."""
    c = cfg(3)
    x0 = O.REFERENCE_X0
    Rho = O.initial_rho(x0, PH, c)
    Phi, Gam, Lam = O.lift(Rho, PH, c)
    G, F = O.cost(Phi, Gam, Lam, x0, c)
    Lin, b = O.constraints(Phi, Gam, Lam, x0, c)
    assert np.all(Lin[2] == 0) and b[2] == pytest.approx(-0.06)
    U, flag, _ = O.qp_solve(G, F, Lin, b)
    assert flag == O.EXIT_INFEASIBLE and np.all(U == 0)
    st = O.mpc_step(x0, Rho, np.full(3, np.inf), PH, c)
    assert st["exitflag"] == -2 and st["u"] == 0


def test_constant_row_tolerance():
    """D22: a constant row (Lin_i = 0) is violated only beyond CONST_ROW_TOL = 1e-9,
    as quadprog judges feasibility to a tolerance (the plant step can leave x_{k+1}
    one ulp outside a bound the plan held it at).  Both oracles agree."""
    G, F = np.eye(3), np.array([1.0, -2.0, 0.5])
    Lin = np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0]])
    for b0, flag in ((-7e-18, O.EXIT_OK), (-0.9e-9, O.EXIT_OK), (-1e-6, O.EXIT_INFEASIBLE)):
        b = np.array([b0, 10.0])
        U, fl, _ = O.qp_solve(G, F, Lin, b)
        Uc, flc, _ = cbind.qp(G, F, Lin, b)
        assert fl == flag and flc == flag
        if flag == O.EXIT_OK:
            np.testing.assert_allclose(U, -F, atol=1e-15)
            np.testing.assert_allclose(Uc, -F, atol=1e-15)


# ------------------------------------------------------------------ QP
def _brute_force_qp(G, F, Lin, b, max_active):
    """Enumerate active sets (<= max_active rows), keep the feasible KKT point."""
    n = G.shape[0]
    best = None
    nz = [i for i in range(Lin.shape[0]) if np.any(Lin[i] != 0)]
    for k in range(0, max_active + 1):
        for A in itertools.combinations(nz, k):
            A = list(A)
            K = np.block([[G, Lin[A].T], [Lin[A], np.zeros((k, k))]]) if k else G
            rhs = np.concatenate([-F, b[A]]) if k else -F
            try:
                sol = np.linalg.solve(K, rhs)
            except np.linalg.LinAlgError:
                continue
            U, lam = sol[:n], sol[n:]
            if np.all(lam >= -1e-9 * max(1, np.max(np.abs(lam), initial=1))) and \
                    np.all(Lin @ U <= b + 1e-7 * np.maximum(1, np.abs(b))):
                f = 0.5 * U @ G @ U + F @ U
                if best is None or f < best[0] - 1e-12 * abs(f):
                    best = (f, U)
    return best


def test_qp_matches_active_set_enumeration():
    """N=3 problems from closed-loop states: the dual active-set result equals the
    exhaustive active-set enumeration (the optimum is unique: G > 0)."""
    c = cfg(3)
    x0s = O.scenario_x0(np.arange(6))
    checked = 0
    for s in range(6):
        x = x0s[s]
        Rho = O.initial_rho(x, PH, c)
        Phi, Gam, Lam = O.lift(Rho, PH, c)
        G, F = O.cost(Phi, Gam, Lam, x, c)
        Lin, b = O.constraints(Phi, Gam, Lam, x, c)
        U, flag, _ = O.qp_solve(G, F, Lin, b)
        if flag != 1:
            continue
        best = _brute_force_qp(G, F, Lin, b, 3)
        assert best is not None
        assert np.max(np.abs(U - best[1])) / c.umax <= 1e-9
        checked += 1
    assert checked >= 4


@pytest.mark.parametrize("name", ["qp_m1_N20", "qp_m2_N20", "qp_m3_N20", "qp_m2_N10", "qp_m0_N10",
                                  pytest.param("qp_m2_N50", marks=pytest.mark.slow),
                                  pytest.param("qp_m3_N50", marks=pytest.mark.slow)])
def test_qp_golden_certified(name):
    """Committed QPs with 50-digit-certified optima: both restatements (NumPy and
    C) land within 1e-13 * umax of the exact KKT point, config 5's N = 50 QPs with
    input-rate rows included (their final value is the long-double KKT solve on
    the active set, accurate_resolve / orc_accurate: the fp64 re-solve alone sat
    up to ~6e-9 umax off there)."""
    d = np.load(GOLD / f"{name}.npz")
    n = d["G"].shape[0]
    rng = range(n) if "N50" not in name else range(0, n, 2)        # N = 50: the NumPy GI is slow
    for i in range(n):
        sc = max(2e6, np.max(np.abs(d["U_exact"][i])))
        Uc, fc, _ = cbind.qp(d["G"][i], d["F"][i], d["Lin"][i] if d["Lin"].shape[1] else None,
                             d["b"][i] if d["Lin"].shape[1] else None)
        assert fc == d["exitflag"][i]
        assert np.max(np.abs(Uc - d["U_exact"][i])) / sc <= 1e-13, (i, np.max(np.abs(Uc - d["U_exact"][i])) / sc)
        if i in rng:
            U, flag, info = O.qp_solve(d["G"][i], d["F"][i], d["Lin"][i], d["b"][i])
            assert flag == d["exitflag"][i]
            assert np.max(np.abs(U - d["U_exact"][i])) / sc <= 1e-13, (i, np.max(np.abs(U - d["U_exact"][i])) / sc)


@pytest.mark.parametrize("name", ["qp_ss_m2_N20", "qp_ss_m3_N50"])
def test_steady_state_fixture_certified(name):
    """The steady-state QP fixtures (closed-loop steps 6-25, every
    inner iteration, NTM_MPC_Sim.m:93-97,123-127) that the GPU test feeds to the
    fused step kernel: each QP rebuilt from its (x_k, rho) by the oracle's lift /
    cost / getWLc (NTM_MPC_Sim.m:97,119-121) has U_exact as its KKT point: primal
    feasible to 1e-12, multipliers >= 0, stationarity G U + F + Lin_A' lam = 0 to
    1e-9 of |F| (fp64 evaluation of the 50-digit point), and the C oracle solves
    it to within 1e-13 umax.  The carried warm-start sets are valid active sets."""
    d = np.load(GOLD / f"{name}.npz")
    N, mode = int(d["N"]), int(d["mode"])
    c = cfg(N, mode)
    for i in range(d["x"].shape[0]):
        Rho = d["rho"][i].reshape(N, 3).T
        Phi, Gam, Lam = O.lift(Rho, PH, c)
        G, F = O.cost(Phi, Gam, Lam, d["x"][i], c)
        Lin, b = O.constraints(Phi, Gam, Lam, d["x"][i], c)
        Ue, q = d["U_exact"][i], int(d["act"][i, N])
        act, lam = d["act"][i, :q], d["lam"][i, :q]
        nz = np.any(Lin != 0, axis=1)
        assert np.all((Lin @ Ue - b)[nz] <= 1e-12 * np.maximum(1.0, np.abs(b[nz])))
        assert np.all(lam >= -1e-12 * max(1.0, np.max(np.abs(lam), initial=0.0)))
        r = G @ Ue + F + Lin[act].T @ lam
        assert np.max(np.abs(r)) <= 1e-9 * np.max(np.abs(F)), (i, np.max(np.abs(r)) / np.max(np.abs(F)))
        Uc, fc, _ = cbind.qp(G, F, Lin, b)
        assert fc == 1 and np.max(np.abs(Uc - Ue)) / c.umax <= 1e-13, (i, np.max(np.abs(Uc - Ue)) / c.umax)
        qc = int(d["cand"][i, N])
        if qc >= 0:
            ids = d["cand"][i, :qc]
            assert len(set(ids.tolist())) == qc and ids.min() >= 0 and ids.max() < Lin.shape[0]


def test_kkt_certificate_50_digits():
    d = np.load(GOLD / "qp_m2_N20.npz")
    for i in range(3):
        U, flag, info = O.qp_solve(d["G"][i], d["F"][i], d["Lin"][i], d["b"][i])
        Ue, lam, cert = O.kkt_polish(d["G"][i], d["F"][i], d["Lin"][i], d["b"][i], info["active"], dps=50)
        assert cert["max_violation"] <= 1e-12 and cert["min_multiplier"] >= -1e-12


def test_input_weight_cost_and_certified_qp():
    """Input weight R_u (ABI v5; SURVEY §2.1 D17 "Q, R_u exposed in config"; the
    reference has R_u = 0, NTM_MPC_Sim.m:59,72-73): the cost sum x'Qx + R_u u^2 adds
    exactly 2 R_u I to G = 2 Gamma' Om Gamma and leaves F alone; Ru = 0 is the
    reference's cost bit for bit.  The QPs of one closed-loop step with R_u > 0 are
    solved by both restatements to within 1e-13 umax of the 50-digit KKT point of
    their active set, which certifies (primal feasible, multipliers >= 0)."""
    N = 20
    x = O.scenario_x0([4])[0]
    c0 = cfg(N, O.MODE_FULL)
    Rho = O.initial_rho(x, PH, c0)
    Phi, Gam, Lam = O.lift(Rho, PH, c0)
    G0, F0 = O.cost(Phi, Gam, Lam, x, c0)
    assert np.array_equal(G0, 2 * Gam.T @ O.omega_blk(c0) @ Gam)
    for Ru in (1e-11, 1e-9):
        c = cfg(N, O.MODE_FULL, Ru=Ru)
        G, F = O.cost(Phi, Gam, Lam, x, c)
        assert np.array_equal(G, G0 + 2 * Ru * np.eye(N)) and np.array_equal(F, F0)
        Lin, b = O.constraints(Phi, Gam, Lam, x, c)
        U, flag, info = O.qp_solve(G, F, Lin, b)
        Uc, fc, _ = cbind.qp(G, F, Lin, b)
        assert flag == fc == 1
        Ue, lam, cert = O.kkt_polish(G, F, Lin, b, info["active"], dps=50)
        assert cert["max_violation"] <= 1e-12 and cert["min_multiplier"] >= -1e-12 * max(1.0, np.max(np.abs(lam)))
        assert np.max(np.abs(U - Ue)) / c.umax <= 1e-13
        assert np.max(np.abs(Uc - Ue)) / c.umax <= 1e-13
    # the weight moves the plans of a closed-loop step (this first QP's plan is held
    # by its active rows alone; the step's later LPV iterations are not)
    xs = O.scenario_x0(np.arange(8)).T
    moved = []
    for Ru in (0.0, 1e-9):
        c = cfg(N, O.MODE_FULL, Ru=Ru)
        moved.append(cbind.step(xs, *cbind.initial_state(xs, c), c)["U"])
    assert np.max(np.abs(moved[1] - moved[0])) / c0.umax > 1e-2


def test_unconstrained_lq_vs_mpmath():
    """BASELINE config 1 (N=10, reference x0, no constraints): U = -G^{-1} F in
    fp64 agrees with a 50-digit solve."""
    import mpmath as mp
    c = cfg(10, O.MODE_NONE)
    x0 = O.REFERENCE_X0
    Rho = O.initial_rho(x0, PH, c)
    Phi, Gam, Lam = O.lift(Rho, PH, c)
    G, F = O.cost(Phi, Gam, Lam, x0, c)
    U, flag, _ = O.qp_solve(G, F, np.zeros((0, 10)), np.zeros(0))
    with mp.workdps(50):
        Ue = mp.lu_solve(mp.matrix([[mp.mpf(float(v)) for v in row] for row in G]),
                         mp.matrix([-mp.mpf(float(v)) for v in F]))
        Ue = np.array([float(v) for v in Ue])
    assert flag == 1
    assert np.max(np.abs(U - Ue)) <= 1e-10 * np.max(np.abs(Ue))


# ------------------------------------------------------------------ closed loop
def test_rate_rows_structure():
    """Config 5 rows (extension): after getWLc's 6N+4 rows, pairs
    U_i - U_{i-1} <= du and U_{i-1} - U_i <= du for i = 1..N-1."""
    N = 5
    c = cfg(N, O.MODE_FULL_DU)
    assert c.m_rows == 8 * N + 2 == O.constraint_rows(N, O.MODE_FULL_DU)
    Rho = O.initial_rho(O.scenario_x0([3])[0], PH, c)
    Phi, Gam, Lam = O.lift(Rho, PH, c)
    Lin, b = O.constraints(Phi, Gam, Lam, O.scenario_x0([3])[0], c)
    L2, b2 = O.constraints(Phi, Gam, Lam, O.scenario_x0([3])[0], cfg(N, O.MODE_FULL))
    np.testing.assert_array_equal(Lin[:6 * N + 4], L2)
    np.testing.assert_array_equal(b[:6 * N + 4], b2)
    U = np.array([1.0, 4.0, 2.0, 2.0, 7.0])
    dU = np.diff(U)
    np.testing.assert_array_equal(Lin[6 * N + 4::2] @ U, dU)
    np.testing.assert_array_equal(Lin[6 * N + 5::2] @ U, -dU)
    assert np.all(b[6 * N + 4:] == c.du_max)


def test_rate_limited_closed_loop_respects_rows():
    """Every applied plan of the mode-3 closed-loop fixture satisfies the rate
    rows and the input box (to rounding), and the rate rows do bind."""
    d = np.load(GOLD / "closed_loop_m3_N20.npz")
    c = cfg(20, O.MODE_FULL_DU)
    Uk = d["Uk"]                                        # (scenarios, N, k_sim)
    assert np.max(np.abs(np.diff(Uk, axis=1))) <= c.du_max * (1 + 1e-9)
    assert np.max(np.abs(np.diff(Uk, axis=1))) >= c.du_max * (1 - 1e-9)
    assert Uk.min() >= c.umin - 1e-9 * c.umax and Uk.max() <= c.umax * (1 + 1e-12)


@pytest.mark.parametrize("name", ["closed_loop_m0_N10.npz", "closed_loop_m2_N3.npz", "closed_loop_m3_N20.npz"])
def test_closed_loop_golden(name):
    """Regression pin: the oracle reproduces its committed closed-loop fixtures."""
    d = np.load(GOLD / name)
    mode = int(name.split("_m")[1][0])
    N = int(name.split("_N")[1].split(".")[0])
    c = cfg(N, mode)
    for s in range(d["x0"].shape[0]):
        out = O.closed_loop(d["x0"][s], PH, c, int(d["k_sim"]))
        np.testing.assert_array_equal(out["exitflag"], d["exitflag"][s])
        np.testing.assert_allclose(out["uk"], d["uk"][s], rtol=0, atol=1e-9 * c.umax)
        np.testing.assert_allclose(out["xk"], d["xk"][s], rtol=1e-9, atol=1e-15)


def test_lpv_loop_semantics():
    """NTM_MPC_Sim.m:94-127: the LPV loop runs at most i_sim QPs, stops when
    sum|U - Uold| < eps, carries rho unshifted (D20) and Uold across steps (D14),
    and the applied input is U(1) of the last QP (D21).  Uold follows the
    reference order: the break at :125 comes before Uold = Uk(:,k) at :127, so
    on the converging iteration Uold stays the previous iterate (within eps of
    U, not necessarily bit-equal); only a loop that ran to i_sim ends with
    Uold == U."""
    for c in (cfg(3), cfg(3, i_sim=3), cfg(3, epsilon=1.0)):
        x0 = O.scenario_x0([0])[0]
        Rho = O.initial_rho(x0, PH, c)
        st = O.mpc_step(x0, Rho, np.full(3, np.inf), PH, c)
        assert 1 <= st["inner_iters"] <= c.i_sim
        assert st["u"] == st["U"][0]
        d = float(np.sum(np.abs(st["Uold"] - st["U"])))
        if st["inner_iters"] < c.i_sim:
            assert d < c.epsilon
        else:
            assert d < c.epsilon or np.array_equal(st["Uold"], st["U"])
    c = cfg(3)
    x0 = O.scenario_x0([0])[0]
    Rho = O.initial_rho(x0, PH, c)
    st = O.mpc_step(x0, Rho, np.full(3, np.inf), PH, c)
    xp, Rn = O.rollout(x0, Rho, st["U"], PH, c)        # rho_i <- rho(x_{i-1})
    np.testing.assert_allclose(Rn[:, 0], O.rho_all(x0, PH, c))
    c1 = cfg(3, i_sim=1)
    assert O.mpc_step(x0, Rho, np.full(3, np.inf), PH, c1)["inner_iters"] == 1


def test_plant_step_literal_switch():
    """D13: CANON plant = prediction model (+C); LITERAL drops C (NTM_MPC_Sim.m:130)."""
    x = np.array([0.1, 6000.0])
    a = O.plant_step(x, 1e6, PH, cfg())
    b = O.plant_step(x, 1e6, PH, cfg(flags=O.LITERAL_PLANT_NO_C))
    np.testing.assert_allclose(a - b, O.C_vec(PH, 0.1), rtol=1e-12)


def test_scenario_generator_ranges():
    x = O.scenario_x0(np.arange(1000))
    assert np.all((x[:, 0] >= 0.07) & (x[:, 0] < 0.14))
    assert np.all((x[:, 1] >= 0.8 * 2000 * math.pi) & (x[:, 1] < 1.2 * 2000 * math.pi))
    np.testing.assert_array_equal(O.scenario_x0([5, 6]), x[5:7])     # counter-based: shard invariant

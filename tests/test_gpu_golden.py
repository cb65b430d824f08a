"""GPU parity against the committed golden fixtures (tests/golden/, written by
make_golden.py from the NumPy oracle and, for every QP, certified by a 50-digit
KKT solve).  These pin the HIP path itself, not only the oracle:

  * qp_m{1,2,3}_N20, qp_m{2,3}_N50 (BASELINE config 5), qp_m{0,2}_N10 (config
    1's horizon): ntm_qp_device (the quadprog call, NTM_MPC_Sim.m:97) and the
    fp32 leg ntm_qp_mixed_device against U_exact, the certified optimum;
  * functions_N{3,20}: ntm_lift/cost/getwlc_device (Rho_to_PhiGammaLambda.m,
    NTM_MPC_Sim.m:120-121, getWLc.m) against the fixture's matrices;
  * functions_lit*_N6: the literal-reference lift switches D4/D6
    (Rho_to_PhiGammaLambda.m:21,32);
  * closed_loop_*: ntm_mpc_run (NTM_MPC_Sim.m:80-131) against the fixture's
    uk, Uk, xk, predicted island width wpred, exit flags and inner iterations;
    closed_loop_gen_*: the same with the scenario generator (plasma scenarios
    and disturbance realisations).

  * qp_ss_m2_N20 (config 3) and qp_ss_m3_N50 (config 5 with rate rows): QPs of
    the closed loop's steady state (steps 6-25, every inner iteration 1..10) fed
    to the FUSED step kernel (ntm_mpc_step_ws, i_sim = 1) with the warm-start
    set the device carries into them, against U_exact.

Tolerances: QP 1e-10 * umax (north_star's control-sequence bound) against the
exact optimum; functions 1e-13 relative (Phi/Gamma/Lambda, getWLc) and 1e-12
of the largest entry (G, F); the short free-running closed-loop fixtures 1e-10
(FIX_TOL): the C oracle itself reproduces these NumPy fixtures to <= 2.1e-14
umax (uk, Uk), 7.4e-16 (xk, wpred) with identical inner iterations
(tools/fixture_drift.py), the GPU to <= 6e-13 umax on uk.
"""
import math
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import ntm_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GOLD = Path(__file__).resolve().parent / "golden"


def T(a):
    return torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device=DEV)


def H(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


# free-running closed loops against the fixtures (short loops: 4-20 steps, 1-4
# scenarios): the C oracle reproduces them to <= 2.1e-14 umax (tools/fixture_drift.py)
# and the GPU measured <= 6e-13 umax on uk (round 5); the bound is north_star's
# per-step 1e-10 (round 4 held these at 1e-6)
FIX_TOL = 1e-10

QP_FIXTURES = ["qp_m1_N20", "qp_m2_N20", "qp_m3_N20", "qp_m2_N50", "qp_m3_N50", "qp_m0_N10", "qp_m2_N10"]


def _qp_args(d):
    n = d["G"].shape[0]
    Gb = np.stack([d["G"][i].reshape(-1, order="F") for i in range(n)], axis=1)
    if d["Lin"].shape[1] == 0:                                    # mode 0: no constraint rows
        return T(Gb), T(d["F"].T), None, None
    Lb = np.stack([d["Lin"][i].reshape(-1, order="F") for i in range(n)], axis=1)
    return T(Gb), T(d["F"].T), T(Lb), T(d["b"].T)


def _qp_scale(d):
    """umax, or the minimiser's own magnitude for the unconstrained LQ (mode 0,
    whose minimisers run to ~1e11: relative control-sequence error)."""
    return np.maximum(2e6, np.max(np.abs(d["U_exact"]), axis=1))[None, :]


@pytest.mark.parametrize("name", QP_FIXTURES)
def test_quadprog_vs_certified_optimum(ctl, name):
    """ntm_qp_device on the certified QPs: max |U_gpu - U_exact| <= 1e-10 umax
    (north_star's control-sequence bound) for every fixture, config 5's N = 50
    QPs with input-rate rows included."""
    d = np.load(GOLD / f"{name}.npz")
    U, flag, _ = ctl.quadprog(*_qp_args(d))
    U, flag = H(U), H(flag)
    np.testing.assert_array_equal(flag, d["exitflag"])
    err = np.max(np.abs(U - d["U_exact"].T) / _qp_scale(d))
    print(f"{name}: max |U_gpu - U_exact| / umax = {err:.3e}")
    assert err <= 1e-10, err


@pytest.mark.parametrize("N", [3, 20])
def test_functions_vs_fixture(ctl, N):
    from ntm_mpc import Config
    d = np.load(GOLD / f"functions_N{N}.npz")
    cfg = Config(N=N, mode=2)
    rho = d["Rho"].reshape(-1, order="F")[:, None]          # 3N x 1 (rho1, rho2, rho3 per stage)
    Phi, Gam, Lam = (H(t)[:, 0] for t in ctl.lift(T(rho), cfg))
    np.testing.assert_allclose(Phi.reshape(2 * N, 2, order="F"), d["Phi"], rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(Gam.reshape(2 * N, N, order="F"), d["Gamma"], rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(Lam, d["Lambda"], rtol=1e-13, atol=1e-300)
    G, F = (H(t)[:, 0] for t in ctl.cost(T(rho), T(d["xk"][:, None]), cfg))
    assert np.max(np.abs(G.reshape(N, N, order="F") - d["G"])) <= 1e-12 * np.max(np.abs(d["G"]))
    assert np.max(np.abs(F - d["F"])) <= 1e-12 * np.max(np.abs(d["F"]))
    W, L, c = (H(t)[:, 0] for t in ctl.getWLc(T(rho), cfg))
    m = 6 * N + 4
    np.testing.assert_allclose(W.reshape(m, 2, order="F"), d["W"], rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(L.reshape(m, N, order="F"), d["L"], rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(c, d["c"], rtol=1e-13, atol=1e-12)
    A, Bv = (H(t)[:, 0] for t in ctl.AB(T(d["Rho"][:, :1])))
    np.testing.assert_allclose(A.reshape(2, 2, order="F"), d["A0"], rtol=1e-14)
    np.testing.assert_allclose(Bv, d["B0"], rtol=1e-14)


@pytest.mark.parametrize("flags", [1, 2, 3])
def test_literal_lift_vs_fixture(ctl, flags):
    """D4 (Phi_{j-1} A_j, Rho_to_PhiGammaLambda.m:21) and D6 (A(rho_{i-j}), :32),
    computable literal variants, on the device's generic kernels."""
    from ntm_mpc import Config
    d = np.load(GOLD / f"functions_lit{flags}_N6.npz")
    N = 6
    cfg = Config(N=N, mode=2, flags=flags)
    rho = d["Rho"].reshape(-1, order="F")[:, None]
    Phi, Gam, Lam = (H(t)[:, 0] for t in ctl.lift(T(rho), cfg))
    np.testing.assert_allclose(Phi.reshape(2 * N, 2, order="F"), d["Phi"], rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(Gam.reshape(2 * N, N, order="F"), d["Gamma"], rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(Lam, d["Lambda"], rtol=1e-13, atol=1e-300)
    # the switches change the answer (the A_i do not commute when rho varies)
    Pc, Gc, _ = (H(t)[:, 0] for t in ctl.lift(T(rho), Config(N=N, mode=2)))
    assert not (np.array_equal(Pc, Phi) and np.array_equal(Gc, Gam))


GOLD_RUNS = ["closed_loop_m0_N10.npz", "closed_loop_m1_N20.npz", "closed_loop_m2_N20.npz",
             "closed_loop_m2_N3.npz", "closed_loop_m3_N20.npz", "closed_loop_m3_N50.npz",
             "closed_loop_gen_m2_N20.npz", "closed_loop_gen_m2_N3.npz"]


@pytest.mark.parametrize("name", GOLD_RUNS)
def test_run_vs_closed_loop_fixture(ctl, name):
    from ntm_mpc import Config, ScenarioGen
    d = np.load(GOLD / name)
    mode = int(name.split("_m")[1][0])
    N = int(name.split("_N")[1].split(".")[0])
    k_sim = int(d["k_sim"])
    S = d["x0"].shape[0]
    cfg = Config(N=N, mode=mode)
    gen = None
    if "gen_seed" in d.files:
        gen = ScenarioGen(seed=int(d["gen_seed"]), first_id=int(d["gen_first_id"]), k0=int(d["gen_k0"]),
                          sigma_w=float(d["gen_sigma_w"]), sigma_omega=float(d["gen_sigma_omega"]),
                          jbs_spread=float(d["gen_jbs_spread"]), wdep_spread=float(d["gen_wdep_spread"]))
    ctl.set_scenarios(gen)
    try:
        out = ctl.run(T(d["x0"].T), k_sim, cfg)
        uk, Uk, xk, wp = H(out["uk"]), H(out["Uk"]), H(out["xk"]), H(out["wpred"])
        fl, its = H(out["exitflag"]), H(out["inner_iters"])
    finally:
        ctl.set_scenarios(None)
    np.testing.assert_array_equal(fl.T, d["exitflag"])
    tol = FIX_TOL
    print(f"{name}: |duk| {np.max(np.abs(uk.T - d['uk'])) / cfg.umax:.2e} umax")
    assert np.max(np.abs(uk.T - d["uk"])) <= tol * cfg.umax
    Ukr = Uk.reshape(k_sim, N, S).transpose(2, 1, 0)             # fixture: (S, N, k_sim)
    assert np.max(np.abs(Ukr - d["Uk"])) <= tol * cfg.umax
    xkr = xk.reshape(k_sim + 1, 2, S).transpose(2, 1, 0)          # fixture: (S, 2, k_sim + 1)
    xs = np.array([0.15, 2000 * math.pi])[None, :, None]
    assert np.max(np.abs(xkr - d["xk"]) / xs) <= tol
    wpr = wp.reshape(k_sim, N + 1, S).transpose(2, 0, 1)          # fixture: (S, k_sim, N + 1)
    assert np.max(np.abs(wpr - d["wpred"])) <= tol * 0.15
    assert (its.T == d["inner_iters"]).mean() >= 0.9


@pytest.mark.parametrize("name", QP_FIXTURES)
def test_quadprog_mixed_vs_certified_optimum(ctl, name):
    """Config 5's fp32 leg (ntm_qp_mixed_device): the fp32 solve on fp32-rounded
    data lands within fp32 accuracy of the certified optimum, and the fp64
    refinement of its active set (fp64 fallback when it does not certify)
    recovers the optimum to the fp64 bound, 1e-10 * umax."""
    d = np.load(GOLD / f"{name}.npz")
    U, U32, flag, info, _ = ctl.quadprog_mixed(*_qp_args(d))
    U, U32, flag, info = H(U), H(U32), H(flag), H(info)
    np.testing.assert_array_equal(flag, d["exitflag"])
    sc = _qp_scale(d)
    err = np.max(np.abs(U - d["U_exact"].T) / sc)
    e32 = np.max(np.abs(U32 - d["U_exact"].T) / sc)
    print(f"{name}: mixed {err:.3e}, fp32 {e32:.3e}, certified {np.mean(info & 1):.2f}")
    assert err <= 1e-10, err
    # the fp32 solve itself is reported, not held to a bound: ~1e-7 umax at N = 20,
    # up to ~0.4 umax at N = 50, where cond(G) ~1e10-1e11 leaves fp32 no digits on the
    # weakly determined inputs (profiles/r04_precision.json)
    assert np.all(np.isfinite(U32)) and e32 <= 1.0, e32


@pytest.mark.parametrize("name,build", [("qp_ss_m2_N20", "far"), ("qp_ss_m2_N20", "lds"), ("qp_ss_m3_N50", "far")])
def test_steady_state_qps_through_step_kernel(ctl, name, build):
    """the steady state the bench times, pinned at 50 digits through
    the hot kernel itself.  Each fixture QP (closed-loop steps 6-25, inner
    iterations 1..10, NTM_MPC_Sim.m:93-97,123-127) goes to ntm_mpc_step_ws with
    i_sim = 1: its x_k and carried rho build the QP inside the fused k_mpc_step,
    and workspace slot 0 holds the set the device carries into that QP (the
    certified re-solve, its repairs, then GI).  U must be within 1e-10 umax of the
    50-digit optimum U_exact, with and without the carried set (cold: the
    Goldfarb-Idnani path on the same QPs), and the set the kernel certified must
    be the exact optimum's active set for >= 90% of them (degenerate rows with zero
    multipliers may differ).  N = 20 runs on both builds (far: the bench's
    kernel at B = 1e5; all-LDS: small batches); N = 50 carries one-collision sets of
    both kinds (d["kind"])."""
    from ntm_mpc import Config
    d = np.load(GOLD / f"{name}.npz")
    N, mode = int(d["N"]), int(d["mode"])
    n = d["x"].shape[0]
    assert n >= 32 and sorted(set(d["iter"].tolist())) == list(range(1, 11))
    assert d["step"].min() >= 6 and d["step"].max() <= 25
    if N == 50:
        assert (d["kind"] == 1).any() and (d["kind"] == 2).any()
    cfg = Config(N=N, mode=mode, i_sim=1)
    ctl.set_small_batch(0 if build == "far" else (1 << 62))
    try:
        assert ctl.step_layout(n, cfg) == build
        for warm in (True, False):
            ws = np.full((2 * (N + 1), n), -1, np.int32)
            if warm:
                ws[:N + 1] = d["cand"].T
            wt = torch.tensor(ws, dtype=torch.int32, device=DEV)
            out = ctl.step(T(d["x"].T), T(d["rho"].T), T(d["U_old"].T), cfg, active_ws=wt)
            np.testing.assert_array_equal(H(out["exitflag"]), 1)
            err = np.max(np.abs(H(out["U"]) - d["U_exact"].T), axis=0) / cfg.umax
            print(f"{name} {build} warm={warm}: max |U - U_exact| / umax {err.max():.2e}")
            assert err.max() <= 1e-10, (int(np.argmax(err)), err.max())
            got = H(wt)
            same = [sorted(got[:got[N, i], i].tolist()) == sorted(d["act"][i, :d["act"][i, N]].tolist())
                    for i in range(n)]
            # the optimum's active set is unique up to degenerate rows (zero multipliers)
            print(f"   certified set == the exact optimum's: {np.mean(same):.3f}")
            assert np.mean(same) >= 0.9, [i for i in range(n) if not same[i]]
    finally:
        ctl.set_small_batch(-1)

"""The C restatement of the oracle (oracle/ntm_oracle.c) agrees with the
NumPy oracle; both are test infrastructure (the checker), never the product."""
import dataclasses

import numpy as np
import pytest

from oracle import cbind
from oracle import ntm_oracle as O

PH = O.Physics()


@pytest.mark.parametrize("N", [3, 20])
def test_c_functions_match_python(N):
    import ctypes as C
    d = np.load(f"tests/golden/functions_N{N}.npz")
    c = O.Config(N=N)
    rho = np.ascontiguousarray(d["Rho"].T.reshape(-1))                 # 3xN col-major
    Phi, Gam, Lam = np.zeros(4 * N), np.zeros(2 * N * N), np.zeros(2 * N)
    lib = cbind.lib()
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))             # noqa: E731
    assert lib.ntm_oracle_lift(C.byref(cbind.phys_c()), C.byref(cbind.cfg_c(c)), dp(rho), dp(Phi), dp(Gam),
                               dp(Lam)) == 0
    np.testing.assert_allclose(Phi.reshape(2, 2 * N).T, d["Phi"], rtol=1e-14)
    np.testing.assert_allclose(Gam.reshape(N, 2 * N).T, d["Gamma"], rtol=1e-14)
    np.testing.assert_allclose(Lam, d["Lambda"], rtol=1e-14)
    G, F = np.zeros(N * N), np.zeros(N)
    xk = np.ascontiguousarray(d["xk"])
    lib.ntm_oracle_cost(C.byref(cbind.phys_c()), C.byref(cbind.cfg_c(c)), dp(rho), dp(xk), dp(G), dp(F))
    assert np.max(np.abs(G.reshape(N, N).T - d["G"])) <= 1e-13 * np.max(np.abs(d["G"]))
    assert np.max(np.abs(F - d["F"])) <= 1e-13 * np.max(np.abs(d["F"]))
    m = 6 * N + 4
    W, L, cv = np.zeros(2 * m), np.zeros(m * N), np.zeros(m)
    lib.ntm_oracle_getwlc(C.byref(cbind.phys_c()), C.byref(cbind.cfg_c(c)), dp(rho), dp(W), dp(L), dp(cv))
    np.testing.assert_allclose(W.reshape(2, m).T, d["W"], rtol=1e-14)
    np.testing.assert_allclose(L.reshape(N, m).T, d["L"], rtol=1e-14)
    np.testing.assert_allclose(cv, d["c"], rtol=1e-14, atol=1e-15)


@pytest.mark.parametrize("name", ["qp_m2_N20.npz", "qp_m1_N20.npz", "qp_m3_N20.npz"])
def test_c_qp_matches_certified(name):
    d = np.load(f"tests/golden/{name}")
    for i in range(d["G"].shape[0]):
        U, flag, _ = cbind.qp(d["G"][i], d["F"][i], d["Lin"][i], d["b"][i])
        assert flag == d["exitflag"][i]
        assert np.max(np.abs(U - d["U_exact"][i])) / 2e6 <= 1e-11


@pytest.mark.parametrize("N,mode,Ru", [(10, 0, 0.0), (3, 2, 0.0), (20, 1, 0.0), (20, 2, 0.0), (20, 3, 0.0),
                                       (4, 3, 0.0), (20, 2, 1e-10), (10, 2, 1e-11), (4, 3, 1e-9)])
def test_c_step_teacher_forced(N, mode, Ru):
    """Per-step agreement (identical inputs every step) of the two oracles, with and
    without an input weight Ru (ABI v5)."""
    c = O.Config(N=N, mode=mode, Ru=Ru)
    B = 6
    x = O.scenario_x0(np.arange(B)).T.copy() if mode else np.tile(O.REFERENCE_X0[:, None], (1, B))
    rho, Uo = cbind.initial_state(x, c)
    for k in range(6 if N >= 20 else 12):
        ref = cbind.step(x, rho, Uo, c, nthreads=2)
        for s in range(B):
            out = O.mpc_step(x[:, s], rho[:, s].reshape(N, 3).T, Uo[:, s], PH, c)
            assert out["exitflag"] == ref["exitflag"][s]
            if mode == 3 and out["inner_iters"] != ref["inner_iters"][s]:
                # with rate rows the LPV loop can stop on its bitwise fixed point
                # (sum|U - Uold| < 1e-14) a few iterations apart in two exact
                # solvers, or 2-cycle instead: compare along the C oracle's path
                pc = dataclasses.replace(c, i_sim=int(ref["inner_iters"][s]), epsilon=-1.0)
                out = O.mpc_step(x[:, s], rho[:, s].reshape(N, 3).T, Uo[:, s], PH, pc)
            # both restatements end every QP with the long-double KKT solve on the
            # final active set, mode 3's rate rows included
            tol = 1e-10
            assert np.max(np.abs(out["U"] - ref["U"][:, s])) <= tol * max(c.umax, np.max(np.abs(out["U"])))
            # atol: 1e-10 of |w| ~ 0.1 m (mode 0 drives w towards 0, where rtol alone is 1e-10 of ~0.02)
            np.testing.assert_allclose(out["xnext"], ref["x_next"][:, s], rtol=1e-10, atol=1e-11)
        x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]


@pytest.mark.parametrize("name", ["closed_loop_m1_N20.npz", "closed_loop_m2_N20.npz", "closed_loop_m2_N3.npz",
                                  "closed_loop_m3_N20.npz",
                                  "closed_loop_m0_N10.npz"])
def test_c_closed_loop_vs_golden(name):
    d = np.load(f"tests/golden/{name}")
    mode = int(name.split("_m")[1][0])
    N = int(name.split("_N")[1].split(".")[0])
    c = O.Config(N=N, mode=mode)
    out = cbind.run(np.ascontiguousarray(d["x0"].T), c, int(d["k_sim"]), nthreads=2)
    np.testing.assert_array_equal(out["exitflag"].T, d["exitflag"])
    # free-running closed loops amplify rounding: 1e-6 of umax
    assert np.max(np.abs(out["uk"].T - d["uk"])) <= 1e-6 * c.umax


def test_c_infeasible_and_nonfinite():
    c = O.Config(N=3, mode=2)
    x = np.array([[0.0, 0.1], [2000 * np.pi, np.nan]])
    rho, Uo = cbind.initial_state(x, c)
    out = cbind.step(x, rho, Uo, c)
    assert out["exitflag"][0] == -2 and np.all(out["U"][:, 0] == 0)
    assert out["exitflag"][1] == -7


def test_c_oracle_under_asan_ubsan():
    """SURVEY.md §5 race/sanitizer row: the C oracle built with AddressSanitizer
    and UBSan (make -C oracle sanitize), driven through every exported entry
    point (every mode, N = 1 and 64, all literal switches, the scenario
    generator, infeasible and non-finite inputs) reports nothing."""
    import os
    import subprocess
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    subprocess.run(["make", "-s", "-C", str(root / "oracle"), "sanitize"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([str(root / "oracle" / "_san" / "ntm_oracle_san")], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr

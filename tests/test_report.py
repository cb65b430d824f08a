"""The report replacement (tools/report.py; NTM_MPC_Sim.m:134-164, SURVEY.md §8f
row 4): the closed loop's workspace variables, the predicted island width wpred
(NTM_MPC_Sim.m:110-117) included, reshaped to the reference's layout and written
to npz/CSV/PNG.

  * CPU: write_report on a committed closed-loop fixture round-trips every
    array, and the CSV carries scenario 0's states, input and predicted w;
  * GPU: closed_loop_report (ntm_mpc_run through the C-ABI) on a fixture's x0
    matches the fixture's uk, Uk, xk, wpred and exit flags (the free-running
    closed-loop fixture tolerance of tests/test_gpu_golden.py, FIX_TOL = 1e-10).
"""
import math
from pathlib import Path

import numpy as np
import pytest

from tools import report

GOLD = Path(__file__).resolve().parent / "golden"


def _fixture_rep(name):
    d = np.load(GOLD / name)
    N = d["Uk"].shape[1]
    return d, {"xk": d["xk"], "uk": d["uk"][:, None, :], "Uk": d["Uk"], "wpred": d["wpred"],
               "exitflag": d["exitflag"], "inner_iters": d["inner_iters"], "N": N, "mode": 2}


def test_write_report_roundtrip(tmp_path):
    d, rep = _fixture_rep("closed_loop_m2_N20.npz")
    out = str(tmp_path / "rep")
    files = report.write_report(rep, out)
    assert files[:2] == [out + ".npz", out + ".csv"]
    back = np.load(out + ".npz")
    for k in ("xk", "uk", "Uk", "wpred", "exitflag", "inner_iters"):
        np.testing.assert_array_equal(back[k], rep[k])
    rows = [r.split(",") for r in open(out + ".csv").read().strip().split("\n")]
    assert rows[0] == ["k", "w_m", "omega_rad_s", "u_W", "exitflag", "inner_iters", "wpred_1_m", "wpred_N_m"]
    K, N = d["uk"].shape[1], rep["N"]
    assert len(rows) == K + 2
    for k in range(K):
        r = rows[1 + k]
        assert float(r[1]) == d["xk"][0, 0, k] and float(r[3]) == d["uk"][0, k]
        assert int(r[4]) == d["exitflag"][0, k]
        assert float(r[6]) == d["wpred"][0, k, 1] and float(r[7]) == d["wpred"][0, k, N]
    # wpred row k starts at the plant state x_k (the rollout's x_0 = x_k, NTM_MPC_Sim.m:110)
    np.testing.assert_array_equal(d["wpred"][:, :, 0], d["xk"][:, 0, :K])
    if len(files) == 3:
        assert Path(files[2]).stat().st_size > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["closed_loop_m2_N20.npz", "closed_loop_m3_N20.npz", "closed_loop_gen_m2_N20.npz"])
def test_closed_loop_report_vs_fixture(ctl, name, tmp_path):
    from ntm_mpc import Config, ScenarioGen
    d = np.load(GOLD / name)
    mode = int(name.split("_m")[1][0])
    N = int(name.split("_N")[1].split(".")[0])
    cfg = Config(N=N, mode=mode)
    gen = None
    if "gen_seed" in d.files:
        gen = ScenarioGen(seed=int(d["gen_seed"]), first_id=int(d["gen_first_id"]), k0=int(d["gen_k0"]),
                          sigma_w=float(d["gen_sigma_w"]), sigma_omega=float(d["gen_sigma_omega"]),
                          jbs_spread=float(d["gen_jbs_spread"]), wdep_spread=float(d["gen_wdep_spread"]))
    rep = report.closed_loop_report(ctl, d["x0"].T, int(d["k_sim"]), cfg, gen=gen)
    np.testing.assert_array_equal(rep["exitflag"], d["exitflag"])
    tol = 1e-10        # test_gpu_golden.FIX_TOL: the C oracle reproduces these fixtures to 2.1e-14
    assert np.max(np.abs(rep["uk"][:, 0, :] - d["uk"])) <= tol * cfg.umax
    assert np.max(np.abs(rep["Uk"] - d["Uk"])) <= tol * cfg.umax
    xs = np.array([0.15, 2000 * math.pi])[None, :, None]
    assert np.max(np.abs(rep["xk"] - d["xk"]) / xs) <= tol
    assert np.max(np.abs(rep["wpred"] - d["wpred"])) <= tol * 0.15
    files = report.write_report(rep, str(tmp_path / "r"), plot=False)
    np.testing.assert_array_equal(np.load(files[0])["wpred"], rep["wpred"])

"""Wider closed-loop parity than test_gpu_parity's 32 scenarios:
256 scenarios x 20 free-running steps against the C oracle where the loop keeps
the 5e-8 bound, and per-step (teacher-forced) parity over 20 steps for the N = 50
mode-3 scenarios whose free-running loop amplifies past it."""
import numpy as np
import pytest

from oracle import cbind
from oracle import ntm_oracle as O
from test_gpu_parity import H, RUN_TOL, T, U_TOL_RATE, _assert_run_close, cfgs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,mode", [(20, 2), (20, 3), (50, 2)])
def test_run_closed_loop_wide(ctl, N, mode):
    B, k_sim = 256, 20
    cfg, ocfg = cfgs(N, mode)
    x0 = O.scenario_x0(np.arange(B)).T
    ref = cbind.run(x0, ocfg, k_sim)
    out = ctl.run(T(x0), k_sim, cfg)
    _assert_run_close(out, ref, cfg, k_sim, tol=RUN_TOL, x0=x0, ocfg=ocfg)


def test_teacher_forced_drifting_scenarios_n50_mode3(ctl):
    """Scenarios 112, 240 and 146 drift up to 3.9e-6 umax free-running (profiles/
    r04_parity_wide.txt); given the oracle's (x_k, rho, U_old) at every step, the
    GPU's plan stays within 1e-10 umax with the same inner-iteration count."""
    N, mode, k_sim = 50, 3, 20
    ids = np.array([112, 240, 146])
    cfg, ocfg = cfgs(N, mode)
    x = O.scenario_x0(ids).T
    rho, Uo = cbind.initial_state(x, ocfg)
    ws = ctl.new_active_ws(len(ids), cfg)
    for k in range(k_sim):
        ref = cbind.step(x, rho, Uo, ocfg)
        out = ctl.step(T(x), T(rho), T(Uo), cfg, active_ws=ws)
        assert (H(out["inner_iters"]) == ref["inner_iters"]).all(), k
        du = np.max(np.abs(H(out["U"]) - ref["U"])) / cfg.umax
        assert du <= U_TOL_RATE, (k, du)
        x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]

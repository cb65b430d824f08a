"""Wider closed-loop parity than test_gpu_parity's 32 scenarios:
256 scenarios x 20 free-running steps against the C oracle for every BASELINE
horizon/mode with constraints (N = 20 modes 2 and 3, N = 50 modes 2 and 3).
Where the closed loop itself amplifies rounding past RUN_TOL (in round 4 only
N = 50 mode 3 did so on the GPU), a scenario's bound is SENS_FACTOR times the
loop's own sensitivity, measured on the C oracle against itself (tests/golden/sensitivity_m{mode}_N{N}.npz, from
make_golden.py; pinned on CPU by tests/test_sensitivity.py); plus per-step
(teacher-forced) parity over 20 steps for the N = 50 mode-3 scenarios whose
free-running loop amplifies most."""
import math
from pathlib import Path

import numpy as np
import pytest

from oracle import cbind
from oracle import ntm_oracle as O
from test_gpu_parity import H, RUN_TOL, T, U_TOL_RATE, _assert_run_close, _replay_along, cfgs

pytestmark = pytest.mark.gpu


GOLD = Path(__file__).resolve().parent / "golden"
# A free-running comparison cannot be tighter than the loop's own response to a
# rounding-size perturbation.  sens[s] is the C oracle's drift (max_k |dU_k| / umax)
# when x_0 moves by 1e-13 relative (w and omega, up and down); the GPU's per-step
# differences are ~1e-12 umax (teacher-forced, measured <= 6.5e-12 over these
# scenarios), injected at every step, so a scenario may drift up to 10 sens[s]
# (round 4 measured GPU / sens <= 1.8 on the three most sensitive ones).
SENS_FACTOR = 10.0
# Only (N = 50, mode 3) needs the sensitivity bound: the other three configs hold
# RUN_TOL on every scenario (keep their 5e-8, so a regression in the
# sensitive scenarios cannot pass silently).  For (50, 3) the number of scenarios
# above RUN_TOL is bounded by the recorded count plus a margin.
SENS_BOUND = {(50, 3)}
# recorded on the round-6 build: 1 scenario above RUN_TOL (3.1e-7 umax, 0.02 of its
# sensitivity bound; round-5 intermediate builds had up to 7, at 3.5e-6)
ABOVE_MAX = {(50, 3): 1 + 3}
# Scenarios whose LPV iteration count or exit flag differs from the oracle's at
# some step (the bitwise stopping rule), replayed along the GPU's
# path: the recorded count per config (256 scenarios, 20 steps) plus a margin,
# instead of a blanket 40%
# Recorded (round 6, gpurun_out/r06a): 26 of 256 at (20, 3), none elsewhere; the
# same 26 with the reference's rollout recursion instead of the lifted one
# (NTM_ROLL_LIFTED=0), so the lifted rollout moves no iteration count
DIV_RECORDED = {(20, 2): 0, (20, 3): 26, (50, 2): 0, (50, 3): 0}
DIV_MARGIN = 8


def _per_scenario_errors(out, ref, cfg, k_sim, x0, ocfg):
    """Max over the k_sim steps of |uk|, |Uk| (/ umax), |xk| (/ |w|, |omega| scale)
    and |wpred| (/ 0.15 m) per scenario, after replaying the scenarios whose
    bitwise LPV stopping rule fired at another iteration (_assert_run_close)."""
    N = cfg.N
    g = {k: H(out[k]) for k in ("uk", "Uk", "xk", "wpred", "exitflag", "inner_iters")}
    div = np.where(((g["inner_iters"] != ref["inner_iters"]) | (g["exitflag"] != ref["exitflag"])).any(axis=0))[0]
    print(f"N={N} mode={cfg.mode}: {len(div)} of {x0.shape[1]} scenarios diverged in their iteration "
          f"counts (replayed along the GPU's path): {[int(s) for s in div[:16]]}")
    assert len(div) <= DIV_RECORDED[(N, cfg.mode)] + DIV_MARGIN, len(div)
    ref = {k: np.array(v, copy=True) for k, v in ref.items()}
    for s in div:
        rp = _replay_along(x0[:, s], ocfg, g["inner_iters"][:, s], None, int(s))
        for k in ref:
            ref[k][:, s] = rp[k][:, 0]
    xs = np.tile(np.array([0.15, 2000 * math.pi]), k_sim + 1)[:, None]
    e = np.max(np.stack([np.max(np.abs(g["uk"] - ref["uk"]), axis=0) / cfg.umax,
                         np.max(np.abs(g["Uk"] - ref["Uk"]), axis=0) / cfg.umax,
                         np.max(np.abs(g["xk"] - ref["xk"]) / xs, axis=0),
                         np.max(np.abs(g["wpred"] - ref["wpred"]), axis=0) / 0.15]), axis=0)
    assert (g["exitflag"] == ref["exitflag"]).mean() > 0.99
    assert g["wpred"].shape == ((N + 1) * k_sim, x0.shape[1])
    return e


@pytest.mark.parametrize("N,mode", [(20, 2), (20, 3), (50, 2), (50, 3)])
def test_run_closed_loop_wide(ctl, N, mode):
    B, k_sim = 256, 20
    cfg, ocfg = cfgs(N, mode)
    x0 = O.scenario_x0(np.arange(B)).T
    ref = cbind.run(x0, ocfg, k_sim)
    out = ctl.run(T(x0), k_sim, cfg)
    d = np.load(GOLD / f"sensitivity_m{mode}_N{N}.npz")
    assert int(d["B"]) == B and int(d["k_sim"]) == k_sim
    sens_bound = (N, mode) in SENS_BOUND
    bound = np.maximum(RUN_TOL, SENS_FACTOR * d["sens"]) if sens_bound else np.full(B, RUN_TOL)
    e = _per_scenario_errors(out, ref, cfg, k_sim, x0, ocfg)
    wide = np.where(bound > RUN_TOL)[0]
    above = int((e > RUN_TOL).sum())
    print(f"N={N} mode={mode}: max err {e.max():.2e} (scenario {int(np.argmax(e))}); {len(wide)} scenarios "
          f"bounded by {SENS_FACTOR:g} x the loop's sensitivity, max err / sens there "
          f"{np.max(e[wide] / d['sens'][wide], initial=0.0):.2f}")
    print(f"   scenarios above RUN_TOL: {above}")
    assert above <= ABOVE_MAX.get((N, mode), 0), above
    bad = np.where(e > bound)[0]
    assert len(bad) == 0, [(int(s), float(e[s]), float(bound[s])) for s in bad]


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

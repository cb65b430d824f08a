"""Diagnostic (not a test): per-step (teacher-forced) parity of chosen scenarios
over a long closed loop: each step the GPU (ntm_mpc_step, active-set workspace
carried) and the C oracle get the same (x_k, rho, U_old), taken from the
oracle's own trajectory, and the step's plan U is compared.  Used on the N = 50
mode-3 scenarios whose free-running loop drifts past 5e-8.

    python tools/teacher_forced_one.py N mode k_sim id [id ...]
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "mpc-ntm-control_amd")]
import numpy as np  # noqa: E402

import test_gpu_parity as tp  # noqa: E402
from ntm_mpc import NtmMpc  # noqa: E402

N, mode, K = (int(a) for a in sys.argv[1:4])
ids = np.array([int(a) for a in sys.argv[4:]])
ctl = NtmMpc()
cfg, ocfg = tp.cfgs(N, mode)
x = tp.O.scenario_x0(ids).T
rho, Uo = tp.cbind.initial_state(x, ocfg)
ws = ctl.new_active_ws(len(ids), cfg)
for k in range(K):
    ref = tp.cbind.step(x, rho, Uo, ocfg)
    out = ctl.step(tp.T(x), tp.T(rho), tp.T(Uo), cfg, active_ws=ws)
    gi = tp.H(out["inner_iters"])
    du = np.max(np.abs(tp.H(out["U"]) - ref["U"]), axis=0) / cfg.umax
    print(f"step {k:2d}: " + "  ".join(
        f"id {s}: |dU|/umax {d:.2e} iters gpu {g} cpu {c}" for s, d, g, c in zip(ids, du, gi, ref["inner_iters"])),
        flush=True)
    x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]

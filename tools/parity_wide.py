"""Diagnostic (not a test): a wider closed-loop parity sweep than the -m gpu
suite's (B = 32): ntm_mpc_run on the GPU against the C oracle's closed loop for
B scenarios and k_sim steps at the given horizons and modes, with the suite's
own comparison (tests/test_gpu_parity.py::_assert_run_close: mode 3 replays the
scenarios whose bitwise LPV stopping rule fired at another iteration).

    python tools/parity_wide.py B k_sim N:mode [N:mode ...]
"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "mpc-ntm-control_amd")]
import numpy as np  # noqa: E402

import test_gpu_parity as tp  # noqa: E402
from ntm_mpc import NtmMpc  # noqa: E402

B, K = int(sys.argv[1]), int(sys.argv[2])
ctl = NtmMpc()
for spec in sys.argv[3:]:
    N, mode = (int(v) for v in spec.split(":"))
    cfg, ocfg = tp.cfgs(N, mode)
    x0 = tp.O.scenario_x0(np.arange(B)).T
    t = time.time()
    ref = tp.cbind.run(x0, ocfg, K)
    t_ref = time.time() - t
    out = ctl.run(tp.T(x0), K, cfg)
    g = {k: tp.H(out[k]) for k in ("uk", "Uk", "xk", "inner_iters", "exitflag")}
    div = int(((g["inner_iters"] != ref["inner_iters"]) | (g["exitflag"] != ref["exitflag"])).any(axis=0).sum())
    raw_du = float(np.max(np.abs(g["Uk"] - ref["Uk"])) / cfg.umax)
    try:
        tp._assert_run_close(out, ref, cfg, K, tol=tp.RUN_TOL, x0=x0, ocfg=ocfg)
        verdict = f"within RUN_TOL={tp.RUN_TOL:g} of the C oracle"
    except AssertionError as e:
        verdict = f"FAILS RUN_TOL={tp.RUN_TOL:g} ({e})"
        # per-scenario errors after the replay, the worst first
        sel = np.where(((g["inner_iters"] != ref["inner_iters"]) | (g["exitflag"] != ref["exitflag"])).any(axis=0))[0]
        rr = {k: np.array(v, copy=True) for k, v in ref.items()}
        for s in sel:
            rp = tp._replay_along(x0[:, s], ocfg, g["inner_iters"][:, s], None, int(s))
            for k in rr:
                rr[k][:, s] = rp[k][:, 0]
        e_s = np.max(np.abs(g["Uk"] - rr["Uk"]), axis=0) / cfg.umax
        for s in np.argsort(-e_s)[:6]:
            e_k = np.max(np.abs(g["Uk"] - rr["Uk"])[:, s].reshape(K, N), axis=1) / cfg.umax
            k1 = int(np.argmax(e_k > tp.RUN_TOL)) if (e_k > tp.RUN_TOL).any() else -1
            print(f"   scenario {s}: max |dU|/umax {e_s[s]:.3e}, first step above RUN_TOL {k1}, "
                  f"replayed {s in set(sel.tolist())}, GPU iters {g['inner_iters'][:, s].tolist()}, "
                  f"GPU flags {g['exitflag'][:, s].tolist()}", flush=True)
    print(f"N={N} mode={mode} B={B} k_sim={K}: {verdict} "
          f"(scenarios on another LPV path, replayed: {div}); max |dU|/umax before replay {raw_du:.3e}; "
          f"oracle {t_ref:.1f} s", flush=True)

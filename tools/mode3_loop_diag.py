"""Diagnostic: free-running closed loops (ntm_mpc_run, NTM_MPC_Sim.m:80-131) on
the GPU against the C oracle, per scenario: the first step whose inner-iteration
count or exit flag differs, and the largest |duk| / umax before and after it.

    python tools/mode3_loop_diag.py [N] [mode] [B] [k_sim] [--gen]
"""
import math
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import cbind  # noqa: E402
from oracle import ntm_oracle as O  # noqa: E402


def main():
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    N = int(a[0]) if a else 20
    mode = int(a[1]) if len(a) > 1 else 3
    B = int(a[2]) if len(a) > 2 else 32
    K = int(a[3]) if len(a) > 3 else 20
    from ntm_mpc import Config, NtmMpc, ScenarioGen
    ctl = NtmMpc()
    cfg, ocfg = Config(N=N, mode=mode), O.Config(N=N, mode=mode)
    gen = ogen = None
    if "--gen" in sys.argv:
        kw = dict(seed=20241220, first_id=0, k0=0, sigma_w=1e-3, sigma_omega=0.0, jbs_spread=0.1, wdep_spread=0.1)
        gen, ogen = ScenarioGen(**kw), O.ScenarioGen(**kw)
    x0 = O.scenario_x0(np.arange(B)).T
    ref = cbind.run(x0, ocfg, K, gen=ogen)
    ctl.set_scenarios(gen)
    out = ctl.run(torch.tensor(np.ascontiguousarray(x0), device="cuda"), K, cfg)
    torch.cuda.synchronize()
    ctl.set_scenarios(None)
    g = {k: v.cpu().numpy() for k, v in out.items()}
    du = np.abs(g["uk"] - ref["uk"]) / cfg.umax                        # (K, B)
    dU = np.abs(g["Uk"] - ref["Uk"]).reshape(K, N, B).max(axis=1) / cfg.umax
    diff = (g["inner_iters"] != ref["inner_iters"]) | (g["exitflag"] != ref["exitflag"])
    print(f"N={N} mode={mode} B={B} K={K} gen={gen is not None}: max |dUk|/umax {dU.max():.3e}, "
          f"scenarios with an iteration/flag difference: {int(diff.any(axis=0).sum())}")
    for s in range(B):
        kd = int(np.argmax(diff[:, s])) if diff[:, s].any() else K
        pre = dU[:kd, s].max(initial=0.0)
        post = dU[kd:, s].max(initial=0.0)
        first_big = int(np.argmax(dU[:, s] > 1e-10)) if (dU[:, s] > 1e-10).any() else -1
        if kd < K or post > 1e-10 or pre > 1e-10:
            print(f"  s={s:3d} first iter/flag diff at k={kd:2d}  pre {pre:.2e} post {post:.2e}  first dU>1e-10 at k={first_big}"
                  f"  iters gpu {g['inner_iters'][kd if kd < K else K - 1, s]} cpu {ref['inner_iters'][kd if kd < K else K - 1, s]}"
                  f"  dU per step {' '.join(f'{v:.0e}' for v in dU[:, s])}")


if __name__ == "__main__":
    main()

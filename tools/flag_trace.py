#!/usr/bin/env python3
"""Per-step exit-flag histogram of the bench's closed loop (B scenarios, the
carried warm-start workspace), plus a teacher-forced oracle check of the
non-optimal scenarios of the first step that has any.

    NTM_MPC_LIB=<lib> python tools/flag_trace.py [B] [K] [N] [mode]

Diagnostic only (imports the C oracle as the checker)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "mpc-ntm-control_amd")]

import ntm_mpc  # noqa: E402
from ntm_mpc import Config, NtmMpc  # noqa: E402
from oracle import cbind  # noqa: E402
from oracle import ntm_oracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 25
N = int(sys.argv[3]) if len(sys.argv) > 3 else 20
mode = int(sys.argv[4]) if len(sys.argv) > 4 else 2
cfg, ocfg = Config(N=N, mode=mode), O.Config(N=N, mode=mode)
ctl = NtmMpc(config=cfg, device=0)
x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(0, B), 0)
rho, U_old = ctl.initial_state(x, cfg)
ws = ctl.new_active_ws(B, cfg)
checked = False
for k in range(K):
    x_in, rho_in, uo_in, ws_in = x.cpu().numpy(), rho.cpu().numpy(), U_old.cpu().numpy(), ws.cpu().numpy()
    out = ctl.step(x, rho, U_old, cfg, active_ws=ws)
    torch.cuda.synchronize()
    fl = out["exitflag"].cpu().numpy()
    vals, cnt = np.unique(fl, return_counts=True)
    its = out["inner_iters"].cpu().numpy()
    print(f"step {k:2d} flags {dict(zip(vals.tolist(), cnt.tolist()))} inner_iters mean {its.mean():.4f}"
          f" U checksum {float(out['U'].double().sum().item()):.10e}", flush=True)
    bad = np.flatnonzero(fl != 1)
    if len(bad) and not checked:
        checked = True
        ids = bad[:8]
        ref = cbind.step(x_in[:, ids], rho_in[:, ids], uo_in[:, ids], ocfg)
        print("  first non-optimal ids", ids.tolist(), "gpu flags", fl[ids].tolist(), "oracle flags",
              ref["exitflag"].tolist(), "oracle iters", ref["inner_iters"].tolist(), "gpu iters", its[ids].tolist())
        print("  x_k", x_in[:, ids].T.tolist())
        np.savez(ROOT / "gpurun_out" / "first_bad.npz", ids=ids, x=x_in[:, ids], rho=rho_in[:, ids],
                 U_old=uo_in[:, ids], ws=ws_in[:, ids], step=k)
    x = out["x_next"].clone()
ctl.close()

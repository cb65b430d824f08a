#!/usr/bin/env python3
"""Closed loop of the bench (B scenarios, carried warm-start workspace) for K
steps; saves every step's U, exit flags and x_next to an npz so two runs (or
two builds: NTM_MPC_LIB) can be compared bit for bit.  Diagnostic only.

    NTM_MPC_LIB=<lib> python tools/determinism.py out.npz [B] [K] [first_id]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "mpc-ntm-control_amd")]
import ntm_mpc  # noqa: E402
from ntm_mpc import Config, NtmMpc  # noqa: E402

out_path = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
K = int(sys.argv[3]) if len(sys.argv) > 3 else 12
first = int(sys.argv[4]) if len(sys.argv) > 4 else 0
cfg = Config(N=20, mode=2)
ctl = NtmMpc(config=cfg, device=0)
x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(first, B), 0)
rho, U_old = ctl.initial_state(x, cfg)
ws = ctl.new_active_ws(B, cfg)
Us, fls, xs = [], [], []
for k in range(K):
    out = ctl.step(x, rho, U_old, cfg, active_ws=ws)
    torch.cuda.synchronize()
    Us.append(out["U"].cpu().numpy().copy())
    fls.append(out["exitflag"].cpu().numpy().copy())
    x = out["x_next"].clone()
    xs.append(x.cpu().numpy().copy())
np.savez(out_path, U=np.stack(Us), flag=np.stack(fls), x=np.stack(xs))
print("saved", out_path, flush=True)
ctl.close()

#!/usr/bin/env python3
"""Re-run one saved scenario (gpurun_out/first_bad.npz from flag_trace.py) as a
B=1 batch with its carried warm-start workspace; with the trace build
(make trace NTM_DEBUG_SCEN=0, NTM_MPC_LIB=lib/libntm_mpc_trace.so) the kernel
prints its QP decisions.  Diagnostic only.

    python tools/repro_scen.py [npz] [index]"""
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

path = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "gpurun_out" / "first_bad.npz")
k = int(sys.argv[2]) if len(sys.argv) > 2 else 0
d = np.load(path)
N = d["rho"].shape[0] // 3
cfg, ocfg = Config(N=N, mode=2), O.Config(N=N, mode=2)
ctl = NtmMpc(config=cfg, device=0)
x, rho, uo, ws = (d[n][:, k:k + 1].copy() for n in ("x", "rho", "U_old", "ws"))
for use_ws in (True, False):
    dws = ntm_mpc.device_tensor(ws, 0, dtype=torch.int32) if use_ws else None
    out = ctl.step(ntm_mpc.device_tensor(x, 0), ntm_mpc.device_tensor(rho, 0), ntm_mpc.device_tensor(uo, 0), cfg,
                   active_ws=dws)
    torch.cuda.synchronize()
    print(f"ws={use_ws}: flag {int(out['exitflag'][0])} iters {int(out['inner_iters'][0])}", flush=True)
ref = cbind.step(x, rho, uo, ocfg)
print("oracle flag", int(ref["exitflag"][0]), "iters", int(ref["inner_iters"][0]))
print("x", x[:, 0].tolist(), "ws", ws[:, 0].tolist())
ctl.close()

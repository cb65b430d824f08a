"""Diagnose a teacher-forced literal-flag step mismatch (GPU vs C oracle)."""
import math
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "mpc-ntm-control_amd"), str(ROOT / "tests")]
import numpy as np
import torch
from oracle import cbind
from oracle import ntm_oracle as O
from ntm_mpc import Config, NtmMpc

N, flags, B, ks = int(sys.argv[1]), int(sys.argv[2]), 48, 4
ctl = NtmMpc()
cfg, ocfg = Config(N=N, mode=2, flags=flags), O.Config(N=N, mode=2, flags=flags)
x = O.scenario_x0(np.arange(B)).T
rho, Uo = cbind.initial_state(x, ocfg)
ws = ctl.new_active_ws(B, cfg)
T = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda:0")
for k in range(ks):
    ref = cbind.step(x, rho, Uo, ocfg)
    out = ctl.step(T(x), T(rho), T(Uo), cfg, active_ws=ws)
    torch.cuda.synchronize()
    U = out["U"].cpu().numpy(); it = out["inner_iters"].cpu().numpy(); fl = out["exitflag"].cpu().numpy()
    xp = out["x_pred"].cpu().numpy()
    dU = np.max(np.abs(U - ref["U"]), axis=0) / 2e6
    dxp = np.max(np.abs(xp - ref["x_pred"]) / np.tile([0.15, 2000 * math.pi], N + 1)[:, None], axis=0)
    s = int(np.argmax(dxp))
    print(f"k={k} worst dxp {dxp[s]:.3e} scen {s} dU {dU[s]:.3e} iters gpu {it[s]} ref {ref['inner_iters'][s]} "
          f"flag {fl[s]}/{ref['exitflag'][s]} x {x[:, s]} max dU all {dU.max():.3e} iters differ {(it != ref['inner_iters']).sum()}")
    if dxp[s] > 1e-9:
        print("  U gpu", U[:, s]); print("  U ref", ref["U"][:, s])
        print("  xp gpu", xp[:, s]); print("  xp ref", ref["x_pred"][:, s])
    x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]

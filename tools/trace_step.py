"""Diagnostic: replay an oracle trajectory to step K, then run one GPU step with
the trace build (make -C mpc-ntm-control_amd trace NTM_DEBUG_SCEN=s).
usage: trace_step.py N mode K"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ["NTM_MPC_LIB"] = os.path.join(ROOT, "mpc-ntm-control_amd", "lib", "libntm_mpc_trace.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]
import numpy as np, torch
from ntm_mpc import NtmMpc, Config
from oracle import ntm_oracle as O, cbind
N, mode, K = (int(a) for a in sys.argv[1:4])
ctl = NtmMpc()
cfg, ocfg = Config(N=N, mode=mode), O.Config(N=N, mode=mode)
B = 48
x = O.scenario_x0(np.arange(B)).T.copy()
rho, Uo = cbind.initial_state(x, ocfg)
for k in range(K):
    ref = cbind.step(x, rho, Uo, ocfg)
    x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]
T = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda")
out = ctl.step(T(x), T(rho), T(Uo), cfg)
torch.cuda.synchronize()
print("GPU U", out["U"].cpu().numpy()[:, 33], "iters", out["inner_iters"].cpu().numpy()[33], flush=True)
s = 33
Rho = rho[:, s].reshape(N, 3).T
Phi, Gam, Lam = O.lift(Rho, O.Physics(), ocfg)
G, F = O.cost(Phi, Gam, Lam, x[:, s], ocfg)
Lin, b = O.constraints(Phi, Gam, Lam, x[:, s], ocfg)
U, flag, info = O.qp_solve(G, F, Lin, b)
print("oracle it1 U", U, "active", sorted(info["active"]), "iters", info.get("iters"))

"""Diagnostic: first teacher-forced mismatch of the GPU step vs the C oracle (mode 3)."""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]
import numpy as np, torch
from ntm_mpc import NtmMpc, Config
from oracle import ntm_oracle as O, cbind
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctl = NtmMpc()
cfg, ocfg = Config(N=N, mode=mode), O.Config(N=N, mode=mode)
B = 48
x = O.scenario_x0(np.arange(B)).T.copy()
rho, Uo = cbind.initial_state(x, ocfg)
T = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda")
for k in range(12):
    ref = cbind.step(x, rho, Uo, ocfg)
    tr, tu = T(rho), T(Uo)
    out = ctl.step(T(x), tr, tu, cfg)
    torch.cuda.synchronize()
    U = out["U"].cpu().numpy()
    e = np.max(np.abs(U - ref["U"]), axis=0) / cfg.umax
    bad = np.where(e > 1e-8)[0]
    if len(bad):
        s = bad[0]
        print("step", k, "bad scenarios", bad, "err", e[bad])
        print("gpu flag/iters", out["exitflag"].cpu().numpy()[s], out["inner_iters"].cpu().numpy()[s],
              "ref", ref["exitflag"][s], ref["inner_iters"][s])
        print("U gpu", U[:, s]); print("U ref", ref["U"][:, s])
        Rho = rho[:, s].reshape(N, 3).T
        Phi, Gam, Lam = O.lift(Rho, O.Physics(), ocfg)
        G, F = O.cost(Phi, Gam, Lam, x[:, s], ocfg)
        Lin, b = O.constraints(Phi, Gam, Lam, x[:, s], ocfg)
        for name, UU in (("gpu", U[:, s]), ("ref", ref["U"][:, s])):
            print(name, "max viol", np.max(Lin @ UU - b), "obj", 0.5 * UU @ G @ UU + F @ UU)
        break
    x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]
else:
    print("no mismatch")

# the failing QP through the dense quadprog entry (same gi_solve, no warm start)
if len(sys.argv) > 3:
    Nq = 4
    c4 = O.Config(N=Nq, mode=3)
    Bq = 48
    xq = O.scenario_x0(np.arange(Bq)).T.copy()
    rq, uq = cbind.initial_state(xq, c4)
    for k in range(10):
        ref = cbind.step(xq, rq, uq, c4)
        xq, rq, uq = ref["x_next"], ref["rho"], ref["U_old"]
    s = 33
    Rho = rq[:, s].reshape(Nq, 3).T
    Phi, Gam, Lam = O.lift(Rho, O.Physics(), c4)
    G, F = O.cost(Phi, Gam, Lam, xq[:, s], c4)
    Lin, b = O.constraints(Phi, Gam, Lam, xq[:, s], c4)
    Gb = T(G.reshape(-1, order="F")[:, None]); Fb = T(F[:, None])
    Lb = T(Lin.reshape(-1, order="F")[:, None]); bb = T(b[:, None])
    U, flag, its = ctl.quadprog(Gb, Fb, Lb, bb)
    torch.cuda.synchronize()
    print("dense quadprog U", U.cpu().numpy()[:, 0], "flag", flag.cpu().numpy(), "its", its.cpu().numpy())
    Uc, fc, ic = cbind.qp(G, F, Lin, b)
    print("C oracle U", Uc, fc, ic)

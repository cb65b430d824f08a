"""Report replacement for NTM_MPC_Sim.m:134-164 (presentation
only, not part of the hot path).

Runs the closed loop on the GPU (ntm_mpc_run through the C-ABI) and writes the
reference's workspace variables for each scenario: xk (2 x k_sim+1), uk
(1 x k_sim), Uk (N x k_sim), exitflag, inner_iters.  Outputs:
  * <out>.npz  (all scenarios),
  * <out>.csv  (scenario 0: k, w, omega, u, exitflag),
  * <out>.png  (scenario 0, the reference's figure: stairs of the states and
    of the input, "Constrained quasi-LPV MPC State and Input Trajectory").

    python tools/report.py [--scenarios B] [--k-sim 20] [--N 20] [--mode 2] [--out gpurun_out/report]
"""
import argparse
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenarios", type=int, default=1)
    ap.add_argument("--k-sim", type=int, default=20)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mode", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "report"))
    args = ap.parse_args()

    import numpy as np
    import torch

    import ntm_mpc
    from ntm_mpc import Config, NtmMpc

    cfg = Config(N=args.N, mode=args.mode)
    ctl = NtmMpc(config=cfg)
    B, K, N = args.scenarios, args.k_sim, args.N
    x0 = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(0, B))
    out = ctl.run(x0, K, cfg)
    torch.cuda.synchronize()
    xk = out["xk"].cpu().numpy().reshape(K + 1, 2, B).transpose(2, 1, 0)       # (B, 2, K+1)
    uk = out["uk"].cpu().numpy().T[:, None, :]                                  # (B, 1, K)
    Uk = out["Uk"].cpu().numpy().reshape(K, N, B).transpose(2, 1, 0)            # (B, N, K)
    flags = out["exitflag"].cpu().numpy().T
    iters = out["inner_iters"].cpu().numpy().T
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    np.savez(args.out + ".npz", xk=xk, uk=uk, Uk=Uk, exitflag=flags, inner_iters=iters, N=N, mode=args.mode)
    with open(args.out + ".csv", "w") as f:
        f.write("k,w_m,omega_rad_s,u_W,exitflag,inner_iters\n")
        for k in range(K + 1):
            u = f"{uk[0, 0, k]:.17g}" if k < K else ""
            fl = str(flags[0, k]) if k < K else ""
            it = str(iters[0, k]) if k < K else ""
            f.write(f"{k},{xk[0, 0, k]:.17g},{xk[0, 1, k]:.17g},{u},{fl},{it}\n")
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:                                                          # pragma: no cover
        print("matplotlib missing: wrote npz/csv only")
        return
    fig, ax = plt.subplots(1, 2, figsize=(11, 4))
    ax[0].step(np.arange(K + 1), xk[0, 0], where="post", label="w [m]")
    ax0b = ax[0].twinx()
    ax0b.step(np.arange(K + 1), xk[0, 1], where="post", color="C1", label="omega [rad/s]")
    ax[0].set_xlabel("k")
    ax[0].set_ylabel("w [m]")
    ax0b.set_ylabel("omega [rad/s]")
    ax[1].step(np.arange(K), uk[0, 0], where="post", label="P_ECCD [W]")
    ax[1].set_xlabel("k")
    ax[1].set_ylabel("u = P_ECCD [W]")
    fig.suptitle("Constrained quasi-LPV MPC State and Input Trajectory (MI355X, scenario 0)")
    fig.tight_layout()
    fig.savefig(args.out + ".png", dpi=120)
    print(f"wrote {args.out}.npz/.csv/.png: {B} scenarios x {K} steps, N={N}, mode={args.mode}")


if __name__ == "__main__":
    main()

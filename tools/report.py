"""Report replacement for NTM_MPC_Sim.m:134-164 (presentation
only, not part of the hot path).

Runs the closed loop on the GPU (ntm_mpc_run through the C-ABI) and writes the
reference's workspace variables for each scenario: xk (2 x k_sim+1), uk
(1 x k_sim), Uk (N x k_sim), the predicted island width wpred (k_sim x N+1: row
k is w of the last rollout of step k, NTM_MPC_Sim.m:110-117), exitflag and
inner_iters.  Outputs:
  * <out>.npz  (all scenarios),
  * <out>.csv  (scenario 0: k, w, omega, u, exitflag, inner iterations, and the
    predicted w one and N steps ahead),
  * <out>.png  (scenario 0, the reference's figure: stairs of the states and of
    the input, "Constrained quasi-LPV MPC State and Input Trajectory", plus a
    panel of every step's predicted island width).

    python tools/report.py [--scenarios B] [--k-sim 20] [--N 20] [--mode 2] [--out gpurun_out/report]

``closed_loop_report`` (the GPU run, reshaped to the reference's layout) and
``write_report`` (the files) are importable; tests/test_report.py drives them.
"""
import argparse
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]

import numpy as np  # noqa: E402


def closed_loop_report(ctl, x0, k_sim, cfg, gen=None):
    """ntm_mpc_run for x0 (2, B) on the GPU; returns the reference's workspace
    variables per scenario: xk (B, 2, k_sim+1), uk (B, 1, k_sim), Uk (B, N,
    k_sim), wpred (B, k_sim, N+1), exitflag and inner_iters (B, k_sim).  ``gen``
    (ntm_mpc.ScenarioGen) attaches the scenario generator for this run."""
    import torch

    import ntm_mpc
    B, N, K = x0.shape[1], cfg.N, k_sim
    ctl.set_scenarios(gen)
    try:
        out = ctl.run(ntm_mpc.device_tensor(np.ascontiguousarray(x0, dtype=np.float64)), K, cfg)
        torch.cuda.synchronize()
        host = {k: v.cpu().numpy() for k, v in out.items()}
    finally:
        if gen is not None:
            ctl.set_scenarios(None)
    return {
        "xk": host["xk"].reshape(K + 1, 2, B).transpose(2, 1, 0),
        "uk": host["uk"].T[:, None, :],
        "Uk": host["Uk"].reshape(K, N, B).transpose(2, 1, 0),
        "wpred": host["wpred"].reshape(K, N + 1, B).transpose(2, 0, 1),
        "exitflag": host["exitflag"].T,
        "inner_iters": host["inner_iters"].T,
        "N": N, "mode": cfg.mode,
    }


def write_report(rep, out, plot=True):
    """Write <out>.npz (all scenarios), <out>.csv (scenario 0) and, with
    matplotlib, <out>.png.  Returns the list of files written."""
    xk, uk, wpred = rep["xk"], rep["uk"], rep["wpred"]
    flags, iters = rep["exitflag"], rep["inner_iters"]
    K = uk.shape[2]
    N = wpred.shape[2] - 1
    os.makedirs(os.path.dirname(os.path.abspath(out)) or ".", exist_ok=True)
    files = [out + ".npz", out + ".csv"]
    np.savez(files[0], **{k: v for k, v in rep.items()})
    with open(files[1], "w") as f:
        f.write("k,w_m,omega_rad_s,u_W,exitflag,inner_iters,wpred_1_m,wpred_N_m\n")
        for k in range(K + 1):
            if k < K:
                tail = (f"{uk[0, 0, k]:.17g},{flags[0, k]},{iters[0, k]},"
                        f"{wpred[0, k, 1]:.17g},{wpred[0, k, N]:.17g}")
            else:
                tail = ",,,,"
            f.write(f"{k},{xk[0, 0, k]:.17g},{xk[0, 1, k]:.17g},{tail}\n")
    if not plot:
        return files
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:                                                          # pragma: no cover
        print("matplotlib missing: wrote npz/csv only")
        return files
    fig, ax = plt.subplots(1, 3, figsize=(16, 4))
    ax[0].step(np.arange(K + 1), xk[0, 0], where="post", label="w [m]")
    ax0b = ax[0].twinx()
    ax0b.step(np.arange(K + 1), xk[0, 1], where="post", color="C1", label="omega [rad/s]")
    ax[0].set_xlabel("k")
    ax[0].set_ylabel("w [m]")
    ax0b.set_ylabel("omega [rad/s]")
    ax[1].step(np.arange(K), uk[0, 0], where="post", label="P_ECCD [W]")
    ax[1].set_xlabel("k")
    ax[1].set_ylabel("u = P_ECCD [W]")
    for k in range(K):                                      # predicted w of every step, i = k .. k+N
        ax[2].plot(np.arange(k, k + N + 1), wpred[0, k], color=plt.cm.viridis(k / max(K - 1, 1)), lw=0.8)
    ax[2].step(np.arange(K + 1), xk[0, 0], where="post", color="k", lw=1.5, label="w (plant)")
    ax[2].set_xlabel("k + i")
    ax[2].set_ylabel("predicted w [m]")
    ax[2].legend(loc="best")
    fig.suptitle("Constrained quasi-LPV MPC State and Input Trajectory (MI355X, scenario 0)")
    fig.tight_layout()
    fig.savefig(out + ".png", dpi=120)
    plt.close(fig)
    files.append(out + ".png")
    return files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenarios", type=int, default=1)
    ap.add_argument("--k-sim", type=int, default=20)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mode", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "report"))
    args = ap.parse_args()

    import ntm_mpc
    from ntm_mpc import Config, NtmMpc

    cfg = Config(N=args.N, mode=args.mode)
    ctl = NtmMpc(config=cfg)
    rep = closed_loop_report(ctl, ntm_mpc.scenarios_x0(0, args.scenarios), args.k_sim, cfg)
    files = write_report(rep, args.out)
    print(f"wrote {', '.join(files)}: {args.scenarios} scenarios x {args.k_sim} steps, N={args.N}, mode={args.mode}")


if __name__ == "__main__":
    main()

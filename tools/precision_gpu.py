"""BASELINE config 5's "fp32 vs fp64 tolerance sweep" on the GPU.

QPs met along oracle closed-loop trajectories (the quadprog call of
NTM_MPC_Sim.m:97, N = 10 / 20 / 50, modes 2 and 3) are solved three ways on
the MI355X and compared with the fp64 C oracle:
  * fp64: ntm_qp_device (the product's QP path);
  * fp32: ntm_qp_mixed_device's fp32 Goldfarb-Idnani on fp32-rounded data (U32);
  * mixed: the fp32 active set re-solved exactly in fp64 and KKT-certified, the
    fp64 solve as fallback (U).
Errors are max |dU| / umax per QP (median / p90 / max over the QPs); the
certified fraction says how often the fp32 active set was already the fp64
optimum's.  Timing: one batch of the QPs replicated to --timing-batch.

    python tools/precision_gpu.py [scenarios] [steps] [--out profiles/r03_precision.json]
"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import cbind  # noqa: E402
from oracle import ntm_oracle as O  # noqa: E402


def qps(N, mode, n_scen, n_steps):
    cfg = O.Config(N=N, mode=mode)
    ph = O.Physics()
    x = O.scenario_x0(np.arange(n_scen)).T.copy()
    rho, Uo = cbind.initial_state(x, cfg)
    out = []
    for _ in range(n_steps):
        for s in range(n_scen):
            Rho = rho[:, s].reshape(N, 3).T
            Phi, Gam, Lam = O.lift(Rho, ph, cfg)
            G, F = O.cost(Phi, Gam, Lam, x[:, s], cfg)
            Lin, b = O.constraints(Phi, Gam, Lam, x[:, s], cfg)
            out.append((G, F, Lin, b))
        ref = cbind.step(x, rho, Uo, cfg)
        x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]
    return out


def stats(e):
    e = np.asarray(e)
    return {"median": float(np.median(e)), "p90": float(np.percentile(e, 90)), "max": float(e.max())}


def run(ctl, N, mode, n_scen, n_steps, timing_batch):
    data = qps(N, mode, n_scen, n_steps)
    n = len(data)
    m = data[0][2].shape[0]
    Gb = np.stack([d[0].reshape(-1, order="F") for d in data], axis=1)
    Fb = np.stack([d[1] for d in data], axis=1)
    Lb = np.stack([d[2].reshape(-1, order="F") for d in data], axis=1)
    bb = np.stack([d[3] for d in data], axis=1)
    T = ctl.tensor
    G_, F_, L_, b_ = T(Gb), T(Fb), T(Lb), T(bb)
    U64, f64, _ = ctl.quadprog(G_, F_, L_, b_)
    U, U32, fm, info, it32 = ctl.quadprog_mixed(G_, F_, L_, b_)
    torch.cuda.synchronize()
    U64, f64, U, U32, fm, info = (t.cpu().numpy() for t in (U64, f64, U, U32, fm, info))
    e64, e32, emx = [], [], []
    for i, (G, F, Lin, b) in enumerate(data):
        Ur, fr, _ = cbind.qp(G, F, Lin, b)
        if fr != 1 or f64[i] != 1 or fm[i] != 1:
            continue
        e64.append(np.max(np.abs(U64[:, i] - Ur)) / 2e6)
        e32.append(np.max(np.abs(U32[:, i] - Ur)) / 2e6)
        emx.append(np.max(np.abs(U[:, i] - Ur)) / 2e6)
    # timing: the batch replicated
    rep = max(1, timing_batch // n)
    big = [t.repeat(1, rep) for t in (G_, F_, L_, b_)]
    times = {}
    for name, fn in (("fp64", lambda: ctl.quadprog(*big)), ("mixed", lambda: ctl.quadprog_mixed(*big))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        times[name] = (time.perf_counter() - t) / 3 * 1e3
    return {"N": N, "mode": mode, "m": m, "qps": n, "compared": len(e64),
            "err_fp64": stats(e64), "err_fp32": stats(e32), "err_mixed": stats(emx),
            "fp32_set_certified_frac": float(np.mean((info & 1) != 0)),
            "fp64_fallback_frac": float(np.mean((info & 2) != 0)),
            "fp32_not_optimal_frac": float(np.mean((info & 4) != 0)),
            "fp32_gi_iters_mean": float(it32.double().mean().item()),
            "timing_batch": n * rep, "ms_fp64_qp_batch": times["fp64"], "ms_mixed_qp_batch": times["mixed"]}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("scen", type=int, nargs="?", default=16)
    ap.add_argument("steps", type=int, nargs="?", default=4)
    ap.add_argument("--timing-batch", type=int, default=20000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from ntm_mpc import NtmMpc
    ctl = NtmMpc()
    rows = []
    for N in (10, 20, 50):
        for mode in (2, 3):
            r = run(ctl, N, mode, a.scen, a.steps, a.timing_batch)
            rows.append(r)
            print(f"N={N:2d} mode={mode} QPs={r['qps']:4d}  |dU|/umax vs oracle: fp64 max {r['err_fp64']['max']:.1e}  "
                  f"fp32 med {r['err_fp32']['median']:.1e} p90 {r['err_fp32']['p90']:.1e} max {r['err_fp32']['max']:.1e}"
                  f"  mixed max {r['err_mixed']['max']:.1e}  certified {r['fp32_set_certified_frac']:.2f} "
                  f"fallback {r['fp64_fallback_frac']:.2f}  ms/batch fp64 {r['ms_fp64_qp_batch']:.2f} "
                  f"mixed {r['ms_mixed_qp_batch']:.2f}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"tool": "tools/precision_gpu.py", "scenarios": a.scen, "steps": a.steps, "rows": rows}, f,
                      indent=1)


if __name__ == "__main__":
    main()

"""Precision study for BASELINE config 5 ("fp32 vs fp64 tolerance sweep").

For QPs met along oracle closed-loop trajectories (N = 10, 20, 50; modes 2 and
3), measures how far the control sequence moves when the QP data (G, F, Lin,
b) are stored in fp32 and the QP is then solved exactly in fp64 on that data.
This is a lower bound on the error of any fp32 or mixed-precision build of the
path: it charges only the rounding of the data and none of the solver's
arithmetic.  The fp64 reference is the oracle's certified solve.  Results go
to DESIGN.md §6 (precision).

    python tools/precision_sweep.py [scenarios] [steps]
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402

from oracle import cbind  # noqa: E402
from oracle import ntm_oracle as O  # noqa: E402


def sweep(N, mode, n_scen, n_steps):
    cfg = O.Config(N=N, mode=mode)
    ph = O.Physics()
    x = O.scenario_x0(np.arange(n_scen)).T.copy()
    rho, Uo = cbind.initial_state(x, cfg)
    errs, conds = [], []
    for k in range(n_steps):
        for s in range(n_scen):
            Rho = rho[:, s].reshape(N, 3).T
            Phi, Gam, Lam = O.lift(Rho, ph, cfg)
            G, F = O.cost(Phi, Gam, Lam, x[:, s], cfg)
            Lin, b = O.constraints(Phi, Gam, Lam, x[:, s], cfg)
            U64, f64, _ = cbind.qp(G, F, Lin, b)
            r32 = lambda a: a.astype(np.float32).astype(np.float64)      # noqa: E731
            U32, f32, _ = cbind.qp(r32(G), r32(F), r32(Lin), r32(b))
            if f64 == 1 and f32 == 1:
                errs.append(np.max(np.abs(U32 - U64)) / cfg.umax)
            conds.append(np.linalg.cond(G))
        ref = cbind.step(x, rho, Uo, cfg)
        x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]
    e = np.array(errs)
    return {"N": N, "mode": mode, "qps": len(conds), "cond_median": float(np.median(conds)),
            "err_median": float(np.median(e)), "err_p90": float(np.percentile(e, 90)), "err_max": float(e.max())}


def main():
    n_scen = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    print(f"{'N':>3} {'mode':>4} {'QPs':>5} {'cond(G) med':>12} {'|dU|/umax med':>14} {'p90':>10} {'max':>10}")
    for N in (10, 20, 50):
        for mode in (2, 3):
            r = sweep(N, mode, n_scen, n_steps)
            print(f"{r['N']:>3} {r['mode']:>4} {r['qps']:>5} {r['cond_median']:>12.2e} {r['err_median']:>14.2e} "
                  f"{r['err_p90']:>10.2e} {r['err_max']:>10.2e}", flush=True)


if __name__ == "__main__":
    main()

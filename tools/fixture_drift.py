"""Diagnostic: the C oracle (oracle/ntm_oracle.c) against the NumPy closed-loop fixtures
(tests/golden/closed_loop_*.npz): max |duk|, |dUk| / umax, |dxk| / (0.15 m, 2000 pi),
|dwpred| / 0.15 m and the fraction of equal inner-iteration counts.  The GPU fixture
tests (tests/test_gpu_golden.py) cite its numbers for their RUN_TOL.

    python tools/fixture_drift.py
"""
import math, numpy as np, sys
sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parent.parent))
from oracle import cbind, ntm_oracle as O
names = ["closed_loop_m0_N10.npz", "closed_loop_m1_N20.npz", "closed_loop_m2_N20.npz", "closed_loop_m2_N3.npz",
         "closed_loop_m3_N20.npz", "closed_loop_m3_N50.npz", "closed_loop_gen_m2_N20.npz", "closed_loop_gen_m2_N3.npz"]
for name in names:
    d = np.load(str(__import__("pathlib").Path(__file__).resolve().parent.parent / "tests" / "golden" / name))
    mode = int(name.split("_m")[1][0]); N = int(name.split("_N")[1].split(".")[0])
    c = O.Config(N=N, mode=mode); K = int(d["k_sim"]); S = d["x0"].shape[0]
    gen = None
    if "gen_seed" in d.files:
        gen = O.ScenarioGen(seed=int(d["gen_seed"]), first_id=int(d["gen_first_id"]), k0=int(d["gen_k0"]),
                            sigma_w=float(d["gen_sigma_w"]), sigma_omega=float(d["gen_sigma_omega"]),
                            jbs_spread=float(d["gen_jbs_spread"]), wdep_spread=float(d["gen_wdep_spread"]))
    out = cbind.run(np.ascontiguousarray(d["x0"].T), c, K, gen=gen)
    sc = max(c.umax, np.max(np.abs(d["Uk"])))
    du = np.max(np.abs(out["uk"].T - d["uk"])) / sc
    dU = np.max(np.abs(out["Uk"].reshape(K, N, S).transpose(2, 1, 0) - d["Uk"])) / sc
    xs = np.array([0.15, 2000 * math.pi])[None, :, None]
    dx = np.max(np.abs(out["xk"].reshape(K + 1, 2, S).transpose(2, 1, 0) - d["xk"]) / xs)
    dw = np.max(np.abs(out["wpred"].reshape(K, N + 1, S).transpose(2, 0, 1) - d["wpred"])) / 0.15
    it = (out["inner_iters"].T == d["inner_iters"]).mean()
    print(f"{name:32s} K={K:2d} S={S} maxU {np.max(np.abs(d['Uk'])):.2e} uk {du:.2e} Uk {dU:.2e} xk {dx:.2e} wpred {dw:.2e} iters_same {it:.2f}")

"""Diagnostic (not a test): which carried active set predicts inner iteration 2's
optimum best (the iteration where 72% of the N = 20 Goldfarb-Idnani fallbacks
start, profiles/r05_phases.txt).  NumPy oracle closed loops (active sets of every
LPV iteration recorded, tests/golden/make_golden._step_record) over steps lo..hi;
for each predictor, the fraction of iteration-2 QPs whose optimal active set it
equals exactly, and within one or two rows (symmetric difference).

    python tools/set_predictor_study.py N mode n_scen lo hi
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]
from make_golden import _step_record  # noqa: E402
from oracle import cbind  # noqa: E402
from oracle import ntm_oracle as O  # noqa: E402

N, mode, S, lo, hi = (int(v) for v in sys.argv[1:6])
ph = O.Physics()
cfg = O.Config(N=N, mode=mode)


def shift(st):
    """The device's receding-horizon shift (ntm_device.h shifted_into_act)."""
    out, dup = [], []
    for i in st:
        if i >= 6 * N + 4:
            j = ((i - (6 * N + 4)) >> 1) + 1
            if j >= 2:
                out.append(i - 2)
            if j == N - 1:
                dup.append(i)
        elif i >= 6 * N:
            out.append(6 * (N - 1) + 2 + (i - 6 * N))
            dup.append(i)
        else:
            blk, rr = divmod(i, 6)
            if blk >= 2 or (blk == 1 and rr < 2):
                out.append(i - 6)
            if blk == N - 1 and rr < 2:
                dup.append(i)
    if len(out) + len(dup) <= N:
        out += dup
    return set(out)


x = O.scenario_x0(np.arange(S)).T.copy()
rho, Uo = cbind.initial_state(x, cfg)
for _ in range(lo - 2):
    r = cbind.step(x, rho, Uo, cfg)
    x, rho, Uo = r["x_next"], r["rho"], r["U_old"]
preds = {}
names = ["prev even (S10 k-1)", "shift(prev even)", "S1 k", "S1 k ^ (S9 ^ S10) k-1", "prev odd (S9 k-1)",
         "shift(S1 k)"]
stats = {n: [0, 0, 0] for n in names}
count = 0
dists = []
for s in range(S):
    xk, Rho, Uold = x[:, s].copy(), rho[:, s].reshape(N, 3).T.copy(), Uo[:, s].copy()
    prev = None
    for k in range(lo - 1, hi + 1):
        recs, xn, Rho, Uold = _step_record(xk, Rho, Uold, ph, cfg)
        sets = {rc["it"]: set(rc["act"]) for rc in recs if rc["flag"] == O.EXIT_OK}
        if k >= lo and prev is not None and 2 in sets and 1 in sets and 9 in prev and 10 in prev:
            tgt = sets[2]
            cands = [prev[10], shift(prev[10]), sets[1], sets[1] ^ (prev[9] ^ prev[10]), prev[9], shift(sets[1])]
            dists.append((len(prev[10] ^ tgt), len(shift(prev[10]) ^ tgt), len(tgt), len(prev[10])))
            for n, c in zip(names, cands):
                d = len(c ^ tgt)
                stats[n][0] += d == 0
                stats[n][1] += d <= 1
                stats[n][2] += d <= 2
            count += 1
        prev = sets
        xk = xn
    print(f"scenario {s} done", flush=True)
print(f"N={N} mode={mode}: {count} iteration-2 QPs, steps {lo}-{hi}, {S} scenarios")
for n in names:
    e, d1, d2 = stats[n]
    print(f"  {n:28s} exact {e / count:.2f}   |diff| <= 1 {d1 / count:.2f}   <= 2 {d2 / count:.2f}")
d = np.array(dists)
print("  min(prev even, shift) exact %.2f  <=1 %.2f  <=2 %.2f" % ((d[:, :2].min(1) == 0).mean(), (d[:, :2].min(1) <= 1).mean(),
                                                                  (d[:, :2].min(1) <= 2).mean()))
print("  |prev even ^ target| histogram:", np.bincount(d[:, 0]).tolist())
print("  |shift ^ target| histogram:", np.bincount(d[:, 1]).tolist())
print("  target sizes:", np.bincount(d[:, 2]).tolist())
far = d[:, 0] >= 3
print("  prev even diff >= 3: %d cases; their |shift ^ target| histogram:" % far.sum(), np.bincount(d[far, 1]).tolist())

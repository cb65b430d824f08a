"""Diagnostic (not a test): box-only QPs (mode 1, BASELINE config 2), offline.

At B = 1024 every scenario runs on a SIMD of its own, so a step-batch lasts as
long as its slowest scenario, and a scenario's step costs about one certified
re-solve per QP plus one per exchange (tools/c2_tail.py, c2_scen_phases.py:
13 exchanges double a scenario's QP time).  This replays the QPs of NumPy-oracle
closed loops (NTM_MPC_Sim.m:94-127) from the carried set the kernel starts from
(qp_phase: the set of inner iteration it-2, the previous step's for it <= 2) and
scores exchange rules by the mean re-solves per QP and by the per-step MAXIMUM
over scenarios of a scenario's re-solves in that step (what sets the batch time).

    python tools/box_study.py n_scen lo hi
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]
from make_golden import _step_record  # noqa: E402
from oracle import cbind  # noqa: E402
from oracle import ntm_oracle as O  # noqa: E402

N = 20
S, lo, hi = (int(v) for v in sys.argv[1:4])
ph = O.Physics()
cfg = O.Config(N=N, mode=O.MODE_BOX)


def solve(G, F, D, act):
    """Re-solve of a set of box rows (ids < N lower, >= N upper bound): (fk, V, lam by
    position, slacks by row id).  fk as the kernel's: 0 certified, 1 dual, 2 primal,
    4 both, 3 colliding."""
    var = [a % N for a in act]
    if len(set(var)) != len(var):
        return 3, None, None, None
    lo_v = cfg.umin / D
    hi_v = cfg.umax / D
    Gt = G * D[:, None] * D[None, :]
    Ft = F * D
    fixed = np.zeros(N, bool)
    V = np.zeros(N)
    for a, j in zip(act, var):
        fixed[j] = True
        V[j] = lo_v[j] if a < N else hi_v[j]
    fr = ~fixed
    if fr.any():
        V[fr] = np.linalg.solve(Gt[np.ix_(fr, fr)], -(Ft[fr] + Gt[np.ix_(fr, fixed)] @ V[fixed]))
    g = Gt @ V + Ft
    # GI form: lower row n = e_j (n'V >= lo), upper n = -e_j; g = sum lam n
    lam = np.array([g[j] if a < N else -g[j] for a, j in zip(act, var)])
    vmax = max(1.0, np.abs(V).max())
    s = np.concatenate([V - lo_v, hi_v - V])
    bc = np.concatenate([lo_v, -hi_v])
    pbad = np.any(s < -1e-9 * np.maximum(vmax, np.abs(bc)))
    dbad = len(act) > 0 and lam.min() < -1e-9 * max(1.0, np.abs(lam).max())
    fk = 0 if not (pbad or dbad) else (1 if not pbad else (2 if not dbad else 4))
    return fk, V, lam, s


def single(G, F, D, act, budget=16, batch_add=False, batch_drop=False):
    """qp_phase's stage 4: a violated bound joins (a negative multiplier leaves in the
    same exchange; in a full set it takes the smallest multiplier's place); a negative
    multiplier alone leaves.  batch_add: every violated bound joins; batch_drop: every
    negative multiplier leaves."""
    act, n = list(act), 0
    while True:
        fk, V, lam, s = solve(G, F, D, act)
        n += 1
        if fk == 0:
            return True, n
        if fk == 3 or n > budget:
            return False, n
        tol = -1e-9 * max(1.0, np.abs(lam).max()) if len(act) else 0.0
        fp = int(np.argmin(lam)) if len(act) else -1
        neg = [k for k in range(len(act)) if lam[k] < tol]
        if fk == 1:
            drop = set(neg) if batch_drop else {fp}
            act = [a for k, a in enumerate(act) if k not in drop]
            continue
        sm = s.copy()
        sm[act] = np.inf
        order = [int(i) for i in np.argsort(sm, kind="stable") if np.isfinite(sm[i]) and sm[i] < 0]
        vmax = max(1.0, np.abs(V).max())
        lo_v = np.concatenate([cfg.umin / D, -cfg.umax / D])
        order = [i for i in order if sm[i] < -1e-9 * max(vmax, abs(lo_v[i]))]
        if not order:
            return False, n
        adds = order if batch_add else order[:1]
        drop = (set(neg) if batch_drop else {fp}) if fk == 4 else set()
        keep = [a for k, a in enumerate(act) if k not in drop]
        for p in adds:
            if len(keep) < N:
                keep.append(p)
            else:
                keep[int(np.argmin([lam[act.index(a)] if a in act else np.inf for a in keep]))] = p
        act = keep


def pdas(G, F, D, act, budget=16):
    """Primal-dual active set: every violated bound in, every negative multiplier out."""
    act, n = list(act), 0
    while True:
        fk, V, lam, s = solve(G, F, D, act)
        n += 1
        if fk == 0:
            return True, n
        if fk == 3 or n > budget:
            return False, n
        tol = -1e-9 * max(1.0, np.abs(lam).max()) if len(act) else 0.0
        keep = [a for k, a in enumerate(act) if lam[k] >= tol]
        vmax = max(1.0, np.abs(V).max())
        lo_v = np.concatenate([cfg.umin / D, -cfg.umax / D])
        viol = [i for i in range(2 * N) if i not in act and s[i] < -1e-9 * max(vmax, abs(lo_v[i]))]
        act = (keep + viol)[:N]


strategies = {
    "single exchanges (kernel)": lambda G, F, D, a: single(G, F, D, a),
    "all violated join": lambda G, F, D, a: single(G, F, D, a, batch_add=True),
    "all negative leave": lambda G, F, D, a: single(G, F, D, a, batch_drop=True),
    "both (batch add + drop)": lambda G, F, D, a: single(G, F, D, a, batch_add=True, batch_drop=True),
    "PDAS": pdas,
}


def shift_box(st):
    """Receding-horizon shift of a box set: stage j's bound moves to stage j-1, the last
    stage's bound is kept (it also holds the new last stage)."""
    out = [a - 1 for a in st if a % N >= 1]
    out += [a for a in st if a % N == N - 1]
    return list(dict.fromkeys(out))


# carried-set rules for the first two inner iterations (k = the step's previous sets)
cands = {
    "kernel (it-2; prev 8+it)": lambda prev, sets, it: prev.get(8 + it),
    "shifted prev 8+it": lambda prev, sets, it: shift_box(prev[8 + it]) if 8 + it in prev else None,
    "shifted prev last": lambda prev, sets, it: shift_box(prev[max(prev)]),
    "it 2: this step's it 1": lambda prev, sets, it: prev.get(9) if it == 1 else sets.get(1),
}
x = O.scenario_x0(np.arange(S)).T.copy()
rho, Uo = cbind.initial_state(x, cfg)
for _ in range(lo - 2):
    r = cbind.step(x, rho, Uo, cfg)
    x, rho, Uo = r["x_next"], r["rho"], r["U_old"]
steps = list(range(lo, hi + 1))
tot = {k: np.zeros((len(steps), S)) for k in strategies}     # re-solves per scenario-step
ctot = {k: np.zeros((len(steps), S)) for k in cands}         # the same, single exchanges, by carried set
fails = {k: 0 for k in strategies}
nqp = 0
for s in range(S):
    xk, Rho, Uold = x[:, s].copy(), rho[:, s].reshape(N, 3).T.copy(), Uo[:, s].copy()
    prev = None
    for k in range(lo - 1, hi + 1):
        recs, xn, Rho, Uold = _step_record(xk, Rho, Uold, ph, cfg)
        sets = {rc["it"]: rc["act"] for rc in recs if rc["flag"] == O.EXIT_OK}
        if k >= lo and prev is not None:
            for rc in recs:
                it = rc["it"]
                cand = sets.get(it - 2) if it > 2 else prev.get(8 + it)
                if cand is None or rc["flag"] != O.EXIT_OK:
                    continue
                D = O.jacobi_scale(rc["G"])
                nqp += 1
                for name, f in strategies.items():
                    ok, n = f(rc["G"], rc["F"], D, cand)
                    fails[name] += not ok
                    tot[name][k - lo, s] += n
                for name, f in cands.items():
                    c2 = f(prev, sets, it) if it <= 2 else cand
                    if c2 is None:
                        c2 = cand
                    ok, n = single(rc["G"], rc["F"], D, c2)
                    ctot[name][k - lo, s] += n + (0 if ok else 16)
        prev = sets
        xk = xn
print(f"N={N} box QPs: {nqp} QPs, steps {lo}-{hi}, {S} scenarios (carried sets as the kernel's)")
for name in strategies:
    t = tot[name]
    print(f"  {name:28s} re-solves per QP {t.sum() / nqp:.3f}  not certified {fails[name]}  "
          f"per step: mean over scenarios {t.mean():.2f}, max over scenarios {t.max(axis=1).mean():.2f} "
          f"(worst {t.max():.0f})")
print("carried set at inner iterations 1-2 (single exchanges; a failure counts 16 more):")
for name in cands:
    t = ctot[name]
    print(f"  {name:28s} per step: mean over scenarios {t.mean():.2f}, max over scenarios {t.max(axis=1).mean():.2f} "
          f"(worst {t.max():.0f})")

"""Diagnostic (not a test): offline replay of the step kernel's certified warm start
at inner iteration 2 (qp_phase in csrc/ntm_device.h: the previous step's last even
set, single-row repairs, the shifted set, then Goldfarb-Idnani), against other
repair strategies, on the QPs of NumPy-oracle closed loops (NTM_MPC_Sim.m:94-127).
Each QP's exact optimum is the oracle's active set; a strategy is scored by how
often it certifies without GI and by the re-solves it spends.

    python tools/repair_study.py N mode n_scen lo hi [iters]

iters: which inner iterations to replay (default "2"; e.g. "2,3,4").
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden"), str(ROOT / "tools")]
from make_golden import _step_record  # noqa: E402
from oracle import cbind  # noqa: E402
from oracle import ntm_oracle as O  # noqa: E402

N, mode, S, lo, hi = (int(v) for v in sys.argv[1:6])
ITERS = [int(v) for v in (sys.argv[6] if len(sys.argv) > 6 else "2").split(",")]
ph = O.Physics()
cfg = O.Config(N=N, mode=mode)


def shift(st):
    """The device's receding-horizon shift (shifted_into_act), as in set_predictor_study."""
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
    return list(dict.fromkeys(out))


class QP:
    """One QP in the device's scaled form: V = U / D, unit-norm rows, slacks
    s = (b - Lin U) / rn (>= 0 feasible), multipliers mu = lambda rn."""

    def __init__(self, G, F, Lin, b):
        self.G, self.F, self.Lin, self.b = G, F, Lin, b
        self.D = O.jacobi_scale(G)
        self.rn = np.linalg.norm(Lin * self.D[None, :], axis=1)
        self.live = self.rn > 0
        nzl = [np.flatnonzero(Lin[i]) for i in range(len(b))]
        self.last = np.array([c[-1] if len(c) else -1 for c in nzl])
        self.nnz = np.array([len(c) for c in nzl])

    def kind(self, i):
        if mode == O.MODE_BOX:
            return 0 if i < N else 1
        if mode == O.MODE_FULL_DU and i >= 6 * N + 4:
            return 4
        if i < 6 * N and i % 6 < 2:
            return i % 6        # 0 lower, 1 upper u bound (full mode)
        return 2

    def solve(self, act):
        """(fk, U, mu, slack): fk 0 certified, 1 dual, 2 primal, 4 both, 3 singular."""
        act = list(act)
        if len(act) > N or len(set(act)) != len(act) or any(not self.live[a] for a in act):
            return 3, None, None, None
        A = self.Lin[act]
        fixed_by = {}
        for a in act:
            if self.nnz[a] == 1:
                j = int(self.last[a])
                if j in fixed_by:
                    return 3, None, None, None
                fixed_by[j] = a
        if act and np.linalg.matrix_rank(A, tol=1e-10 * np.abs(A).max()) < len(act):
            return 3, None, None, None
        q = len(act)
        M = np.zeros((N + q, N + q))
        M[:N, :N] = self.G
        M[:N, N:] = A.T
        M[N:, :N] = A
        rhs = np.concatenate([-self.F, self.b[act]])
        try:
            sol = np.linalg.solve(M, rhs)
        except np.linalg.LinAlgError:
            return 3, None, None, None
        U, lam = sol[:N], sol[N:]
        V = U / self.D
        vmax = max(1.0, np.abs(V).max())
        s = np.where(self.live, (self.b - self.Lin @ U) / np.where(self.live, self.rn, 1.0), np.inf)
        bc = -self.b / np.where(self.live, self.rn, 1.0)
        pbad = np.any(s < -1e-9 * np.maximum(vmax, np.abs(bc)))
        mu = lam * self.rn[act]
        mabs = max(1.0, np.abs(mu).max()) if q else 1.0
        dbad = q > 0 and mu.min() < -1e-9 * mabs
        fk = 0 if not (pbad or dbad) else (1 if not pbad else (2 if not dbad else 4))
        return fk, U, mu, s


def device_repair(qp, cand, alt_set, budget=8, multi_drop=False, out=None):
    """qp_phase's loop: returns (certified, re-solves); out[0]: the last set."""
    act, n = list(cand), 0
    alt = alt_set is not None
    rep = 0
    while True:
        fk, U, mu, s = qp.solve(act)
        n += 1
        if fk == 0:
            return True, n
        stop = rep >= budget or rep < 0 or fk == 3
        if not stop and fk in (2, 4):
            sm = s.copy()
            sm[act] = np.inf
            p = int(np.argmin(sm))            # ties: lowest id
            if not np.isfinite(sm[p]):
                stop = True
            else:
                fp = int(np.argmin(mu))
                jl = int(qp.last[p]) if qp.kind(p) >= 2 else -1
                keep = [a for k2, a in enumerate(act)
                        if not ((jl >= 0 and qp.kind(a) < 2 and qp.last[a] == jl) or (fk == 4 and k2 == fp)
                                or (multi_drop and mu[k2] < -1e-9 * max(1.0, np.abs(mu).max())))]
                if len(keep) < N:
                    act = keep + [p]
                else:
                    act = list(act)
                    act[fp] = p
        elif not stop:
            fp = int(np.argmin(mu))
            act = [a for k2, a in enumerate(act) if k2 != fp]
        if stop:
            if not alt:
                if out is not None:
                    out.append(act)
                return False, n
            alt = False
            act = list(alt_set)
            rep = -2
        rep += 1


def hybrid(qp, cand, alt_set, reps, budget=64):
    """reps single-row repairs, then the certified dual path from the set they reach."""
    out = []
    ok, n = device_repair(qp, cand, None, reps, out=out)
    if ok:
        return True, n
    ok2, n2 = gi_resolve(qp, out[0] if out else cand, None, budget)
    return ok2, n + n2


def device_revert(qp, cand, alt_set, budget=8, max_skip=99):
    """device_repair, but a repair that makes the set singular is undone: back to
    the set before it, with the row it added excluded from the next pick (the
    device: a skip flag next to kActiveRow in aflag)."""
    act, n = list(cand), 0
    alt = alt_set is not None
    rep, prev_act, skip, last_p = 0, None, set(), None
    while True:
        fk, U, mu, s = qp.solve(act)
        n += 1
        if fk == 0:
            return True, n
        if fk == 3 and prev_act is not None and rep <= budget and len(skip) < max_skip:
            skip.add(last_p)
            act = prev_act
            fk, U, mu, s = prev_fk, prev_U, prev_mu, prev_s
        stop = rep >= budget or rep < 0 or fk == 3
        if not stop and fk in (2, 4):
            sm = s.copy()
            sm[act] = np.inf
            for i in skip:
                sm[i] = np.inf
            p = int(np.argmin(sm))
            if not np.isfinite(sm[p]) or sm[p] >= -1e-9 * max(1.0, np.abs(U / qp.D).max(), abs(qp.b[p] / max(qp.rn[p], 1e-300))):
                if fk == 4:          # nothing else violated: the dual part alone
                    fp = int(np.argmin(mu))
                    prev_act, prev_fk, prev_U, prev_mu, prev_s, last_p = list(act), fk, U, mu, s, None
                    act = [a for k2, a in enumerate(act) if k2 != fp]
                else:
                    stop = True
            else:
                fp = int(np.argmin(mu))
                jl = int(qp.last[p]) if qp.kind(p) >= 2 else -1
                keep = [a for k2, a in enumerate(act)
                        if not ((jl >= 0 and qp.kind(a) < 2 and qp.last[a] == jl) or (fk == 4 and k2 == fp))]
                prev_act, prev_fk, prev_U, prev_mu, prev_s, last_p = list(act), fk, U, mu, s, p
                if len(keep) < N:
                    act = keep + [p]
                else:
                    act = list(act)
                    act[fp] = p
        elif not stop:
            fp = int(np.argmin(mu))
            prev_act, prev_fk, prev_U, prev_mu, prev_s, last_p = list(act), fk, U, mu, s, None
            act = [a for k2, a in enumerate(act) if k2 != fp]
        if stop:
            if not alt:
                return False, n
            alt = False
            act = list(alt_set)
            prev_act = None
            rep = -2
        rep += 1


def gi_resolve(qp, cand, alt_set, budget=16, dual_first=True, hint=None):
    """Goldfarb-Idnani's dual path evaluated by certified re-solves: from a dual
    feasible set A (multipliers u0 >= 0 at its equality-constrained optimum V0),
    add the most violated row p: the re-solve on A + {p} is the full step's end
    point; a multiplier of A that is negative there is dropped at the fraction of
    the (linear) path where it reaches zero, and A - {i} + {p} is re-solved again.
    Dual feasibility first: drop the most negative multiplier until none is."""
    act, n = list(cand), 0
    fk, U, mu, s = qp.solve(act)
    n += 1
    if fk == 0:
        return True, n
    while fk in (1, 4) or fk == 3:              # dual phase: drop the most negative multiplier
        if fk == 3 or n > budget:
            return False, n
        fp = int(np.argmin(mu))
        act = [a for k2, a in enumerate(act) if k2 != fp]
        fk, U, mu, s = qp.solve(act)
        n += 1
        if fk == 0:
            return True, n
    V0, u0 = U / qp.D, dict(zip(act, mu))
    while n <= budget:
        sm = s.copy()
        sm[act] = np.inf
        p = int(np.argmin(sm))
        vmax = max(1.0, np.abs(V0).max())
        if not (sm[p] < -1e-9 * max(vmax, abs(qp.b[p] / qp.rn[p]))):
            return True, n                     # (certified by the last re-solve)
        if hint is not None:                   # steer: a violated row of the hint set first
            hv = [i for i in hint if i not in act and sm[i] < -1e-9 * max(vmax, abs(qp.b[i] / qp.rn[i]))]
            if hv:
                p = min(hv, key=lambda i: sm[i])
        up = 0.0
        while True:
            A1 = act + [p]
            fk, U1, mu1, s1 = qp.solve(A1)
            n += 1
            if fk == 3:
                # n_p dependent on A: the dual-only step, n_p = sum r_i n_i (the
                # certificate's multiplier solve with n_p as the right-hand side)
                Nn = -(qp.Lin * qp.D[None, :]) / np.where(qp.live, qp.rn, 1.0)[:, None]
                r, *_ = np.linalg.lstsq(Nn[act].T, Nn[p], rcond=None)
                if np.linalg.norm(Nn[act].T @ r - Nn[p]) > 1e-8 * np.linalg.norm(Nn[p]):
                    return False, n            # singular for another reason
                cands = [(u0[a] / r[k2], a) for k2, a in enumerate(act) if r[k2] > 1e-12]
                if not cands:
                    return False, n            # infeasible
                t, i = min(cands)
                u0 = {a: u0[a] - t * r[k2] for k2, a in enumerate(act) if a != i}
                act = [a for a in act if a != i]
                if n > budget:
                    return False, n
                continue
            m1 = dict(zip(A1, mu1))
            neg = [(u0[a] / (u0[a] - m1[a]), a) for a in act if m1[a] < 0]
            if not neg:
                act = A1
                V0 = U1 / qp.D
                u0 = m1
                s = s1
                if fk == 0:
                    return True, n
                break
            th, i = min(neg)
            V1 = U1 / qp.D
            V0 = V0 + th * (V1 - V0)
            u0 = {a: u0[a] + th * (m1[a] - u0[a]) for a in act if a != i}
            act = [a for a in act if a != i]
            if n > budget:
                return False, n
    return False, n


def pdas(qp, cand, alt_set, budget=8, cap_add=None):
    """Primal-dual active-set exchange: drop every negative multiplier, add every
    violated row (a state row whose last variable is held by a u bound replaces
    that bound), keep at most N rows."""
    act, n = list(cand), 0
    tried_alt = alt_set is None
    for rep in range(budget + 1):
        fk, U, mu, s = qp.solve(act)
        n += 1
        if fk == 0:
            return True, n
        if fk == 3:
            break
        mtol = -1e-9 * max(1.0, np.abs(mu).max()) if len(act) else 0
        keep = [a for k2, a in enumerate(act) if mu[k2] >= mtol]
        sm = s.copy()
        sm[act] = np.inf
        viol = [int(i) for i in np.argsort(sm) if sm[i] < -1e-9 * max(1.0, np.abs(U / qp.D).max())]
        if cap_add:
            viol = viol[:cap_add]
        for p in viol:
            jl = int(qp.last[p]) if qp.kind(p) >= 2 else -1
            if jl >= 0:
                keep = [a for a in keep if not (qp.kind(a) < 2 and qp.last[a] == jl)]
            if p not in keep:
                keep.append(p)
        if len(keep) > N:
            keep = keep[:N]
        act = keep
    if not tried_alt:
        fk, *_ = qp.solve(alt_set)
        n += 1
        if fk == 0:
            return True, n
    return False, n


def pdas_then_gi(qp, cand, k):
    """k primal-dual exchanges (every violated row in, every negative multiplier out),
    then the certified dual path from the last set (steered by the shifted set)."""
    act, n = list(cand), 0
    for rep in range(k):
        fk, U, mu, s = qp.solve(act)
        n += 1
        if fk == 0:
            return True, n
        if fk == 3:
            break
        mtol = -1e-9 * max(1.0, np.abs(mu).max()) if len(act) else 0
        keep = [a for k2, a in enumerate(act) if mu[k2] >= mtol]
        sm = s.copy()
        sm[act] = np.inf
        viol = [int(i) for i in np.argsort(sm) if sm[i] < -1e-9 * max(1.0, np.abs(U / qp.D).max())]
        for p in viol:
            jl = int(qp.last[p]) if qp.kind(p) >= 2 else -1
            if jl >= 0:
                keep = [a for a in keep if not (qp.kind(a) < 2 and qp.last[a] == jl)]
            if p not in keep:
                keep.append(p)
        act = keep[:N]
    ok, n2 = gi_resolve(qp, act, None, 64, hint=HINTS.get("s10"))
    return ok, n + n2


x = O.scenario_x0(np.arange(S)).T.copy()
rho, Uo = cbind.initial_state(x, cfg)
for _ in range(lo - 2):
    r = cbind.step(x, rho, Uo, cfg)
    x, rho, Uo = r["x_next"], r["rho"], r["U_old"]
HINTS = {}
strategies = {
    "device (8 repairs)": lambda q, c, a: device_repair(q, c, a, 8),
    "GI: hint shift(prev 10)": lambda q, c, a: gi_resolve(q, c, a, 64, hint=HINTS.get("s10")),
    "GI: hint prev 2": lambda q, c, a: gi_resolve(q, c, a, 64, hint=HINTS.get("p2")),
    "GI: hint shift(prev 2)": lambda q, c, a: gi_resolve(q, c, a, 64, hint=HINTS.get("s2")),
    "GI: hint shift(p10) + shift(p2)": lambda q, c, a: gi_resolve(q, c, a, 64, hint=HINTS.get("u")),
    "GI by re-solves (64)": lambda q, c, a: gi_resolve(q, c, a, 64),
    # round 6: the odd plan's set change at this step (O_{k+1} vs O_k) carried to the even set
    "GI: hint shift(p10) + odd delta": lambda q, c, a: gi_resolve(q, c, a, 64, hint=HINTS.get("sd")),
    "GI: delta cand + hint shift(p10)": lambda q, c, a: gi_resolve(q, HINTS.get("dc", c), a, 64, hint=HINTS.get("s10")),
    "PDAS (8)": lambda q, c, a: pdas(q, c, None, 8),
    "PDAS (2) then GI path": lambda q, c, a: pdas_then_gi(q, c, 2),
    # box-only QPs (mode 1, BASELINE config 2): the kernel's 16 single-row exchanges vs PDAS
    "device (16 exchanges)": lambda q, c, a: device_repair(q, c, None, 16),
    "PDAS (16)": lambda q, c, a: pdas(q, c, None, 16),
}
import os  # noqa: E402
if os.environ.get("STRATS"):                     # e.g. STRATS="device (16,PDAS (16"
    keys = os.environ["STRATS"].split(",")
    strategies = {k: f for k, f in strategies.items() if any(k.startswith(p) for p in keys)}
res = {it: {k: [0, 0, 0] for k in strategies} for it in ITERS}   # certified, re-solves, count
exact = {it: 0 for it in ITERS}
first_fail = {it: 0 for it in ITERS}
hist = {it: [] for it in ITERS}
for s in range(S):
    xk, Rho, Uold = x[:, s].copy(), rho[:, s].reshape(N, 3).T.copy(), Uo[:, s].copy()
    prev = None
    for k in range(lo - 1, hi + 1):
        recs, xn, Rho, Uold = _step_record(xk, Rho, Uold, ph, cfg)
        sets = {rc["it"]: rc["act"] for rc in recs if rc["flag"] == O.EXIT_OK}
        if k >= lo and prev is not None:
            for it in ITERS:
                if it not in sets:
                    continue
                rc = recs[it - 1]
                if it <= 2:
                    if 8 + it not in prev:
                        continue
                    cand, alt = prev[8 + it], (shift(prev[10]) if it == 2 else None)
                else:
                    if it - 2 not in sets:
                        continue
                    cand, alt = sets[it - 2], None
                qp = QP(rc["G"], rc["F"], rc["Lin"], rc["b"])
                HINTS.clear()
                if it == 2 and 2 in prev:
                    HINTS.update(s10=shift(prev[10]), p2=list(prev[2]), s2=shift(prev[2]),
                                 u=list(dict.fromkeys(shift(prev[10]) + shift(prev[2]))))
                    if 1 in sets and 9 in prev:
                        add = [i for i in sets[1] if i not in prev[9]]
                        drop = set(i for i in prev[9] if i not in sets[1])
                        HINTS.update(sd=list(dict.fromkeys(add + shift(prev[10]))))
                        dc = [i for i in cand if i not in drop] + [i for i in add if i not in cand]
                        if len(dc) <= N:
                            HINTS.update(dc=dc)
                elif it == 1:
                    HINTS.update(s10=shift(prev[9]), p2=list(prev[10]), s2=list(prev[1]) if 1 in prev else None)
                elif it >= 3 and it - 1 in sets:
                    HINTS.update(s10=list(sets[it - 1]), p2=list(prev[it]) if it in prev else None,
                                 s2=shift(prev[it]) if it in prev else None)
                exact[it] += set(cand) == set(sets[it])
                first_fail[it] += QP(rc["G"], rc["F"], rc["Lin"], rc["b"]).solve(cand)[0] != 0
                for name, f in strategies.items():
                    ok, n = f(qp, cand, alt)
                    r3 = res[it][name]
                    r3[0] += ok
                    r3[1] += n
                    r3[2] += 1
                    if name.startswith("GI by re-solves (64)"):
                        hist[it].append(n if ok else -n)
        prev = sets
        xk = xn
    print(f"scenario {s} done", flush=True)
for it in ITERS:
    cnt = max(1, next(iter(res[it].values()))[2])
    print(f"N={N} mode={mode} iteration {it}: {cnt} QPs, steps {lo}-{hi}, {S} scenarios; candidate exact {exact[it] / cnt:.2f}, first try fails {first_fail[it] / cnt:.2f}")
    for name, (ok, n, c) in res[it].items():
        print(f"  {name:30s} certified {ok / cnt:.3f}  GI {1 - ok / cnt:.3f}  re-solves {n / cnt:.2f}")
    h = np.array(hist[it], dtype=np.int64)
    if not len(h):
        continue
    print("  GI by re-solves (64): re-solve counts of certified QPs", np.bincount(h[h > 0]).tolist(), "failed", int((h < 0).sum()))

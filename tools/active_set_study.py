"""Offline study (not a test): how the QP active sets of the closed loop evolve,
on the NumPy oracle (CPU).  The figures quoted in DESIGN.md §4 come from here.

    python tools/active_set_study.py hits   [scenarios] [steps] [N] [mode]
    python tools/active_set_study.py repair [scenarios] [steps] [N] [mode]
    python tools/active_set_study.py shape  [scenarios] [steps] [N] [mode]
    python tools/active_set_study.py collide [scenarios] [steps] [N] [mode]

hits   - how often the previous step's last odd / even active set (carried
         unshifted or shifted by one stage) equals the set of inner iteration 1 / 2,
         and how often iteration it's set equals iteration it-2's
repair - of the misses, how many single-row repairs recover the optimal set
         (exact active-set solves), without and with the bound-row swap
shape  - the shape of the optimal sets: echelon (every general row ends in its
         own free column) and the null-space dimension k = n_F - n_S
collide - the non-echelon optimal sets by k, collisions and bordered size n_F + n_S
Steps 0-4 are the transient ("early"), later steps the steady state ("late").
"""
import sys
from collections import Counter
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "mpc-ntm-control_amd")]
from oracle import ntm_oracle as O  # noqa: E402


def active_set(Lin, b, U):
    s = b - Lin @ U
    return frozenset(np.flatnonzero(s <= 1e-9 * np.maximum(1.0, np.abs(b))))


def shift(S, N):
    """Receding-horizon shift (the device's shifted_into_act, full getWLc rows)."""
    out = set()
    for r in S:
        blk, rr = divmod(r, 6)
        if r >= 6 * N:                      # terminal rows -> stage N-1, and kept
            out.update((6 * (N - 1) + 2 + (r - 6 * N), r))
        elif blk >= 2 or (blk == 1 and rr < 2):   # x_1's state rows would become x_0 rows: dropped
            out.add(r - 6)
        if blk == N - 1 and rr < 2:        # the old last input's bounds are kept
            out.add(r)
    return frozenset(out)


def solve_set(G, F, Lin, b, S):
    """Equality-constrained optimum on S in the scaled, normalised form; None if singular."""
    S = sorted(S)
    n = len(F)
    D = 1 / np.sqrt(np.diag(G))
    Gs, Fs, Ls = G * D[:, None] * D[None, :], F * D, Lin * D[None, :]
    rn = np.linalg.norm(Ls, axis=1)
    rn[rn == 0] = 1
    Ln, bn = Ls / rn[:, None], b / rn
    A, k = Ln[S], len(S)
    K = np.block([[Gs, A.T], [A, np.zeros((k, k))]])
    if np.linalg.cond(K) > 1e15:
        return None
    sol = np.linalg.solve(K, np.concatenate([-Fs, bn[S]]))
    return sol[:n], sol[n:], bn - Ln @ sol[:n], S


def repair(G, F, Lin, b, S0, N, swap, maxrep=8):
    S = set(S0)
    for _ in range(maxrep + 1):
        r = solve_set(G, F, Lin, b, S)
        if r is None:
            return None
        V, lam, slack, Ss = r
        vmax = max(1.0, np.max(np.abs(V)))
        act = np.zeros(len(slack), bool)
        act[Ss] = True
        pv = [i for i in np.flatnonzero(~act) if slack[i] < -1e-9 * vmax]
        ls = max(1.0, np.max(np.abs(lam))) if len(lam) else 1.0
        dv = [Ss[j] for j in range(len(Ss)) if lam[j] < -1e-9 * ls]
        if not pv and not dv:
            return frozenset(S)
        if dv:
            S.discard(min(dv, key=lambda i: lam[Ss.index(i)]))
        if pv:
            a = min(pv, key=lambda i: slack[i])
            if swap and not (a < 6 * N and a % 6 < 2):
                nz = np.flatnonzero(Lin[a])
                jl = nz[-1] if len(nz) else -1
                S -= {r for r in S if r < 6 * N and r % 6 < 2 and r // 6 == jl}
            S.add(a)
    return None


def shape(Lin, S, N):
    fixed, gen = set(), []
    for r in sorted(S):
        nz = np.flatnonzero(Lin[r])
        (fixed.add(nz[0]) if len(nz) == 1 else gen.append(r))
    free = [j for j in range(N) if j not in fixed]
    if not gen:
        return True, len(free)
    E = Lin[np.ix_(gen, free)]
    last = [max((a for a in range(len(free)) if E[i, a] != 0), default=-1) for i in range(len(gen))]
    return (len(set(last)) == len(gen) and min(last) >= 0), len(free) - len(gen)


def collisions(Lin, S, N):
    """Non-echelon optimal sets: (k = n_F - n_S, collisions = rows that do not own their
    last free column, n_F + n_S, whether the square E (k = 0) is nonsingular)."""
    fixed, gen = set(), []
    for r in sorted(S):
        nz = np.flatnonzero(Lin[r])
        (fixed.add(nz[0]) if len(nz) == 1 else gen.append(r))
    free = [j for j in range(N) if j not in fixed]
    if not gen:
        return [("all",)]
    E = Lin[np.ix_(gen, free)]
    last = [max((a for a in range(len(free)) if E[i, a] != 0), default=-1) for i in range(len(gen))]
    ncol = len(gen) - len(set(last))
    kk = len(free) - len(gen)
    out = [("all",)]
    if ncol == 0 and min(last) >= 0:
        out.append(("echelon", f"k={kk}"))
    else:
        sing = ""
        if kk == 0:
            sing = "E nonsingular" if np.linalg.matrix_rank(E) == len(gen) else "E singular"
        out.append(("not echelon", f"k={kk}", f"collisions={min(ncol, 4)}", sing))
        out.append(("not echelon nt", f"nt<=40" if len(free) + len(gen) <= 40 else ("nt<=61" if len(free) + len(gen) <= 61 else "nt>61")))
    return out


def main():
    what = sys.argv[1]
    ns, K = int(sys.argv[2]) if len(sys.argv) > 2 else 12, int(sys.argv[3]) if len(sys.argv) > 3 else 20
    N, mode = int(sys.argv[4]) if len(sys.argv) > 4 else 20, int(sys.argv[5]) if len(sys.argv) > 5 else 2
    ph, cfg = O.Physics(), O.Config(N=N, mode=mode)
    cnt = Counter()
    for x0 in O.scenario_x0(np.arange(ns)):
        xk, Rho, Uold, prev = x0.copy(), O.initial_rho(x0, ph, cfg), np.full(N, np.inf), None
        for k in range(K):
            tag, sets = ("early" if k < 5 else "late"), []
            for it in range(1, cfg.i_sim + 1):
                Phi, Gam, Lam = O.lift(Rho, ph, cfg)
                G, F = O.cost(Phi, Gam, Lam, xk, cfg)
                Lin, b = O.constraints(Phi, Gam, Lam, xk, cfg)
                U, _, _ = O.qp_solve(G, F, Lin, b)
                S = active_set(Lin, b, U)
                sets.append(S)
                cand = None
                if it <= 2 and prev is not None and len(prev) >= it:
                    cand = [x for i, x in enumerate(prev) if i % 2 == it - 1][-1]
                elif it > 2:
                    cand = sets[it - 3]
                if what == "hits" and cand is not None:
                    cnt[(tag, f"it{min(it, 3)}", "n")] += 1
                    cnt[(tag, f"it{min(it, 3)}", "unshifted")] += S == cand
                    if it == 2:
                        cnt[(tag, "it2", "shifted")] += S == shift(cand, N)
                        cnt[(tag, "it2", "either")] += S in (cand, shift(cand, N))
                elif what == "repair" and cand is not None and S != cand:
                    key = (tag, f"it{min(it, 3)}")
                    cnt[key + ("misses",)] += 1
                    for sw in (False, True):
                        cnt[key + ("repaired", "swap" if sw else "no swap")] += repair(G, F, Lin, b, cand, N, sw) == S
                elif what == "shape" and k >= 3:
                    ech, kk = shape(Lin, S, N)
                    cnt[("echelon" if ech else "not echelon", f"k={kk}" if ech else "")] += 1
                elif what == "collide" and k >= 3:
                    for key in collisions(Lin, S, N):
                        cnt[key] += 1
                _, Rho = O.rollout(xk, Rho, U, ph, cfg)
                if np.sum(np.abs(Uold - U)) < cfg.epsilon:
                    break
                Uold = U.copy()
            prev = sets
            xk = O.plant_step(xk, U[0], ph, cfg)
    for key in sorted(cnt, key=str):
        print(key, cnt[key])


if __name__ == "__main__":
    main()

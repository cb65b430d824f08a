#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the Python
oracle (oracle/ntm_oracle.py).  The reference (MATLAB) cannot run in this
image (no MATLAB/Octave) and ships no fixtures of its own, so these vectors
are produced by the oracle, whose correctness is pinned by the invariant
tests in tests/test_oracle.py and by 50-digit KKT certificates stored with
every QP fixture.  Re-run after any change to the canonical semantics:

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import ntm_oracle as O  # noqa: E402


def functions_fixture(N):
    ph = O.Physics()
    cfg = O.Config(N=N, mode=O.MODE_FULL)
    rng = np.random.default_rng(1000 + N)
    xs = np.stack([rng.uniform(0.06, 0.15, N), rng.uniform(0.8, 1.2, N) * 2000 * np.pi])
    Rho = np.stack([O.rho_all(xs[:, i], ph, cfg) for i in range(N)], axis=1)       # 3 x N
    xk = np.array([0.1, 2000 * np.pi])
    Phi, Gam, Lam = O.lift(Rho, ph, cfg)
    G, F = O.cost(Phi, Gam, Lam, xk, cfg)
    W, L, c = O.getWLc(cfg.xmax, cfg.xmin, cfg.umax, cfg.umin, Gam, Phi, Lam)
    A0 = O.A_mat(Rho[0, 0], Rho[1, 0], ph, cfg.Ts)
    B0 = O.B_mat(Rho[2, 0], ph, cfg.Ts)
    np.savez(HERE / f"functions_N{N}.npz", xs=xs, Rho=Rho, xk=xk, Phi=Phi, Gamma=Gam, Lambda=Lam, G=G, F=F,
             W=W, L=L, c=c, A0=A0, B0=B0, C=O.C_vec(ph, cfg.Ts), kappa=ph.kappa(), zeta=ph.zeta())


def closed_loop_fixture(N, mode, ids, k_sim, gen=None, name=None):
    """Closed loops (NTM_MPC_Sim.m:80-131).  wpred (k_sim, N+1) is the predicted
    island width of every step's last rollout (:110-117); with ``gen`` the
    scenarios are global ids gen.first_id + s of the scenario generator."""
    ph = O.Physics()
    cfg = O.Config(N=N, mode=mode)
    x0 = O.scenario_x0(ids) if mode != O.MODE_NONE else np.tile(O.REFERENCE_X0, (len(ids), 1))
    outs = [O.closed_loop(x0[s], ph, cfg, k_sim, gen=gen, sid=s) for s in range(len(ids))]
    extra = {}
    if gen is not None:
        extra = dict(gen_seed=gen.seed, gen_first_id=gen.first_id, gen_k0=gen.k0, gen_sigma_w=gen.sigma_w,
                     gen_sigma_omega=gen.sigma_omega, gen_jbs_spread=gen.jbs_spread,
                     gen_wdep_spread=gen.wdep_spread)
    np.savez(HERE / (name or f"closed_loop_m{mode}_N{N}.npz"), x0=x0, ids=np.asarray(ids),
             xk=np.stack([o["xk"] for o in outs]), uk=np.stack([o["uk"] for o in outs]),
             Uk=np.stack([o["Uk"] for o in outs]), wpred=np.stack([o["xpred"][:, 0, :] for o in outs]),
             exitflag=np.stack([o["exitflag"] for o in outs]),
             inner_iters=np.stack([o["inner_iters"] for o in outs]), k_sim=k_sim, **extra)


def literal_functions_fixture(N, flags):
    """Rho_to_PhiGammaLambda.m with the literal-reference switches D4
    (Phi_{j-1} A_j, :21) and D6 (A(rho_{i-j}), :32)."""
    ph = O.Physics()
    cfg = O.Config(N=N, mode=O.MODE_FULL, flags=flags)
    rng = np.random.default_rng(2000 + N + flags)
    xs = np.stack([rng.uniform(0.06, 0.15, N), rng.uniform(0.8, 1.2, N) * 2000 * np.pi])
    Rho = np.stack([O.rho_all(xs[:, i], ph, cfg) for i in range(N)], axis=1)
    Phi, Gam, Lam = O.lift(Rho, ph, cfg)
    np.savez(HERE / f"functions_lit{flags}_N{N}.npz", Rho=Rho, Phi=Phi, Gamma=Gam, Lambda=Lam, flags=flags)


def qp_fixture(N, mode, n):
    """QPs met along closed-loop trajectories, with the certified exact optimum."""
    ph = O.Physics()
    cfg = O.Config(N=N, mode=mode)
    Gs, Fs, Ls, bs, Us, flags = [], [], [], [], [], []
    x0 = O.scenario_x0(np.arange(n))
    for s in range(n):
        xk = x0[s]
        Rho = O.initial_rho(xk, ph, cfg)
        for it in range(1 + s % 4):
            Phi, Gam, Lam = O.lift(Rho, ph, cfg)
            G, F = O.cost(Phi, Gam, Lam, xk, cfg)
            Lin, b = O.constraints(Phi, Gam, Lam, xk, cfg)
            U, flag, info = O.qp_solve(G, F, Lin, b)
            _, Rho = O.rollout(xk, Rho, U, ph, cfg)
        Phi, Gam, Lam = O.lift(Rho, ph, cfg)
        G, F = O.cost(Phi, Gam, Lam, xk, cfg)
        Lin, b = O.constraints(Phi, Gam, Lam, xk, cfg)
        U, flag, info = O.qp_solve(G, F, Lin, b)
        Ue, _, cert = O.kkt_polish(G, F, Lin, b, info["active"], dps=50)
        assert cert["max_violation"] <= 1e-12 and cert["min_multiplier"] >= -1e-12, cert
        Gs.append(G), Fs.append(F), Ls.append(Lin), bs.append(b), Us.append(Ue), flags.append(flag)
    np.savez(HERE / f"qp_m{mode}_N{N}.npz", G=np.stack(Gs), F=np.stack(Fs), Lin=np.stack(Ls), b=np.stack(bs),
             U_exact=np.stack(Us), exitflag=np.asarray(flags))


def qp_traj_fixture(N, mode, n_scen, steps, name=None, dps=50):
    """QPs along closed-loop trajectories of the C oracle (NTM_MPC_Sim.m:93-131):
    for every scenario and step, the QP of the first inner iteration (the data
    built from the carried rho, :94-97) with its optimum certified at ``dps``
    digits on the NumPy oracle's final active set.  Mode 0 (BASELINE config 1)
    starts from the reference x0 (NTM_MPC_Sim.m:34) with omega perturbed per
    scenario, where the unconstrained LQ is well posed."""
    from oracle import cbind
    ph = O.Physics()
    cfg = O.Config(N=N, mode=mode)
    if mode == O.MODE_NONE:
        x = np.tile(O.REFERENCE_X0[:, None], (1, n_scen))
        x[1] *= 1.0 + 1e-3 * np.arange(n_scen)
    else:
        x = O.scenario_x0(np.arange(n_scen)).T.copy()
    rho, Uo = cbind.initial_state(x, cfg)
    Gs, Fs, Ls, bs, Us, flags, ks = [], [], [], [], [], [], []
    for k in range(steps):
        for s in range(n_scen):
            Rho = rho[:, s].reshape(N, 3).T
            Phi, Gam, Lam = O.lift(Rho, ph, cfg)
            G, F = O.cost(Phi, Gam, Lam, x[:, s], cfg)
            Lin, b = O.constraints(Phi, Gam, Lam, x[:, s], cfg)
            U, flag, info = O.qp_solve(G, F, Lin, b)
            if flag != O.EXIT_OK:
                continue
            Ue, _, cert = O.kkt_polish(G, F, Lin, b, info["active"], dps=dps)
            assert cert["max_violation"] <= 1e-12 and cert["min_multiplier"] >= -1e-12, cert
            Gs.append(G), Fs.append(F), Ls.append(Lin), bs.append(b), Us.append(Ue), flags.append(flag)
            ks.append(k)
        ref = cbind.step(x, rho, Uo, cfg)
        x, rho, Uo = ref["x_next"], ref["rho"], ref["U_old"]
    np.savez(HERE / (name or f"qp_m{mode}_N{N}.npz"), G=np.stack(Gs), F=np.stack(Fs), Lin=np.stack(Ls),
             b=np.stack(bs), U_exact=np.stack(Us), exitflag=np.asarray(flags), step=np.asarray(ks))
    print(f"qp_m{mode}_N{N}: {len(Us)} certified QPs")


def _step_record(xk, Rho, Uold, ph, cfg):
    """O.mpc_step (NTM_MPC_Sim.m:94-130) with every inner iteration's QP recorded:
    its inputs (the carried rho and U_old), its active set and solution."""
    recs = []
    U = np.zeros(cfg.N)
    for it in range(1, cfg.i_sim + 1):
        Phi, Gam, Lam = O.lift(Rho, ph, cfg)
        G, F = O.cost(Phi, Gam, Lam, xk, cfg)
        Lin, b = O.constraints(Phi, Gam, Lam, xk, cfg)
        U, flag, info = O.qp_solve(G, F, Lin, b)
        recs.append(dict(it=it, Rho=Rho.copy(), Uold=Uold.copy(), G=G, F=F, Lin=Lin, b=b, U=U, flag=flag,
                         act=[int(a) for a in info.get("active", [])]))
        _, Rho = O.rollout(xk, Rho, U, ph, cfg)
        if np.sum(np.abs(Uold - U)) < cfg.epsilon:
            break
        Uold = U.copy()
    return recs, O.plant_step(xk, U[0], ph, cfg), Rho, Uold


def collision_kind(Lin, act, N):
    """The long-horizon one-collision shapes of the device's echelon re-solve (DESIGN
    §4): exactly one general row does not own the last free column it ends in, with
    k = n_F - n_S = 0 (kind 1) or k = 1 (kind 2); 0 for any other set."""
    nz = [np.nonzero(np.abs(Lin[r]) > 0)[0] for r in act]
    fixed = {int(c[0]) for c in nz if len(c) == 1}
    free = [j for j in range(N) if j not in fixed]
    gen = [c for c in nz if len(c) > 1]
    k = len(free) - len(gen)
    if k not in (0, 1) or not gen:
        return 0
    last = [max(j for j in c if j not in fixed) if any(j not in fixed for j in c) else -1 for c in gen]
    holes = [j for j in free if j not in last]
    if -1 in last or len(holes) != k + 1 or len(set(last)) != len(gen) - 1:
        return 0
    return 1 + k


def qp_steady_fixture(N, mode, scen, n_want, name, k_lo=6, k_hi=25, per_kind=6, dps=50):
    """Steady-state QPs of the closed loop: every inner iteration
    (1..10) of closed-loop steps k_lo..k_hi (the bench's timed steps 6-25,
    NTM_MPC_Sim.m:93-97, 123-127), each with the inputs the fused step kernel takes
    for it: x_k, the carried rho and U_old, and the warm-start set the device
    carries into that QP (the active set of the last QP of the same iteration
    parity: iteration it-2 of this step, or for it = 1, 2 the previous step's last
    odd / even one), plus the 50-digit KKT optimum U_exact and its multipliers.
    Steps 0..k_lo-2 run on the C oracle, steps k_lo-1.. on the NumPy oracle (whose
    active sets are recorded).  Selection: the one-collision sets of both kinds
    first (up to per_kind each), then round robin over (iteration, step)."""
    from oracle import cbind
    ph = O.Physics()
    cfg = O.Config(N=N, mode=mode)
    x = O.scenario_x0(np.asarray(scen)).T.copy()
    rho, Uo = cbind.initial_state(x, cfg)
    for _ in range(k_lo - 1):
        r = cbind.step(x, rho, Uo, cfg)
        x, rho, Uo = r["x_next"], r["rho"], r["U_old"]
    pool = []
    for si, sid in enumerate(scen):
        xk, Rho, Uold = x[:, si].copy(), rho[:, si].reshape(N, 3).T.copy(), Uo[:, si].copy()
        last = {1: None, 0: None}                  # last active set per iteration parity
        for k in range(k_lo - 1, k_hi + 1):
            recs, xn, Rho, Uold = _step_record(xk, Rho, Uold, ph, cfg)
            for rc in recs:
                par = rc["it"] & 1
                if k >= k_lo and rc["flag"] == O.EXIT_OK:
                    rc.update(k=k, sid=sid, xk=xk.copy(), cand=last[par],
                              kind=collision_kind(rc["Lin"], rc["act"], N))
                    pool.append(rc)
                last[par] = rc["act"] if rc["flag"] == O.EXIT_OK else None
            xk = xn
        print(f"  scenario {sid}: steps {k_lo}-{k_hi} recorded", flush=True)
    chosen = []
    for kind in (1, 2):
        chosen += [p for p in pool if p["kind"] == kind][:per_kind]
    rest = [p for p in pool if all(p is not c for c in chosen)]
    rest.sort(key=lambda p: ((p["k"] * 7 + p["it"] * 3 + p["sid"]) % 11, p["it"], p["k"], p["sid"]))
    by_it = {it: [p for p in rest if p["it"] == it] for it in range(1, cfg.i_sim + 1)}
    while len(chosen) < n_want and any(by_it.values()):
        for it in range(1, cfg.i_sim + 1):
            if by_it[it] and len(chosen) < n_want:
                chosen.append(by_it[it].pop(0))
    out = {k: [] for k in ("x", "rho", "U_old", "cand", "U_exact", "lam", "act", "step", "iter", "sid", "kind")}
    for p in chosen:
        Ue, lam, cert = O.kkt_polish(p["G"], p["F"], p["Lin"], p["b"], p["act"], dps=dps)
        assert cert["max_violation"] <= 1e-12 and cert["min_multiplier"] >= -1e-12 * max(1.0, np.max(np.abs(lam))), cert
        cand = np.full(N + 1, -1, np.int32)
        if p["cand"] is not None:
            cand[:len(p["cand"])] = p["cand"]
            cand[N] = len(p["cand"])
        act = np.full(N + 1, -1, np.int32)
        act[:len(p["act"])] = p["act"]
        act[N] = len(p["act"])
        lm = np.zeros(N + 1)
        lm[:len(lam)] = lam
        out["x"].append(p["xk"]), out["rho"].append(p["Rho"].T.reshape(-1)), out["U_old"].append(p["Uold"])
        out["cand"].append(cand), out["U_exact"].append(Ue), out["lam"].append(lm), out["act"].append(act)
        out["step"].append(p["k"]), out["iter"].append(p["it"]), out["sid"].append(p["sid"])
        out["kind"].append(p["kind"])
    np.savez(HERE / name, **{k: np.asarray(v) for k, v in out.items()}, N=N, mode=mode)
    kinds = np.bincount(np.asarray(out["kind"]), minlength=3)
    print(f"{name}: {len(chosen)} certified QPs (of {len(pool)}), iterations "
          f"{np.bincount(np.asarray(out['iter']), minlength=11)[1:].tolist()}, one-collision kinds {kinds.tolist()}")


def run_along(x0, cfg, iters, k_sim):
    """The C oracle's closed loop from x0 (2, B) with step k of scenario s running
    exactly iters[k, s] LPV iterations (no early stop; same U, x_next and rho as a
    loop that stopped there), batched by iteration count.  Returns Uk (N k_sim, B)."""
    import dataclasses
    from oracle import cbind
    N, B = cfg.N, x0.shape[1]
    x = np.ascontiguousarray(x0, dtype=np.float64)
    rho, Uo = cbind.initial_state_gen(x, cfg)          # the C oracle's own rho(x_0), as ntm_oracle_run
    Uk = np.zeros((N * k_sim, B))
    for k in range(k_sim):
        xn, rn, un = np.zeros_like(x), np.zeros_like(rho), np.zeros_like(Uo)
        for it in np.unique(iters[k]):
            sel = np.where(iters[k] == it)[0]
            r = cbind.step(np.ascontiguousarray(x[:, sel]), np.ascontiguousarray(rho[:, sel]),
                           np.ascontiguousarray(Uo[:, sel]), dataclasses.replace(cfg, i_sim=int(it), epsilon=-1.0))
            Uk[k * N:(k + 1) * N, sel] = r["U"]
            xn[:, sel], rn[:, sel], un[:, sel] = r["x_next"], r["rho"], r["U_old"]
        x, rho, Uo = xn, rn, un
    return Uk


def sensitivity_fixture(N, mode, B=256, k_sim=20, eps=1e-13, name=None):
    """The closed loop's own sensitivity: the C oracle against
    itself with x_0 perturbed by eps relative, w and omega each up and down (four
    runs), for the first B synthetic scenarios; sens[s] is the largest drift
    max_k |U_k' - U_k| / umax of scenario s over the four.  The perturbed loops run
    along the unperturbed loop's LPV iteration counts (run_along), as the GPU test
    replays a scenario whose bitwise stopping rule (NTM_MPC_Sim.m:123-125) fired at
    another iteration: sens is the continuous amplification of NTM_MPC_Sim.m:110-130
    (each step's state fed back through rho(x)), not a switch of path.  A
    free-running GPU-vs-oracle comparison cannot be tighter than the loop itself."""
    from oracle import cbind
    cfg = O.Config(N=N, mode=mode)
    x0 = np.ascontiguousarray(O.scenario_x0(np.arange(B)).T)
    ref = cbind.run(x0, cfg, k_sim)
    base = run_along(x0, cfg, ref["inner_iters"], k_sim)
    assert np.array_equal(base, ref["Uk"])
    sens = np.zeros(B)
    for c in range(2):
        for sgn in (1.0, -1.0):
            xp = x0.copy()
            xp[c] = xp[c] * (1.0 + sgn * eps)
            Up = run_along(xp, cfg, ref["inner_iters"], k_sim)
            sens = np.maximum(sens, np.max(np.abs(Up - base), axis=0) / cfg.umax)
    np.savez(HERE / (name or f"sensitivity_m{mode}_N{N}.npz"), sens=sens, eps=eps, k_sim=k_sim, B=B, N=N, mode=mode,
             inner_iters=ref["inner_iters"])
    print(f"sensitivity N={N} mode={mode}: median {np.median(sens):.2e}, max {sens.max():.2e} "
          f"(scenario {int(np.argmax(sens))}), > 5e-9: {int((sens > 5e-9).sum())}", flush=True)


GEN = O.ScenarioGen(seed=20241220, first_id=0, k0=0, sigma_w=1e-3, sigma_omega=0.0, jbs_spread=0.1,
                    wdep_spread=0.1)


ALL = ("functions", "closed_loop", "qp", "literal", "gen", "qp_long", "closed_loop_long", "qp_steady", "sensitivity")


def main(which=ALL):
    if "literal" in which:
        for flags in (O.LITERAL_PHI_RIGHTMUL, O.LITERAL_GAMMA_INDEX,
                      O.LITERAL_PHI_RIGHTMUL | O.LITERAL_GAMMA_INDEX):
            literal_functions_fixture(6, flags)
    if "gen" in which:
        # disturbance realisations + plasma scenarios (SURVEY.md §8d sigma_w = 1e-3 m)
        closed_loop_fixture(20, O.MODE_FULL, [0, 1, 2], 8, gen=GEN, name="closed_loop_gen_m2_N20.npz")
        closed_loop_fixture(3, O.MODE_FULL, [0, 1, 2, 3], 20, gen=GEN, name="closed_loop_gen_m2_N3.npz")
    if "functions" in which:
        for N in (3, 20):
            functions_fixture(N)
    if "closed_loop" in which:
        closed_loop_fixture(10, O.MODE_NONE, [0], 20)          # BASELINE config 1
        closed_loop_fixture(3, O.MODE_FULL, [0, 1, 2, 3], 20)
        closed_loop_fixture(20, O.MODE_BOX, [0, 1], 6)          # config 2 shape
        closed_loop_fixture(20, O.MODE_FULL, [0, 1, 2], 6)      # config 3 shape
        # BASELINE config 5 row structure (input-rate rows, an extension of getWLc)
        closed_loop_fixture(20, O.MODE_FULL_DU, [0, 1], 6)
    if "qp" in which:
        qp_fixture(20, O.MODE_FULL, 12)
        qp_fixture(20, O.MODE_BOX, 8)
        qp_fixture(20, O.MODE_FULL_DU, 8)
    if "qp_long" in which:
        # BASELINE config 5 (N = 50, modes 2 and 3) and config 1 (N = 10, unconstrained)
        qp_traj_fixture(50, O.MODE_FULL, 4, 4)
        qp_traj_fixture(50, O.MODE_FULL_DU, 4, 4)
        qp_traj_fixture(10, O.MODE_NONE, 4, 4)
        qp_traj_fixture(10, O.MODE_FULL, 4, 4)
    if "closed_loop_long" in which:
        closed_loop_fixture(50, O.MODE_FULL_DU, [0, 1], 4)     # config 5 shape
    if "qp_steady" in which:
        # the bench's timed steps 6-25 at BASELINE config 3 (N = 20, mode 2) and config 5
        # with rate rows (N = 50, mode 3; scenario 112 is the most loop-sensitive one)
        qp_steady_fixture(20, O.MODE_FULL, [0, 1, 2, 3], 40, "qp_ss_m2_N20.npz")
        qp_steady_fixture(50, O.MODE_FULL_DU, [0, 112, 5], 40, "qp_ss_m3_N50.npz")
    if "sensitivity" in which:
        for N, mode in ((20, O.MODE_FULL), (20, O.MODE_FULL_DU), (50, O.MODE_FULL), (50, O.MODE_FULL_DU)):
            sensitivity_fixture(N, mode)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ALL)

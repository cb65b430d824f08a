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


GEN = O.ScenarioGen(seed=20241220, first_id=0, k0=0, sigma_w=1e-3, sigma_omega=0.0, jbs_spread=0.1,
                    wdep_spread=0.1)


def main(which=("functions", "closed_loop", "qp", "literal", "gen", "qp_long", "closed_loop_long")):
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
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ("functions", "closed_loop", "qp", "literal", "gen", "qp_long", "closed_loop_long"))

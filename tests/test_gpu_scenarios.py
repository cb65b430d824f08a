"""GPU tests of the scenario generator (plasma scenarios and disturbance
realisations, SURVEY.md §8d / §8(f)1, ntm_ctx_set_scenarios) and of the
literal-reference switches at the time-step level (SURVEY.md §2.1 D4, D6, D13,
D18), all through the C-ABI against the C oracle.

Tolerances as tests/test_gpu_parity.py: teacher-forced steps 1e-10 * umax on U
and 1e-9 on the states; free-running closed loops 1e-6.
"""
import dataclasses
import math

import numpy as np
import pytest
import torch

from oracle import cbind
from oracle import ntm_oracle as O

from test_gpu_parity import RUN_TOL, H, T, _assert_run_close, _teacher_forced, cfgs

pytestmark = pytest.mark.gpu

GEN = O.ScenarioGen(seed=20241220, first_id=0, k0=0, sigma_w=1e-3, sigma_omega=0.0, jbs_spread=0.1,
                    wdep_spread=0.1)


def dev_gen(g: O.ScenarioGen, **kw):
    from ntm_mpc import ScenarioGen
    return ScenarioGen(**{**dataclasses.asdict(g), **kw})


# ------------------------------------------------------------ generator
@pytest.mark.parametrize("N,mode,warm", [(20, 2, True), (20, 1, False), (3, 2, False), (50, 2, True)])
def test_step_teacher_forced_with_generator(ctl, N, mode, warm):
    """Each scenario's own plasma in the model and the plant, plus step k's
    disturbance at time index k (gen.k0 = k), identical inputs every step."""
    _teacher_forced(ctl, N, mode, warm, k_sim=6, gen=GEN)


def test_step_teacher_forced_with_omega_disturbance(ctl):
    _teacher_forced(ctl, 20, 2, True, k_sim=5, gen=dataclasses.replace(GEN, sigma_omega=50.0, first_id=977))


@pytest.mark.parametrize("N,mode", [(20, 2), (20, 3), (10, 1)])
def test_run_with_generator_matches_oracle(ctl, N, mode):
    B, k_sim = 32, 20
    cfg, ocfg = cfgs(N, mode)
    x0 = O.scenario_x0(np.arange(B)).T
    g = dataclasses.replace(GEN, first_id=5000, k0=3)
    ref = cbind.run(x0, ocfg, k_sim, gen=g)
    ctl.set_scenarios(dev_gen(g))
    try:
        out = ctl.run(T(x0), k_sim, cfg)
    finally:
        ctl.set_scenarios(None)
    _assert_run_close(out, ref, cfg, k_sim, tol=RUN_TOL, x0=x0, ocfg=ocfg, gen=g)


def test_initial_state_per_scenario_plasma(ctl):
    """ntm_mpc_init with the generator: rho3 uses each scenario's w_dep (rho3.m:2)."""
    B, N = 40, 20
    cfg, ocfg = cfgs(N, 2)
    x0 = O.scenario_x0(np.arange(B)).T
    ctl.set_scenarios(dev_gen(GEN))
    try:
        rho, uo = ctl.initial_state(T(x0), cfg)
    finally:
        ctl.set_scenarios(None)
    r_ref, _ = cbind.initial_state_gen(x0, ocfg, GEN)
    np.testing.assert_allclose(H(rho), r_ref, rtol=1e-15, atol=0)
    r_nom, _ = ctl.initial_state(T(x0), cfg)
    assert not np.array_equal(H(r_nom), H(rho))                  # the spread did change rho3


def test_disturbance_is_the_sampled_realisation(ctl):
    """x_next with the generator minus x_next without it, from identical inputs,
    is sigma * n(id, k0) of the host sampler (the QP never sees the disturbance),
    to one rounding of x."""
    from ntm_mpc import scenario_sample
    B, N = 64, 20
    cfg, ocfg = cfgs(N, 2)
    x = O.scenario_x0(np.arange(100, 100 + B)).T
    rho, Uo = cbind.initial_state(x, ocfg)
    g = dev_gen(O.ScenarioGen(seed=99, first_id=100, k0=7, sigma_w=2e-3, sigma_omega=30.0))
    a = ctl.step(T(x), T(rho), T(Uo), cfg)
    ctl.set_scenarios(g)
    try:
        b = ctl.step(T(x), T(rho), T(Uo), cfg)
    finally:
        ctl.set_scenarios(None)
    assert torch.equal(a["U"], b["U"])
    smp = scenario_sample(g, B, 7)
    d = H(b["x_next"]) - H(a["x_next"])
    np.testing.assert_allclose(d[0], 2e-3 * smp[:, 2], rtol=0, atol=1e-16)
    np.testing.assert_allclose(d[1], 30.0 * smp[:, 3], rtol=0, atol=2e-12)


def test_generator_is_shard_invariant(ctl):
    """Counter-based on the global scenario id: a batch split into shards with
    first_id offsets (how the multi-GPU bench shards) reproduces the one-batch
    closed loop bit for bit, disturbances and plasma included."""
    B, k_sim, N = 48, 8, 20
    cfg, _ = cfgs(N, 2)
    x0 = O.scenario_x0(np.arange(B)).T
    g = dev_gen(GEN, first_id=0)
    ctl.set_scenarios(g)
    try:
        full = ctl.run(T(x0), k_sim, cfg)
        parts = []
        for lo, hi in ((0, 20), (20, 48)):
            ctl.set_scenarios(dev_gen(GEN, first_id=lo))
            parts.append(ctl.run(T(x0[:, lo:hi]), k_sim, cfg))
    finally:
        ctl.set_scenarios(None)
    for k in full:
        assert torch.equal(full[k], torch.cat([parts[0][k], parts[1][k]], dim=1)), k


def test_generator_off_restores_nominal_loop(ctl):
    B, k_sim, N = 16, 5, 20
    cfg, _ = cfgs(N, 2)
    x0 = T(O.scenario_x0(np.arange(B)).T)
    a = ctl.run(x0, k_sim, cfg)
    ctl.set_scenarios(dev_gen(GEN))
    try:
        b = ctl.run(x0, k_sim, cfg)
    finally:
        ctl.set_scenarios(None)
    c = ctl.run(x0, k_sim, cfg)
    for k in a:
        assert torch.equal(a[k], c[k]), k
    assert not torch.equal(a["xk"], b["xk"])


def test_generator_arguments_validated(ctl):
    from ntm_mpc import NtmLibraryError
    for bad in (dict(sigma_w=-1.0), dict(jbs_spread=1.0), dict(wdep_spread=float("nan")), dict(k0=-1)):
        with pytest.raises(NtmLibraryError):
            ctl.set_scenarios(dev_gen(GEN, **bad))
    ctl.set_scenarios(None)


# ------------------------------------------------------------ literal switches at the step level
@pytest.mark.parametrize("flags", [O.LITERAL_PHI_RIGHTMUL, O.LITERAL_GAMMA_INDEX,
                                   O.LITERAL_PHI_RIGHTMUL | O.LITERAL_GAMMA_INDEX,
                                   O.LITERAL_PLANT_NO_C, O.RHO1_SQUARED])
@pytest.mark.parametrize("N", [6, 20])
def test_step_teacher_forced_literal(ctl, N, flags):
    """One MPC step with each literal-reference switch (D4 Rho_to_PhiGammaLambda.m:21,
    D6 :32, D13 NTM_MPC_Sim.m:130, D18 rhos.m:18) against the oracle with the same
    switch (D4/D6 run on the generic kernels)."""
    _teacher_forced(ctl, N, 2, True, k_sim=4, flags=flags)


@pytest.mark.parametrize("N", [6, 20])
def test_lift_literal_matches_oracle(ctl, N):
    from ntm_mpc import Config
    from test_gpu_parity import random_rho
    B = 9
    rho = random_rho(N, B, 11)
    for flags in (1, 2, 3):
        Phi, Gam, Lam = (H(t) for t in ctl.lift(T(rho), Config(N=N, mode=2, flags=flags)))
        ocfg = O.Config(N=N, mode=2, flags=flags)
        for s in range(B):
            P_, G_, L_ = O.lift(rho[:, s].reshape(N, 3).T, O.Physics(), ocfg)
            np.testing.assert_allclose(Phi[:, s].reshape(2 * N, 2, order="F"), P_, rtol=1e-13, atol=1e-300)
            np.testing.assert_allclose(Gam[:, s].reshape(2 * N, N, order="F"), G_, rtol=1e-13, atol=1e-300)
            np.testing.assert_allclose(Lam[:, s], L_, rtol=1e-13, atol=1e-300)


def test_unknown_flags_rejected(ctl):
    """The boundary refuses semantics it does not implement: unknown flag bits
    are NTM_E_UNSUPPORTED, never a silently canonical result."""
    from ntm_mpc import Config, NtmLibraryError
    x0 = T(O.scenario_x0(np.arange(4)).T)
    for f in (1 << 4, 1 << 9, -1):
        with pytest.raises(NtmLibraryError, match=r"\(-4\)"):
            ctl.run(x0, 1, Config(N=20, mode=2, flags=f))

"""ctypes binding of the C oracle (oracle/libntm_oracle.so) — TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
Arrays are numpy (E, B) (element e of scenario s at [e, s]), staged C-contiguous
(the oracle's own scenario-minor interface; any (E, B) array is accepted).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

from . import ntm_oracle as O

HERE = Path(__file__).resolve().parent
LIB = HERE / "libntm_oracle.so"

PHYSICS_FIELDS = ("j_BS w_dep w_marg w_sat tau_r rs a eta_CD tau_E0 tau_E mu0 Lq B_pol m Cw "
                  "tau_A0 tau_w omega0").split()


class CPhys(C.Structure):
    _fields_ = [(n, C.c_double) for n in PHYSICS_FIELDS]


class CCfg(C.Structure):
    _fields_ = [("N", C.c_int32), ("i_sim", C.c_int32), ("mode", C.c_int32), ("flags", C.c_int32),
                ("Ts", C.c_double), ("xmin", C.c_double * 2), ("xmax", C.c_double * 2),
                ("umin", C.c_double), ("umax", C.c_double), ("Q", C.c_double * 4),
                ("r", C.c_double * 2), ("epsilon", C.c_double), ("du_max", C.c_double),
                ("Ru", C.c_double)]


class CGen(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("first_id", C.c_int64), ("k0", C.c_int32), ("reserved", C.c_int32),
                ("sigma_w", C.c_double), ("sigma_omega", C.c_double), ("jbs_spread", C.c_double),
                ("wdep_spread", C.c_double)]


def gen_c(g: "O.ScenarioGen | None"):
    if g is None:
        return None
    return C.byref(CGen(g.seed, g.first_id, g.k0, 0, g.sigma_w, g.sigma_omega, g.jbs_spread, g.wdep_spread))


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
    return _lib


def phys_c(ph: O.Physics | None = None) -> CPhys:
    ph = ph or O.Physics()
    return CPhys(*[float(getattr(ph, n)) for n in PHYSICS_FIELDS])


def cfg_c(cfg: O.Config) -> CCfg:
    return CCfg(cfg.N, cfg.i_sim, cfg.mode, cfg.flags, cfg.Ts, (C.c_double * 2)(*cfg.xmin),
                (C.c_double * 2)(*cfg.xmax), cfg.umin, cfg.umax, (C.c_double * 4)(*cfg.Q),
                (C.c_double * 2)(*cfg.r), cfg.epsilon, cfg.du_max, cfg.Ru)


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32)) if a is not None else None


def run(x0, cfg: O.Config, k_sim: int, ph: O.Physics | None = None, nthreads: int = 0, gen=None):
    """Closed loop (NTM_MPC_Sim.m:80-131) for x0 (2, B).  Same output layout as ntm_mpc_run;
    ``gen`` (O.ScenarioGen) adds the scenario generator."""
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    B = x0.shape[1]
    N = cfg.N
    out = {"xk": np.zeros((2 * (k_sim + 1), B)), "uk": np.zeros((k_sim, B)), "Uk": np.zeros((N * k_sim, B)),
           "wpred": np.zeros(((N + 1) * k_sim, B)), "exitflag": np.zeros((k_sim, B), np.int32),
           "inner_iters": np.zeros((k_sim, B), np.int32)}
    rc = lib().ntm_oracle_run_gen(C.byref(phys_c(ph)), C.byref(cfg_c(cfg)), gen_c(gen), C.c_int64(B), k_sim,
                                  _dp(x0), _dp(out["xk"]), _dp(out["uk"]), _dp(out["Uk"]), _dp(out["wpred"]),
                                  _ip(out["exitflag"]), _ip(out["inner_iters"]), nthreads)
    assert rc == 0, rc
    return out


def step(x_k, rho, U_old, cfg: O.Config, ph: O.Physics | None = None, nthreads: int = 0, gen=None):
    """One MPC step (NTM_MPC_Sim.m:94-130) for a batch; rho / U_old are copied, not modified.
    ``gen`` (O.ScenarioGen) adds the scenario generator (plant step at time index gen.k0)."""
    x_k = np.ascontiguousarray(x_k, dtype=np.float64)
    rho = np.array(rho, dtype=np.float64, order="C")
    U_old = np.array(U_old, dtype=np.float64, order="C")
    B = x_k.shape[1]
    N = cfg.N
    out = {"U": np.zeros((N, B)), "x_pred": np.zeros((2 * (N + 1), B)), "x_next": np.zeros((2, B)),
           "exitflag": np.zeros(B, np.int32), "inner_iters": np.zeros(B, np.int32)}
    rc = lib().ntm_oracle_step_gen(C.byref(phys_c(ph)), C.byref(cfg_c(cfg)), gen_c(gen), C.c_int64(B), _dp(x_k),
                                   _dp(rho), _dp(U_old), _dp(out["U"]), _dp(out["x_pred"]), _dp(out["x_next"]),
                                   _ip(out["exitflag"]), _ip(out["inner_iters"]), nthreads)
    assert rc == 0, rc
    out["rho"] = rho
    out["U_old"] = U_old
    return out


def qp(G, F, Lin, b):
    """Single-scenario QP (column-major matrices) -> (U, exitflag, iterations)."""
    n = F.shape[0]
    m = 0 if Lin is None else Lin.shape[0]
    Gf = np.asfortranarray(G, dtype=np.float64)
    Lf = np.asfortranarray(Lin, dtype=np.float64) if m else None
    bb = np.ascontiguousarray(b, dtype=np.float64) if m else None
    U = np.zeros(n)
    its = C.c_int(0)
    flag = lib().ntm_oracle_qp(n, m, _dp(Gf), _dp(np.ascontiguousarray(F, dtype=np.float64)), _dp(Lf), _dp(bb),
                               _dp(U), C.byref(its))
    return U, flag, its.value


def initial_state(x0, cfg: O.Config, ph: O.Physics | None = None):
    """rho (3N, B) = repmat(rho(x0)) and U_old (N, B) = +inf."""
    ph = ph or O.Physics()
    B = x0.shape[1]
    rho = np.zeros((3 * cfg.N, B))
    for s in range(B):
        r = O.rho_all(x0[:, s], ph, cfg)
        rho[:, s] = np.tile(r, cfg.N)
    return rho, np.full((cfg.N, B), np.inf)


def initial_state_gen(x0, cfg: O.Config, gen=None, ph: O.Physics | None = None):
    """ntm_oracle_init_gen: rho (3N, B) of each scenario's own plasma and U_old = +inf."""
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    B = x0.shape[1]
    rho = np.zeros((3 * cfg.N, B))
    U_old = np.zeros((cfg.N, B))
    rc = lib().ntm_oracle_init_gen(C.byref(phys_c(ph)), C.byref(cfg_c(cfg)), gen_c(gen), C.c_int64(B), _dp(x0),
                                   _dp(rho), _dp(U_old))
    assert rc == 0, rc
    return rho, U_old


def scenario_sample(gen, B: int, k: int):
    """(B, 4) samples of the generator: j_BS factor, w_dep factor, n_w(k), n_omega(k)."""
    out = np.zeros((B, 4))
    lib().ntm_oracle_scenario_sample(gen_c(gen), C.c_int64(B), C.c_int32(k), _dp(out))
    return out

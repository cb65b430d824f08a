"""The MATLAB MEX gateway (integration/matlab/ntm_mpc_mex.c, row (f)2) compiled
against a TEST-ONLY minimal mx*/mex* implementation (tests/mex_shim/) and driven
like MATLAB would drive it: 'init' / 'step' / 'run' / 'scenarios' / 'close',
cfg structs, E-by-B arrays, error identifiers.

CPU tests check the argument parsing and error paths (no GPU: the context
cannot be created, and that must surface as an ntm:library error); GPU tests
check that every output is bit-identical to the ctypes path over the same
C-ABI, i.e. that the gateway marshals without copies or transposes going
wrong.  MATLAB itself is not in this image, so this is the
closest exercise of NTM_MPC_Sim_gpu.m's calls available here.
"""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
LIBDIR = ROOT / "mpc-ntm-control_amd" / "lib"

DOUBLE, INT32, CHAR, STRUCT = 3, 4, 2, 1


@pytest.fixture(scope="module")
def mex():
    # built by __graft_entry__.build() (tests/mex_shim/Makefile, in-tree); make is a
    # no-op when it is up to date
    shim = ROOT / "tests" / "mex_shim"
    out = shim / "libmex_test.so"
    subprocess.run(["make", "-s", "-C", str(shim)], check=True)
    lib = C.CDLL(str(out))
    P = C.c_void_p
    for name, res, args in (("t_double", P, [C.c_size_t, C.c_size_t, P]), ("t_int32", P, [C.c_size_t, C.c_size_t, P]),
                            ("t_char", P, [C.c_char_p]), ("t_struct", P, []),
                            ("t_struct_set", None, [P, C.c_char_p, P]), ("t_class", C.c_int, [P]),
                            ("t_m", C.c_size_t, [P]), ("t_n", C.c_size_t, [P]), ("t_data", P, [P]),
                            ("t_free", None, [P]), ("t_err_id", C.c_char_p, []), ("t_err_msg", C.c_char_p, []),
                            ("t_call", C.c_int, [C.c_int, P, C.c_int, P]), ("t_clear", C.c_int, [])):
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return Mex(lib)


class MexError(Exception):
    def __init__(self, ident, msg):
        super().__init__(f"{ident}: {msg}")
        self.ident = ident


class Mex:
    """MATLAB-like calls: ntm(cmd, *args, nout=k) -> list of numpy arrays."""

    def __init__(self, lib):
        self.lib = lib

    def arg(self, v):
        L = self.lib
        if isinstance(v, str):
            return L.t_char(v.encode())
        if isinstance(v, dict):
            s = L.t_struct()
            for k, x in v.items():
                L.t_struct_set(s, k.encode(), self.arg(x))
            return s
        a = np.asarray(v)
        if a.ndim == 0:
            a = a.reshape(1, 1)
        elif a.ndim == 1:
            a = a.reshape(1, -1)
        if a.dtype == np.int32:
            f = np.asfortranarray(a)
            return L.t_int32(a.shape[0], a.shape[1], f.ctypes.data)
        f = np.asfortranarray(a, dtype=np.float64)
        return L.t_double(a.shape[0], a.shape[1], f.ctypes.data)

    def out(self, p):
        L = self.lib
        cls, m, n = L.t_class(p), L.t_m(p), L.t_n(p)
        ct = {DOUBLE: C.c_double, INT32: C.c_int32}[cls]
        buf = (ct * (m * n)).from_address(L.t_data(p))
        a = np.ctypeslib.as_array(buf).copy().reshape(n, m).T           # column-major E-by-B
        L.t_free(p)
        return a

    def __call__(self, cmd, *args, nout=1):
        ins = [self.arg(cmd)] + [self.arg(a) for a in args]
        prhs = (C.c_void_p * len(ins))(*ins)
        plhs = (C.c_void_p * max(nout, 1))()
        rc = self.lib.t_call(nout, plhs, len(ins), prhs)
        if rc:
            raise MexError(self.lib.t_err_id().decode(), self.lib.t_err_msg().decode())
        return [self.out(plhs[i]) for i in range(nout) if plhs[i]]


# ---------------------------------------------------------------- CPU: parsing and errors
def test_mex_rejects_bad_commands_and_shapes(mex):
    with pytest.raises(MexError) as e:
        mex("frobnicate")
    assert e.value.ident == "ntm:arg"
    with pytest.raises(MexError) as e:
        mex(np.ones(2))
    assert e.value.ident == "ntm:arg"
    B, N = 3, 4
    good = dict(x=np.ones((2, B)), rho=np.ones((3 * N, B)), uo=np.ones((N, B)))
    cfg = {"N": 4.0}
    for bad, what in ((dict(good, x=np.ones((3, B))), "x_k"), (dict(good, rho=np.ones((3 * N + 1, B))), "rho"),
                      (dict(good, uo=np.ones((N, B + 1))), "Uold")):
        with pytest.raises(MexError, match=what) as e:
            mex("step", bad["x"], bad["rho"], bad["uo"], cfg)
        assert e.value.ident == "ntm:arg"
    with pytest.raises(MexError) as e:                         # warm-start workspace must be int32
        mex("step", good["x"], good["rho"], good["uo"], cfg, np.ones((2 * (N + 1), B)))
    assert e.value.ident == "ntm:arg"
    with pytest.raises(MexError) as e:
        mex("step", good["x"], good["rho"], good["uo"], 3.0)
    assert e.value.ident == "ntm:cfg"
    with pytest.raises(MexError) as e:
        mex("run", good["x"], 5.0, {"N": 4.0, "xmin": np.ones(3)})
    assert e.value.ident == "ntm:cfg"
    with pytest.raises(MexError) as e:
        mex("run", good["x"], 0.0, cfg)
    assert e.value.ident == "ntm:arg"
    with pytest.raises(MexError):
        mex("scenarios", 5.0)


def test_mex_library_errors_surface_as_matlab_errors(mex):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: the context can be created")
    with pytest.raises(MexError, match="ntm_ctx_create") as e:
        mex("init", np.ones((2, 3)), {"N": 4.0})
    assert e.value.ident == "ntm:library"


# ---------------------------------------------------------------- GPU: bit-identical to ctypes
def _skip_if_variant():
    """The gateway is linked to the product library (rpath); a bitwise comparison
    with a variant build loaded through NTM_MPC_LIB (A/B suites) would compare two
    different builds."""
    from ntm_mpc import _lib
    if _lib.LIB_PATH.resolve() != (LIBDIR / "libntm_mpc.so").resolve():
        pytest.skip(f"ctypes path loads {_lib.LIB_PATH.name} (NTM_MPC_LIB), the gateway libntm_mpc.so")


@pytest.mark.gpu
def test_mex_input_weight_field(mex, ctl):
    """cfg.Ru (ABI v5, the input weight) reaches the library through the gateway: a
    'step' with Ru = 1e-10 equals the ctypes call with the same Config, bit for bit,
    and differs from the Ru = 0 step."""
    from ntm_mpc import Config, scenarios_x0
    _skip_if_variant()
    B, N = 8, 20
    x0 = np.ascontiguousarray(scenarios_x0(0, B))
    outs = []
    for Ru in (1e-10, 0.0):
        mcfg = {"N": float(N), "mode": 2.0, "Ru": Ru}
        cfg = Config(N=N, mode=2, Ru=Ru)
        rho_m, uo_m = mex("init", x0, mcfg, nout=2)
        rho_h, uo_h = ctl.initial_state_host(x0, cfg)
        U = mex("step", x0, rho_m, uo_m, mcfg, nout=1)[0]
        h = ctl.step_host(x0, rho_h, uo_h, cfg)
        np.testing.assert_array_equal(U, h["U"])
        outs.append(U)
    assert np.max(np.abs(outs[0] - outs[1])) > 0


@pytest.mark.gpu
def test_mex_matches_ctypes_path(mex, ctl):
    """'init' / 'step' (warm-start workspace carried) / 'run' / 'scenarios'
    through the gateway == the same calls through ctypes, bit for bit, with a
    cfg struct that sets every field the gateway reads (Q given as MATLAB's
    column-major 2x2)."""
    import torch
    from ntm_mpc import Config, ScenarioGen, scenarios_x0
    _skip_if_variant()
    B, N, k_sim = 12, 20, 4
    Qm = np.array([[2.0e4, 3.0], [3.0, 2.0e-2]])
    mcfg = {"N": float(N), "i_sim": 10.0, "mode": 2.0, "flags": 0.0, "Ts": 0.1, "xmin": [0.06, 200 * np.pi],
            "xmax": [0.15, 10000 * np.pi], "umin": 0.0, "umax": 2e6, "Q": Qm, "r": [0.09, 1800 * np.pi],
            "epsilon": 1e-14, "du_max": 5e5, "Ru": 0.0}
    cfg = Config(N=N, mode=2, Q=tuple(Qm.reshape(-1)), r=(0.09, 1800 * np.pi))
    x0 = np.ascontiguousarray(scenarios_x0(0, B))
    rho_m, uo_m = mex("init", x0, mcfg, nout=2)
    rho_h, uo_h = ctl.initial_state_host(x0, cfg)
    np.testing.assert_array_equal(rho_m, rho_h)
    np.testing.assert_array_equal(uo_m, uo_h)
    ws_m = -np.ones((2 * (N + 1), B), np.int32)
    ws_h = ws_m.copy()
    x = x0
    for _ in range(3):
        U, xp, xn, fl, it, rho_m, uo_m, ws_m = mex("step", x, rho_m, uo_m, mcfg, ws_m, nout=8)
        h = ctl.step_host(x, rho_h, uo_h, cfg, active_ws=ws_h)
        for a, b in ((U, h["U"]), (xp, h["x_pred"]), (xn, h["x_next"]), (rho_m, rho_h), (uo_m, uo_h),
                     (ws_m, ws_h)):
            np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(fl[0], h["exitflag"])
        np.testing.assert_array_equal(it[0], h["inner_iters"])
        x = np.ascontiguousarray(xn)
    outs = mex("run", x0, float(k_sim), mcfg, nout=6)
    ref = ctl.run_host(x0, k_sim, cfg)
    for a, k in zip(outs, ("xk", "uk", "Uk", "wpred", "exitflag", "inner_iters")):
        np.testing.assert_array_equal(a, ref[k], err_msg=k)
    # the scenario generator through the gateway
    gen = {"seed": 7.0, "first_id": 3.0, "sigma_w": 1e-3, "jbs_spread": 0.1, "wdep_spread": 0.1}
    mex("scenarios", gen, nout=0)
    outs = mex("run", x0, float(k_sim), mcfg, nout=6)
    mex("scenarios", np.zeros((0, 0)), nout=0)
    ctl.set_scenarios(ScenarioGen(seed=7, first_id=3, sigma_w=1e-3, jbs_spread=0.1, wdep_spread=0.1))
    try:
        ref = ctl.run_host(x0, k_sim, cfg)
    finally:
        ctl.set_scenarios(None)
    for a, k in zip(outs, ("xk", "uk", "Uk", "wpred", "exitflag", "inner_iters")):
        np.testing.assert_array_equal(a, ref[k], err_msg=k)
    mex("close", nout=0)
    assert mex.lib.t_clear() in (0, 1)
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["closed_loop_m0_N10.npz", "closed_loop_m2_N20.npz", "closed_loop_m3_N20.npz",
                                  "closed_loop_gen_m2_N20.npz"])
def test_mex_run_vs_closed_loop_fixture(mex, ctl, name):
    """NTM_MPC_Sim_gpu.m's 'run' call (ntm_mpc_mex('run', x0, k_sim, cfg), with
    'scenarios' first for a generator fixture) against the committed oracle
    fixture directly: uk, Uk, xk, wpred, exit flags (exact) at the free-running
    closed-loop tolerance of tests/test_gpu_golden.py (1e-6)."""
    import math
    d = np.load(ROOT / "tests" / "golden" / name)
    mode = int(name.split("_m")[1][0])
    N = int(name.split("_N")[1].split(".")[0])
    k_sim = int(d["k_sim"])
    S = d["x0"].shape[0]
    if "gen_seed" in d.files:
        mex("scenarios", {"seed": float(d["gen_seed"]), "first_id": float(d["gen_first_id"]), "k0": float(d["gen_k0"]),
                          "sigma_w": float(d["gen_sigma_w"]), "sigma_omega": float(d["gen_sigma_omega"]),
                          "jbs_spread": float(d["gen_jbs_spread"]), "wdep_spread": float(d["gen_wdep_spread"])},
            nout=0)
    try:
        xk, uk, Uk, wp, fl, its = mex("run", np.ascontiguousarray(d["x0"].T), float(k_sim),
                                      {"N": float(N), "mode": float(mode)}, nout=6)
    finally:
        mex("scenarios", np.zeros((0, 0)), nout=0)
    np.testing.assert_array_equal(fl.T, d["exitflag"])
    tol, umax = 1e-6, 2e6
    assert np.max(np.abs(uk.T - d["uk"])) <= tol * umax
    assert np.max(np.abs(Uk.reshape(k_sim, N, S).transpose(2, 1, 0) - d["Uk"])) <= tol * umax
    xs = np.array([0.15, 2000 * math.pi])[None, :, None]
    assert np.max(np.abs(xk.reshape(k_sim + 1, 2, S).transpose(2, 1, 0) - d["xk"]) / xs) <= tol
    assert np.max(np.abs(wp.reshape(k_sim, N + 1, S).transpose(2, 0, 1) - d["wpred"])) <= tol * 0.15
    assert (its.T == d["inner_iters"]).mean() >= 0.9

"""Host-side mirror of the reference's MATLAB interface over the HIP C-ABI.

The reference (IsaacSavona/MPC-NTM-Control) is a MATLAB script whose hot path
is a handful of functions resolved by name.  MATLAB is not available in this
image, so the host side is Python; it keeps the reference's names, argument
meaning and error behaviour, batched over scenarios:

    rho1 / rho2 / rho3          rho1.m, rho2.m, rho3.m
    A / B                       A.m, B.m
    Rho_to_PhiGammaLambda       Rho_to_PhiGammaLambda.m
    cost (G, F)                 NTM_MPC_Sim.m:120-121
    getWLc                      getWLc.m
    quadprog                    NTM_MPC_Sim.m:97 (exitflag semantics :98-103)
    NtmMpc.step                 NTM_MPC_Sim.m:94-130  (one time step, drop-in)
    NtmMpc.run / NTM_MPC_Sim    NTM_MPC_Sim.m:80-131  (closed loop)

All batched arrays have shape (E, B) — element e of scenario s at [e, s] —
and their storage is the C-ABI's scenario-major layout: each scenario's
E-record is contiguous, [s*E + e], i.e. the transpose of a contiguous (B, E)
array (MATLAB's E-by-B arrays, one column per scenario).  Arrays this module
returns are laid out that way, so passing them back costs nothing; any other
(E, B) array is accepted too, through a staged copy (in/out arguments are
copied back).  ``device_tensor`` builds a device tensor in the ABI layout from
host data.  PyTorch is only plumbing (device memory, streams); every
computation runs in the HIP kernels of lib/libntm_mpc.so.  There is no CPU
fallback: without the library or a GPU, calls raise.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib as L
from ._lib import NtmConfig, NtmLibraryError, NtmPhysics, NtmScenarioGen


STATS_ROWS = 6   # include/ntm_mpc.h NTM_STATS_ROWS


@dataclass
class Physics:
    """Physics constants, NTM_MPC_Sim.m:5-22."""
    j_BS: float = 73e3
    w_dep: float = 0.024
    w_marg: float = 0.02
    w_sat: float = 0.32
    tau_r: float = 293.0
    rs: float = 1.55
    a: float = 2.0
    eta_CD: float = 0.9
    tau_E0: float = 3.7
    tau_E: float = 3.7
    mu0: float = 4e-7 * math.pi
    Lq: float = 0.87
    B_pol: float = 0.97
    m: float = 2.0
    Cw: float = 1.0
    tau_A0: float = 3e-6
    tau_w: float = 0.188
    omega0: float = 2 * math.pi * 420

    def to_c(self) -> NtmPhysics:
        return NtmPhysics(*[float(getattr(self, n)) for n in L.PHYSICS_FIELDS])


@dataclass
class Config:
    """Controller configuration, NTM_MPC_Sim.m:30-60, 80-88 (mode/flags: SURVEY.md §2.1)."""
    N: int = 20
    Ts: float = 0.1
    xmin: tuple = (0.06, 100 * 2 * math.pi)
    xmax: tuple = (0.15, 5000 * 2 * math.pi)
    umin: float = 0.0
    umax: float = 2e6
    Q: tuple = (1.0, 0.0, 0.0, 1.0)
    r: tuple = (0.0, 1000 * 2 * math.pi)
    i_sim: int = 10
    epsilon: float = 1e-14
    mode: int = L.MODE_FULL
    flags: int = 0
    du_max: float = 5e5      # NTM_MODE_FULL_DU (config 5, extension): |U_i - U_{i-1}| <= du_max
    Ru: float = 0.0          # input weight (ABI v5): G = 2 Gamma' Om Gamma + 2 Ru I; the reference: 0

    def to_c(self) -> NtmConfig:
        return NtmConfig(int(self.N), int(self.i_sim), int(self.mode), int(self.flags), float(self.Ts),
                         (C.c_double * 2)(*self.xmin), (C.c_double * 2)(*self.xmax), float(self.umin),
                         float(self.umax), (C.c_double * 4)(*self.Q), (C.c_double * 2)(*self.r),
                         float(self.epsilon), float(self.du_max), float(self.Ru))

    @property
    def m(self) -> int:
        if self.mode == L.MODE_NONE:
            return 0
        if self.mode == L.MODE_BOX:
            return 2 * self.N
        return 6 * self.N + 4 + (2 * (self.N - 1) if self.mode == L.MODE_FULL_DU else 0)


@dataclass
class ScenarioGen:
    """ntm_scenario_gen: independent plasma scenarios (j_BS, w_dep of NTM_MPC_Sim.m:5-6,
    each scaled by 1 + spread (2u - 1)) and additive plant disturbances (on
    NTM_MPC_Sim.m:130, unit-variance Irwin-Hall samples times sigma), all
    counter-based on (seed, global scenario id, time index)."""
    seed: int = 20241220
    first_id: int = 0          # global id of the batch's scenario 0 (a shard's offset)
    k0: int = 0                # time index of the next launch's first plant step
    sigma_w: float = 0.0       # [m]
    sigma_omega: float = 0.0   # [rad/s]
    jbs_spread: float = 0.0
    wdep_spread: float = 0.0

    def to_c(self) -> NtmScenarioGen:
        return NtmScenarioGen(int(self.seed) & 0xFFFFFFFFFFFFFFFF, int(self.first_id), int(self.k0), 0,
                              float(self.sigma_w), float(self.sigma_omega), float(self.jbs_spread),
                              float(self.wdep_spread))


def scenario_sample(gen: ScenarioGen, B: int, k: int = 0) -> np.ndarray:
    """(B, 4) host-side samples of the generator for scenarios gen.first_id + s: j_BS
    factor, w_dep factor, n_w(k), n_omega(k) (ntm_scenario_sample; no GPU needed)."""
    out = np.zeros((B, 4))
    L.load().ntm_scenario_sample(C.byref(gen.to_c()), B, k, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def _check_dev(t: torch.Tensor, shape, dtype=torch.float64, name="tensor"):
    """Plain contiguous CUDA array (instrumentation counters, SoA)."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def is_scenario_major(a) -> bool:
    """(E, B) array whose storage is scenario-major ([s*E + e]); 1-D arrays trivially."""
    if isinstance(a, np.ndarray):
        return a.ndim < 2 or a.T.flags.c_contiguous
    return a.dim() < 2 or a.T.is_contiguous()


def _dev_arg(t, shape, dtype=torch.float64, name="tensor"):
    """Validate an (E, B) CUDA argument; return (array in the ABI layout, staged?)."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if is_scenario_major(t):
        return t, False
    return t.T.contiguous().T, True


def _host_arg(a, shape, dtype=np.float64, name="array"):
    """Validate an (E, B) host argument; return (array in the ABI layout, staged?)."""
    if not isinstance(a, np.ndarray) or a.shape != tuple(shape) or a.dtype != dtype:
        raise ValueError(f"{name}: expected {np.dtype(dtype).name} {tuple(shape)}")
    if is_scenario_major(a):
        return a, False
    return np.asfortranarray(a), True


def _host_empty(*shape, dtype=np.float64):
    return np.empty(shape[::-1], dtype).T if len(shape) == 2 else np.empty(shape, dtype)


def device_tensor(a, device=None, dtype=torch.float64) -> torch.Tensor:
    """(E, B) host data -> (E, B) CUDA tensor in the ABI's scenario-major layout."""
    a = np.asarray(a)
    if device is None:
        device = torch.cuda.current_device()
    dev = device if isinstance(device, (str, torch.device)) else torch.device("cuda", int(device))
    return torch.tensor(np.ascontiguousarray(a.T), dtype=dtype, device=dev).T


class NtmMpc:
    """Batched LPV-MPC controller on one MI355X (one ``ntm_ctx`` per device)."""

    def __init__(self, physics: Physics | None = None, config: Config | None = None, device: int | None = None):
        self.lib = L.load()
        if not torch.cuda.is_available():
            raise NtmLibraryError("no GPU visible: the HIP path has no CPU fallback")
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.physics = physics or Physics()
        self.config = config or Config()
        self.gen = None
        self._ctx = C.c_void_p()
        rc = self.lib.ntm_ctx_create(C.byref(self._ctx), self.device)
        if rc != L.NTM_OK:
            raise NtmLibraryError(f"ntm_ctx_create failed ({rc})")

    def close(self):
        if self._ctx:
            self.lib.ntm_ctx_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ helpers
    def _cfg(self, cfg: Config | None):
        return (cfg or self.config).to_c()

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _raise(self, rc, what):
        if rc != L.NTM_OK:
            raise NtmLibraryError(f"{what} failed ({rc}): {self.lib.ntm_last_error(self._ctx).decode()}")

    def _empty(self, *shape, dtype=torch.float64):
        """(E, B) output in the ABI's scenario-major layout (1-D: plain)."""
        dev = f"cuda:{self.device}"
        if len(shape) == 2:
            return torch.empty(shape[1], shape[0], dtype=dtype, device=dev).T
        return torch.empty(*shape, dtype=dtype, device=dev)

    def tensor(self, a, dtype=torch.float64) -> torch.Tensor:
        """(E, B) host data -> device tensor in the ABI layout on this controller's GPU."""
        return device_tensor(a, self.device, dtype)

    def set_stats(self, stats: torch.Tensor | None):
        """Accumulate per-scenario counters (NTM_STATS_ROWS=6, B) int32 (plain
        contiguous rows) into ``stats`` during subsequent step/run launches: QP
        solves, GI iterations, final active rows, state rows in the final active
        set, warm-start candidate verifications, full GI solves; None disables."""
        if stats is not None:
            if stats.dim() != 2 or stats.shape[0] != STATS_ROWS:
                raise ValueError(f"stats must be ({STATS_ROWS}, B) int32")
            _check_dev(stats, tuple(stats.shape), dtype=torch.int32, name="stats")
        self._raise(self.lib.ntm_ctx_set_stats(self._ctx, _ptr(stats)), "ntm_ctx_set_stats")

    def set_small_batch(self, max_scenarios: int = -1):
        """ntm_ctx_set_small_batch: N = 20 batches of at most ``max_scenarios``
        run on the all-LDS build, larger ones on the far-workspace 4-wave build;
        -1 restores the default (8 x the compute units), 0 always uses the far
        build."""
        self._raise(self.lib.ntm_ctx_set_small_batch(self._ctx, int(max_scenarios)), "ntm_ctx_set_small_batch")

    def set_one_wave_batch(self, max_scenarios: int = -1):
        """ntm_ctx_set_one_wave_batch: all-LDS N = 20 batches of at most
        ``max_scenarios`` use the one-wave register budget (bit-identical results);
        -1 restores the default (4 x the compute units), 0 never."""
        self._raise(self.lib.ntm_ctx_set_one_wave_batch(self._ctx, int(max_scenarios)), "ntm_ctx_set_one_wave_batch")

    def step_build(self, B: int, cfg: Config | None = None) -> str:
        """The build a launch of B scenarios takes: "far", "lds" or "lds1" (the
        all-LDS build with the one-wave register budget; ntm_ctx_step_build)."""
        b = C.c_int32()
        self._raise(self.lib.ntm_ctx_step_build(self._ctx, C.byref((cfg or self.config).to_c()), int(B), C.byref(b)),
                    "ntm_ctx_step_build")
        return ("far", "lds", "lds1")[b.value]

    def set_scenarios(self, gen: ScenarioGen | None):
        """Attach a scenario generator (ntm_ctx_set_scenarios): subsequent
        initial_state / step / run launches use each scenario's own plasma and
        add its disturbance realisation to the plant step; None restores the
        nominal, disturbance-free loop of the reference."""
        self.gen = gen
        self._raise(self.lib.ntm_ctx_set_scenarios(self._ctx, None if gen is None else C.byref(gen.to_c())),
                    "ntm_ctx_set_scenarios")

    def _layout(self, B: int, cfg: Config):
        far, lanes, nn = C.c_int32(), C.c_int32(), C.c_int32()
        self._raise(self.lib.ntm_ctx_step_layout_cfg(self._ctx, C.byref(cfg.to_c()), int(B), C.byref(far),
                                                     C.byref(lanes), C.byref(nn)), "ntm_ctx_step_layout_cfg")
        return ("far" if far.value else "lds"), lanes.value, nn.value

    def step_layout(self, B: int, cfg: Config | None = None) -> str:
        """Workspace layout of the build a launch of B scenarios with ``cfg``
        (flags included) takes: "far" (J/R in a per-scenario HBM block) or "lds"
        (ntm_ctx_step_layout_cfg)."""
        return self._layout(B, cfg or self.config)[0]

    def step_kernel_name(self, B: int, cfg: Config | None = None) -> str:
        """Name of the fused step kernel specialisation a launch uses (reporting)."""
        layout, lanes, nn = self._layout(B, cfg or self.config)
        build = self.step_build(B, cfg)
        return f"k_mpc_step<P={lanes},NN={nn},{layout}>" + (" (one-wave budget)" if build == "lds1" else "")

    # ------------------------------------------------------------ hot path
    def initial_state(self, x0: torch.Tensor, cfg: Config | None = None):
        """Rho = repmat(rho(x0), 1, N) (NTM_MPC_Sim.m:63-65); U_old = +inf (D14)."""
        cfg = cfg or self.config
        Bn = x0.shape[1]
        x0, _ = _dev_arg(x0, (2, Bn), name="x0")
        rho, U_old = self._empty(3 * cfg.N, Bn), self._empty(cfg.N, Bn)
        self._raise(self.lib.ntm_mpc_init_device(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn,
                                                 _ptr(x0), _ptr(rho), _ptr(U_old), self._stream()),
                    "ntm_mpc_init_device")
        return rho, U_old

    def initial_state_host(self, x0: np.ndarray, cfg: Config | None = None):
        """ntm_mpc_init with host arrays (the MEX path)."""
        cfg = cfg or self.config
        Bn = x0.shape[1]
        x0, _ = _host_arg(x0, (2, Bn), name="x0")
        rho, U_old = _host_empty(3 * cfg.N, Bn), _host_empty(cfg.N, Bn)
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))          # noqa: E731
        self._raise(self.lib.ntm_mpc_init(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn,
                                          dp(x0), dp(rho), dp(U_old)), "ntm_mpc_init")
        return rho, U_old

    def new_active_ws(self, B: int, cfg: Config | None = None) -> torch.Tensor:
        """Empty warm-start workspace for step(..., active_ws=): (2(N+1), B) int32 of -1."""
        cfg = cfg or self.config
        return self._empty(2 * (cfg.N + 1), B, dtype=torch.int32).fill_(-1)

    def step(self, x_k: torch.Tensor, rho: torch.Tensor, U_old: torch.Tensor, cfg: Config | None = None,
             out: dict | None = None, active_ws: torch.Tensor | None = None):
        """One MPC time step for a batch (NTM_MPC_Sim.m:94-130).  ``rho`` (3N, B) and
        ``U_old`` (N, B) are updated in place.  ``active_ws`` (see new_active_ws)
        carries the last two active sets from step to step as verified warm
        starts (ntm_mpc_step_ws_device).  Returns dict U, x_pred, x_next,
        exitflag, inner_iters (all CUDA tensors); ``out`` (a dict this method
        returned earlier) is reused."""
        cfg = cfg or self.config
        N, Bn = cfg.N, x_k.shape[1]
        xk, _ = _dev_arg(x_k, (2, Bn), name="x_k")
        rh, rho_st = _dev_arg(rho, (3 * N, Bn), name="rho")
        uo, uo_st = _dev_arg(U_old, (N, Bn), name="U_old")
        ws, ws_st = (None, False) if active_ws is None else _dev_arg(active_ws, (2 * (N + 1), Bn), torch.int32,
                                                                     "active_ws")
        if out is None:
            out = {"U": self._empty(N, Bn), "x_pred": self._empty(2 * (N + 1), Bn), "x_next": self._empty(2, Bn),
                   "exitflag": self._empty(Bn, dtype=torch.int32), "inner_iters": self._empty(Bn, dtype=torch.int32)}
        else:
            for k, shp in (("U", (N, Bn)), ("x_pred", (2 * (N + 1), Bn)), ("x_next", (2, Bn))):
                if tuple(out[k].shape) != shp or not is_scenario_major(out[k]):
                    raise ValueError(f"out[{k!r}] must be a {shp} array from an earlier step()")
        rc = self.lib.ntm_mpc_step_ws_device(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn,
                                             _ptr(xk), _ptr(rh), _ptr(uo), _ptr(out["U"]), _ptr(out["x_pred"]),
                                             _ptr(out["x_next"]), _ptr(out["exitflag"]), _ptr(out["inner_iters"]),
                                             _ptr(ws), self._stream())
        self._raise(rc, "ntm_mpc_step_ws_device")
        for staged, dst, src in ((rho_st, rho, rh), (uo_st, U_old, uo), (ws_st, active_ws, ws)):
            if staged:
                dst.copy_(src)
        return out

    def run(self, x0: torch.Tensor, k_sim: int = 20, cfg: Config | None = None):
        """Closed loop NTM_MPC_Sim.m:80-131 on device.  Returns the workspace
        variables xk (2(k_sim+1), B), uk (k_sim, B), Uk (N k_sim, B), wpred
        ((N+1) k_sim, B), exitflag / inner_iters (k_sim, B)."""
        cfg = cfg or self.config
        N, Bn = cfg.N, x0.shape[1]
        x0, _ = _dev_arg(x0, (2, Bn), name="x0")
        out = {"xk": self._empty(2 * (k_sim + 1), Bn), "uk": self._empty(k_sim, Bn), "Uk": self._empty(N * k_sim, Bn),
               "wpred": self._empty((N + 1) * k_sim, Bn), "exitflag": self._empty(k_sim, Bn, dtype=torch.int32),
               "inner_iters": self._empty(k_sim, Bn, dtype=torch.int32)}
        rc = self.lib.ntm_mpc_run_device(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn, k_sim,
                                         _ptr(x0), _ptr(out["xk"]), _ptr(out["uk"]), _ptr(out["Uk"]),
                                         _ptr(out["wpred"]), _ptr(out["exitflag"]), _ptr(out["inner_iters"]),
                                         self._stream())
        self._raise(rc, "ntm_mpc_run_device")
        return out

    # ------------------------------------------------------------ host-buffer entry points (the MEX path)
    def step_host(self, x_k: np.ndarray, rho: np.ndarray, U_old: np.ndarray, cfg: Config | None = None,
                  active_ws: np.ndarray | None = None):
        """ntm_mpc_step with host (NumPy fp64) arrays, as a MEX gateway calls it:
        the library stages through its own device buffers.  ``rho`` and
        ``U_old`` (and ``active_ws``) are updated in place."""
        cfg = cfg or self.config
        N, Bn = cfg.N, x_k.shape[1]
        xk, _ = _host_arg(x_k, (2, Bn), name="x_k")
        rh, rho_st = _host_arg(rho, (3 * N, Bn), name="rho")
        uo, uo_st = _host_arg(U_old, (N, Bn), name="U_old")
        ws, ws_st = (None, False) if active_ws is None else _host_arg(active_ws, (2 * (N + 1), Bn), np.int32,
                                                                      "active_ws")
        out = {"U": _host_empty(N, Bn), "x_pred": _host_empty(2 * (N + 1), Bn), "x_next": _host_empty(2, Bn),
               "exitflag": np.empty(Bn, np.int32), "inner_iters": np.empty(Bn, np.int32)}
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))          # noqa: E731
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))           # noqa: E731
        rc = self.lib.ntm_mpc_step_ws(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn, dp(xk),
                                      dp(rh), dp(uo), dp(out["U"]), dp(out["x_pred"]), dp(out["x_next"]),
                                      ip(out["exitflag"]), ip(out["inner_iters"]), None if ws is None else ip(ws))
        self._raise(rc, "ntm_mpc_step_ws")
        for staged, dst, src in ((rho_st, rho, rh), (uo_st, U_old, uo), (ws_st, active_ws, ws)):
            if staged:
                dst[...] = src
        return out

    def run_host(self, x0: np.ndarray, k_sim: int = 20, cfg: Config | None = None):
        """ntm_mpc_run with host arrays (NTM_MPC_Sim.m:80-131 for a batch)."""
        cfg = cfg or self.config
        N, Bn = cfg.N, x0.shape[1]
        x0, _ = _host_arg(x0, (2, Bn), name="x0")
        out = {"xk": _host_empty(2 * (k_sim + 1), Bn), "uk": _host_empty(k_sim, Bn),
               "Uk": _host_empty(N * k_sim, Bn), "wpred": _host_empty((N + 1) * k_sim, Bn),
               "exitflag": _host_empty(k_sim, Bn, dtype=np.int32), "inner_iters": _host_empty(k_sim, Bn, dtype=np.int32)}
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))          # noqa: E731
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))           # noqa: E731
        rc = self.lib.ntm_mpc_run(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn, k_sim, dp(x0),
                                  dp(out["xk"]), dp(out["uk"]), dp(out["Uk"]), dp(out["wpred"]),
                                  ip(out["exitflag"]), ip(out["inner_iters"]))
        self._raise(rc, "ntm_mpc_run")
        return out

    # ------------------------------------------------------------ function level
    def rho(self, x: torch.Tensor, cfg: Config | None = None, physics: Physics | None = None):
        """rho1.m / rho2.m / rho3.m at x (2, B) -> (3, B) (``physics`` overrides w_marg / w_dep)."""
        Bn = x.shape[1]
        x, _ = _dev_arg(x, (2, Bn), name="x")
        out = self._empty(3, Bn)
        ph = physics or self.physics
        self._raise(self.lib.ntm_rho_device(self._ctx, C.byref(ph.to_c()), C.byref(self._cfg(cfg)), Bn,
                                            _ptr(x), _ptr(out), self._stream()), "ntm_rho_device")
        return out

    def AB(self, rho: torch.Tensor, cfg: Config | None = None):
        """A.m / B.m at rho (3, B) -> A (4, B) col-major 2x2, B (2, B) column (D5)."""
        Bn = rho.shape[1]
        rho, _ = _dev_arg(rho, (3, Bn), name="rho")
        A, Bv = self._empty(4, Bn), self._empty(2, Bn)
        self._raise(self.lib.ntm_AB_device(self._ctx, C.byref(self.physics.to_c()), C.byref(self._cfg(cfg)), Bn,
                                           _ptr(rho), _ptr(A), _ptr(Bv), self._stream()), "ntm_AB_device")
        return A, Bv

    def lift(self, rho: torch.Tensor, cfg: Config | None = None):
        """Rho_to_PhiGammaLambda.m: rho (3N, B) -> Phi (4N, B), Gamma (2N*N, B), Lambda (2N, B)."""
        cfg = cfg or self.config
        N, Bn = cfg.N, rho.shape[1]
        rho, _ = _dev_arg(rho, (3 * N, Bn), name="rho")
        Phi, Gam, Lam = self._empty(4 * N, Bn), self._empty(2 * N * N, Bn), self._empty(2 * N, Bn)
        self._raise(self.lib.ntm_lift_device(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn,
                                             _ptr(rho), _ptr(Phi), _ptr(Gam), _ptr(Lam), self._stream()),
                    "ntm_lift_device")
        return Phi, Gam, Lam

    def cost(self, rho: torch.Tensor, x_k: torch.Tensor, cfg: Config | None = None):
        """NTM_MPC_Sim.m:120-121 -> G (N*N, B), F (N, B)."""
        cfg = cfg or self.config
        N, Bn = cfg.N, rho.shape[1]
        rho, _ = _dev_arg(rho, (3 * N, Bn), name="rho")
        x_k, _ = _dev_arg(x_k, (2, Bn), name="x_k")
        G, F = self._empty(N * N, Bn), self._empty(N, Bn)
        self._raise(self.lib.ntm_cost_device(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn,
                                             _ptr(rho), _ptr(x_k), _ptr(G), _ptr(F), self._stream()),
                    "ntm_cost_device")
        return G, F

    def getWLc(self, rho: torch.Tensor, cfg: Config | None = None):
        """getWLc.m -> W (2m, B), L (m*N, B), c (m, B), m = 6N+4 (column-major per scenario)."""
        cfg = cfg or self.config
        N, Bn = cfg.N, rho.shape[1]
        m = 6 * N + 4
        rho, _ = _dev_arg(rho, (3 * N, Bn), name="rho")
        W, Lm, c = self._empty(2 * m, Bn), self._empty(m * N, Bn), self._empty(m, Bn)
        self._raise(self.lib.ntm_getwlc_device(self._ctx, C.byref(self.physics.to_c()), C.byref(cfg.to_c()), Bn,
                                               _ptr(rho), _ptr(W), _ptr(Lm), _ptr(c), self._stream()),
                    "ntm_getwlc_device")
        return W, Lm, c

    def quadprog(self, H: torch.Tensor, f: torch.Tensor, Lin: torch.Tensor | None, b: torch.Tensor | None):
        """quadprog(H, f, A, b) for a batch: min 1/2 U'HU + f'U s.t. Lin U <= b.
        H (N*N, B), f (N, B), Lin (m*N, B) column-major per scenario, b (m, B).
        Returns (U (N, B), exitflag (B,), iterations (B,)); exitflag as quadprog
        (1 optimal, 0 max iterations, -2 infeasible -> U = 0, -7 non-finite)."""
        N, Bn = f.shape
        m = 0 if Lin is None else b.shape[0]
        H, _ = _dev_arg(H, (N * N, Bn), name="H")
        f, _ = _dev_arg(f, (N, Bn), name="f")
        if m:
            Lin, _ = _dev_arg(Lin, (m * N, Bn), name="A")
            b, _ = _dev_arg(b, (m, Bn), name="b")
        U = self._empty(N, Bn)
        flag = self._empty(Bn, dtype=torch.int32)
        its = self._empty(Bn, dtype=torch.int32)
        self._raise(self.lib.ntm_qp_device(self._ctx, Bn, N, m, _ptr(H), _ptr(f), _ptr(Lin) if m else None,
                                           _ptr(b) if m else None, _ptr(U), _ptr(flag), _ptr(its), self._stream()),
                    "ntm_qp_device")
        return U, flag, its


def _quadprog_mixed(self, H: torch.Tensor, f: torch.Tensor, Lin: torch.Tensor | None, b: torch.Tensor | None):
    """Config 5's fp32 leg (ntm_qp_mixed_device; not the fp64 product path): the QP
    solved in fp32 on fp32-rounded data, its active set then re-solved exactly in
    fp64 and certified (fp64 fallback otherwise).  Returns (U refined (N, B),
    U32 fp32 solution (N, B), exitflag (B,), info (B,) bit 0 certified / bit 1
    fp64 fallback / bit 2 fp32 not optimal, fp32 GI iterations (B,))."""
    N, Bn = f.shape
    m = 0 if Lin is None else b.shape[0]
    H, _ = _dev_arg(H, (N * N, Bn), name="H")
    f, _ = _dev_arg(f, (N, Bn), name="f")
    if m:
        Lin, _ = _dev_arg(Lin, (m * N, Bn), name="A")
        b, _ = _dev_arg(b, (m, Bn), name="b")
    U, U32 = self._empty(N, Bn), self._empty(N, Bn)
    flag, info, its = (self._empty(Bn, dtype=torch.int32) for _ in range(3))
    self._raise(self.lib.ntm_qp_mixed_device(self._ctx, Bn, N, m, _ptr(H), _ptr(f), _ptr(Lin) if m else None,
                                             _ptr(b) if m else None, _ptr(U), _ptr(U32), _ptr(flag), _ptr(info),
                                             _ptr(its), self._stream()), "ntm_qp_mixed_device")
    return U, U32, flag, info, its


NtmMpc.quadprog_mixed = _quadprog_mixed


def scenarios_x0(first_id: int, B: int, seed: int = 20241220):
    """Synthetic initial states for global ids first_id..first_id+B-1:
    (2, B) float64 numpy array in the ABI layout (each scenario's [w, omega] contiguous)."""
    x0 = _host_empty(2, B)
    L.load().ntm_scenarios_x0(C.c_uint64(seed), first_id, B, x0.ctypes.data_as(C.POINTER(C.c_double)))
    return x0


# ---- MATLAB-named thin wrappers (reference function names) ----------------

_default = None


def _ctl():
    global _default
    if _default is None:
        _default = NtmMpc()
    return _default


def _phys_with(**kw):
    ph = _ctl().physics
    kw = {k: float(v) for k, v in kw.items() if v is not None}
    return dataclasses.replace(ph, **kw) if kw else ph


def rho1(x, wmarg=None):
    """rho1.m (batched): rho1(x, wmarg) = 1/(x(1) + wmarg^2), x (2, B) CUDA -> (B,).
    ``wmarg`` defaults to the controller's physics (NTM_MPC_Sim.m:7)."""
    return _ctl().rho(x, physics=_phys_with(w_marg=wmarg))[0]


def rho2(x):
    """rho2.m (batched): x(1)^2 / x(2)."""
    return _ctl().rho(x)[1]


def rho3(x, w_dep=None):
    """rho3.m (batched): rho3(x, w_dep); ``w_dep`` defaults to the controller's physics (:6)."""
    return _ctl().rho(x, physics=_phys_with(w_dep=w_dep))[2]


def Rho_to_PhiGammaLambda(Rho1, Rho2, Rho3, cfg: Config | None = None):
    """Rho_to_PhiGammaLambda.m (batched): Rho1/2/3 (N, B) -> Phi, Gamma, Lambda."""
    rho = torch.stack([Rho1, Rho2, Rho3], dim=1).reshape(-1, Rho1.shape[1])
    return _ctl().lift(rho, cfg)


def quadprog(H, f, A=None, b=None):
    """quadprog stand-in (NTM_MPC_Sim.m:97)."""
    return _ctl().quadprog(H, f, A, b)


def NTM_MPC_Sim(x0, k_sim: int = 20, cfg: Config | None = None):
    """The driver NTM_MPC_Sim.m:80-131 for a batch of initial states x0 (2, B)."""
    return _ctl().run(x0, k_sim, cfg)

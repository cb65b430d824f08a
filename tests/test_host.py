"""Host-side checks that need no GPU: the HIP library builds for gfx950, loads,
exports every symbol include/ntm_mpc.h declares, and the Python mirror's
host logic (configs, defaults, layouts, scenario generator, flop model)."""
import ctypes as C
import math
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "ntm_mpc.h"


def declared_functions():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ntm_[A-Za-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    import ntm_mpc
    lib = ntm_mpc.load()
    names = declared_functions()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), n
    from ntm_mpc._lib import EXPORTS
    assert set(EXPORTS) == set(names)


def test_library_is_gfx950_code_object(tmp_path):
    import shutil
    import subprocess
    lib = tmp_path / "libntm_mpc.so"          # llvm-objdump extracts bundles next to its input
    shutil.copy(ROOT / "mpc-ntm-control_amd" / "lib" / "libntm_mpc.so", lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)], capture_output=True,
                         text=True, cwd=tmp_path)
    assert "gfx950" in (out.stdout + out.stderr)


def test_defaults_match_reference_literals():
    from ntm_mpc import _lib as L
    from ntm_mpc.api import Config, Physics
    p = L.default_physics()
    ref = Physics()
    for n in L.PHYSICS_FIELDS:
        assert getattr(p, n) == pytest.approx(getattr(ref, n), rel=1e-15), n
    c = L.default_config(20)
    assert (c.N, c.i_sim, c.mode) == (20, 10, 2)
    assert c.Ts == 0.1 and c.umax == 2e6 and c.umin == 0
    assert tuple(c.xmin) == pytest.approx((0.06, 200 * math.pi))
    assert tuple(c.xmax) == pytest.approx((0.15, 10000 * math.pi))
    assert c.r[1] == pytest.approx(2000 * math.pi) and c.epsilon == 1e-14
    py = Config(N=20).to_c()
    for f, _ in L.NtmConfig._fields_:
        a, b = getattr(py, f), getattr(c, f)
        if hasattr(a, "__len__"):
            assert list(a) == pytest.approx(list(b))
        else:
            assert a == pytest.approx(b)


def test_config_rows():
    from ntm_mpc.api import Config
    assert Config(N=20, mode=2).m == 124
    assert Config(N=20, mode=1).m == 40
    assert Config(N=20, mode=0).m == 0


def test_scenario_generator_matches_oracle():
    """ntm_scenarios_x0 (C-ABI) == oracle scenario_x0: shard-invariant synthetic inputs."""
    import ntm_mpc
    from oracle import ntm_oracle as O
    x = ntm_mpc.scenarios_x0(1000, 257)
    np.testing.assert_array_equal(x.T, O.scenario_x0(np.arange(1000, 1257)))
    a = ntm_mpc.scenarios_x0(0, 10)
    b = ntm_mpc.scenarios_x0(5, 5)
    np.testing.assert_array_equal(a[:, 5:], b)


def test_disturbance_generator_matches_both_oracles():
    """ntm_scenario_sample (the device's generator code compiled for the host) ==
    the C oracle == the NumPy oracle, bit for bit, for plasma factors and
    disturbance samples; counter-based (a shard's first_id offset reproduces the
    same values); the samples have zero mean and unit variance and the factors
    stay inside 1 +- spread."""
    import ntm_mpc
    from oracle import cbind
    from oracle import ntm_oracle as O
    for seed, first, k in ((20241220, 0, 0), (7, -5, 13), (2 ** 64 - 1, 10 ** 12, 2 ** 31 - 1)):
        g = O.ScenarioGen(seed=seed, first_id=first, k0=0, sigma_w=1e-3, sigma_omega=1.0, jbs_spread=0.1,
                          wdep_spread=0.37)
        lib = ntm_mpc.scenario_sample(ntm_mpc.ScenarioGen(**vars(g)), 300, k)
        np.testing.assert_array_equal(lib, cbind.scenario_sample(g, 300, k))
        py = np.array([[O.gen_factor(seed, first + s, 0, 0.1), O.gen_factor(seed, first + s, 1, 0.37),
                        O.gen_normal(seed, first + s, k, 0), O.gen_normal(seed, first + s, k, 1)]
                       for s in range(300)])
        np.testing.assert_array_equal(lib, py)
        shard = ntm_mpc.scenario_sample(ntm_mpc.ScenarioGen(**{**vars(g), "first_id": first + 100}), 200, k)
        np.testing.assert_array_equal(shard, lib[100:])
    big = ntm_mpc.scenario_sample(ntm_mpc.ScenarioGen(seed=3, jbs_spread=0.1, wdep_spread=0.1), 200_000, 5)
    n = big[:, 2:].ravel()
    assert abs(n.mean()) < 0.01 and abs(n.std() - 1.0) < 0.01
    assert np.abs(n).max() <= 2 * math.sqrt(3)
    assert big[:, :2].min() >= 0.9 and big[:, :2].max() < 1.1
    assert abs(np.corrcoef(big[:, 2], big[:, 3])[0, 1]) < 0.01
    # different time indices give independent draws
    other = ntm_mpc.scenario_sample(ntm_mpc.ScenarioGen(seed=3), 200_000, 6)
    assert abs(np.corrcoef(big[:, 2], other[:, 2])[0, 1]) < 0.01


def test_scenario_gen_struct_layout():
    """ctypes mirrors of ntm_scenario_gen agree with the C layout (56 bytes)."""
    from ntm_mpc._lib import NtmScenarioGen
    from oracle.cbind import CGen
    assert C.sizeof(NtmScenarioGen) == C.sizeof(CGen) == 56
    assert NtmScenarioGen.sigma_w.offset == 24 and NtmScenarioGen.wdep_spread.offset == 48


def test_no_gpu_raises_not_falls_back():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ntm_mpc import NtmLibraryError, NtmMpc
    with pytest.raises(NtmLibraryError):
        NtmMpc()


def test_ctx_create_without_gpu_is_an_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ntm_mpc
    ctx = C.c_void_p()
    assert ntm_mpc.load().ntm_ctx_create(C.byref(ctx), 0) != 0


def test_flop_model_monotone():
    from ntm_mpc import flops
    # qps, tries, giruns, K (per step); q, s (per QP)
    a = flops.per_step(20, 2, 8, 6, 2, 60, 19, 5)
    b = flops.per_step(20, 2, 8, 6, 2, 90, 19, 5)
    c = flops.per_step(20, 2, 8, 4, 4, 60, 19, 5)        # a full GI solve costs more than a verify
    assert 0 < a < b and a < c
    # never above the survey's IPM-based count (6.47e6 flop/step at N=20)
    assert flops.per_step(20, 2, 10, 0, 10, 400, 20, 10) < 6.47e6
    assert flops.hbm_bytes_per_step(20) == 8 * (2 + 120 + 40 + 20 + 42 + 2) + 8


def test_launch_info_dispatch():
    """The kernel specialisation per horizon (host logic, no GPU needed)."""
    import ntm_mpc
    lib = ntm_mpc.load()
    lanes, nn = C.c_int32(), C.c_int32()
    for N, want in [(3, (16, 0)), (10, (16, 10)), (20, (64, 20)), (33, (64, 0)), (50, (64, 50))]:
        assert lib.ntm_step_launch_info(N, C.byref(lanes), C.byref(nn)) == 0
        assert (lanes.value, nn.value) == want, N
    assert lib.ntm_step_launch_info(0, C.byref(lanes), C.byref(nn)) != 0


def test_product_never_imports_oracle():
    """The product package must not import, link or execute the oracle (checker)."""
    pkg = ROOT / "mpc-ntm-control_amd"
    bad = re.compile(r"(import\s+oracle|from\s+oracle|libntm_oracle|cbind|ntm_oracle_)")
    for f in list(pkg.rglob("*.py")) + list(pkg.rglob("*.hip")) + list(pkg.rglob("*.h")) + [pkg / "Makefile"]:
        assert not bad.search(f.read_text()), f


def test_bench_record_histories():
    """bench.py's closed-loop record: the step kernels write scenario-major (K, B, E)
    slots (each an (E, B) ABI view), and _histories forms the (..., B) histories the
    gather and the report use: uk = U(1), Uk, xk (with x_0), wpred = x_pred(1:2:end)."""
    import importlib.util
    import torch
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    K, B, N = 3, 5, 4
    g = torch.Generator().manual_seed(0)
    raw = {"U": torch.randn(K, B, N, generator=g, dtype=torch.float64),
           "x_pred": torch.randn(K, B, 2 * (N + 1), generator=g, dtype=torch.float64),
           "x_next": torch.randn(K + 1, B, 2, generator=g, dtype=torch.float64),
           "exitflag": torch.ones(K, B, dtype=torch.int32), "inner_iters": torch.full((K, B), 10, dtype=torch.int32)}
    for i in range(K):                              # the per-step views the kernels write
        assert raw["U"][i].T.shape == (N, B) and raw["U"][i].T.T.is_contiguous()
    h = bench._histories({"hist": {"raw": dict(raw)}})
    assert h["Uk"].shape == (K, N, B) and h["xk"].shape == (K + 1, 2, B) and h["wpred"].shape == (K, N + 1, B)
    for i in range(K):
        assert torch.equal(h["uk"][i], raw["U"][i][:, 0])
        assert torch.equal(h["Uk"][i], raw["U"][i].T)
        assert torch.equal(h["wpred"][i], raw["x_pred"][i].T[0::2])
    for i in range(K + 1):
        assert torch.equal(h["xk"][i], raw["x_next"][i].T)
    assert bench._histories({"hist": h}) is h       # idempotent

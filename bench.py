#!/usr/bin/env python3
"""Benchmark: MPC steps/s (whole node) at horizon N=20, batch 1e5 scenarios/GPU.

One "step" = one MPC time step (NTM_MPC_Sim.m:94-130: up to i_sim=10 LPV
iterations of lift + cost + getWLc + QP + rollout, then the plant step) for
every scenario of the batch: one launch of the fused HIP kernel through the
C-ABI (ntm_mpc_step_device).  Workload = BASELINE config 3 (B=1e5 scenarios
per GPU, N=20, full getWLc constraints, fp64); per-GPU work is fixed as the
GPU count grows (weak scaling, scenarios sharded by global id, no
communication inside the loop).  The per-step outputs (u_k, x_{k+1}) are
gathered over RCCL at the end of the timed region (the end-of-batch gather).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu]
    torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no WORLD_SIZE in the environment, the script starts the
N ranks itself (torch.distributed.run as a child process, before any GPU
call); under a launcher, WORLD_SIZE must equal --gpus or it exits with 2.

Rank 0 prints ONE JSON line (bench contract).  roofline.achieved uses this
build's own algorithmic flop count (ntm_mpc/flops.py),
driven by the kernel's own solver counters accumulated over exactly the K
timed launches, over the kernel's HIP-event-timed average duration.  A second
leg ("disturbed") runs the same workload with the scenario generator on
(per-step w disturbance sigma_w = 1e-3 m and +-10% j_BS / w_dep plasma
scenarios) and reports its rate and warm-start statistics.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for p in (str(ROOT), str(ROOT / "mpc-ntm-control_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

FP64_PEAK_TFLOPS = 78.6     # MI355X dense fp64 (vector = matrix), spec
HBM_PEAK_GBS = 8000.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=100_000, help="scenarios per GPU")
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mode", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-disturbed", action="store_true", help="skip the disturbed-loop leg")
    ap.add_argument("--sigma-w", type=float, default=1e-3, help="disturbed leg: w disturbance per step [m]")
    ap.add_argument("--spread", type=float, default=0.1, help="disturbed leg: j_BS / w_dep spread over scenarios")
    ap.add_argument("--verify", type=int, default=64, help="scenarios rank 0 recomputes after the gather")
    ap.add_argument("--no-stats", action="store_true",
                    help="A/B only: leave the solver counters off in the timed region (roofline then unavailable)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU sample length")
    ap.add_argument("--small-batch", type=int, default=-1,
                    help="N=20: batches up to this size run on the all-LDS build (-1: library default, 0: never)")
    ap.add_argument("--one-wave-batch", type=int, default=-1,
                    help="N=20: all-LDS batches up to this size use the one-wave register budget "
                         "(-1: library default, 4 x the compute units; 0: never)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL over xGMI) for real runs; gloo only to rehearse the multi-rank "
                         "control flow with more ranks than GPUs (ranks share devices, timing not meaningful)")
    ap.add_argument("--stub-rank", action="store_true",
                    help="test only: each rank joins a gloo group and reports its rank, no GPU work "
                         "(exercises the --gpus launcher on a CPU-only host)")
    return ap.parse_args(argv)


def launch_plan(gpus, env):
    """How this process takes part in a --gpus run (one process per GPU):
    ("here", None) when it is a rank of a launched job (WORLD_SIZE set and equal
    to --gpus) or the only process (--gpus 1); ("spawn", n) when it must start
    n ranks itself; ("error", message) when WORLD_SIZE and --gpus disagree, so a
    launcher mistake never yields a one-GPU line labelled as a scaling point."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "error", f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}"
        return "here", None
    if gpus < 1:
        return "error", f"bench.py: --gpus {gpus}"
    return ("spawn", gpus) if gpus > 1 else ("here", None)


def spawn_ranks(n, argv):
    """Start n ranks of this script under torch.distributed.run (one node,
    rendezvous on 127.0.0.1) as a CHILD process and return its exit code.  The
    caller has made no GPU call (no HIP initialisation in the parent: the
    ranks own the devices); rank 0's JSON line reaches stdout through the
    launcher."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this pool (RCCL)
    return subprocess.run(cmd, env=env).returncode


def stub_rank(world, rank):
    """--stub-rank: the rank's part of the launcher test, on CPU (gloo)."""
    import torch
    import torch.distributed as dist
    per_rank = [rank]
    if world > 1:
        dist.init_process_group("gloo")
        allr = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, torch.tensor([rank], dtype=torch.int64))
        per_rank = [int(t.item()) for t in allr]
    if rank == 0:
        print(json.dumps({"stub": True, "n_gpus": world, "per_rank": {"rank": per_rank}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    """Threads of the CPU leg: the box's CPU share (OMP_NUM_THREADS, which the GPU
    pool sets to 16 per GPU and asks jobs to keep), bounded by this process's
    CPU affinity.  nproc is recorded alongside."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    want = int(os.environ.get("OMP_NUM_THREADS", "0")) or aff
    return max(1, min(want, aff)), aff


def cpu_baseline(N, mode, target_s, warm_steps=5, timed_steps=20):
    """C restatement of the oracle (oracle/ntm_oracle.c, the "port"), OpenMP over
    scenarios on this host, timed on a bounded sample of the same workload and
    the same closed-loop steps as the GPU (steps warm_steps+1 .. warm_steps+
    timed_steps, after warm_steps untimed ones); plus the same on one core and
    the NumPy oracle (single thread, the interpreted stand-in for MATLAB).  The
    port solves every QP cold: Goldfarb-Idnani from the empty set plus the exact
    active-set polish, no carried active sets (the GPU kernel's certified
    warm-start re-solves are its own algorithm)."""
    import numpy as np
    from oracle import cbind
    from oracle import ntm_oracle as O
    import ntm_mpc
    threads, aff = _cpu_threads()
    cfg = O.Config(N=N, mode=mode)

    def steady(B, nthreads, steps):
        x = ntm_mpc.scenarios_x0(0, B)
        x = np.ascontiguousarray(x)
        rho, uo = cbind.initial_state_gen(x, cfg)
        for _ in range(warm_steps):                       # untimed: steps 1..warm_steps
            r = cbind.step(x, rho, uo, cfg, nthreads=nthreads)
            x, rho, uo = r["x_next"], r["rho"], r["U_old"]
        t = time.perf_counter()
        for _ in range(steps):
            r = cbind.step(x, rho, uo, cfg, nthreads=nthreads)
            x, rho, uo = r["x_next"], r["rho"], r["U_old"]
        return time.perf_counter() - t

    steady(threads, threads, 1)                               # load the library, start the thread pool
    B = 64 * threads
    dt = steady(B, threads, 2)
    B2 = int(min(400_000, max(B, B * 2 * target_s / (timed_steps * max(dt, 1e-3)))))
    dt = steady(B2, threads, timed_steps)
    b1 = 8
    d1 = steady(b1, 1, 2)
    b1 = int(min(20_000, max(b1, b1 * 2 * 3.0 / (timed_steps * max(d1, 1e-3)))))   # ~3 s on one core
    d1 = steady(b1, 1, timed_steps)
    ph, nb = O.Physics(), 30
    t = time.perf_counter()
    for s in range(nb):                                         # NumPy oracle, one step each
        x = ntm_mpc.scenarios_x0(s, 1)[:, 0]
        O.mpc_step(x, O.initial_rho(x, ph, cfg), np.full(N, np.inf), ph, cfg)
    dpy = time.perf_counter() - t
    return {"value": B2 * timed_steps / dt, "unit": "MPC steps/s", "cores": threads, "kind": "port",
            "sample": f"{B2} scenarios (ids 0..{B2 - 1}) x closed-loop steps {warm_steps + 1}-"
                      f"{warm_steps + timed_steps} (after {warm_steps} untimed), N={N}, mode={mode}, "
                      f"{threads} OpenMP threads, {dt:.1f} s",
            "solver": "C port of the oracle: cold Goldfarb-Idnani per QP + exact active-set polish, "
                      "no carried active sets",
            "one_core_value": b1 * timed_steps / d1,
            "one_core_sample": f"{b1} scenarios x steps {warm_steps + 1}-{warm_steps + timed_steps}, 1 thread, "
                               f"{d1:.1f} s",
            "interpreted_numpy_value": nb / dpy,
            "interpreted_sample": f"NumPy oracle, {nb} scenarios x 1 step (cold), 1 thread, {dpy:.1f} s",
            "host": {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": _cpu_model(),
                     "note": "threads = the GPU pool's per-GPU CPU share (OMP_NUM_THREADS), not every core "
                             "of the shared host: the pool asks jobs to keep to it"}}


def _workload(N, mode, B):
    kind = {0: "unconstrained LQ", 1: "box-constrained u", 2: "full getWLc constraints",
            3: "full getWLc + input-rate rows"}[mode]
    cfgs = {(20, 2, 100_000): "BASELINE config 3", (20, 1, 1024): "BASELINE config 2",
            (50, 3, 100_000): "BASELINE config 5 (rate rows)", (50, 2, 100_000): "BASELINE config 5 shape (N=50)",
            (10, 0, 1): "BASELINE config 1"}
    tag = cfgs.get((N, mode, B), "custom")
    return f"{tag}: LPV-MPC closed-loop step, N={N}, {kind}, B={B} per GPU, fp64"


def _run_leg(ctl, cfg, B, K, W, x0, rank, world, gen=None, collect=False, stats_on=True):
    """W untimed warmup steps then K timed steps of the closed loop through the
    step entry point, the solver counters accumulated over exactly the K timed
    launches.  Returns timing, per-step counters and (collect) the histories."""
    import torch
    import torch.distributed as dist
    from ntm_mpc.api import STATS_ROWS
    dev = f"cuda:{ctl.device}"
    ctl.set_scenarios(gen)
    x = x0
    rho, U_old = ctl.initial_state(x, cfg)
    active_ws = ctl.new_active_ws(B, cfg)       # last two active sets, carried step to step
    outs = [None, None]

    def one_step(i, xin):
        if gen is not None:
            gen.k0 = i                          # the plant step's time index
            ctl.set_scenarios(gen)
        out = ctl.step(xin, rho, U_old, cfg, out=outs[i & 1], active_ws=active_ws)
        outs[i & 1] = out
        return out

    for i in range(W):
        x = one_step(i, x)["x_next"].clone()
    N = cfg.N
    hist = raw = None
    if collect:
        # The closed-loop record (NTM_MPC_Sim.m:106-131 keeps uk, Uk, xk per step): each
        # timed step's kernel writes its outputs straight into their slot of the record,
        # scenario-major as the ABI wants (no copy kernels between steps; uk and wpred
        # are views of the stored U and x_pred, extracted after the timed region)
        raw = {"U": torch.empty(K, B, N, dtype=torch.float64, device=dev),
               "x_pred": torch.empty(K, B, 2 * (N + 1), dtype=torch.float64, device=dev),
               "x_next": torch.empty(K + 1, B, 2, dtype=torch.float64, device=dev),
               "exitflag": torch.empty(K, B, dtype=torch.int32, device=dev),
               "inner_iters": torch.empty(K, B, dtype=torch.int32, device=dev)}
        raw["x_next"][0].copy_(x.T)
        x = raw["x_next"][0].T
    stats = torch.zeros(STATS_ROWS, B, dtype=torch.int32, device=dev)
    ctl.set_stats(stats if stats_on else None)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    xin = x
    for i in range(K):
        if collect:
            outs[(W + i) & 1] = {"U": raw["U"][i].T, "x_pred": raw["x_pred"][i].T, "x_next": raw["x_next"][i + 1].T,
                                 "exitflag": raw["exitflag"][i], "inner_iters": raw["inner_iters"][i]}
        ev[i][0].record()
        out = one_step(W + i, xin)
        ev[i][1].record()
        xin = out["x_next"]
    if collect:
        hist = {"raw": raw}
    return {"t0": t0, "ev": ev, "stats": stats, "out": out, "hist": hist}


def _histories(leg):
    """The step kernels' (K, B, E) records as the (..., B) histories uk, Uk, xk, wpred,
    exitflag, inner_iters (the gather's and the report's layout); idempotent."""
    h = leg["hist"]
    if h is not None and "raw" in h:
        raw = h.pop("raw")
        h.update({"uk": raw["U"][:, :, 0].contiguous(), "Uk": raw["U"].permute(0, 2, 1).contiguous(),
                  "xk": raw["x_next"].permute(0, 2, 1).contiguous(),
                  "wpred": raw["x_pred"][:, :, 0::2].permute(0, 2, 1).contiguous(),
                  "exitflag": raw["exitflag"], "inner_iters": raw["inner_iters"]})
    return h


def _finish_leg(ctl, leg, K):
    import torch
    torch.cuda.synchronize()
    _histories(leg)
    ctl.set_stats(None)
    ctl.set_scenarios(None)
    kern_ms = sum(a.elapsed_time(b) for a, b in leg["ev"]) / K
    B = leg["stats"].shape[1]
    st = leg["stats"].double().sum(dim=1).cpu().numpy() / (B * K)          # per MPC step
    flags = leg["out"]["exitflag"]
    return {"kern_ms": kern_ms, "qps": st[0], "Kgi": st[1], "tries": st[4], "giruns": st[5],
            "qact": st[2] / st[0], "sgen": st[3] / st[0],
            "optimal_frac": float((flags == 1).double().mean().item()),
            "inner_iters_mean": float(leg["out"]["inner_iters"].double().mean().item())}


def _verify_gathered(ctl, cfg, B_total, K, W, g, n_verify, seed=12345):
    """Rank 0: recompute a seeded sample of the gathered scenarios from their
    global ids alone (one process, one GPU) and require bit-identical histories."""
    import numpy as np
    import torch
    import ntm_mpc
    rng = np.random.default_rng(seed)
    ids = np.sort(rng.choice(B_total, size=min(n_verify, B_total), replace=False))
    x0 = np.concatenate([ntm_mpc.scenarios_x0(int(i), 1) for i in ids], axis=1)
    x = ctl.tensor(x0)
    n = len(ids)
    # the context is pinned to the build the whole batch takes on one GPU
    # (dist.pin_layout in main), so the recompute runs the build the ranks ran
    leg = _run_leg(ctl, cfg, n, K, W, x, 0, 1, collect=True)
    _finish_leg(ctl, leg, K)
    sel = torch.as_tensor(ids, device=leg["hist"]["uk"].device)
    bad = [k for k, v in leg["hist"].items() if not bool((v == g[k].index_select(-1, sel)).all().item())]
    return {"scenarios": n, "ids_seed": seed, "bitwise_equal": not bad, "mismatched": bad}


def main():
    args = parse()
    # --gpus N: the driver launches N ranks itself (torch.distributed.run, WORLD_SIZE
    # set); a bare `python bench.py --gpus N` starts them here, before any GPU call
    plan, arg = launch_plan(args.gpus, os.environ)
    if plan == "error":
        print(arg, file=sys.stderr, flush=True)
        return 2
    if plan == "spawn":
        return spawn_ranks(arg, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub_rank:
        stub_rank(world, rank)
        return 0
    import torch
    import torch.distributed as dist

    rehearsal = args.dist_backend == "gloo"
    if rehearsal:                       # ranks fold onto the available devices
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

    import ntm_mpc
    from ntm_mpc import Config, NtmMpc, ScenarioGen
    from ntm_mpc import flops as FL
    from ntm_mpc.dist import gather_to_root, pin_layout

    B, N, K, W = args.batch, args.N, args.steps, args.warmup
    cfg = Config(N=N, mode=args.mode)
    ctl = NtmMpc(config=cfg, device=local)
    if args.small_batch < 0:
        # every rank, and rank 0's recompute, on the build one GPU takes for the whole batch
        pin_layout(ctl, world * B, cfg)
    else:
        ctl.set_small_batch(args.small_batch)
    ctl.set_one_wave_batch(args.one_wave_batch)
    # shard: global scenario ids [rank*B, (rank+1)*B)  (shard-invariant inputs)
    x0 = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(rank * B, B), local)

    leg = _run_leg(ctl, cfg, B, K, W, x0, rank, world, collect=True, stats_on=not args.no_stats)
    # end-of-batch gather of every per-scenario output history into rank 0 (RCCL
    # point-to-point over xGMI; gloo rehearsal through host memory), scenario
    # order = global id order
    g = None
    if world > 1:
        tot = world * B
        g = {k: gather_to_root(v.cpu() if rehearsal else v, tot) for k, v in _histories(leg).items()}
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - leg["t0"]
    r = _finish_leg(ctl, leg, K)
    # per-rank timings: each rank's own wall time of the K steps and
    # its HIP-event kernel average, so a scaling run shows which rank set the max
    per_rank = {"elapsed_s": [elapsed], "kernel_avg_ms": [r["kern_ms"]]}
    if world > 1:
        tdev = "cpu" if rehearsal else f"cuda:{local}"
        mine = torch.tensor([elapsed, r["kern_ms"]], dtype=torch.float64, device=tdev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = {"elapsed_s": [float(t[0].item()) for t in allr],
                    "kernel_avg_ms": [float(t[1].item()) for t in allr]}
        elapsed = max(per_rank["elapsed_s"])                  # the max over ranks
    if world == 1:
        g = leg["hist"]
    verify = None
    if rank == 0 and args.verify > 0:
        gd = {k: v.to(f"cuda:{local}") for k, v in g.items()}
        verify = _verify_gathered(ctl, cfg, world * B, K, W, gd, args.verify)
        del gd
    del g, leg

    value = world * B * K / elapsed
    flop_step = FL.per_step(N, args.mode, r["qps"], r["tries"], r["giruns"], r["Kgi"], r["qact"], r["sgen"])
    achieved = flop_step * B / (r["kern_ms"] * 1e-3) / 1e12
    traffic, traffic_source = None, None
    # PMC-measured HBM bytes per launch of this workload (tools/traffic_run.py,
    # separate FETCH_SIZE / WRITE_SIZE passes under rocprofv3, which this run cannot
    # take itself): the latest round's committed file that matches, named in the line
    for prof in sorted((ROOT / "profiles").glob("traffic_r*.json"), reverse=True):
        try:
            tj = json.loads(prof.read_text())
        except Exception:
            continue
        if tj.get("B") == B and tj.get("N") == N and tj.get("mode", 2) == args.mode:
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_source = {"file": str(prof.relative_to(ROOT)), "round": prof.stem.split("_r")[-1],
                              "measured_in_this_run": False,
                              "build": tj.get("build") or tj.get("commit"),
                              "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the same workload "
                                      "(tools/traffic_run.py), not this process"}
            break
    res = {
        "metric": "MPC steps/sec (whole node) at horizon N=20, batch=1e5 scenarios",
        "value": value,
        "unit": "MPC steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: counter-based x0 (w0~U[0.07,0.14] m, omega0~U[0.8,1.2]*2000pi), nominal physics "
                "NTM_MPC_Sim.m:5-60, closed loop advanced step to step",
        "config": {"workload": _workload(N, args.mode, B),
                   "scenarios_per_gpu": B, "global_batch": world * B, "N": N, "mode": args.mode, "i_sim": 10,
                   "timed_closed_loop_steps": f"{W + 1}-{W + K}",
                   "parallelism": f"scenario-sharded x{world} (weak), end-of-batch gather into rank 0 of uk, Uk, xk, "
                                  "wpred, exitflag, inner_iters"
                       + (" [gloo rehearsal: ranks share devices]" if rehearsal and world > 1 else "")},
        "roofline": {"bound": "valu-fp64", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_source,
                     "kernel": ctl.step_kernel_name(B, cfg), "kernel_avg_ms": r["kern_ms"],
                     "flop_per_step": flop_step,
                     "flop_counters": "solver counters of the K timed launches (ntm_ctx_set_stats on in the "
                                      "timed region)",
                     "hbm_algorithmic_bytes_per_launch": FL.hbm_bytes_per_step(N, workspace=True) * B,
                     "note": ("fp64 VALU work (DPP/LDS, no MFMA at this horizon: DESIGN.md §6)" if N <= 32 else
                              "fp64 VALU work plus GI's full Gram on V_MFMA_F64_16X16X4F64 (gram_mfma, DESIGN.md §6)")
                             + "; peak = MI355X fp64 vector rate (78.6 TF, equal to the fp64 matrix rate)"},
        "solver": {"inner_iters_mean": r["inner_iters_mean"], "qp_per_step": r["qps"],
                   "warm_verify_per_step": r["tries"], "gi_solves_per_step": r["giruns"],
                   "gi_iters_per_step": r["Kgi"], "active_rows_per_qp": r["qact"], "state_rows_per_qp": r["sgen"],
                   "warm_hit_rate": 1.0 - r["giruns"] / r["qps"], "optimal_frac": r["optimal_frac"]},
        "gather_verify": verify,
        "per_rank": {**per_rank, "kernel_avg_ms_max": max(per_rank["kernel_avg_ms"]),
                     "note": "elapsed_s: each rank's wall time of the K timed steps (barrier + synchronize "
                             "bracketed, gather included); value uses their max"},
    }
    if not args.no_disturbed:
        gen = ScenarioGen(seed=20241220, first_id=rank * B, k0=0, sigma_w=args.sigma_w, sigma_omega=0.0,
                          jbs_spread=args.spread, wdep_spread=args.spread)
        dl = _run_leg(ctl, cfg, B, K, W, x0, rank, world, gen=gen)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        d_el = time.perf_counter() - dl["t0"]
        d = _finish_leg(ctl, dl, K)
        res["disturbed"] = {
            "value": world * B * K / d_el, "ms_per_step": d_el / K * 1e3, "kernel_avg_ms": d["kern_ms"],
            "generator": {"sigma_w_m": args.sigma_w, "jbs_spread": args.spread, "wdep_spread": args.spread,
                          "seed": 20241220, "disturbance": "Irwin-Hall(4) unit variance x sigma_w per plant step"},
            "inner_iters_mean": d["inner_iters_mean"], "qp_per_step": d["qps"], "warm_verify_per_step": d["tries"],
            "gi_solves_per_step": d["giruns"], "gi_iters_per_step": d["Kgi"],
            "warm_hit_rate": 1.0 - d["giruns"] / d["qps"], "optimal_frac": d["optimal_frac"],
            "flop_per_step": FL.per_step(N, args.mode, d["qps"], d["tries"], d["giruns"], d["Kgi"], d["qact"],
                                         d["sgen"])}
    if rank == 0 and not args.no_cpu:
        try:
            res["cpu_baseline"] = cpu_baseline(N, args.mode, args.cpu_seconds)
        except Exception as e:  # pragma: no cover
            res["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctl.close()
    if world > 1:
        dist.barrier()                  # rank 0 may still be timing the CPU baseline
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

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

Rank 0 prints ONE JSON line (bench contract).  roofline.achieved uses this
build's own algorithmic flop count (ntm_mpc/flops.py)
over the kernel's HIP-event-timed average duration.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=100_000, help="scenarios per GPU")
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mode", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU sample length")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL over xGMI) for real runs; gloo only to rehearse the multi-rank "
                         "control flow with more ranks than GPUs (ranks share devices, timing not meaningful)")
    return ap.parse_args()


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(N, mode, target_s):
    """C restatement of the oracle (oracle/ntm_oracle.c, the "port"), OpenMP over
    scenarios on this host, timed on a bounded sample of the same workload; plus
    the same on one core and the NumPy oracle (single thread, the interpreted
    stand-in for MATLAB) on a few scenarios (BASELINE.md CPU-baseline plan)."""
    import numpy as np
    from oracle import cbind
    from oracle import ntm_oracle as O
    import ntm_mpc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    threads = max(1, min(threads, os.cpu_count() or 1))
    cfg = O.Config(N=N, mode=mode)
    k = 2

    def timed(B, nthreads):
        x0 = ntm_mpc.scenarios_x0(0, B)
        t = time.perf_counter()
        cbind.run(x0, cfg, k, nthreads=nthreads)
        return time.perf_counter() - t

    B = 64 * threads
    dt = timed(B, threads)
    B2 = int(min(400_000, max(B, B * target_s / max(dt, 1e-3))))
    dt = timed(B2, threads)
    b1 = 64
    d1 = timed(b1, 1)
    b1 = int(min(20_000, max(b1, b1 * 3.0 / max(d1, 1e-3))))   # ~3 s on one core
    d1 = timed(b1, 1)
    ph, nb = O.Physics(), 30
    t = time.perf_counter()
    for s in range(nb):                                         # NumPy oracle, one step each
        x = ntm_mpc.scenarios_x0(s, 1)[:, 0]
        O.mpc_step(x, O.initial_rho(x, ph, cfg), np.full(N, np.inf), ph, cfg)
    dpy = time.perf_counter() - t
    return {"value": B2 * k / dt, "unit": "MPC steps/s", "cores": threads, "kind": "port",
            "sample": f"{B2} scenarios x {k} closed-loop steps (ids 0..{B2 - 1}), N={N}, mode={mode}, "
                      f"{threads} OpenMP threads, {dt:.1f} s",
            "one_core_value": b1 * k / d1, "one_core_sample": f"{b1} scenarios x {k} steps, 1 thread, {d1:.1f} s",
            "interpreted_numpy_value": nb / dpy,
            "interpreted_sample": f"NumPy oracle, {nb} scenarios x 1 step, 1 thread, {dpy:.1f} s",
            "host": {"nproc": os.cpu_count(), "cpu_model": _cpu_model()}}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
    from ntm_mpc import Config, NtmMpc
    from ntm_mpc import flops as FL
    from ntm_mpc.api import STATS_ROWS

    B, N, K, W = args.batch, args.N, args.steps, args.warmup
    cfg = Config(N=N, mode=args.mode)
    ctl = NtmMpc(config=cfg, device=local)
    dev = f"cuda:{local}"
    # shard: global scenario ids [rank*B, (rank+1)*B)  (shard-invariant inputs)
    x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(rank * B, B), local)
    rho, U_old = ctl.initial_state(x, cfg)
    active_ws = ctl.new_active_ws(B, cfg)       # last two active sets, carried step to step
    outs = [None, None]

    def one_step(i, xin):
        out = ctl.step(xin, rho, U_old, cfg, out=outs[i & 1], active_ws=active_ws)
        outs[i & 1] = out
        return out

    # warmup (untimed): also advances the closed loop
    for i in range(W):
        x = one_step(i, x)["x_next"].clone()
    # instrumentation pass (untimed, separate launch on a copy of the state)
    stats = torch.zeros(STATS_ROWS, B, dtype=torch.int32, device=dev)
    rho_s, uo_s, ws_s = rho.clone(), U_old.clone(), active_ws.clone()
    ctl.set_stats(stats)
    ctl.step(x, rho_s, uo_s, cfg, active_ws=ws_s)
    ctl.set_stats(None)
    torch.cuda.synchronize()
    st = stats.double().sum(dim=1).cpu().numpy()
    qps, Kgi, tries, giruns = st[0] / B, st[1] / B, st[4] / B, st[5] / B     # per MPC step
    qact, sgen = st[2] / st[0], st[3] / st[0]                                 # per QP
    del rho_s, uo_s, ws_s

    hist_u = torch.empty(K, B, dtype=torch.float64, device=dev)
    hist_x = torch.empty(K, 2, B, dtype=torch.float64, device=dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    xin = x
    for i in range(K):
        ev[i][0].record()
        out = one_step(W + i, xin)
        ev[i][1].record()
        hist_u[i].copy_(out["U"][0])
        hist_x[i].copy_(out["x_next"])
        xin = out["x_next"]
    # end-of-batch gather of the control sequence and trajectory (RCCL over xGMI)
    if world > 1 and not rehearsal:
        g_u = torch.empty(world * K * B, dtype=torch.float64, device=dev)
        g_x = torch.empty(world * K * 2 * B, dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(g_u, hist_u.reshape(-1))
        dist.all_gather_into_tensor(g_x, hist_x.reshape(-1))
    elif world > 1:                     # gloo rehearsal: same exchange through host memory
        g_u = [torch.empty(K * B, dtype=torch.float64) for _ in range(world)]
        g_x = [torch.empty(K * 2 * B, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(g_u, hist_u.reshape(-1).cpu())
        dist.all_gather(g_x, hist_x.reshape(-1).cpu())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearsal else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / K
    flags = out["exitflag"]
    n_opt = int((flags == 1).sum().item())
    iters = out["inner_iters"].double().mean().item()

    value = world * B * K / elapsed
    flop_step = FL.per_step(N, args.mode, qps, tries, giruns, Kgi, qact, sgen)
    achieved = flop_step * B / (kern_ms * 1e-3) / 1e12
    traffic = None
    # PMC-measured HBM bytes per launch of this workload (tools/traffic_run.py,
    # separate FETCH_SIZE / WRITE_SIZE passes): the latest round's file that matches
    for prof in sorted((ROOT / "profiles").glob("traffic_r*.json"), reverse=True):
        try:
            tj = json.loads(prof.read_text())
        except Exception:
            continue
        if tj.get("B") == B and tj.get("N") == N and tj.get("mode", 2) == args.mode:
            traffic = tj.get("hbm_bytes_per_launch")
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
        "config": {"workload": "BASELINE config 3: LPV-MPC closed-loop step, full getWLc constraints, fp64",
                   "scenarios_per_gpu": B, "global_batch": world * B, "N": N, "mode": args.mode, "i_sim": 10,
                   "parallelism": f"scenario-sharded x{world} (weak), end-of-batch all_gather"
                       + (" [gloo rehearsal: ranks share devices]" if rehearsal and world > 1 else "")},
        "roofline": {"bound": "valu-fp64", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "kernel": ctl.step_kernel_name(B, cfg), "kernel_avg_ms": kern_ms,
                     "flop_per_step": flop_step,
                     "hbm_algorithmic_bytes_per_launch": FL.hbm_bytes_per_step(N, workspace=True) * B,
                     "note": "fp64 VALU work (DPP/LDS, no MFMA: DESIGN.md §6); peak = MI355X fp64 vector rate "
                             "(78.6 TF, equal to the fp64 matrix rate)"},
        "solver": {"inner_iters_mean": iters, "qp_per_step": qps, "warm_verify_per_step": tries,
                   "gi_solves_per_step": giruns, "gi_iters_per_step": Kgi,
                   "active_rows_per_qp": qact, "state_rows_per_qp": sgen, "optimal_frac": n_opt / B},
    }
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


if __name__ == "__main__":
    main()

"""Diagnostic (not a test): config 2's step latency against its slowest scenario.

At B = 1024 every scenario has a SIMD of its own, so a step-batch lasts as long
as its slowest wave.  Per closed-loop step this prints the distribution of the
LPV iteration counts (inner_iters) and the step's HIP-event time, and then the
time of a batch made only of the slowest scenario repeated (the chain's latency
for one scenario) and of the median one.

    python tools/c2_tail.py [B] [mode] [warm steps] [measured steps]
"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "mpc-ntm-control_amd")]
import numpy as np, torch, ntm_mpc
from ntm_mpc import NtmMpc, Config

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
cfg = Config(N=20, mode=int(sys.argv[2]) if len(sys.argv) > 2 else 1)
WARM = int(sys.argv[3]) if len(sys.argv) > 3 else 5
K = int(sys.argv[4]) if len(sys.argv) > 4 else 20
ctl = NtmMpc(config=cfg)
print("kernel:", ctl.step_kernel_name(B, cfg))


def timed_step(x, rho, uo, ws):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    out = ctl.step(x, rho, uo, cfg, active_ws=ws)
    e.record()
    torch.cuda.synchronize()
    return out, s.elapsed_time(e)


x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(0, B))
rho, uo = ctl.initial_state(x, cfg)
ws = ctl.new_active_ws(B, cfg)
snaps = []
for k in range(WARM + K):
    if k >= WARM:
        snaps.append((x.clone(), rho.clone(), uo.clone(), ws.clone()))
    out, ms = timed_step(x, rho, uo, ws)
    it = out["inner_iters"].cpu().numpy()
    if k >= WARM:
        h = np.bincount(it, minlength=11)
        print(f"step {k + 1:3d}: {ms:.4f} ms  iters mean {it.mean():.2f} max {it.max()}  hist {h[1:].tolist()}")
    x = out["x_next"].clone()

# replay step WARM+1 with the batch made of one scenario repeated
x0, r0, u0, w0 = snaps[0]
out, ms = timed_step(x0.clone(), r0.clone(), u0.clone(), w0.clone())
it = out["inner_iters"].cpu().numpy()
order = np.argsort(it, kind="stable")
for name, s in (("slowest", int(order[-1])), ("median", int(order[len(order) // 2])), ("fastest", int(order[0]))):
    idx = torch.full((B,), s, dtype=torch.long, device=x0.device)
    xs, rs, us, wsr = (t.T[idx].contiguous().T for t in (x0, r0, u0, w0))   # keep the ABI layout
    times = []
    for _ in range(5):
        _, ms = timed_step(xs.clone(), rs.clone(), us.clone(), wsr.clone())
        times.append(ms)
    print(f"batch of the {name} scenario ({s}, {it[s]} iterations) x {B}: {min(times):.4f} ms")

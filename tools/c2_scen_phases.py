"""Diagnostic (not a test): the phase stamps of ONE scenario's step (a batch of
that scenario repeated), on the -DNTM_STAMPS build, for scenarios picked by
their step time (tools/c2_tail.py found config 2 scenarios with the same
iteration count running 0.11 to 0.18 ms).

    NTM_MPC_LIB=.../libntm_mpc_diag.so python tools/c2_scen_phases.py [B] [mode] [warm steps] [scenarios...]
"""
import ctypes as C, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "mpc-ntm-control_amd")]
import numpy as np, torch, ntm_mpc
from ntm_mpc import NtmMpc, Config

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
cfg = Config(N=20, mode=int(sys.argv[2]) if len(sys.argv) > 2 else 1)
WARM = int(sys.argv[3]) if len(sys.argv) > 3 else 5
picks = [int(s) for s in sys.argv[4:]] or [1023, 386]
ctl = NtmMpc(config=cfg)
lib = ntm_mpc.load()
buf = (C.c_ulonglong * 104)()
x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(0, B))
rho, uo = ctl.initial_state(x, cfg)
ws = ctl.new_active_ws(B, cfg)
for _ in range(WARM):
    out = ctl.step(x, rho, uo, cfg, active_ws=ws)
    torch.cuda.synchronize()
    x = out["x_next"].clone()
major = "lift cost scale cand regram gi polish roll".split()
fine = "k_y k_chk k_grad k_mu k_sub c_a c_b c_y c_sq sc_col sc_row sc_end l_coef l_loop".split()
rows = {}
for s in picks:
    idx = torch.full((B,), s, dtype=torch.long, device=x.device)
    xs, rs, us, wsr = (t.T[idx].contiguous().T for t in (x, rho, uo, ws))
    lib.ntm_debug_stamps(buf, 1)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    out = ctl.step(xs, rs, us, cfg, active_ws=wsr)
    ev1.record()
    torch.cuda.synchronize()
    assert lib.ntm_debug_stamps(buf, 1) == 0
    it = int(out["inner_iters"][0].item())
    v = {n: buf[i] / B for i, n in enumerate(major)}
    v.update({n: buf[46 + i] / B for i, n in enumerate(fine)})
    v.update({"p_gram": buf[16 + 1] / B, "p_bwd": buf[16 + 4] / B, "p_kkt": buf[16 + 5] / B,
              "s_E+h": buf[24] / B, "s_Y": buf[25] / B, "s_cholK": buf[27] / B, "s_solve": buf[28] / B,
              "sets": buf[14] / B, "drops": buf[67] / B, "iters": it, "us": 1e3 * ev0.elapsed_time(ev1)})
    rows[s] = v
names = list(next(iter(rows.values())).keys())
print(f"B={B} mode {cfg.mode} step {WARM + 1}: cycles per wave-step by phase, batch of one scenario repeated")
print("phase      " + "".join(f"{s:>12d}" for s in picks))
for n in names:
    print(f"{n:10s} " + "".join(f"{rows[s][n]:12.0f}" if rows[s][n] >= 10 else f"{rows[s][n]:12.2f}" for s in picks))
print("total      " + "".join(f"{sum(rows[s][n] for n in major):12.0f}" for s in picks))

"""Workload for the HBM-traffic PMC passes (tools/prof_r01.sh): the bench's
steady state -- three warm steps of the closed loop with the carried
warm-start workspace, then one measured k_mpc_step dispatch at B scenarios
(N=20, full getWLc constraints) -- and a calibration copy of a known byte count
(512 MiB read + 512 MiB written, above the 256 MiB Infinity Cache) so the
FETCH_SIZE / WRITE_SIZE units can be checked against bytes in the same run."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]
import torch  # noqa: E402

import ntm_mpc  # noqa: E402
from ntm_mpc import Config, NtmMpc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
cfg = Config(N=20, mode=2)
ctl = NtmMpc(config=cfg)
x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(0, B))
rho, uo = ctl.initial_state(x, cfg)
ws = ctl.new_active_ws(B, cfg)
for _ in range(3):                                    # warm steps (advance the loop, fill the workspace)
    out = ctl.step(x, rho, uo, cfg, active_ws=ws)
    x = out["x_next"].clone()
torch.cuda.synchronize()
out = ctl.step(x, rho, uo, cfg, active_ws=ws)         # measured dispatch
torch.cuda.synchronize()
src = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
dst = torch.empty_like(src)
dst.copy_(src)                                        # calibration: 512 MiB in, 512 MiB out
torch.cuda.synchronize()
print("ok", B)

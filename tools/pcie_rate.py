"""PCIe-inclusive rate of the host-buffer boundary (ntm_mpc_step with host
arrays, what a MEX gateway calls): H2D of x_k/rho/U_old, the step kernel, D2H
of every output, per call.  Reported in DESIGN.md next to the device-resident
bench value; never the bench `value`."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ntm_mpc  # noqa: E402
from ntm_mpc import Config, NtmMpc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = Config(N=20, mode=2)
ctl = NtmMpc(config=cfg)
x = ntm_mpc.scenarios_x0(0, B)                         # (2, B) in the ABI layout: no staging copies
rho, uo = ctl.initial_state_host(x, cfg)
out = ctl.step_host(x, rho, uo, cfg)                   # warmup
x = out["x_next"]
t = time.perf_counter()
for _ in range(K):
    out = ctl.step_host(x, rho, uo, cfg)
    x = out["x_next"]
dt = (time.perf_counter() - t) / K
bytes_moved = B * 8 * (2 + 2 * 3 * 20 + 2 * 20 + 20 + 2 * 21 + 2) + B * 8
print(json.dumps({"B": B, "steps": K, "ms_per_step": dt * 1e3, "steps_per_s": B / dt,
                  "pcie_bytes_per_step": bytes_moved}))

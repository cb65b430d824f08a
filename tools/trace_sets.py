"""Diagnostic: the warm-start candidate and final active sets of one traced
scenario (the trace build, make -C mpc-ntm-control_amd trace NTM_DEBUG_SCEN=0),
over K closed-loop steps with the carried workspace, written as lines
"SET it <it> cand|final <q>: ids" on stdout (device printf).

    python tools/trace_sets.py N mode K > gpurun_out/trace_sets.log
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("NTM_MPC_LIB", os.path.join(ROOT, "mpc-ntm-control_amd", "lib", "libntm_mpc_trace.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-ntm-control_amd")]
import torch  # noqa: E402

import ntm_mpc  # noqa: E402
from ntm_mpc import Config, NtmMpc  # noqa: E402

N, mode, K = (int(a) for a in sys.argv[1:4])
B = 8
ctl = NtmMpc()
cfg = Config(N=N, mode=mode)
x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(0, B))
rho, uo = ctl.initial_state(x, cfg)
ws = ctl.new_active_ws(B, cfg)
for k in range(K):
    print(f"STEP {k}", flush=True)
    out = ctl.step(x, rho, uo, cfg, active_ws=ws)
    torch.cuda.synchronize()
    sys.stdout.flush()
    x = out["x_next"].clone()

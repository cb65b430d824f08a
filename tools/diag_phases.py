"""Diagnostic (not a test): per-phase cycle breakdown of the fused step kernel
using the -DNTM_STAMPS build (lib/libntm_mpc_diag.so).

    python tools/diag_phases.py [B] [N] [mode] [warm steps] [measured steps]
"""
import ctypes as C, os, sys, time
os.environ.setdefault("NTM_MPC_LIB", os.path.join(os.path.dirname(__file__), "..", "mpc-ntm-control_amd", "lib", "libntm_mpc_diag.so"))
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "mpc-ntm-control_amd")]
import torch, ntm_mpc
from ntm_mpc import NtmMpc, Config
B = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = Config(N=N, mode=int(sys.argv[3]) if len(sys.argv) > 3 else 2)
ctl = NtmMpc(config=cfg)
lib = ntm_mpc.load()
buf = (C.c_ulonglong * 104)()
x = ntm_mpc.device_tensor(ntm_mpc.scenarios_x0(0, B))
rho, uo = ctl.initial_state(x, cfg)
ws = ctl.new_active_ws(B, cfg)
WARM = int(sys.argv[4]) if len(sys.argv) > 4 else 6   # steps before the measured one (bench: 5 warmup)
for _ in range(WARM):
    out = ctl.step(x, rho, uo, cfg, active_ws=ws); torch.cuda.synchronize()
    x = out["x_next"].clone()
K = int(sys.argv[5]) if len(sys.argv) > 5 else 1      # measured steps (bench: 20, steps 6-25)
lib.ntm_debug_stamps(buf, 1)
t = time.time()
for _ in range(K):
    out = ctl.step(x, rho, uo, cfg, active_ws=ws); torch.cuda.synchronize()
    x = out["x_next"].clone()
dt = (time.time() - t) / K
assert lib.ntm_debug_stamps(buf, 1) == 0
B = B * K                                               # every figure below is per wave-step
names = "lift cost scale cand regram gi polish roll gi_fact gi_check gi_dir gi_add gi_drop".split()
tot = sum(buf[i] for i in range(8))
print(f"B={B // K} N={N} steps {WARM + 1}-{WARM + K} {dt*1e3:.1f} ms; cycles per wave-step by phase (s_memtime):")
for i, n in enumerate(names):
    print(f"  {n:9s} {buf[i]/B:12.0f}  {100*buf[i]/tot:5.1f}%")
print(f"per wave-step: check calls {buf[13]/B:.1f}, candidate sets {buf[14]/B:.2f}, hits {buf[15]/B:.2f} (after repair {buf[22]/B:.2f}), GI solves {buf[23]/B:.2f}")
sub = "p_class p_gram p_chol p_schur p_bwd p_kkt".split()
print("certified re-solve (cand + polish) sub-phases, cycles per wave-step:")
for i, n in enumerate(sub):
    print(f"  {n:9s} {buf[16 + i]/B:12.0f}")
print(f"  first tries at it<=2: {buf[29]/B:.2f}, failed {buf[30]/B:.2f}; failed at it>2: {buf[31]/B:.2f}")
sch = "s_E+h s_Y s_K s_cholK s_solve".split()
print("  Schur part:")
for i, n in enumerate(sch):
    print(f"    {n:9s} {buf[24 + i]/B:12.0f}")
print(f"per wave-step: tries it=1 {buf[37]/B:.2f} failed {buf[32]/B:.2f}; tries it=2 {buf[38]/B:.2f} failed {buf[33]/B:.2f}; "
      f"GI solves at it=1 {buf[34]/B:.2f}, it=2 {buf[35]/B:.2f}, later {buf[36]/B:.2f}")
print(f"per wave-step: GI warm starts tried {buf[39]/B:.2f}, accepted {buf[40]/B:.2f}; "
      f"warm-start adds {buf[66]/B:.0f} cycles (inside gi, apart from gi_check)")
print(f"  dependent rows skipped {buf[41]/B:.3f}; rejected: negative multiplier {buf[42]/B:.3f}; stopped at N rows {buf[43]/B:.3f}")
print(f"per wave-step: the other form (shifted or unshifted) of the carried set at it=2 tried {buf[44]/B:.2f}, hits {buf[45]/B:.2f}")
fine = "k_y k_chk k_grad k_mu k_sub c_a c_b c_y c_sq sc_col sc_row sc_end l_coef l_loop".split()
print("certificate / classification detail, cycles per wave-step:")
for i, n in enumerate(fine):
    print(f"  {n:9s} {buf[46 + i]/B:12.0f}")
print(f"exact 2-cycle study: steps whose rho and U after iteration it equal those after it-2 (it >= 3): "
      f"{buf[60]/B:.4f} per wave-step; iterations a shortcut could skip {buf[61]/B:.4f} per wave-step")
print(f"certified dual path per wave-step: negative-multiplier drops {buf[67]/B:.3f}, A+p re-solves {buf[68]/B:.3f}, "
      f"partial steps {buf[69]/B:.3f}, dual-only directions {buf[70]/B:.3f}, handed to GI {buf[71]/B:.3f}")
print(f"  handed to GI because: candidate singular {buf[72]/B:.3f}, singular in the dual phase {buf[73]/B:.3f}, budget {buf[74]/B:.3f}, "
      f"direction on a non-echelon set {buf[75]/B:.3f}, no violated row {buf[76]/B:.3f}, dual failure at a full step {buf[77]/B:.3f}, "
      f"no row can leave {buf[78]/B:.3f}, non-finite end-point multiplier {buf[88]/B:.4f}")
print(f"re-solves with non-finite multipliers per wave-step, by path: bordered {buf[89]/B:.4f}, echelon k=0 {buf[90]/B:.4f}, "
      f"k=1 {buf[91]/B:.4f}, k=2 {buf[92]/B:.4f}, one collision {buf[93]/B:.4f}, two collisions {buf[94]/B:.4f}; "
      f"of them primal check failed {buf[95]/B:.4f}, V non-finite {buf[96]/B:.4f}")
print(f"bordered re-solves by shape per wave-step: not classified (nS = 0 or k >= 3) {buf[101]/B:.3f}, "
      f"a row with no free column {buf[100]/B:.3f}, one row left out {buf[97]/B:.3f}, two {buf[98]/B:.3f}, "
      f"three or more {buf[99]/B:.3f}")
print(f"dual path: rows skipped after a non-finite end point {buf[102]/B:.3f} per wave-step, dual-only steps of a skipped row {buf[103]/B:.3f}")
print(f"re-solve paths per wave-step: echelon k=0 {buf[84]/B:.2f}, k=1 {buf[85]/B:.2f}, k=2 {buf[86]/B:.2f}, one collision {buf[87]/B:.2f}; "
      f"bordered with k = nF - nS = 0 {buf[79]/B:.2f}, 1 {buf[80]/B:.2f}, 2 {buf[81]/B:.2f}, 3 {buf[82]/B:.2f}, >= 4 {buf[83]/B:.2f}")
print(f"first tries at it<=2 that failed, by kind, per wave-step: dual {buf[62]/B:.3f}, primal {buf[63]/B:.3f}, "
      f"singular/colliding {buf[64]/B:.3f}, primal and dual {buf[65]/B:.3f}")

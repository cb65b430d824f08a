# Round-end GPU pass, part A: parity suite, phase diagnostics (N = 20 and config
# 5), the default bench (20 steps) and the bench with its CPU leg, then the rocprof
# kernel trace and FETCH/WRITE passes.  TAG=r06 bash tools/gpu_round_a.sh
# (build first: make, make diag, make diag20; the N = 20 phases use the diag20 build,
# which carries the N = 20 far TU's scheduler flags, the N = 50 ones the diag build)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/parity.log 2>&1
rc=$?
tail -4 gpurun_out/parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
NTM_MPC_LIB=$PWD/mpc-ntm-control_amd/lib/libntm_mpc_diag20.so timeout -k 10 300 python tools/diag_phases.py 100000 20 2 5 20 > gpurun_out/phases.log 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > gpurun_out/phases_n50m2.log 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 3 5 5 > gpurun_out/phases_n50m3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_cpu.json 2> gpurun_out/bench_cpu.err || exit $?
TAG=$TAG bash tools/prof_r01.sh > gpurun_out/prof.log 2>&1 || exit $?
echo part A done

# Round-end GPU pass: parity suite + phase diagnostics + short bench (gpu_cmd.sh),
# the default bench with its CPU leg, then the rocprof collections
# (kernel trace + FETCH/WRITE passes, SQ passes).  Copy the results into profiles/.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_cmd.sh || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_cpu.json 2> gpurun_out/bench_cpu.err || exit $?
TAG=${TAG:-r02} bash tools/prof_r01.sh > gpurun_out/prof.log 2>&1 || exit $?
TAG=${TAG:-r02} bash tools/prof_pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
bash tools/gpu_configs.sh || exit $?

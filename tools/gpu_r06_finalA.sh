# Round 6 final pass, call 1: smoke() (the driver's round-end check), then part A
# (parity suite, phases, benches, rocprof kernel trace and FETCH/WRITE)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final_smoke.log
TAG=r06 bash tools/gpu_round_a.sh

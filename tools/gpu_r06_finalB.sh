# Round 6 final pass, call 2: part B (SQ counters, configs 2 and 5, PCIe rate, the
# multi-rank rehearsals including the bare --gpus launcher, N = 50 MFMA counters)
set -o pipefail
TAG=r06 bash tools/gpu_round_b.sh
# the shapes of the sets N = 50 still sends to the bordered elimination (diagnostic build)
mkdir -p gpurun_out/r06h
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > gpurun_out/r06h/phases_n50m2.txt 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 3 5 5 > gpurun_out/r06h/phases_n50m3.txt 2>&1 || exit $?
grep -h "bordered re-solves by shape" gpurun_out/r06h/phases_n50m2.txt gpurun_out/r06h/phases_n50m3.txt

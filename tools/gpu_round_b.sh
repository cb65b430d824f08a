# Round-end GPU pass, part B: SQ counter passes, BASELINE configs 2 and 5 and the
# PCIe-inclusive rate, the multi-rank rehearsal, the N = 50 MFMA counters, and the
# warm-start set trace of one N = 50 scenario.  TAG=r06 bash tools/gpu_round_b.sh
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r06}
TAG=$TAG bash tools/prof_pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
bash tools/gpu_configs.sh || exit $?
bash tools/gpu_dist.sh > gpurun_out/dist.log 2>&1 || exit $?
bash tools/prof_mfma.sh > gpurun_out/mfma.log 2>&1 || exit $?
echo part B done

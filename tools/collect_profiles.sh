# Copy the outputs of one round-end GPU pass (tools/gpu_round.sh + gpu_dist.sh +
# the N = 50 diag_phases runs + prof_mfma.sh, all under gpurun_out/) into
# profiles/ under the round's tag:   bash tools/collect_profiles.sh r03
set -e
T=${1:?round tag}
G=gpurun_out
P=profiles
cp $G/bench_cpu.json $P/${T}_bench.json
cp $G/bench.json $P/${T}_bench_20steps.json
cp $G/prof_$T/ktrace_kernel_stats.csv $P/${T}_kernel_stats.csv
(head -1 $G/prof_$T/ktrace_kernel_trace.csv; grep 'k_mpc_step' $G/prof_$T/ktrace_kernel_trace.csv) > $P/${T}_kernel_trace_step.csv
cp $G/prof_$T/bench_under_rocprof.json $P/${T}_bench_under_rocprof.json
cp $G/prof_$T/fetch_counter_collection.csv $P/${T}_pmc_fetch.csv
cp $G/prof_$T/write_counter_collection.csv $P/${T}_pmc_write.csv
cp $G/prof_$T/traffic_$T.json $P/traffic_$T.json
(cat $G/pmc/pmc1_counter_collection.csv; tail -n +2 $G/pmc/pmc2_counter_collection.csv) > $P/${T}_pmc_sq.csv
cp $G/pmc/sq_$T.json $P/sq_$T.json
(cat $G/phases.log; echo; echo "== N=50, mode 2 (B=20000) =="; cat $G/phases_n50m2.log; echo
 echo "== N=50, mode 3 (B=20000) =="; cat $G/phases_n50m3.log) | grep -v amdgpu.ids > $P/${T}_phases.txt
mkdir -p $P/${T}_configs $P/${T}_dist
cp $G/cfg/c2.json $G/cfg/c5m2.json $G/cfg/c5m3.json $G/cfg/pcie.log $P/${T}_configs/
cp $G/dist/w1_nccl.json $G/dist/w2_gloo.json $P/${T}_dist/
[ -f $G/dist/w2_launcher.json ] && cp $G/dist/w2_launcher.json $P/${T}_dist/
tail -3 $G/parity.log > $P/${T}_gpu_tests.txt
cp $G/mfma_pmc/mfma_counter_collection.csv $P/${T}_pmc_mfma_n50.csv
echo "copied into $P/ (${T})"

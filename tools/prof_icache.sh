# Instruction-cache counters of the step kernel (VALU/LDS-latency study): the
# counter list, then one --pmc pass of the SQC instruction-cache counters over one
# bench step (B = 1e5, N = 20).  Results: gpurun_out/icache/
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/icache
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -iE "ICACHE|IFETCH|SQC_" $OUT/counters.txt | head -60 > $OUT/icache_names.txt || true
A="--steps 1 --warmup 1 --no-cpu --no-disturbed --verify 0 ${EXTRA:-}"
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE} --kernel-trace -d $OUT -o ic1 --output-format csv -- python3 $R/bench.py $A > $OUT/ic1.log 2>&1 || exit $?
echo icache done

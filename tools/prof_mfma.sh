# MFMA evidence for the long-horizon Gram (gram_mfma, N = 50): one --pmc pass of
# the matrix-core counters over config 5 (mode 2, one warmup + one timed step),
# kernel trace only.  Results: gpurun_out/mfma_pmc/
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/mfma_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $OUT -o mfma --output-format csv -- python3 $R/bench.py --N 50 --mode 2 --steps 1 --warmup 1 --no-cpu --no-disturbed --verify 0 > $OUT/mfma.log 2>&1 || exit $?
echo mfma pmc done

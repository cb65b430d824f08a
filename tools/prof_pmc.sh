# SQ instruction-mix / wait counters of the step kernel (separate --pmc passes,
# kernel trace only; B=1e5, one warmup + one timed step), reduced by sq_parse.py.
# Results: gpurun_out/pmc/
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A="--steps 1 --warmup 1 --no-cpu --no-disturbed --verify 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY -d $OUT -o pmc1 --output-format csv -- python3 $R/bench.py $A > $OUT/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d $OUT -o pmc2 --output-format csv -- python3 $R/bench.py $A > $OUT/pmc2.log 2>&1 || exit $?
cd $R && python3 tools/sq_parse.py $OUT $TAG > $OUT/sq.log 2>&1 || exit $?
echo pmc done

set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export NTM_LANES=64
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o ktrace --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY -d $R/gpurun_out/prof2 -o pmc1 --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu --batch 20000 >> $R/gpurun_out/prof2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d $R/gpurun_out/prof2 -o pmc2 --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu --batch 20000 >> $R/gpurun_out/prof2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof2 -o pmc3 --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu >> $R/gpurun_out/prof2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof2 -o pmc4 --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu >> $R/gpurun_out/prof2.log 2>&1 || exit $?
echo done

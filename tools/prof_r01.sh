# Round-1 profile collection (run on the GPU box through gpurun):
#   kernel-trace stats of the default bench, then FETCH_SIZE and WRITE_SIZE
#   in separate --pmc passes (never combined with runtime/sys traces).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o ktrace --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-disturbed --verify 0 > $OUT/bench_under_rocprof.json 2> $OUT/ktrace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT -o fetch --output-format csv -- python3 $R/tools/traffic_run.py 100000 > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT -o write --output-format csv -- python3 $R/tools/traffic_run.py 100000 > $OUT/write.log 2>&1 || exit $?
cd $R && python3 tools/traffic_parse.py $OUT 100000 $TAG > $OUT/traffic.log 2>&1 || exit $?
echo prof done

# Parity suite (every -m gpu test) + the default bench; each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/parity.log 2>&1
rc=$?
tail -15 gpurun_out/parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json

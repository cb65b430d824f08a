# Parity suite + a short bench (no CPU leg); each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/parity.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/parity.log; exit 1; }
tail -3 gpurun_out/parity.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_phases.py 100000 > gpurun_out/phases.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?

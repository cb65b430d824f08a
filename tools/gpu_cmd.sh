set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -x > gpurun_out/parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/parity.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_phases.py 20000 > gpurun_out/phases.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?

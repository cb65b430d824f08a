# Parity suite (every -m gpu test), then config 5's fp32-vs-fp64 sweep on the GPU
# (tools/precision_gpu.py at N = 10/20/50, modes 2 and 3, timed at B = 1e5).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/parity.log 2>&1
rc=$?
tail -15 gpurun_out/parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/precision_gpu.py 16 4 --timing-batch 100000 --out gpurun_out/r04_precision.json > gpurun_out/precision.log 2>&1 || exit $?
cat gpurun_out/precision.log

# One GPU call: the -m gpu suite (log in gpurun_out/$1_tests.txt), then, unless the
# suite crashed (pytest exit 0 = passed, 1 = test failures; anything else stops the
# call), an A/B bench of two library builds: bash tools/gpu_tests_then_ab.sh TAG libA libB [bench args]
set -o pipefail
mkdir -p gpurun_out
tag=$1; A=$2; B=$3; shift 3
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_bench.sh "$A" "$B" "$@" 2>&1 | tee gpurun_out/${tag}_ab.txt

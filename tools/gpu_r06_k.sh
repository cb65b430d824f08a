# Round 6, call K: the product with both N = 50 changes (two-collision k = 1 sets in
# the mode-3 build, zero-row rejection): -m gpu suite, configs 2 and 5, default bench
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/gpu_configs.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit $?
for f in gpurun_out/cfg/c2.json gpurun_out/cfg/c5m2.json gpurun_out/cfg/c5m3.json $O/bench.json; do python -c "import json; d=json.loads(open('$f').read().strip().split(chr(10))[-1]); print('$f', round(d['ms_per_step'], 3), d['value'])"; done

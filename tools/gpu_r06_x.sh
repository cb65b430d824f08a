# Round 6, call X: the product with the skipped-row dual-only step: -m gpu suite and config 5 mode 2
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu --N 50 --steps 10 --warmup 5 --no-disturbed > $O/c5m2.json 2>/dev/null || exit 1
python -c "
import json
d = json.loads(open('$O/c5m2.json').read().strip().split(chr(10))[-1])
print('c5m2', round(d['ms_per_step'], 3), d['solver'], d.get('gather_verify'))
"

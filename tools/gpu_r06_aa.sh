# Round 6, call AA: readlane indices in the N = 50 E build (and, mode 3, the sparse pass)
# in the product: -m gpu suite, config 5 modes 2 and 3, config 3
set -o pipefail
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu --N 50 --steps 10 --warmup 5 --no-disturbed > $O/c5m2.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --no-cpu --N 50 --mode 3 --steps 10 --warmup 5 --no-disturbed > $O/c5m3.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 --no-disturbed > $O/c3.json 2>/dev/null || exit 1
python -c "
import json
for f in ('c5m2', 'c5m3', 'c3'):
    d = json.loads(open('$O/' + f + '.json').read().strip().split(chr(10))[-1])
    print(f, round(d['ms_per_step'], 3), d['solver']['optimal_frac'], d['solver']['gi_solves_per_step'], d.get('gather_verify', {}).get('bitwise_equal'))
"

# Round 6, call T: the fused column sums at N = 50 in the product: -m gpu suite,
# config 5 mode 3 A/B against the unfused mode-3 TU, config 5 mode 2 and config 3
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
echo "config 5 mode 3"
bash tools/ab_multi.sh $L/libntm_mpc_nofuse3.so $L/libntm_mpc.so -- --N 50 --mode 3 --steps 10 --warmup 5 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m3.txt || exit 1
echo "config 5 mode 2, config 3 (product)"
timeout -k 10 300 python bench.py --no-cpu --N 50 --steps 10 --warmup 5 --no-disturbed > $O/c5m2.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 --no-disturbed > $O/c3.json 2>/dev/null || exit 1
python -c "
import json
for f in ('c5m2', 'c3'):
    d = json.loads(open('$O/' + f + '.json').read().strip().split(chr(10))[-1])
    print(f, round(d['ms_per_step'], 3), d['solver']['optimal_frac'], d.get('gather_verify'))
"

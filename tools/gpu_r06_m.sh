# Round 6, call M: the constant-row feasibility test folded into the scaling pass
# (product) against the previous commit (base): -m gpu suite, A/B at configs 3, 2, 5
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --no-disturbed --verify 0 2>&1 | tee $O/ab_c3.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 20 --warmup 2 --batch 1024 --mode 1 --no-disturbed --verify 0 2>&1 | tee $O/ab_c2.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 5 --warmup 5 --N 50 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m2.txt

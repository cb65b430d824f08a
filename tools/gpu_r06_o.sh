# Round 6, call O: the one-wave all-LDS N = 20 build in the product: -m gpu suite
# (the bitwise test against the two-wave build included), A/B at config 2 against
# the previous commit (base), and the default bench
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 20 --warmup 2 --batch 1024 --mode 1 --no-disturbed --verify 0 2>&1 | tee $O/ab_c2.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 20 --warmup 5 --batch 2048 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_2048.txt

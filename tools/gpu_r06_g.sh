# Round 6, call G: N = 50 split by mode with the plane minimisation as one helper
# (the modes 0-2 build compiles as before the three-hole path): -m gpu suite, A/B
# at config 5 against the previous commit's build
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 5 --warmup 5 --N 50 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m2.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 5 --warmup 5 --N 50 --mode 3 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m3.txt

# Round 6, call F: N = 50 split by mode (ntm_n50.hip without the three-hole path,
# ntm_n50m3.hip with it): the -m gpu suite, then A/B at config 5 (both modes) and
# config 3 against the previous commit's build (base)
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 5 --warmup 5 --N 50 --mode 3 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m3.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so -- --steps 5 --warmup 5 --N 50 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m2.txt || exit 1
NTM_MPC_LIB=$L/libntm_mpc_fusey.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "20 and not wide" > $O/tests_fusey.txt 2>&1; echo "fusey: $(tail -1 $O/tests_fusey.txt)"
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc.so $L/libntm_mpc_fusey.so -- --no-disturbed --verify 0 2>&1 | tee $O/ab_c3.txt

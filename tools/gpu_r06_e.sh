# Round 6, call E: k = 2 sets with one collision (three holes) on the null-space
# path (NTM_COLL3): the -m gpu suite, A/B at config 5 against the build without it,
# and the diagnostic counters of the re-solve paths
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc_nocoll3.so $L/libntm_mpc.so -- --steps 5 --warmup 5 --N 50 --mode 3 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m3.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc_nocoll3.so $L/libntm_mpc.so -- --steps 5 --warmup 5 --N 50 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m2.txt || exit 1
timeout -k 10 300 python tools/diag_phases.py 20000 50 3 5 5 > $O/phases_n50m3.txt 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > $O/phases_n50m2.txt 2>&1 || exit $?
grep -h "re-solve paths\|GI solves\|cand  " $O/phases_n50m3.txt $O/phases_n50m2.txt

# Round 6, call J: sets with a zero row of E rejected before the bordered elimination
# (N = 50, variant nofree): parity at N = 50, A/B at config 5 mode 2
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
NTM_MPC_LIB=$L/libntm_mpc_nofree.so timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "50" > $O/tests_nofree.txt 2>&1
rc=$?
echo "nofree: $(tail -1 $O/tests_nofree.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc_nofree.so -- --steps 5 --warmup 5 --N 50 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m2.txt

# Round 6, call I: k = 1 sets with two collisions (three holes) on the null-space path
# in the mode-3 N = 50 build (variant twoorph): parity at N = 50 / mode 3, A/B at config 5 mode 3
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
NTM_MPC_LIB=$L/libntm_mpc_twoorph.so timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "50 or m3 or mode3 or 3]" > $O/tests_twoorph.txt 2>&1
rc=$?
echo "twoorph: $(tail -1 $O/tests_twoorph.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_twoorph.so -- --steps 5 --warmup 5 --N 50 --mode 3 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m3.txt

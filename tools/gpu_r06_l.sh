# Round 6, call L: the dual path skips a row whose A + {p} end point is non-finite
# (variant skip, N = 50 modes 0-2 build): parity at N = 50, A/B at config 5 mode 2,
# and the diagnostic counters (skips, GI solves)
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
NTM_MPC_LIB=$L/libntm_mpc_skip.so timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "50" > $O/tests_skip.txt 2>&1
rc=$?
echo "skip: $(tail -1 $O/tests_skip.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc_skip.so -- --steps 5 --warmup 5 --N 50 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_c5m2.txt || exit 1
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > $O/phases_n50m2.txt 2>&1 || exit $?
grep -h "GI solves\|handed to GI\|skipped\|  gi  " $O/phases_n50m2.txt

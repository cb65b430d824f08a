# Round 6, call B: parity of the most aggressive split builds (all-LDS and far,
# both N = 20 builds exercised by the suite's batch sizes and small-batch
# settings), then A/B timing: config 3 (far build) base vs far split 1/2/3 and
# the GI-removed timing probe; config 2 and B = 2048 mode 2 (all-LDS build) base
# vs near split 1/2/3.
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_product.txt 2>&1
rc=$?
echo "product: $(tail -1 $O/tests_product.txt)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
for v in near3 far3; do
  NTM_MPC_LIB=$L/libntm_mpc_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x -k "not wide" > $O/tests_$v.txt 2>&1
  rc=$?
  echo "$v: $(tail -1 $O/tests_$v.txt)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
done
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_far1.so $L/libntm_mpc_far2.so $L/libntm_mpc_far3.so $L/libntm_mpc_gidefer.so -- --no-disturbed --verify 0 2>&1 | tee $O/ab_far.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_near1.so $L/libntm_mpc_near2.so $L/libntm_mpc_near3.so -- --steps 20 --warmup 2 --batch 1024 --mode 1 --no-disturbed --verify 0 2>&1 | tee $O/ab_near_c2.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_near1.so $L/libntm_mpc_near3.so -- --steps 20 --warmup 5 --batch 2048 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_near_2048.txt
# N = 50: the dual path's signed partial step (product) vs without (nosigned); the
# diagnostic build's counters of the reasons the path hands QPs to GI
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_nosigned.so -- --steps 5 --warmup 5 --N 50 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_n50m2.txt || exit 1
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > $O/phases_n50m2.txt 2>&1 || exit $?

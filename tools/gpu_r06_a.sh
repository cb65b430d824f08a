# Round 6, first call: the --gpus launcher rehearsal (gloo, two ranks on one GPU),
# the -m gpu suite on the product build (wide closed-loop counts printed), the wide
# test on the recursive-rollout variant (divergence with
# NTM_ROLL_LIFTED=0), and the GI-deferral probe timed against the product.
set -o pipefail
mkdir -p gpurun_out/r06a
O=gpurun_out/r06a
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --batch 8192 --steps 3 --warmup 1 > $O/launch_gloo2.json 2> $O/launch_gloo2.err || exit $?
python -c "import json; d=json.loads(open('$O/launch_gloo2.json').read().strip().split(chr(10))[-1]); print('launcher', d['n_gpus'], d['per_rank'], d['gather_verify'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
NTM_MPC_LIB=$PWD/mpc-ntm-control_amd/lib/libntm_mpc_rollrec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_wide.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k closed_loop_wide > $O/wide_rollrec.txt 2>&1
rc=$?
tail -3 $O/wide_rollrec.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh mpc-ntm-control_amd/lib/libntm_mpc.so mpc-ntm-control_amd/lib/libntm_mpc_gidefer.so -- --no-disturbed --verify 0 2>&1 | tee $O/ab_gidefer.txt

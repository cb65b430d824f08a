# Round 6, call AD: the free-response recursion on every lane in the fused N = 50 lift (NTM_FUSE_LOCAL_E), config 5
set -o pipefail
L=mpc-ntm-control_amd/lib
echo "config 5 mode 2"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_locale.so -- --N 50 --steps 10 --warmup 5 --no-disturbed --verify 0 || exit 1
echo "config 5 mode 3"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_locale3.so -- --N 50 --mode 3 --steps 10 --warmup 5 --no-disturbed --verify 0 || exit 1
python -c "
import json
for f in ('abm_libntm_mpc_2', 'abm_libntm_mpc_locale_2', 'abm_libntm_mpc_locale3_2'):
    d = json.load(open('gpurun_out/' + f + '.json'))
    print(f, {k: v for k, v in d['solver'].items() if 'gi' in k or 'optimal' in k})
"

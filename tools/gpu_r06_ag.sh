# Round 6, call AG: prescaled echelon substitutions at N = 50 (NTM_SUB_PRESCALE), config 5
set -o pipefail
L=mpc-ntm-control_amd/lib
echo "config 5 mode 2"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_presc.so -- --N 50 --steps 10 --warmup 5 --no-disturbed --verify 0 || exit 1
echo "config 5 mode 3"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_presc3.so -- --N 50 --mode 3 --steps 10 --warmup 5 --no-disturbed --verify 0 || exit 1
python -c "
import json
for f in ('abm_libntm_mpc_2', 'abm_libntm_mpc_presc_2', 'abm_libntm_mpc_presc3_2'):
    d = json.load(open('gpurun_out/' + f + '.json'))
    print(f, {k: v for k, v in d['solver'].items() if 'gi' in k or 'optimal' in k})
"

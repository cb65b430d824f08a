# Round 6, call AC: E prefetched 3 steps ahead in the N = 50 forward substitution (NTM_SUB_AHEAD)
set -o pipefail
L=mpc-ntm-control_amd/lib
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_ahead1.so $L/libntm_mpc_ahead3.so -- --N 50 --steps 10 --warmup 5 --no-disturbed --verify 0

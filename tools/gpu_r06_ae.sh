# Round 6, call AE: E prefetched 1 / 2 / 4 steps ahead in the N = 50 multipliers' back substitution (NTM_MU_AHEAD)
set -o pipefail
L=mpc-ntm-control_amd/lib
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_mua1.so $L/libntm_mpc_mua2.so $L/libntm_mpc_mua4.so -- --N 50 --steps 10 --warmup 5 --no-disturbed --verify 0

# Round 6, call U: the row norms two rows per lane at N = 50 (NTM_ROW_PAIRS), config 5 modes 2 and 3
set -o pipefail
L=mpc-ntm-control_amd/lib
echo "config 5 mode 2"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_pairs.so -- --N 50 --steps 10 --warmup 5 --no-disturbed --verify 0 || exit 1
echo "config 5 mode 3"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_pairs3.so -- --N 50 --mode 3 --steps 10 --warmup 5 --no-disturbed --verify 0

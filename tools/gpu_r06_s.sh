# Round 6, call S: column sums accumulated by the slim lift (NTM_FUSE_COLSUM), config 3 and config 5 mode 2
set -o pipefail
L=mpc-ntm-control_amd/lib
echo "config 3"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_fuse.so -- --steps 20 --warmup 5 --no-disturbed --verify 0 || exit 1
echo "config 5 mode 2"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_fuse50.so -- --N 50 --steps 10 --warmup 5 --no-disturbed --verify 0

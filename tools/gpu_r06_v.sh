# Round 6, call V: column sums accumulated by the all-LDS N = 20 lift (NTM_FUSE_COLSUM bit 2)
set -o pipefail
L=mpc-ntm-control_amd/lib
echo "config 2 (B = 1024 mode 1, one-wave build)"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_fnear1.so -- --steps 20 --warmup 2 --batch 1024 --mode 1 --no-disturbed --verify 0 || exit 1
echo "B = 1024 mode 2 (one-wave build)"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_fnear1.so -- --steps 20 --warmup 5 --batch 1024 --mode 2 --no-disturbed --verify 0 || exit 1
echo "B = 2048 mode 2 (two-wave build)"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_fnear.so -- --steps 20 --warmup 5 --batch 2048 --mode 2 --no-disturbed --verify 0

# Round 6, call AB: the row-per-lane E build (with readlane column indices) at N = 20
set -o pipefail
L=mpc-ntm-control_amd/lib
echo "config 3 (far)"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_rowe2.so -- --steps 20 --warmup 5 --no-disturbed --verify 0 || exit 1
echo "B = 2048 mode 2 (all-LDS)"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_rowen.so -- --steps 20 --warmup 5 --batch 2048 --mode 2 --no-disturbed --verify 0

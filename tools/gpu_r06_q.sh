# Round 6, call Q: CH (terms per LDS round trip) of the one-wave all-LDS build, config 2 and B = 1024 mode 2
set -o pipefail
L=mpc-ntm-control_amd/lib
echo "config 2 (B = 1024, mode 1)"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_ch5.so $L/libntm_mpc_ch10.so $L/libntm_mpc_ch20.so -- --steps 20 --warmup 2 --batch 1024 --mode 1 --no-disturbed --verify 0 || exit 1
echo "B = 1024, mode 2"
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_ch5.so $L/libntm_mpc_ch10.so $L/libntm_mpc_ch20.so -- --steps 20 --warmup 5 --batch 1024 --mode 2 --no-disturbed --verify 0

# Round 6, call N: the all-LDS N = 20 build with a one-wave register budget (near1w)
# at config 2 (B = 1024, one wave per SIMD) against the product
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
L=$PWD/mpc-ntm-control_amd/lib
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc_near1w.so -- --steps 20 --warmup 2 --batch 1024 --mode 1 --no-disturbed --verify 0 2>&1 | tee $O/ab_c2.txt || exit 1
bash tools/ab_multi.sh $L/libntm_mpc_base.so $L/libntm_mpc_near1w.so -- --steps 20 --warmup 5 --batch 1024 --mode 2 --no-disturbed --verify 0 2>&1 | tee $O/ab_1024m2.txt

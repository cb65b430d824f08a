# Round 6, call R: row-per-lane E at N = 20 (config 3 A/B) and config 2 per-scenario phases
set -o pipefail
L=mpc-ntm-control_amd/lib
bash tools/ab_multi.sh $L/libntm_mpc.so $L/libntm_mpc_rowe.so -- --steps 20 --warmup 5 --no-disturbed --verify 0 || exit 1
NTM_MPC_LIB=$L/libntm_mpc_diag.so timeout -k 10 200 python -u tools/c2_scen_phases.py 1024 1 5 1023 386 0 100 500 700 900 > gpurun_out/r06r_scen.txt 2>&1 || exit 1
cat gpurun_out/r06r_scen.txt

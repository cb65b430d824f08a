# Round 6, call P: config 2's tail (iteration counts vs step time, batches of
# one scenario repeated) and its phase stamps on the diagnostic build
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 200 python -u tools/c2_tail.py 1024 1 5 20 > $O/c2_tail.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/c2_tail.py 1024 2 5 10 > $O/b1024m2_tail.txt 2>&1 || exit 1
NTM_MPC_LIB=mpc-ntm-control_amd/lib/libntm_mpc_diag.so timeout -k 10 200 python -u tools/diag_phases.py 1024 20 1 5 20 > $O/c2_phases.txt 2>&1 || exit 1
cat $O/c2_tail.txt $O/b1024m2_tail.txt
head -30 $O/c2_phases.txt

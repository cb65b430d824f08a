# Occupancy sensitivity of the N=20 step kernel:
#   base  : the product library (8 scenarios per CU, 2 waves per SIMD)
#   pad6  : -DNTM_LDS_PAD=4096   (6 scenarios per CU)
#   pad4  : -DNTM_LDS_PAD=14336  (4 scenarios per CU, 1 wave per SIMD)
#   w3    : -DNTM_HOT_WAVES_PER_EU=3 (168 VGPRs + scratch spills, still LDS-capped at 8 per CU)
# Built beforehand in mpc-ntm-control_amd/lib/; results in gpurun_out/occ_*.json.
set -o pipefail
mkdir -p gpurun_out
L=mpc-ntm-control_amd/lib
for r in 1 2; do
  for v in base pad6 pad4 w3; do
    lib=$L/libntm_mpc.so; [ $v != base ] && lib=$L/libntm_mpc_$v.so
    NTM_MPC_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/occ_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/occ_${v}_$r.json')); print('$v', $r, round(d['ms_per_step'], 3))"
  done
done

# Configs 2 and 5 for several builds (alternating), then the phase profiles of the
# diagnostic build at config 2 and config 5.  Results: gpurun_out/$TAG/
#   TAG=x bash tools/gpu_cfg_ab.sh lib1.so lib2.so ...
set -o pipefail
TAG=${TAG:-cfg}
O=gpurun_out/$TAG
mkdir -p $O
for lib in "$@"; do
  t=$(basename $lib .so)
  NTM_MPC_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu --batch 1024 --mode 1 > $O/c2_$t.json 2> $O/c2_$t.err || exit $?
  NTM_MPC_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 5 --no-cpu --N 50 --mode 2 > $O/c5m2_$t.json 2> $O/c5m2_$t.err || exit $?
  NTM_MPC_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 5 --no-cpu --N 50 --mode 3 > $O/c5m3_$t.json 2> $O/c5m3_$t.err || exit $?
  for c in c2 c5m2 c5m3; do python -c "import json; d=json.load(open('$O/${c}_$t.json')); print('$c $t', round(d['ms_per_step'], 3), d['solver']['gi_solves_per_step'], d['solver']['warm_verify_per_step'])"; done
done
if [ -z "$NO_PHASES" ]; then
timeout -k 10 120 python tools/diag_phases.py 1024 20 1 2 20 > $O/phases_c2.txt 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > $O/phases_n50m2.txt 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 3 5 5 > $O/phases_n50m3.txt 2>&1 || exit $?
fi
echo done

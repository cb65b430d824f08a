# A/B timing of two builds of the library on one box (alternating, 2 rounds):
#   bash tools/ab_bench.sh <libA.so> <libB.so> [bench args...]
# Prints ms_per_step of each run; results in gpurun_out/ab_*.json.
set -o pipefail
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for r in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    NTM_MPC_LIB=$lib timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/ab_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${v}_$r.json')); print('$v', $r, round(d['ms_per_step'], 3))"
  done
done

# A/B timing of several builds of the library on one box (alternating, 2 rounds):
#   bash tools/ab_multi.sh <lib1.so> <lib2.so> ... -- [bench args...]
# Prints ms_per_step of each run; results in gpurun_out/abm_*.json.
set -o pipefail
mkdir -p gpurun_out
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in 1 2; do
  for lib in "${libs[@]}"; do
    tag=$(basename "$lib" .so)
    NTM_MPC_LIB=$lib timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/abm_${tag}_$r.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abm_${tag}_$r.json')); print('$tag', $r, round(d['ms_per_step'], 4), d['solver']['optimal_frac'])"
  done
done

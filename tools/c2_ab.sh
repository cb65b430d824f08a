# Small-batch A/B (the all-LDS N = 20 build): config 2 (mode 1, B = 1024) and mode 2 at
# B = 1024 / 2048 for several libraries, alternating, 2 rounds.
#   bash tools/c2_ab.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out/c2ab
for r in 1 2; do
  for lib in "$@"; do
    t=$(basename $lib .so)
    for cfg in "1 1024" "2 1024" "2 2048"; do
      m=${cfg% *}; b=${cfg#* }
      NTM_MPC_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --mode $m --batch $b --steps 20 --warmup 2 > gpurun_out/c2ab/${t}_m${m}_b${b}_$r.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('gpurun_out/c2ab/${t}_m${m}_b${b}_$r.json')); print('$t mode $m B $b round $r', round(d['ms_per_step'], 4))"
    done
  done
done

# Small-batch layout sweep (ms per step-batch, N = 20): the all-LDS build against the
# far (slim) build at several batch sizes; config 2 (mode 1, B = 1024) first.
set -o pipefail
mkdir -p gpurun_out/lsweep
run() {  # mode B small_batch steps
  timeout -k 10 120 python bench.py --no-cpu --mode $1 --batch $2 --small-batch $3 --steps $4 --warmup 2 > gpurun_out/lsweep/m$1_b$2_s$3.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/lsweep/m$1_b$2_s$3.json')); print('mode $1 B $2', 'lds' if $3 > 0 else 'far', round(d['ms_per_step'], 4))"
}
for r in 1 2; do
  run 1 1024 1000000000 20; run 1 1024 0 20
  for b in 2048 4096 8192 16384; do run 2 $b 1000000000 20; run 2 $b 0 20; done
done

# Round 6, call O2: config 2 and B = 1024 mode 2 with the one-wave budget (default)
# and without it (--one-wave-batch 0), alternating, on the product build
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
for r in 1 2; do
  for ow in 0 -1; do
    timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 2 --batch 1024 --mode 1 --no-disturbed --verify 0 --one-wave-batch $ow > $O/c2_${ow}_${r}.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/c2_${ow}_${r}.json').read().strip().split(chr(10))[-1]); print('c2 one-wave-batch $ow', $r, round(d['ms_per_step'], 4), d['roofline']['kernel'])"
    timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 5 --batch 1024 --mode 2 --no-disturbed --verify 0 --one-wave-batch $ow > $O/m2_${ow}_${r}.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/m2_${ow}_${r}.json').read().strip().split(chr(10))[-1]); print('B1024m2 one-wave-batch $ow', $r, round(d['ms_per_step'], 4))"
  done
done

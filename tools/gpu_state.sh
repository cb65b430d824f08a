# One GPU call measuring where the current tree stands: the -m gpu suite, the
# default bench, configs 2 and 5, and the phase profiles over the bench's steps
# (N = 20 at B = 1e5, config 2, config 5 modes 2/3).  Results: gpurun_out/$TAG/
#   TAG=r05a bash tools/gpu_state.sh [skip-tests]
set -o pipefail
TAG=${TAG:-state}
O=gpurun_out/$TAG
mkdir -p $O
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -rf > $O/tests.txt 2>&1
  rc=$?
  tail -3 $O/tests.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 200 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu --batch 1024 --mode 1 > $O/c2.json 2> $O/c2.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 5 --no-cpu --N 50 --mode 2 > $O/c5m2.json 2> $O/c5m2.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 5 --no-cpu --N 50 --mode 3 > $O/c5m3.json 2> $O/c5m3.err || exit $?
timeout -k 10 300 python tools/diag_phases.py 100000 20 2 5 20 > $O/phases_n20.txt 2>&1 || exit $?
timeout -k 10 120 python tools/diag_phases.py 1024 20 1 2 20 > $O/phases_c2.txt 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > $O/phases_n50m2.txt 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 3 5 5 > $O/phases_n50m3.txt 2>&1 || exit $?
for f in bench c2 c5m2 c5m3; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', round(d['ms_per_step'], 3))"; done
echo done

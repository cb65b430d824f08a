# The driver's round-end checks on the final tree: smoke(), the -m gpu suite and
# the default bench line.  Results: gpurun_out/final_*.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final_smoke.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/final_parity.log 2>&1
rc=$?
tail -3 gpurun_out/final_parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/final_bench.json').read().strip().split(chr(10))[-1]); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['traffic_source']['file'])"

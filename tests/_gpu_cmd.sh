set -o pipefail
R=$GRAFT_REPO_ROOT
hipcc --offload-arch=gfx950 -O3 -o /tmp/dpp_check tests/_dpp_check.hip 2>/dev/null && timeout -k 5 60 /tmp/dpp_check > gpurun_out/dpp.log 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -x > gpurun_out/parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/parity.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?

# Parity suite (every -m gpu test), then the command given as arguments (an A/B
# or a bench) unless the suite crashed, hung or hit its time limit (pytest exit
# codes 0 and 1 = ran to completion).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/parity.log 2>&1
rc=$?
tail -12 gpurun_out/parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ $# -eq 0 ] || "$@"

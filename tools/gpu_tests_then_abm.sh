# One GPU call: the -m gpu suite on the library NTM_MPC_LIB names (default: the
# product build; log in gpurun_out/$TAG_tests.txt), then, unless the suite crashed
# (pytest exit 0 = passed, 1 = test failures; anything else stops the call), an
# alternating A/B of several builds (tools/ab_multi.sh):
#   bash tools/gpu_tests_then_abm.sh TAG lib1.so lib2.so ... -- [bench args]
# K=<pytest -k expression> narrows the suite.
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/${tag}_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
unset NTM_MPC_LIB
bash tools/ab_multi.sh "$@" 2>&1 | tee gpurun_out/${tag}_ab.txt

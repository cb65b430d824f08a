# BASELINE configs 2 and 5 (config 3 is the default bench) and the PCIe-inclusive
# rate of the host-buffer entry point.  Results: gpurun_out/cfg/
set -o pipefail
mkdir -p gpurun_out/cfg
timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu --batch 1024 --mode 1 > gpurun_out/cfg/c2.json 2>gpurun_out/cfg/c2.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 5 --no-cpu --N 50 --mode 2 > gpurun_out/cfg/c5m2.json 2>gpurun_out/cfg/c5m2.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 5 --no-cpu --N 50 --mode 3 > gpurun_out/cfg/c5m3.json 2>gpurun_out/cfg/c5m3.err || exit $?
timeout -k 10 300 python tools/pcie_rate.py > gpurun_out/cfg/pcie.log 2>&1 || exit $?

# Register / scratch report of one translation unit's step kernel, built with the
# product flags (the N = 20 far TU adds the register-pressure trackers, Makefile N20FLAGS):
#   bash tools/ru_tu.sh csrc/ntm_n20.hip 'k_mpc_stepILi64ELi20ELb0ELb1E' [extra flags]
cd "$(dirname "$0")/../mpc-ntm-control_amd" || exit 1
tu=$1; pat=$2; shift 2
extra=""
case $tu in *ntm_n20.hip) extra="-mllvm -amdgpu-use-amdgpu-trackers=1";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -Wno-unused-variable $extra "$@" \
    --cuda-device-only -c -o /tmp/ru_tu.o "$tu" -Rpass-analysis=kernel-resource-usage 2>&1 |
    grep -A12 "$pat" | grep -E "VGPRs:|AGPRs|ScratchSize|Spill|Occupancy" | head -7

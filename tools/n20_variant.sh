# Fast A/B variant of the N = 20 far translation unit only: compiles csrc/ntm_n20.hip
# with extra flags and links it with the product's other objects (lib/obj/).  Only for
# changes that leave the host side alone (ws_bytes, far_doubles, launch settings):
# a layout change needs `make variant` (the launches size the LDS from the host TU)
#   bash tools/n20_variant.sh NAME "-DNTM_N20_CH=4 ..."   ->  lib/libntm_mpc_NAME.so
set -e
cd "$(dirname "$0")/../mpc-ntm-control_amd"
V=$1; F=$2
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function"
mkdir -p lib/obj_$V
SCHED=${SCHED:--mllvm -amdgpu-use-amdgpu-trackers=1}   # the product flags of ntm_n20.o (Makefile N20FLAGS)
$H $SCHED $F -c -o lib/obj_$V/ntm_n20.o csrc/ntm_n20.hip
$H -shared -o lib/libntm_mpc_$V.so lib/obj/ntm_kernels.o lib/obj_$V/ntm_n20.o lib/obj/ntm_n20near.o lib/obj/ntm_n50.o lib/obj/ntm_n50m3.o
echo built lib/libntm_mpc_$V.so

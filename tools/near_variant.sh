# Fast A/B variant of the all-LDS N = 20 translation unit only (ntm_n20near.hip),
# linked with the product's other objects (lib/obj/), like tools/n20_variant.sh:
#   bash tools/near_variant.sh NAME "-DNTM_SPLIT_CERT=3 ..."  ->  lib/libntm_mpc_NAME.so
set -e
cd "$(dirname "$0")/../mpc-ntm-control_amd"
V=$1; F=$2
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function"
mkdir -p lib/obj_$V
$H $F -c -o lib/obj_$V/ntm_n20near.o csrc/ntm_n20near.hip
$H -shared -o lib/libntm_mpc_$V.so lib/obj/ntm_kernels.o lib/obj/ntm_n20.o lib/obj_$V/ntm_n20near.o lib/obj/ntm_n50.o lib/obj/ntm_n50m3.o
echo built lib/libntm_mpc_$V.so

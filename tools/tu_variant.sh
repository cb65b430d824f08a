# Fast A/B variant of ONE translation unit (n20 | n20near | n20near1w | n50 | n50m3 | kernels), linked
# with the product's other objects (lib/obj/):
#   bash tools/tu_variant.sh n50 NAME "-DNTM_CDP_SIGNED=0"  ->  lib/libntm_mpc_NAME.so
# (the N = 20 far TU gets its product scheduler flags, Makefile N20FLAGS)
set -e
cd "$(dirname "$0")/../mpc-ntm-control_amd"
T=$1; V=$2; F=$3
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function"
case $T in n20) X="-mllvm -amdgpu-use-amdgpu-trackers=1";; *) X="";; esac
mkdir -p lib/obj_$V
objs=""
for t in kernels n20 n20near n20near1w n50 n50m3; do
  if [ "$t" = "$T" ]; then
    $H $X $F -c -o lib/obj_$V/ntm_$t.o csrc/ntm_$t.hip
    objs="$objs lib/obj_$V/ntm_$t.o"
  else
    objs="$objs lib/obj/ntm_$t.o"
  fi
done
$H -shared -o lib/libntm_mpc_$V.so $objs
echo built lib/libntm_mpc_$V.so

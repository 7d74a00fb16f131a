#!/bin/bash
# Build an A/B variant of libelect_ec.so with extra defines (kernels and host path):
#   tools/ab_build.sh NAME -DFOO -DBAR=1   ->  elect_amd/_ab/libelect_ec_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p elect_amd/_ab
python -m elect_amd.build >/dev/null
H=/opt/rocm/bin/hipcc
C="$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include"
objs=""
$C "$@" -x hip -c elect_amd/csrc/rs_kernels.hip -o elect_amd/_ab/rs_kernels_$name.o &
objs="$objs elect_amd/_ab/rs_kernels_$name.o"
# host_path.cpp has no device code: host C++ (elect_amd/build.py HOST_SOURCES)
$H -O3 -std=c++17 -fPIC -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ "$@" -x c++ \
    -c elect_amd/csrc/host_path.cpp -o elect_amd/_ab/host_path_$name.o &
objs="$objs elect_amd/_ab/host_path_$name.o"
for k in $(seq 1 16); do  # rs_inst.hip once per source-column count, 8 at a time
    $C "$@" -DELECT_EC_INST_K=$k -x hip -c elect_amd/csrc/rs_inst.hip -o elect_amd/_ab/rs_inst_k${k}_$name.o &
    objs="$objs elect_amd/_ab/rs_inst_k${k}_$name.o"
    [ $((k % 8)) -eq 0 ] && wait
done
wait
$H --offload-arch=gfx950 -shared -fPIC -o elect_amd/_ab/libelect_ec_$name.so elect_amd/_build/ec_capi.o $objs
rm $objs
echo elect_amd/_ab/libelect_ec_$name.so

#!/bin/bash
# Build an A/B variant of libelect_ec.so with extra defines (kernels and host path):
#   tools/ab_build.sh NAME -DFOO -DBAR=1   ->  elect_amd/_ab/libelect_ec_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p elect_amd/_ab
python -m elect_amd.build >/dev/null
H=/opt/rocm/bin/hipcc
for f in rs_kernels.hip host_path.cpp; do
    $H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include "$@" -x hip -c elect_amd/csrc/$f -o elect_amd/_ab/${f%.*}_$name.o &
done
wait
$H --offload-arch=gfx950 -shared -fPIC -o elect_amd/_ab/libelect_ec_$name.so elect_amd/_build/ec_capi.o \
    elect_amd/_ab/host_path_$name.o elect_amd/_ab/rs_kernels_$name.o
rm elect_amd/_ab/rs_kernels_$name.o elect_amd/_ab/host_path_$name.o
echo elect_amd/_ab/libelect_ec_$name.so

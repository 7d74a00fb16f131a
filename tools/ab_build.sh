#!/bin/bash
# Build an A/B variant of libelect_ec.so with extra defines:
#   tools/ab_build.sh NAME -DFOO -DBAR=1   ->  elect_amd/_ab/libelect_ec_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p elect_amd/_ab
python -m elect_amd.build >/dev/null
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include "$@" -x hip -c elect_amd/csrc/rs_kernels.hip -o elect_amd/_ab/rk_$name.o
$H --offload-arch=gfx950 -shared -fPIC -o elect_amd/_ab/libelect_ec_$name.so elect_amd/_build/ec_capi.o elect_amd/_build/host_path.o elect_amd/_ab/rk_$name.o
rm elect_amd/_ab/rk_$name.o
echo elect_amd/_ab/libelect_ec_$name.so

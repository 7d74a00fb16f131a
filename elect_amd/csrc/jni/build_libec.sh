#!/bin/bash
# Build the drop-in libec.so (JNI shim + MI355X engine) for ELECT.
# Needs a JDK (for <jni.h>) and ROCm hipcc.  Not built in the CI image, which
# has no JDK.  Usage: JAVA_HOME=/path/to/jdk elect_amd/csrc/jni/build_libec.sh [out_dir]
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../../.." && pwd)
OUT=${1:-$ROOT/build/libec}
: "${JAVA_HOME:=$(dirname "$(dirname "$(readlink -f "$(which javac)")")")}"
[ -f "$JAVA_HOME/include/jni.h" ] || { echo "no jni.h under JAVA_HOME=$JAVA_HOME" >&2; exit 1; }
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
gcc -O2 -fPIC -Wall -c -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I"$ROOT/include" \
    "$HERE/libec_jni.c" -o "$OUT/libec_jni.o"
"$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -x hip -c \
    "$ROOT/elect_amd/csrc/ec_capi.cpp" -o "$OUT/ec_capi.o"
"$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -x hip -c \
    "$ROOT/elect_amd/csrc/host_path.cpp" -o "$OUT/host_path.o"
"$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -x hip -c \
    "$ROOT/elect_amd/csrc/rs_kernels.hip" -o "$OUT/rs_kernels.o"
INST=""
for k in $(seq 1 16); do  # the kernel instances, once per source-column count
    "$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -DELECT_EC_INST_K=$k -x hip -c \
        "$ROOT/elect_amd/csrc/rs_inst.hip" -o "$OUT/rs_inst_k$k.o" &
    INST="$INST $OUT/rs_inst_k$k.o"
    [ $((k % 8)) -eq 0 ] && wait
done
wait
"$HIPCC" --offload-arch=gfx950 -shared -fPIC -o "$OUT/libec.so" \
    "$OUT/libec_jni.o" "$OUT/ec_capi.o" "$OUT/host_path.o" "$OUT/rs_kernels.o" $INST
echo "built $OUT/libec.so — copy it to \$CASSANDRA_HOME/lib/sigar-bin (README.md:60)"

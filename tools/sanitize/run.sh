#!/bin/bash
# Build the engine's HOST code with AddressSanitizer + UndefinedBehaviorSanitizer
# (device code is not instrumented: GPU sanitizers are unavailable on this pool)
# and run the concurrency stress driver.  Build here (no GPU needed), run on the box:
#   tools/sanitize/run.sh build     -> tools/sanitize/out/{libelect_ec_san.so,host_stress}
#   tools/sanitize/run.sh run [T] [N]
#   SANITIZER=tsan tools/sanitize/run.sh build|run   (ThreadSanitizer instead)
set -eu
cd "$(dirname "$0")/../.."
OUT=tools/sanitize/out
H=/opt/rocm/bin/hipcc
if [ "${SANITIZER:-asan}" = tsan ]; then  # ThreadSanitizer build: tools/sanitize/out_tsan
    SAN="-Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer"
    OUT=tools/sanitize/out_tsan
else
    SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
fi
case "${1:-build}" in
build)
    mkdir -p $OUT
    C="$H --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -I include $SAN"
    objs=""
    for f in ec_capi.cpp rs_kernels.hip; do
        $C -x hip -c elect_amd/csrc/$f -o $OUT/${f%.*}.o &
        objs="$objs $OUT/${f%.*}.o"
    done
    # host_path.cpp has no device code: host C++ (elect_amd/build.py HOST_SOURCES)
    $H -O1 -g -std=c++17 -fPIC -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ $SAN -x c++ \
        -c elect_amd/csrc/host_path.cpp -o $OUT/host_path.o &
    objs="$objs $OUT/host_path.o"
    for k in $(seq 1 16); do  # rs_inst.hip once per source-column count
        $C -DELECT_EC_INST_K=$k -x hip -c elect_amd/csrc/rs_inst.hip -o $OUT/rs_inst_k$k.o &
        objs="$objs $OUT/rs_inst_k$k.o"
        [ $((k % 8)) -eq 0 ] && wait
    done
    wait
    $H --offload-arch=gfx950 -shared -fPIC $SAN -o $OUT/libelect_ec_san.so $objs -L/opt/rocm/lib -lhsa-runtime64
    $H --offload-arch=gfx950 -O1 -g -std=c++17 -I include $SAN -x hip tools/sanitize/host_stress.cpp -o $OUT/host_stress \
        -L $OUT -lelect_ec_san -Wl,-rpath,'$ORIGIN' -pthread
    rm -f $OUT/*.o
    echo built $OUT/host_stress ;;
run)
    # the pool's harness preloads a library of its own, so ASan cannot come first in the link order
    ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=0 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    TSAN_OPTIONS=report_signal_unsafe=0:second_deadlock_stack=1 \
        $OUT/host_stress "${2:-24}" "${3:-12}" "${4:-1}" ;;
esac

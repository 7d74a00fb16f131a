#!/bin/bash
# Copy a `tools/gpu_run.sh final` call's artefacts from gpurun_out/ (scratch) into
# profiles/$TAG/ (tracked).   usage: TAG=r04 tools/collect_final.sh
set -eu
cd "$(dirname "$0")/.."
TAG=${TAG:-r04}
D=profiles/$TAG
mkdir -p $D/configs
line() { grep -m1 '^{' "$1"; }
[ -f gpurun_out/pytest_gpu.log ] && tail -3 gpurun_out/pytest_gpu.log > $D/pytest_gpu_final.txt
[ -f gpurun_out/smoke.log ] && grep -v amdgpu.ids gpurun_out/smoke.log > $D/smoke_final.txt
[ -f gpurun_out/bench_driver.log ] && line gpurun_out/bench_driver.log > $D/bench_final.json
[ -f gpurun_out/prof_$TAG/run_kernel_stats.csv ] && cp gpurun_out/prof_$TAG/run_kernel_stats.csv $D/kernel_stats_final.csv
if [ -d gpurun_out/pmc_fetch_$TAG ] && [ -d gpurun_out/pmc_write_$TAG ]; then
    python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG profiles/${TAG}_pmc_traffic.json
fi
for f in gpurun_out/cfg_*.log; do
    [ -e "$f" ] || continue
    n=$(basename "$f" .log); n=${n#cfg_}
    line "$f" > $D/configs/bench_$n.json || true
done
git status --short profiles

#!/bin/bash
# Copy the judged artefacts of the last gpurun call from gpurun_out/ (scratch)
# into profiles/ (tracked): bench JSON lines, rocprof kernel stats, PMC traffic,
# the GPU test summary.   usage: tools/collect_profiles.sh [TAG]
set -eu
cd "$(dirname "$0")/.."
TAG=${1:-r01}
for f in gpurun_out/bench*.log; do
    [ -e "$f" ] || continue
    name=$(basename "$f" .log)
    line=$(grep -m1 '^{' "$f" || true)
    [ -n "$line" ] && echo "$line" > "profiles/${TAG}_${name}.json"
done
if [ -f gpurun_out/prof_$TAG/run_kernel_stats.csv ]; then
    cp gpurun_out/prof_$TAG/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
fi
if [ -d gpurun_out/pmc_fetch_$TAG ] && [ -d gpurun_out/pmc_write_$TAG ]; then
    python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG profiles/${TAG}_pmc_traffic.json
fi
if [ -f gpurun_out/pytest_gpu.log ]; then
    tail -3 gpurun_out/pytest_gpu.log > profiles/${TAG}_pytest_gpu.log
fi
git status --short profiles

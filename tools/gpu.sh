#!/bin/bash
# Local wrapper: clear stale logs, run tools/gpu_run.sh steps on the GPU box, summarise.
# usage: tools/gpu.sh TIMEOUT step [step ...]
cd "$(dirname "$0")/.."
T=$1; shift
rm -f gpurun_out/*.log gpurun_out/status.txt
/usr/local/graft/bin/gpurun --timeout "$T" -- "${GPU_ENV:-} tools/gpu_run.sh $*" > /tmp/gpurun_last.log 2>&1
rc=$?
echo "gpurun exit=$rc"; sed -n 2,3p /tmp/gpurun_last.log
[ -f gpurun_out/pytest_gpu.log ] && tail -2 gpurun_out/pytest_gpu.log
python3 tools/summarize.py 2>/dev/null | grep -v start
exit $rc

# rocprofv3 kernel-trace stats of every --config line (round 4); summaries copied to profiles/r04/kernel_stats_configs/
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in "flows_elect:--config flows --chunk 4404020 --stripes 256" "hashed:--config hashed" "update:--config update" "padded:--config padded" "rs12:--config rs12" "mixed:--config mixed"; do
  n=${c%%:*}; a=${c#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cfgprof_$n -o run -- python3 $R/bench.py $a --no-cpu --no-host --steps 20 > $R/gpurun_out/cfgprof_$n.log 2>&1
done

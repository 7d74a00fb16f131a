"""Table of tools/gpu_run.sh hostreg logs (gpurun_out/bench_hostpath_reg*.log)."""
import glob, json, sys
rows = []
for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/bench_hostpath_*.log')):
    lines = [l for l in open(f) if l.startswith('{')]
    if not lines:
        print(f, "no result"); continue
    o = json.loads(lines[-1]); st = o['host_path_stats']
    gib = o['value'] * 0 + o['steps'] * o['callers'] * 4 * 4404020 / 2**30 if 'callers' in o else 1
    per = lambda k: round(st.get(k, 0) / gib, 1) if gib else None
    print(f"{f.split('/')[-1]:40s} {o['value']:7.2f} GiB/s  core-ms/GiB {o['cpu_core_ms_per_GiB']:7.1f}  ceiling {o['cpu_bound_ceiling_GiB/s']}  "
          f"reg {st.get('registered',0)} staged {st.get('batched',0)} fb {st.get('register_fallback',0)} unregfail {st.get('unregister_failures',0)}  "
          f"ms/GiB reg {per('register_cpu_ms')} unreg {per('unregister_cpu_ms')} issue {per('dispatch_issue_cpu_ms')}")

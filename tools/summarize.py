#!/usr/bin/env python3
"""Print one line per bench log under gpurun_out/ (missing logs are reported, not raised)."""
import glob
import json
import os
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for path in sorted(glob.glob(os.path.join(out, "bench*.log"))):
    line = next((l for l in open(path) if l.startswith("{")), None)
    name = os.path.basename(path)[:-4]
    if line is None:
        print(f"{name}: no JSON line ({open(path).read()[-300:]!r})")
        continue
    d = json.loads(line)
    rf = d.get("roofline") or {}
    extra = {k: d[k] for k in ("kernels", "host_inclusive_GiB/s", "cpu_baseline") if k in d}
    print(f"{name}: {d['value']} {d['unit']} verified={d.get('verified')} "
          f"roofline={rf.get('achieved')} GB/s frac={rf.get('frac')} {json.dumps(extra)[:400]}")
status = os.path.join(out, "status.txt")
if os.path.exists(status):
    print(open(status).read())

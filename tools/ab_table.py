"""Tabulate gpurun_out/ab_<variant>_<config>_<i>.log bench lines: mean value and
fractions per (variant, config).  Usage: python tools/ab_table.py"""
import collections
import glob
import json
import os

rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab_*.log")):
    v, c, _ = os.path.basename(f)[3:-4].split("_", 2) if f.count("_") >= 3 else (None, None, None)
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print("no result:", f)
        continue
    d = json.loads(lines[-1])
    fr = {n: k["frac"] for n, k in d.get("kernels", {}).items() if "frac" in k}
    fr["roof"] = (d.get("roofline") or {}).get("frac")
    rows[(c, v)].append((d["value"], fr))
for (c, v), rs in sorted(rows.items()):
    val = sum(r[0] for r in rs) / len(rs)
    keys = rs[0][1].keys()
    fr = {k: round(sum(r[1][k] or 0 for r in rs) / len(rs), 4) for k in keys}
    print(f"{c:10s} {v}  value={val:9.2f}  n={len(rs)}  {fr}")

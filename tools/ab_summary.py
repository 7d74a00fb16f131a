#!/usr/bin/env python3
"""Summarise interleaved A/B bench logs: gpurun_out/<PREFIX><variant>_<config>_<i>.log.

  python tools/ab_summary.py PREFIX      e.g. persist  ->  persist0_headline_1.log ...
Prints per (config, variant): value mean [min-max], and the kernel fractions
the lines carry (headline encode/decode, rs12 decode, mixed classes)."""
import collections
import glob
import json
import os
import statistics as st
import sys


def fracs(d):
    out = {}
    for n, k in d.get("kernels", {}).items():
        if isinstance(k, dict) and "frac" in k:
            out[n] = k["frac"]
    for n, c in d.get("classes", {}).items():
        out[f"{n}.enc"] = c["encode_frac"]
        out[f"{n}.dec"] = c["decode_frac"]
    return out


def main():
    prefix = sys.argv[1]
    rows = collections.defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/{prefix}*.log")):
        stem = os.path.basename(f)[len(prefix):-4]
        parts = stem.split("_")
        if len(parts) < 3 or not parts[-1].isdigit():
            continue
        v, c = parts[0], "_".join(parts[1:-1])
        lines = [x for x in open(f) if x.startswith("{")]
        if not lines:
            print("no result:", f)
            continue
        d = json.loads(lines[-1])
        rows[(c, v)].append((d["value"], fracs(d)))
    for (c, v), rs in sorted(rows.items()):
        vals = [r[0] for r in rs]
        fr = {k: round(st.mean(r[1][k] for r in rs if k in r[1]), 4) for k in rs[0][1]}
        print(f"{c:12s} {v:8s} value {st.mean(vals):9.2f} [{min(vals):.0f}-{max(vals):.0f}] n={len(rs)}  {fr}")


if __name__ == "__main__":
    main()

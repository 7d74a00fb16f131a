#!/usr/bin/env python3
"""Per-dispatch PMC counters joined with kernel-trace wall time (rocprofv3
--pmc ... --kernel-trace, csv).  For each pass directory: the dispatches of
kernels matching --kernel, their counters, wall time and effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / wall, MI355X_MICROARCH.md 'DVFS give-back').

  python tools/pmc_dispatch.py --kernel 'gf_apply_x16u<8, 2' [--last N] DIR [DIR ...]
"""
import argparse
import csv
import glob
import os
import statistics as st
from collections import defaultdict


def load(d, kernel):
    trace = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                trace[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ctr = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                c = ctr[r["Dispatch_Id"]]
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return trace, ctr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--bytes", type=float, default=0.0, help="algorithmic bytes per dispatch (for the HBM fraction)")
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    for d in a.dirs:
        trace, ctr = load(d, a.kernel)
        ids = sorted(set(trace) | set(ctr), key=int)[-a.last:]
        if not ids:
            print(d, "no dispatches")
            continue
        names = sorted({n for i in ids for n in ctr.get(i, {})})
        walls = [trace[i] for i in ids if i in trace]
        line = [f"{os.path.basename(d.rstrip('/'))}: {len(ids)} dispatches"]
        if walls:
            w = st.median(walls)
            line.append(f"wall {w * 1e6:.1f} us")
            if a.bytes:
                line.append(f"frac {a.bytes / w / 8e12:.4f}")
        for n in names:
            v = [ctr[i][n] for i in ids if n in ctr.get(i, {})]
            line.append(f"{n} {st.median(v):.4g}")
            if n == "GRBM_GUI_ACTIVE" and walls:
                clk = [ctr[i][n] / 8 / trace[i] / 1e9 for i in ids if i in trace and n in ctr.get(i, {})]
                line.append(f"eff_clock {st.median(clk):.3f} GHz")
        print("  ".join(line))


if __name__ == "__main__":
    main()

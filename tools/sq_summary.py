"""Summarise tools/gpu_run.sh sqpmc passes (rocprofv3 --pmc ... --kernel-trace CSVs).

  python tools/sq_summary.py gpurun_out/sqpmc_<cfg>_{A,B,C} ...   (any number of pass dirs)

For every gf_apply / gf_update / hash_reduce kernel in the passes: median over its
last 15 dispatches of each counter and of the wall time, then the derived columns
of profiles/r04/sq_bound_pmc.txt: effective clock = GRBM_GUI_ACTIVE / 8 XCDs /
wall, VALU instructions per wave, VALU busy = SQ_ACTIVE_INST_VALU x 4 / 1024
SIMDs / (wall x clock), LDS instructions per wave."""
import csv
import re
import os
import statistics
import sys
from collections import defaultdict

KEEP = ("gf_apply", "gf_update", "hash_reduce")


def short(name: str) -> str:
    m = re.search(r"(gf_\w+|hash_reduce)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")).replace(" ", "") if m else name[:60]


def load(d):
    """{kernel: {counter: [values in dispatch order]}, plus 'wall_us'}"""
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter -> value
    wall = {}
    for r in rows:
        if not any(k in r["Kernel_Name"] for k in KEEP):
            continue
        kn, disp = short(r["Kernel_Name"]), int(r["Dispatch_Id"])
        per[kn][disp][r["Counter_Name"]] = float(r["Counter_Value"])
        per[kn][disp]["grid"] = float(r["Grid_Size"])
        per[kn][disp]["wg"] = float(r["Workgroup_Size"])
    kt = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(kt):
        for r in csv.DictReader(open(kt)):
            wall[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = {}
    for kn, disps in per.items():
        last = sorted(disps)[-15:]
        agg = {}
        for c in set().union(*(disps[x].keys() for x in last)):
            agg[c] = statistics.median(disps[x][c] for x in last if c in disps[x])
        ws = [wall[x] for x in last if x in wall]
        if ws:
            agg["wall_us"] = statistics.median(ws)
        out[kn] = agg
    return out


def main(dirs):
    merged = defaultdict(dict)
    for d in dirs:
        tag = os.path.basename(d.rstrip("/"))
        for kn, agg in load(d).items():
            merged[kn][tag] = agg
    print("| kernel | pass | wall us | eff. clock GHz | waves | VALU/wave | VALU busy | LDS/wave | other counters |")
    print("|---|---|---|---|---|---|---|---|---|")
    for kn, passes in sorted(merged.items()):
        waves = next((p["SQ_WAVES"] for p in passes.values() if "SQ_WAVES" in p), None)
        if waves is None:
            g = next(iter(passes.values()))
            waves = g["grid"] / 64
        for tag, p in sorted(passes.items()):
            w = p.get("wall_us")
            clk = p["GRBM_GUI_ACTIVE"] / 8 / (w * 1e3) if w and "GRBM_GUI_ACTIVE" in p else None
            valu = p.get("SQ_INSTS_VALU")
            busy = (p["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (w * 1e-6 * clk * 1e9)
                    if "SQ_ACTIVE_INST_VALU" in p and clk else None)
            lds = p.get("SQ_INSTS_LDS")
            rest = {c: v for c, v in p.items() if c not in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_LDS",
                                                          "GRBM_GUI_ACTIVE", "wall_us", "grid", "wg", "SQ_WAVES")}
            f = lambda x, fmt: (fmt % x) if x is not None else "-"  # noqa: E731
            print(f"| {kn} | {tag} | {f(w, '%.1f')} | {f(clk, '%.2f')} | {waves:.0f} | "
                  f"{f(valu / waves if valu else None, '%.0f')} | {f(busy * 100 if busy else None, '%.0f %%')} | "
                  f"{f(lds / waves if lds else None, '%.1f')} | "
                  + ", ".join(f"{c}={v:.3g}" for c, v in sorted(rest.items())) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])

"""Summarise tools/gpu_run.sh hostab logs: one row per (variant, op, callers),
every repetition's GiB/s and core-ms per GiB (and per-call latency where the
record has it)."""
import collections
import json
import re
import sys

rows = collections.defaultdict(list)
flags = [a for a in sys.argv[1:] if a.startswith("-")]
for path in [a for a in sys.argv[1:] if not a.startswith("-")]:
    m = re.search(r"hostab_(.+)_(encode_ex|encode|decode|update)_T(\d+)_(\d+)\.log$", path)
    if not m:
        continue
    rec = None
    for line in open(path, errors="replace"):
        if line.startswith("{"):
            try:
                rec = json.loads(line)
            except ValueError:
                pass
    rows[(m.group(1), m.group(2), int(m.group(3)))].append(rec)
for (name, op, T), recs in sorted(rows.items(), key=lambda x: (x[0][1], x[0][2], x[0][0])):
    cells = []
    for r in recs:
        if not r:
            cells.append("FAIL")
            continue
        lat = r.get("call_latency_ms") or {}
        extra = f" p50 {lat['p50']:.3f} p99 {lat['p99']:.3f} ms" if lat else ""
        ok = "" if r.get("verified") else " UNVERIFIED"
        st = r.get("host_path_stats") or {}
        ph = st.get("phase_ms")
        if ph and "-v" in flags:  # per call (us): lock fill queue | per batch: issue device | per call: wake unlock
            calls = max(1, st["batched"] + st["direct"] + st["registered"])
            nb = max(1, st.get("batches", 1))
            extra += (" [us/call lock {:.0f} fill {:.0f} queue {:.0f} wake {:.0f} unlock {:.0f};"
                      " us/batch issue {:.0f} device {:.0f}; {:.1f} calls/batch]").format(
                *(ph[x] * 1e3 / calls for x in ("lock", "fill", "queue", "wake", "unlock")),
                ph["issue"] * 1e3 / nb, ph["device"] * 1e3 / nb, calls / nb)
        cells.append(f"{r['value']:6.2f} GiB/s @ {r['cpu_core_ms_per_GiB']:5.2f}{extra}{ok}")
    print(f"{op:9s} T{T:<3d} {name:14s} " + " | ".join(cells))

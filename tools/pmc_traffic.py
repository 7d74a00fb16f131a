#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
streaming read, so hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
The two counters come from separate passes (TCC slot limits).

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [--filter elect]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read(dirpath, counter, filt):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or filt not in r["Kernel_Name"]:
                continue
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    filt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else "elect"
    fetch = read(fetch_dir, "FETCH_SIZE", filt)
    write = read(write_dir, "WRITE_SIZE", filt)
    res = {}
    for name in sorted(set(fetch) | set(write)):
        fk = sum(fetch[name]) / len(fetch[name]) if fetch.get(name) else None
        wk = sum(write[name]) / len(write[name]) if write.get(name) else None
        hbm = None if fk is None or wk is None else int(round(2 * fk * 1024 + wk * 1024))
        res[name] = {"fetch_size_kb": fk, "write_size_kb": wk, "launches": len(fetch.get(name, [])),
                     "hbm_bytes_per_launch": hbm}
    doc = {"method": "hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE reports half of "
                     "a 16B/lane streaming read; MI355X_MICROARCH.md HBM section); separate --pmc passes",
           "kernels": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for n, r in res.items():
        print(n[:90], r)


if __name__ == "__main__":
    main()

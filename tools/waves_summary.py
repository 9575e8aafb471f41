#!/usr/bin/env python3
"""Table of tools/waves_sweep.sh: per resident-wave cap the bench rate and kernel time (two runs), and
the decode kernel's per-launch HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md's gfx950
correction) and clock (GRBM_GUI_ACTIVE / 8 over the kernel duration).

usage: waves_summary.py OUT_DIR caps..."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def pmc(d, counter):
    vals = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    dec = [k for k in durs if "persist" in k]
    if not dec:
        return None, None
    k = dec[0]
    xs = [v for i, v in vals.items() if names[i] == k]
    ds = durs[k]
    return (sum(xs) / len(xs) if xs else None), sum(ds) / len(ds)


def main():
    out, caps = sys.argv[1], sys.argv[2:]
    rows = []
    for w in caps:
        runs = []
        for rep in (1, 2):
            try:
                d = json.loads(open(os.path.join(out, f"bench_w{w}_{rep}.log")).read().strip().splitlines()[-1])
                runs.append((d["value"] / 1e3, d["kernel_ms"]))
            except (OSError, ValueError, IndexError, KeyError):
                pass
        fetch, ns = pmc(os.path.join(out, f"w{w}_FETCH_SIZE"), "FETCH_SIZE")
        write, _ = pmc(os.path.join(out, f"w{w}_WRITE_SIZE"), "WRITE_SIZE")
        grbm, gns = pmc(os.path.join(out, f"w{w}_GRBM_GUI_ACTIVE"), "GRBM_GUI_ACTIVE")
        hbm = (fetch * 2 + write) * 1024 if fetch is not None and write is not None else None
        rows.append({"waves_per_cu": int(w), "gbit_s": [r[0] for r in runs], "kernel_ms": [r[1] for r in runs],
                     "hbm_gb_per_launch": round(hbm / 1e9, 4) if hbm else None,
                     "fetch_gb": round(fetch * 2 * 1024 / 1e9, 4) if fetch else None,
                     "write_gb": round(write * 1024 / 1e9, 4) if write else None,
                     "clock_ghz": round(grbm / 8 / gns, 3) if grbm and gns else None})
    print(json.dumps(rows, indent=1))
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

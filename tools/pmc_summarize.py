#!/usr/bin/env python3
"""Per-launch HBM traffic of the decoder kernel from the two PMC passes of tools/pmc_traffic.sh.

Writes <root>/pmc_traffic*.json (copy it into profiles/ to have bench.py report it).
FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (summed over the XCDs' L2 channels).
MI355X_MICROARCH.md (HBM): on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide coalesced
streaming read; other widths are uncalibrated. The probe's copy kernel moves a known byte count with
wide streaming loads/stores, so its measured/known ratios are the calibration we apply.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    out = defaultdict(list)
    for d, v in vals.items():
        out[names[d]].append(v * 1024.0)
    return out


def main():
    root = sys.argv[1]
    args = sys.argv[2:]
    opt = dict(zip(args[::2], args[1::2]))
    fetch = per_kernel(os.path.join(root, "FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(root, "WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    log = open(os.path.join(root, "FETCH_SIZE.log")).read().split()
    copy_bytes = int(log[log.index("copy_bytes") + 1])
    nblocks = int(log[log.index("nblocks") + 1])
    copy_k = [k for k in fetch if "copy" in k.lower() or "elementwise" in k.lower()]
    dec_k = [k for k in fetch if "viterbi" in k]
    avg = lambda xs: sum(xs) / len(xs)   # noqa: E731
    c_fetch, c_write = avg(fetch[copy_k[0]]), avg(write[copy_k[0]])
    read_scale = copy_bytes / c_fetch          # expected ~2 on gfx950
    write_scale = copy_bytes / c_write
    d_fetch, d_write = avg(fetch[dec_k[0]]), avg(write[dec_k[0]])
    traffic = d_fetch * read_scale + d_write * write_scale
    res = {
        "workload_key": f"{opt.get('--code', 'k7')}:frames{opt.get('--frames', '64')}:{opt.get('--layout', 'block')}",
        "kernel": dec_k[0],
        "nblocks": nblocks,
        "raw_fetch_bytes_per_launch": d_fetch,
        "raw_write_bytes_per_launch": d_write,
        "calibration": {"copy_kernel": copy_k[0], "copy_bytes": copy_bytes,
                        "raw_fetch": c_fetch, "raw_write": c_write,
                        "read_scale": read_scale, "write_scale": write_scale},
        "hbm_bytes_per_launch": int(traffic),
        "note": "HBM bytes = FETCH_SIZE*1024*read_scale + WRITE_SIZE*1024*write_scale, scales from a "
                "device copy of a known byte count profiled in the same run (MI355X_MICROARCH.md: "
                "FETCH_SIZE counts half of a wide streaming read on gfx950); Infinity-Cache hits are "
                "counted by these L2-side counters",
    }
    name = "pmc_traffic.json" if res["workload_key"] == "k7:frames64:block" else \
        f"pmc_traffic_{res['workload_key'].replace(':', '_')}.json"
    with open(os.path.join(root, name), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise the three PMC passes of tools/pmc_workload.sh into per-launch figures of the workload's
dominant kernel, merged into a JSON keyed like bench.py's workload_key_of() (copy it to
profiles/pmc_workloads.json to have bench.py report traffic / traffic_frac / valu_frac).

HBM bytes = FETCH_SIZE * 1024 * read_scale + WRITE_SIZE * 1024 * write_scale, the scales from a device
copy of a known byte count profiled in the same run (MI355X_MICROARCH.md: FETCH_SIZE counts half of a
wide streaming read on gfx950). SQ / GRBM counters are the device totals rocprofv3 reports per
dispatch (GRBM_GUI_ACTIVE summed over the 8 XCDs). The kernel is the one with the largest total
duration among the probe's dispatches (the decode).

usage: pmc_workload.py PASS_DIR OUT_JSON [workload args...]
       pmc_workload.py --rederive profiles/pmc_workloads.json   (calibrations from the committed CSVs)
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def counter_rows(paths):
    """Per dispatch of the counter CSVs: {dispatch: (kernel, grid size, {counter: value})}."""
    out = {}
    for f in paths:
        for r in csv.DictReader(open(f)):
            d = r["Dispatch_Id"]
            k, g, cs = out.get(d, (r["Kernel_Name"], int(r.get("Grid_Size") or 0), defaultdict(float)))
            cs[r["Counter_Name"]] += float(r["Counter_Value"])
            out[d] = (k, g, cs)
    return out


def calibration(fetch_rows, write_rows, copy_bytes):
    """Byte scales of FETCH_SIZE and WRITE_SIZE from the run's calibration copy of copy_bytes: the
    mean over the copy kernel's dispatches of the LARGEST grid only -- the run also holds small
    copies of the same kernel (a 512-thread 1.6 KiB one), and averaging them in read 2.67 / 1.33
    instead of the true 2.00 / 1.00. None when the run holds no copy."""
    def scale(rows, counter):
        copies = [(g, cs[counter]) for k, g, cs in rows.values()
                  if ("copy" in k.lower() or "elementwise" in k.lower()) and counter in cs]
        if not copies:
            return None, None
        gmax = max(g for g, _ in copies)
        vals = [v for g, v in copies if g == gmax]
        return copy_bytes / (sum(vals) / len(vals) * 1024), len(vals)
    rs, rn = scale(fetch_rows, "FETCH_SIZE")
    ws, wn = scale(write_rows, "WRITE_SIZE")
    if rs is None or ws is None:
        return None
    return {"read_scale": rs, "write_scale": ws, "copies_averaged": [rn, wn],
            "rule": "copy dispatches of the largest grid only"}


def counters(pass_dir):
    """{kernel: {counter: [per-dispatch value]}}, {kernel: [duration ns]}"""
    vals = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = r["Dispatch_Id"]
            vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(pass_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = defaultdict(lambda: defaultdict(list))
    for d, cs in vals.items():
        for c, v in cs.items():
            out[names[d]][c].append(v)
    return out, durs


def avg(xs):
    return sum(xs) / len(xs) if xs else None


GUIDE_READ_SCALE, GUIDE_WRITE_SCALE = 2.0, 1.0


def committed_csvs(source):
    """The committed FETCH / WRITE CSVs a pmc_workloads.json record names in its "source" field
    ("profiles/r0N_pmc/<tag>_{FETCH,...}.csv", or a gpurun_out pass directory "committed as
    profiles/r0N_pmc/<tag>_{...}.csv" with <tag> its basename). (fetch, write) paths or None."""
    import re
    m = re.search(r"(profiles/r0\d_pmc/)(\S*?)_\{FETCH,WRITE", source)
    if not m:
        return None
    prefix = m.group(2)
    if prefix == "<tag>":
        prefix = os.path.basename(source.split(" ")[0])
    base = os.path.join(REPO, m.group(1) + prefix)
    paths = (base + "_FETCH.csv", base + "_WRITE.csv")
    return paths if all(os.path.exists(p) for p in paths) else None


def rederive(json_path):
    """Recompute the calibration field of every record from its committed CSVs (the largest-grid
    rule); the traffic figures use the guide's scales and do not change."""
    doc = json.load(open(json_path))
    for key, rec in sorted(doc.items()):
        paths = committed_csvs(rec.get("source", ""))
        old = rec.get("calibration") or {}
        if not paths or "copy_bytes" not in old:
            print(f"{key}: no committed CSVs found, calibration left as is")
            continue
        cal = calibration(counter_rows([paths[0]]), counter_rows([paths[1]]), old["copy_bytes"])
        if cal:
            rec["calibration"] = {"copy_kernel": old.get("copy_kernel"), "copy_bytes": old["copy_bytes"], **cal}
        print(f"{key}: read_scale {old.get('read_scale', 0):.3f} -> {cal and cal['read_scale']:.4f}, "
              f"write_scale {old.get('write_scale', 0):.3f} -> {cal and cal['write_scale']:.4f}")
    with open(json_path, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--rederive":
        return rederive(sys.argv[2])
    root, out_json = sys.argv[1], sys.argv[2]
    ap = argparse.ArgumentParser()
    for a, d in (("--code", None), ("--frames", "104"), ("--layout", "block"), ("--channel", "awgn"),
                 ("--decoder", "viterbi"), ("--ebn0", "4.0"), ("--p-ppm", "50000"), ("--reps", "3")):
        ap.add_argument(a, default=d)
    ap.add_argument("--iq", action="store_true")
    args = ap.parse_args(sys.argv[3:])
    args.code = args.code or ("k7" if args.decoder == "viterbi" else "k15")
    args.frames = int(args.frames)
    import bench
    key = bench.workload_key_of(args) + (":iq" if args.iq else "")
    fetch, durs = counters(os.path.join(root, "FETCH"))
    write, _ = counters(os.path.join(root, "WRITE"))
    sq, sq_durs = counters(os.path.join(root, "SQ"))
    stall, _ = counters(os.path.join(root, "STALL"))
    copy_k = [k for k in fetch if "copy" in k.lower() or "elementwise" in k.lower()]
    dec_k = max((k for k in durs if k not in copy_k), key=lambda k: sum(durs[k]))
    log = open(os.path.join(root, "FETCH.log")).read().split()
    copy_bytes = int(log[log.index("copy_bytes") + 1])
    cal = calibration(
        counter_rows(glob.glob(os.path.join(root, "FETCH", "**", "*counter_collection.csv"), recursive=True)),
        counter_rows(glob.glob(os.path.join(root, "WRITE", "**", "*counter_collection.csv"), recursive=True)),
        copy_bytes)
    d_fetch = avg(fetch[dec_k]["FETCH_SIZE"]) * 1024
    d_write = avg(write[dec_k]["WRITE_SIZE"]) * 1024
    rec = {
        "kernel": dec_k,
        "launches_profiled": len(durs[dec_k]),
        "kernel_ns": avg(sq_durs.get(dec_k, durs[dec_k])),
        # the guide's correction (MI355X_MICROARCH.md HBM/rocprofv3: FETCH_SIZE x 2 on gfx950,
        # WRITE_SIZE exact), which the in-run copy calibration reproduces (2.00 / 1.00)
        "hbm_bytes_per_launch": int(d_fetch * GUIDE_READ_SCALE + d_write * GUIDE_WRITE_SCALE),
        "raw_fetch_bytes_per_launch": d_fetch, "raw_write_bytes_per_launch": d_write,
        "calibration": {"copy_kernel": copy_k[0], "copy_bytes": copy_bytes, **(cal or {})},
        "source": os.path.relpath(root) + " (committed as profiles/r05_pmc/<tag>_{FETCH,WRITE,SQ,STALL}.csv)",
    }
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_BUSY_CYCLES",
              "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"):
        v = avg(sq[dec_k].get(c, []))
        if v is not None:
            rec[c.lower()] = v
    st = {}
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_WAVE_CYCLES"):
        v = avg(stall.get(dec_k, {}).get(c, []))
        if v is not None:
            st[c.lower()] = v
    if st.get("sq_wave_cycles"):
        # disjoint split of wave lifetime (MI355X_MICROARCH.md PMC table): parked on s_waitcnt /
        # barrier, issue-stalled, issuing
        for c in ("sq_wait_any", "sq_wait_inst_any", "sq_active_inst_any"):
            if c in st:
                st[c + "_frac"] = st[c] / st["sq_wave_cycles"]
        rec["stall"] = st
    if rec.get("sq_insts_valu") and rec.get("grbm_gui_active"):
        rec["valu_frac"] = rec["sq_insts_valu"] / (512.0 * rec["grbm_gui_active"] / 8.0)
        rec["clock_ghz"] = rec["grbm_gui_active"] / 8.0 / rec["kernel_ns"]
    try:
        doc = json.load(open(out_json))
    except (OSError, ValueError):
        doc = {}
    doc[key] = rec
    os.makedirs(os.path.dirname(os.path.abspath(out_json)), exist_ok=True)
    with open(out_json, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print(key, json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()

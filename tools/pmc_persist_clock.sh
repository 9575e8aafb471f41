#!/bin/bash
# Clock (GRBM_GUI_ACTIVE / duration / 8 XCDs) and VALU counts per persist_bench kernel variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_persist
mkdir -p $OUT
for set in "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES" "SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- \
      ./tools/persist_bench > $OUT/$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $OUT/$tag.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list)); dur = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/*/run_kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        dur[f][r["Dispatch_Id"]] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    tf = f.replace("counter_collection", "kernel_trace")
    for r in csv.DictReader(open(f)):
        name, d = dur[tf][r["Dispatch_Id"]]
        key = name[name.find("Li40E"):][:24] + (" true" if "Li1EEELi40" in name else " ref")
        rows[key][r["Counter_Name"]].append((float(r["Counter_Value"]), d))
for k, cs in sorted(rows.items()):
    out = []
    for c, v in sorted(cs.items()):
        val = sorted(x for x, _ in v)[len(v) // 2]
        d = sorted(y for _, y in v)[len(v) // 2]
        out.append(f"{c}={val:.4g}" + (f" ({val / d / 8:.3f} GHz, dur {d/1e3:.0f} us)" if c == "GRBM_GUI_ACTIVE" else ""))
    print(k, " ".join(out))
PY

#!/bin/bash
# Clock (GRBM_GUI_ACTIVE / duration / 8 XCDs) and VALU counts per persist_bench kernel variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_persist
mkdir -p $OUT
SETS=${PMC_SETS:-"GRBM_GUI_ACTIVE,SQ_INSTS_VALU,SQ_WAVES;SQ_BUSY_CU_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU"}
IFS=';' read -ra SETLIST <<< "$SETS"
for set in "${SETLIST[@]}"; do
  set=${set//,/ }
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- \
      ./tools/persist_bench > $OUT/$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $OUT/$tag.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, re, sys
OUT = sys.argv[1]
dur = {}
for f in glob.glob(OUT + "/*/run_kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        dur[(f.split('/')[-2], r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                    r.get("Grid_Size_X") or r.get("Grid_Size"))
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(OUT + "/*/run_counter_collection.csv"):
    tag = f.split('/')[-2]
    for r in csv.DictReader(open(f)):
        name, d, grid = dur[(tag, r["Dispatch_Id"])]
        m = re.search(r', 40, (\d+)>', name)
        key = ("true" if "ul}, 1}" in name else "ref", m.group(1) if m else "?", grid)
        rows[key][r["Counter_Name"]].append((float(r["Counter_Value"]), d))
for k, cs in sorted(rows.items()):
    out = []
    for c, v in sorted(cs.items()):
        val = sorted(x for x, _ in v)[len(v) // 2]
        d = sorted(y for _, y in v)[len(v) // 2]
        out.append(f"{c}={val:.4g}" + (f" ({val / d / 8:.3f} GHz, {d / 1e3:.0f}us)" if c == "GRBM_GUI_ACTIVE" else ""))
    print("ablate", k, " ".join(out))
PY

#!/bin/bash
# Clock and busy counters of one bench.py kernel (one counter set per rocprofv3 pass).
# Usage: tools/pmc_clock.sh TAG KERNEL_SUBSTRING bench.py-args...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; KSUB=$2; shift 2
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
for set in "GRBM_COUNT GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU" "SQ_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- \
      python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fused-channel "$@" > $OUT/$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $OUT/$tag.log; continue; }
done
python3 - "$OUT" "$KSUB" <<'PY'
import csv, sys, glob, collections
acc = collections.defaultdict(float); n = collections.Counter(); dur = []
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for f in glob.glob(sys.argv[1] + "/*/run_kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r.get("Kernel_Name", ""):
            dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
d = sorted(dur)[len(dur) // 2] if dur else 0
print(f"median kernel duration {d/1e3:.1f} us over {len(dur)} launches")
for k in sorted(acc):
    v = acc[k] / n[k]
    print(f"{k:24s} {v:.4g}" + (f"   -> {v / d:.3f} per ns" if d and k.startswith("GRBM") else ""))
PY

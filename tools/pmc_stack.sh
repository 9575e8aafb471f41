#!/bin/bash
# Occupancy / instruction-mix counters for the stack decoder (bench.py --decoder stack), one counter
# set per rocprofv3 pass (kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_stack
mkdir -p $OUT
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_LEVEL_WAVES"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- \
      python bench.py --decoder stack --frames 4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
done
for f in $(find $OUT -name '*counter_collection.csv'); do
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(float)
for r in rows:
    if "stack_decode" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[1].split("/")[-3], dict(acc))
PY
done

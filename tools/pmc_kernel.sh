#!/bin/bash
# Occupancy / instruction-mix counters for one kernel of a bench.py run, one counter set per
# rocprofv3 pass (kernel trace only). Usage: tools/pmc_kernel.sh TAG KERNEL_SUBSTRING bench.py-args...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; KSUB=$2; shift 2
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_LEVEL_WAVES"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- \
      python bench.py "$@" > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
done
for f in $(find $OUT -name '*counter_collection.csv'); do
  python3 - "$f" "$KSUB" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(float)
n = set()
for r in rows:
    if sys.argv[2] in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n.add(r.get("Dispatch_Id"))
print(f"{len(n)} dispatches", {k: f"{v:.4g}" for k, v in acc.items()})
PY
done

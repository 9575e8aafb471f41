#!/bin/bash
# Instruction-fetch counters (i-cache hits/misses, fetch stalls) of the K=7 bench kernel, one counter
# set per rocprofv3 pass. Usage: tools/pmc_icache.sh [traffic_probe.py args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_icache
mkdir -p $OUT
ARGS="${*:---code k7 --frames 64 --layout block}"
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o 'SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z0-9_]*\|SQ_WAIT_INST[A-Z0-9_]*\|SQ_INST_LEVEL[A-Z_]*' $OUT/avail.txt | sort -u > $OUT/names.txt || true
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU" \
           "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_WAVES"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- \
      python tools/traffic_probe.py $ARGS > $OUT/$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $OUT/$tag.log; continue; }
done
for f in $(find $OUT -name '*counter_collection.csv'); do
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", "")
    if "viterbi" in k:
        acc[(k[:60], r["Counter_Name"])] += float(r["Counter_Value"]); n[(k[:60], r["Counter_Name"])] += 1
for (k, c), v in sorted(acc.items()):
    print(f"{k:60s} {c:28s} {v/n[(k,c)]:.4g} per dispatch ({n[(k,c)]} dispatches)")
PY
done

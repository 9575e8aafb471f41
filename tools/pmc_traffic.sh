#!/bin/bash
# Two rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE: they cannot share a pass on gfx950) over
# tools/traffic_probe.py, then tools/pmc_summarize.py -> profiles/pmc_traffic*.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
ARGS="${*:---code k7 --frames 104 --layout block}"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $OUT/$ctr -o run -- \
      python tools/traffic_probe.py $ARGS > $OUT/$ctr.log 2>&1 || { tail -20 $OUT/$ctr.log; exit 1; }
done
python tools/pmc_summarize.py $OUT $ARGS

#!/bin/bash
# Resident-wave cap of the persistent K=7 kernel vs its HBM traffic and time:
# for each cap W (CCV_PERSIST_WAVES_PER_CU) a short bench.py run (kernel time, Gbit/s) and one
# FETCH_SIZE / WRITE_SIZE / GRBM pass over tools/traffic_probe.py. Logs in gpurun_out/waves/.
# Usage: tools/waves_sweep.sh [caps...]   (default 8 6 5 4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
OUT=gpurun_out/waves
mkdir -p $OUT
CAPS="${*:-8 6 5 4}"
for w in $CAPS; do
  for rep in 1 2; do
    CCV_PERSIST_WAVES_PER_CU=$w timeout -k 10 240 python bench.py --steps 20 --no-cpu-baseline \
        --no-fused-channel > $OUT/bench_w${w}_$rep.log 2>&1 || { echo "bench w=$w failed"; tail -5 $OUT/bench_w${w}_$rep.log; exit 1; }
    echo "w=$w rep=$rep $(tail -1 $OUT/bench_w${w}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_ms"])')"
  done
done
for w in $CAPS; do
  for pass in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
    CCV_PERSIST_WAVES_PER_CU=$w timeout -k 10 240 rocprofv3 --kernel-trace --pmc $pass --output-format csv \
        -d $OUT/w${w}_$pass -o run -- python3 tools/traffic_probe.py --reps 5 > $OUT/w${w}_$pass.log 2>&1 \
        || { echo "pmc w=$w $pass failed"; tail -5 $OUT/w${w}_$pass.log; exit 1; }
  done
done
python3 tools/waves_summary.py $OUT $CAPS

#!/bin/bash
# Round-robin A/B of bench.py over builds: tools/ab_bench.sh "bench args" NAME... (NAME "head" = the
# working tree's lib/, others = convolutional-codes_amd/build_ab/NAME/lib). REPS rounds (default 3);
# prints value and kernel_ms per run. Logs in gpurun_out/ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=$1; shift
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-3}); do
  for name in "$@"; do
    if [ "$name" = head ]; then dir=$PWD/convolutional-codes_amd/lib; else dir=$PWD/convolutional-codes_amd/build_ab/$name/lib; fi
    log=gpurun_out/ab/${TAG:-ab}_${name}_$rep.log
    CCV_LIB_DIR=$dir timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-fused-channel --no-hbm-probe > $log 2>&1 \
        || { echo "$name failed"; tail -5 $log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('$name rep $rep', d['value'], d['kernel_ms'])"
  done
done

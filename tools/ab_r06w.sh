#!/bin/bash
# Round-6 A/B: the headline soft kernel at 3 waves per SIMD on the group queue (build_ab/w3) against
# production, and the BSC K=7 kernel capped at 2 waves per SIMD (CCV_PERSIST_WAVES_PER_CU=8) against
# its 3. Logs in gpurun_out/ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
TAG=w3 REPS=3 bash tools/ab_bench.sh "" head w3 || exit 1
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for cap in 0 8; do
    log=gpurun_out/ab/bscw_${cap}_$rep.log
    if [ $cap = 0 ]; then env_cap=""; else env_cap="CCV_PERSIST_WAVES_PER_CU=$cap"; fi
    env $env_cap timeout -k 10 200 python bench.py --channel bsc --no-cpu-baseline --no-fused-channel --no-hbm-probe --curve-frames 0 > $log 2>&1 || { tail -5 $log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('bsc cap $cap rep $rep', d['value'], d['kernel_ms'])"
  done
done

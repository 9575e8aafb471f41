#!/bin/bash
# Fano soft: received-row access mode A/B at the bench size with the round-2 queue order
# (CCV_FANO_ROWS: 0 direct (default for soft), 2 prefetched from global memory, 1 LDS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
for db in 6 4; do
  for rm in 0 2 1; do
    CCV_FANO_ROWS=$rm timeout -k 10 600 python bench.py --decoder fano --ebn0 $db --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_fano_rm_${db}_$rm.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('$O/bench_fano_rm_${db}_$rm.log').read().strip().splitlines()[-1])
print('fano $db dB rows=$rm', d['value'], 'Mbit/s', d['kernel_ms'], 'ms')"
  done
done

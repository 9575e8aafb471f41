#!/bin/bash
# Persistent-kernel occupancy study: bench at 8/12 waves per CU + PMC of the soft kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for w in 8 12 4; do
  CCV_PERSIST_WAVES_PER_CU=$w timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fused-channel > $OUT/bench_w$w.log 2>&1 || exit $?
  CCV_PERSIST_WAVES_PER_CU=$w timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fused-channel --channel bsc > $OUT/bench_bsc_w$w.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('$OUT/bench_w$w.log').read().strip().splitlines()[-1]); e=json.loads(open('$OUT/bench_bsc_w$w.log').read().strip().splitlines()[-1])
print('waves/CU $w soft', d['value'], d['kernel_ms'], 'bsc', e['value'], e['kernel_ms'])"
done
bash tools/pmc_icache.sh > $OUT/pmc_icache.log 2>&1; tail -12 $OUT/pmc_icache.log

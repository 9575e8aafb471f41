#!/bin/bash
# Stack decoder session: parity tests, then the config-5 bench (AWGN and BSC) with the four-rows
# kernel and, for A/B, the one-search-per-wave kernel (CCV_STACK_WAVE=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_stack.log 2>&1
rc=$?; tail -3 $O/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
for ch in awgn bsc; do
  CCV_STACK_DEBUG=1 timeout -k 10 300 python bench.py --decoder stack --frames ${FRAMES:-4} --steps 5 --warmup 1 --channel $ch > $O/bench_stack_$ch.log 2>&1 || exit 1
  CCV_STACK_WAVE=1 timeout -k 10 300 python bench.py --decoder stack --frames ${FRAMES:-4} --steps 5 --warmup 1 --channel $ch --no-cpu-baseline > $O/bench_stack_wave_$ch.log 2>&1 || exit 1
  python3 -c "
import json
for tag in ('', 'wave_'):
    d=json.loads(open('$O/bench_stack_'+tag+'$ch.log').read().strip().splitlines()[-1])
    print('$ch', tag or 'rows', d['value'], d['kernel_ms'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
done
grep -h "stack rows" $O/bench_stack_awgn.log | head -2

#!/bin/bash
# Focused GPU session: new-kernel parity tests, then A/B benches (persistent on/off), soft and BSC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "${TESTS_K:-persistent or selected or dropped}" > $OUT/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
for v in on off; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fused-channel --persistent $v > $OUT/bench_soft_$v.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fused-channel --channel bsc --persistent $v > $OUT/bench_bsc_$v.log 2>&1 || exit $?
done
for f in soft_on soft_off bsc_on bsc_off; do python3 -c "
import json,sys; d=json.loads(open('$OUT/bench_$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['kernel_ms'], d['config']['variant'], d['roofline']['frac'], d['ber']['ber'])"; done

#!/bin/bash
# Stack-decoder variants on the GPU: parity tests with the default kernel and with 8 lanes per
# search, then the config-5 bench for each variant (CCV_STACK_ROWL = lanes per search,
# CCV_STACK_SYMTAB=0: parities per iteration instead of the expected-symbol table).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_stack.log 2>&1
rc=$?; tail -2 $O/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
CCV_STACK_ROWL=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_stack_rl8.log 2>&1
rc=$?; tail -2 $O/pytest_stack_rl8.log; [ $rc -ne 0 ] && exit $rc
for ch in awgn bsc; do
  for v in "16 1" "16 0" "8 1" "8 0"; do
    set -- $v
    CCV_STACK_DEBUG=1 CCV_STACK_ROWL=$1 CCV_STACK_SYMTAB=$2 timeout -k 10 300 python bench.py --decoder stack --frames ${FRAMES:-4} --steps 5 --warmup 1 --channel $ch --no-cpu-baseline > $O/bench_stack_${ch}_$1_$2.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('$O/bench_stack_${ch}_$1_$2.log').read().strip().splitlines()[-1])
print('$ch rl=$1 table=$2', d['value'], d['kernel_ms'])"
    grep -h "stack rows" $O/bench_stack_${ch}_$1_$2.log | head -1
  done
done

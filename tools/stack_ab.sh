#!/bin/bash
# Stack-decoder variants on the GPU: parity tests with the default kernels and with the alternative
# rows variants (16 lanes per search and no packed keys for hard input), then the config-5 bench per
# variant. Variables: CCV_STACK_ROWL = lanes per search, CCV_STACK_SYMTAB=0 parities per iteration,
# CCV_STACK_KEYS=0 separate metric and index reductions (hard input).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_stack.log 2>&1
rc=$?; tail -2 $O/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
CCV_STACK_ROWL=16 CCV_STACK_KEYS=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_stack_alt.log 2>&1
rc=$?; tail -2 $O/pytest_stack_alt.log; [ $rc -ne 0 ] && exit $rc
i=0
while read -r ch rl tab keys; do
  [ -z "$ch" ] && continue
  i=$((i+1))
  log=$O/bench_stack_ab_$i.log
  CCV_STACK_DEBUG=1 CCV_STACK_ROWL=$rl CCV_STACK_SYMTAB=$tab CCV_STACK_KEYS=$keys timeout -k 10 300 python bench.py --decoder stack --frames ${FRAMES:-4} --steps 5 --warmup 1 --channel $ch --no-cpu-baseline > $log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('$ch rl=$rl table=$tab keys=$keys', d['value'], 'Mbit/s', d['kernel_ms'], 'ms')"
  grep -h "stack rows" $log | head -1
done <<EOF
${VARIANTS:-awgn 16 1 1
bsc 8 1 1
bsc 8 1 0
bsc 16 1 1}
EOF

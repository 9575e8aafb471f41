#!/bin/bash
# stack + Fano parity after a change to the shared symbol table / record layout, then the benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack.py tests/test_gpu_fano.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_pack.log 2>&1
rc=$?; tail -2 $O/pytest_pack.log; [ $rc -ne 0 ] && exit $rc
for ch in awgn bsc; do
  CCV_STACK_DEBUG=1 timeout -k 10 300 python bench.py --decoder stack --frames 4 --steps 5 --warmup 1 --channel $ch --no-cpu-baseline > $O/bench_pack_$ch.log 2>&1 || exit 1
  grep -h "stack rows" $O/bench_pack_$ch.log | head -1
  grep -h '"metric"' $O/bench_pack_$ch.log | cut -c1-140
done
timeout -k 10 600 python bench.py --decoder fano --ebn0 6 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_pack_fano6.log 2>&1 || exit 1
grep -h '"metric"' $O/bench_pack_fano6.log | cut -c1-140

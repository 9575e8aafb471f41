set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_stack.log 2>&1
rc=$?; tail -3 $O/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
for ch in awgn bsc; do
  timeout -k 10 300 python bench.py --decoder stack --frames 4 --steps 5 --warmup 1 --channel $ch > $O/bench_stack_$ch.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/bench_stack_$ch.log').read().strip().splitlines()[-1]); print('$ch', d['value'], d['kernel_ms'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
done

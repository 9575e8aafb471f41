set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 ./tools/persist_bench ab > $O/persist_bench.txt 2>&1 || exit 1
cat $O/persist_bench.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused-channel > $O/bench_soft.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused-channel --channel bsc > $O/bench_bsc.log 2>&1 || exit 1
for f in soft bsc; do python3 -c "
import json; d=json.loads(open('$O/bench_$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['kernel_ms'], d['config']['variant'], d['roofline']['frac'])"; done

set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 ./tools/persist_bench abh > $O/persist_abh.txt 2>&1 || exit 1
tail -2 $O/persist_abh.txt
for c in "soft:" "bsc:--channel bsc" "k9:--code k9 --frames 16"; do
  tag=${c%%:*}; args=${c#*:}
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused-channel $args > $O/bench_$tag.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/bench_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['kernel_ms'], d['config']['variant'], d['roofline']['frac'])"
done

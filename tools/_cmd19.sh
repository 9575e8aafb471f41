set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "channel or device or simulate or sim" > $O/pytest_ch.log 2>&1
rc=$?; tail -3 $O/pytest_ch.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 ./tools/divcheck > $O/divcheck.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_ch.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads(open('$O/bench_ch.log').read().strip().splitlines()[-1]); print(d['value'], d['fused_channel'])"

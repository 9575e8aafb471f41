set -u
O=gpurun_out
timeout -k 10 60 ./tools/raterbench7 > $O/rates7.txt 2>&1 || exit 1
tail -7 $O/rates7.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for d in register hbm; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --decisions $d > $O/bench_ch_$d.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/bench_ch_$d.log').read().strip().splitlines()[-1]); print('$d', d['value'], d['fused_channel'])"
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --channel bsc > $O/bench_ch_bsc.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads(open('$O/bench_ch_bsc.log').read().strip().splitlines()[-1]); print('bsc', d['value'], d['fused_channel'])"

set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "device_channel" > $O/pytest_ch.log 2>&1
rc=$?; tail -3 $O/pytest_ch.log; [ $rc -ne 0 ] && exit $rc
for ch in awgn bsc; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --channel $ch > $O/bench_ch_$ch.log 2>&1 || exit 1
  CCV_CHANNEL_LDS_DECISIONS=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --channel $ch > $O/bench_ch_${ch}_lds.log 2>&1 || exit 1
  for f in $ch ${ch}_lds; do python3 -c "
import json; d=json.loads(open('$O/bench_ch_$f.log').read().strip().splitlines()[-1]); print('$f', d['fused_channel']['mbit_s'], d['fused_channel']['kernel_ms'])"; done
done

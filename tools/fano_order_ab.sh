#!/bin/bash
# Fano noisiest-first queue order: probe (do noise scores predict long searches?), parity tests with
# the order, then the soft bench with and without it (CCV_FANO_ORDER=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
CCV_FANO_ORDER=0 timeout -k 10 300 python tools/fano_order_probe.py > $O/fano_order_probe.txt 2>&1 || { tail $O/fano_order_probe.txt; exit 1; }
cat $O/fano_order_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_fano.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_fano.log 2>&1
rc=$?; tail -2 $O/pytest_fano.log; [ $rc -ne 0 ] && exit $rc
for db in 4 6; do
  for ord in 1 0; do
    CCV_FANO_DEBUG=1 CCV_FANO_ORDER=$ord timeout -k 10 600 python bench.py --decoder fano --ebn0 $db --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_fano_ord_${db}_$ord.log 2>&1 || exit 1
    grep -h "lane utilisation" $O/bench_fano_ord_${db}_$ord.log | tail -1
    python3 -c "
import json; d=json.loads(open('$O/bench_fano_ord_${db}_$ord.log').read().strip().splitlines()[-1])
print('fano $db dB order=$ord', d['value'], 'Mbit/s', d['kernel_ms'], 'ms')"
  done
done

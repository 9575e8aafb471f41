#!/bin/bash
# Fano decoder: parity tests with the default kernel (expected-symbol table) and with
# CCV_FANO_SYMTAB=0 (parities per pass), then the bench (soft 4 dB and 6 dB, BSC) for both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fano.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_fano.log 2>&1
rc=$?; tail -2 $O/pytest_fano.log; [ $rc -ne 0 ] && exit $rc
CCV_FANO_SYMTAB=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_fano.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "seeded or golden" > $O/pytest_fano_notab.log 2>&1
rc=$?; tail -2 $O/pytest_fano_notab.log; [ $rc -ne 0 ] && exit $rc
for args in "--ebn0 4" "--ebn0 6" "--channel bsc"; do
  for tab in 1 0; do
    tag=$(echo "$args" | tr -d ' -')_$tab
    CCV_FANO_SYMTAB=$tab timeout -k 10 600 python bench.py --decoder fano $args --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_fano_ab_$tag.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('$O/bench_fano_ab_$tag.log').read().strip().splitlines()[-1])
print('fano $args table=$tab', d['value'], 'Mbit/s', d['kernel_ms'], 'ms')"
  done
done

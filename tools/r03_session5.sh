#!/bin/bash
# Fano two-pass: parity tests, lane utilisation (CCV_FANO_DEBUG) and benches with and without the
# second pass at 4 and 6 dB and BSC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fano.py -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $OUT/pytest_fano.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_fano.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cap in 0 default; do
  if [ $cap = default ]; then unset CCV_FANO_CAP; else export CCV_FANO_CAP=$cap; fi
  CCV_FANO_DEBUG=1 timeout -k 10 300 python bench.py --decoder fano --steps 1 --warmup 0 --no-cpu-baseline --frames 104 \
      > $OUT/fano_dbg_$cap.log 2>&1 || { tail $OUT/fano_dbg_$cap.log; exit 1; }
  grep "fano:" $OUT/fano_dbg_$cap.log | tail -2
  timeout -k 10 600 python bench.py --decoder fano --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_fano_$cap.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --decoder fano --ebn0 6 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_fano6_$cap.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --decoder fano --channel bsc --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_fano_bsc_$cap.log 2>&1 || exit 1
  for f in bench_fano_$cap bench_fano6_$cap bench_fano_bsc_$cap; do echo "$f $(tail -1 $OUT/$f.log | cut -c70-150)"; done
done
exit 0

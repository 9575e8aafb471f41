#!/bin/bash
# K=9 traceback A/B + ablations, streaming-shim latency, then the K=9 / shim / persistent GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./tools/k9_bench 16 > $OUT/k9_bench.txt 2>&1; rc=$?; cat $OUT/k9_bench.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shim_latency.py 2000 > $OUT/shim_latency.txt 2>&1; rc=$?; cat $OUT/shim_latency.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "k9 or multi or persistent or shim or golden or ragged or streaming or reference" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
exit $rc

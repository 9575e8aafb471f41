#!/bin/bash
# Full GPU test suite + smoke on the current build, then the K=9 / headline / BSC benches and the
# K=9 PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && { tail -30 $OUT/smoke.log; exit $rc; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --code k9 --frames 16 --no-cpu-baseline > $OUT/bench_k9.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --channel bsc > $OUT/bench_bsc.log 2>&1 || exit 1
for f in bench bench_k9 bench_bsc; do tail -1 $OUT/$f.log | cut -c1-300; done
bash tools/pmc_workload.sh --code k9 --frames 16 > $OUT/pmc_k9.log 2>&1; tail -3 $OUT/pmc_k9.log
exit 0

#!/bin/bash
# Round-3 GPU session: smoke -> GPU tests -> bench -> BER curves. Each GPU step has its own time
# limit; a crash / timeout stops the session (a test FAILURE does not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && { tail -30 $OUT/smoke.log; exit $rc; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ "${PHASE:-all}" = tests ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 $OUT/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
bash tools/ber_curves.sh 1

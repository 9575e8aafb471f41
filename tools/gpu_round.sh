#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel trace of the bench.
# Stops at the first crash / timeout (a test FAILURE, exit 1, does not stop the session).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-20}
# PHASE=tests: smoke + parity tests only; PHASE=bench: benches + rocprof only; default: both
if [ "${PHASE:-all}" != bench ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && { tail -30 $OUT/smoke.log; exit $rc; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ "${PHASE:-all}" = tests ] && exit $rc
fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 > $OUT/bench.log 2>&1 && timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 --layout step --no-cpu-baseline > $OUT/bench_step.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --code k9 --frames 16 --steps $STEPS --warmup 3 --no-cpu-baseline > $OUT/bench_k9.log 2>&1 && \
timeout -k 10 300 python bench.py --channel bsc --steps $STEPS --warmup 3 > $OUT/bench_bsc.log 2>&1 && \
timeout -k 10 300 python bench.py --decoder stack --frames 4 --steps 5 --warmup 1 > $OUT/bench_stack.log 2>&1 && \
timeout -k 10 600 python bench.py --decoder fano --steps 3 --warmup 1 > $OUT/bench_fano.log 2>&1 && \
timeout -k 10 600 python bench.py --decoder fano --channel bsc --steps 3 --warmup 1 > $OUT/bench_fano_bsc.log 2>&1
rc=$?; echo "extra benches rc=$rc"; for f in k9 bsc stack fano fano_bsc; do echo "$f: $(tail -1 $OUT/bench_$f.log | cut -c60-140)"; done; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python bench.py --steps $STEPS --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/prof.log; exit $rc; }
find $OUT/prof -name '*stats*' | head
exit 0

#!/bin/bash
# One GPU-box session over the committed build: smoke -> every GPU test -> the bench of every
# BASELINE config (+ Fano) -> rocprofv3 kernel stats of the headline bench. Each GPU step has its own
# time limit; a crash / timeout stops the session (test FAILURES do not). PHASE=tests / bench limits
# it to one half. Logs in gpurun_out/ (copy what is judged into profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
OUT=gpurun_out
mkdir -p $OUT
if [ "${PHASE:-all}" != bench ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && { tail -30 $OUT/smoke.log; exit $rc; }
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ "${PHASE:-all}" = tests ] && exit $rc
fi
run() {   # name, limit, bench.py args
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > $OUT/bench_$name.log 2>&1 || { echo "bench $name failed"; tail -5 $OUT/bench_$name.log; exit 1; }
  echo "$name: $(tail -1 $OUT/bench_$name.log | cut -c90-200)"
}
run k7 300                                                     # config 2 (headline)
run k7_step 300 --layout step --no-cpu-baseline
run bsc 300 --channel bsc                                      # config 4
run code0_bsc 300 --code code0 --channel bsc                   # config 1 code at GPU scale
run k9 300 --code k9 --frames 32                               # config 3 (port + AVX2 baselines)
run k7_true 300 --code k7:true                                 # textbook (171,133)
run k9_true 300 --code k9:true --frames 32                     # textbook (561,753)
run stack 300 --decoder stack --frames 16 --steps 5 --warmup 1  # config 5 (16 frames: DESIGN 4.5)
run stack_bsc 300 --decoder stack --channel bsc --frames 16 --steps 5 --warmup 1
run fano 600 --decoder fano --steps 3 --warmup 1 --no-cpu-baseline
run fano_bsc 600 --decoder fano --channel bsc --steps 3 --warmup 1 --no-cpu-baseline
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/prof.log; exit $rc; }
cut -c1-160 $OUT/prof/run_kernel_stats.csv | head -6
exit 0

#!/bin/bash
# One GPU-box session over the committed build, in phases (PHASE = a comma list, default
# "tests,bench,prof"):
#   tests     smoke, then every GPU test
#   bench     the bench line of every BASELINE config (+ the textbook codes, Fano), CPU baselines
#   prof      rocprofv3 kernel stats of the headline bench
#   sweeps    Eb/N0 sweeps of configs 2 and 3 with the on-device channel (800 M bits per point)
#   noise     the same sweeps (k9, k7, seed-paired) with the opt-in fp32 Box-Muller against the default
#             double one (tools/noise_compare.py), and the exhaustive fp32 error check
#             (tools/chanmath_f32_check, built on the CPU side beforehand)
#   refdriver the unchanged reference AWGN driver (AWGN-channel/main.c) over libccv_awgn.so, code 0,
#             all eight points, checked against the published table (~7 minutes)
# Each GPU step has its own time limit; a crash / timeout ends the session (test FAILURES do not).
# Logs in gpurun_out/ (copy what is judged into profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
OUT=gpurun_out
mkdir -p $OUT
PHASES=",${PHASE:-tests,bench,prof},"
has() { [[ "$PHASES" == *",$1,"* ]]; }

if has tests; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && { tail -30 $OUT/smoke.log; exit $rc; }
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
run() {   # name, limit, bench.py args
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > $OUT/bench_$name.log 2>&1 || { echo "bench $name failed"; tail -5 $OUT/bench_$name.log; exit 1; }
  echo "$name: $(tail -1 $OUT/bench_$name.log | cut -c90-200)"
}
if has bench; then
  run k7 300                                                     # config 2 (headline)
  run k7_step 300 --layout step --no-cpu-baseline
  run bsc 300 --channel bsc                                      # config 4
  run code0_bsc 300 --code code0 --channel bsc                   # config 1 code at GPU scale
  run k9 300 --code k9 --frames 32                               # config 3 (port + AVX2 baselines)
  run k7_true 300 --code k7:true                                 # textbook (171,133)
  run k9_true 300 --code k9:true --frames 32                     # textbook (561,753)
  run k9_bsc 300 --code k9 --channel bsc --frames 32             # K = 9 BSC (soft kernel on Hamming rows)
  run stack 300 --decoder stack --frames 16 --steps 5 --warmup 1  # config 5 (16 frames: DESIGN 4.5)
  run stack_bsc 300 --decoder stack --channel bsc --frames 16 --steps 5 --warmup 1
  run fano 900 --decoder fano --steps 3 --warmup 1               # bounded reference-decoder sample
  run fano_bsc 900 --decoder fano --channel bsc --steps 3 --warmup 1
fi
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
      python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/prof.log; exit $rc; }
  cut -c1-160 $OUT/prof/run_kernel_stats.csv | head -6
fi
if has sweeps; then
  for c in k9 k7 k9:true k7:true; do
    tag=$(echo $c | tr -d ':')
    timeout -k 10 300 python -m ccviterbi.sim --code $c --points 10:14 --device-channel > $OUT/sweep_$tag.log 2>&1 \
        || { echo "sweep $c failed"; tail -3 $OUT/sweep_$tag.log; exit 1; }
    grep '^{' $OUT/sweep_$tag.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$c', d['ebn0_db'], d['errors'], d['bits'], d['mbit_s'])"
  done
fi
if has noise; then
  if [ -x tools/chanmath_f32_check ]; then
    timeout -k 10 120 tools/chanmath_f32_check > $OUT/chanmath_f32_check.txt 2>&1 \
        || { echo "chanmath_f32_check failed"; tail -5 $OUT/chanmath_f32_check.txt; exit 1; }
    cat $OUT/chanmath_f32_check.txt
  fi
  for c in k9 k7 k9:true k7:true; do
    tag=$(echo $c | tr -d ':')
    for nz in f64 f32; do
      timeout -k 10 300 python -m ccviterbi.sim --code $c --points 10:14 --device-channel --noise $nz \
          > $OUT/noise_${tag}_$nz.log 2>&1 || { echo "sweep $c $nz failed"; tail -3 $OUT/noise_${tag}_$nz.log; exit 1; }
    done
    python tools/noise_compare.py $OUT/noise_${tag}_f64.log $OUT/noise_${tag}_f32.log $OUT/noise_${tag}.json
  done
fi
if has refdriver; then
  mkdir -p $OUT/refdriver
  start=$(date +%s)
  timeout -k 10 1040 oracle/_ref/awgn-simulation-ccv 0 > $OUT/refdriver/awgn_code0.log 2>&1
  rc=$?; echo "driver rc=$rc after $(( $(date +%s) - start )) s"; [ $rc -ne 0 ] && exit $rc
  python tools/ref_driver_check.py $OUT/refdriver/awgn_code0.log 0 $OUT/refdriver/awgn_code0_check.json
fi
exit 0

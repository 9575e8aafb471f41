#!/bin/bash
# Fano decoder A/B: the GPU Fano tests on a variant build, then bench.py soft (4 dB) and BSC lines
# for the tree's libraries and the variant, round-robin, two rounds. Usage: sess_fano_ab.sh VARIANT
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/fano; mkdir -p $O
V=$1
CCV_LIB_DIR=$PWD/convolutional-codes_amd/build_ab/$V/lib timeout -k 10 400 python -u -m pytest tests/test_gpu_fano.py -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_$V.log 2>&1
rc=$?; echo "fano tests ($V) rc=$rc: $(tail -1 $O/tests_$V.log)"; [ $rc -gt 1 ] && exit $rc
for rep in 1 2; do
  for v in cur $V; do
    if [ $v = cur ]; then unset CCV_LIB_DIR; else export CCV_LIB_DIR=$PWD/convolutional-codes_amd/build_ab/$v/lib; fi
    for ch in awgn bsc; do
      timeout -k 10 300 python bench.py --decoder fano --channel $ch --steps 3 --warmup 1 --no-cpu-baseline \
          --no-hbm-probe --no-fused-channel > $O/bench_${v}_${ch}_$rep.log 2>&1 || { echo "bench $v $ch failed"; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_ms'])" $O/bench_${v}_${ch}_$rep.log "$v $ch $rep"
    done
  done
done

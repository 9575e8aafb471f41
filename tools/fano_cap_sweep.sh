#!/bin/bash
# Fano park cap sweep (bench.py --option fano_cap=N; 0 = one pass), round-robin repeats.
#   CHANNEL=bsc|awgn CAPS="216000 0" REPS=4 STEPS=5 bash tools/fano_cap_sweep.sh
set -u
CH=${CHANNEL:-bsc}
mkdir -p gpurun_out/cap
for rep in $(seq 1 ${REPS:-4}); do
for cap in ${CAPS:-216000 54000 0}; do
  timeout -k 10 200 python bench.py --decoder fano --channel $CH --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-fused-channel --option fano_cap=$cap > gpurun_out/cap/${CH}_${cap}_${rep}.log 2>&1 || exit 1
  echo "$CH cap $cap rep $rep $(grep -o '"value": [0-9.]*' gpurun_out/cap/${CH}_${cap}_${rep}.log | head -1)"
done
done

#!/bin/bash
# Fano GPU tests + two bench lines per channel (defaults, with the CPU baseline sample); gpurun_out/fcheck/.
set -u
mkdir -p gpurun_out/fcheck
timeout -k 10 400 python -u -m pytest tests/test_gpu_fano.py tests/test_gpu_seq_fuzz.py -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/fcheck/pytest.log 2>&1 || { tail -20 gpurun_out/fcheck/pytest.log; exit 1; }
tail -1 gpurun_out/fcheck/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --decoder fano --steps 3 --warmup 1 > gpurun_out/fcheck/bench_fano_${rep}.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --decoder fano --channel bsc --steps 3 --warmup 1 > gpurun_out/fcheck/bench_fano_bsc_${rep}.log 2>&1 || exit 1
  echo "rep $rep soft $(grep -o '"value": [0-9.]*' gpurun_out/fcheck/bench_fano_${rep}.log | head -1) iq $(grep -o '"fano_received_points": {"mbit_s": [0-9.]*' gpurun_out/fcheck/bench_fano_${rep}.log | grep -o '[0-9.]*$') bsc $(grep -o '"value": [0-9.]*' gpurun_out/fcheck/bench_fano_bsc_${rep}.log | head -1)"
done

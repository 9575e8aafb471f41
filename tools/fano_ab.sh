#!/bin/bash
# A/B of a Fano kernel change on one box: GPU tests of the new build, then bench.py soft (4 dB, with
# the received-points line) and BSC, round-robin against a copy of the previous core library
# (lib/libccv_core_r6base.so, loaded through CCV_CORE_LIB: copy lib/libccv_core.so there before
# rebuilding with the change, delete it afterwards -- lib/ travels with every gpurun call). Logs in gpurun_out/fab/.
set -u
mkdir -p gpurun_out/fab
timeout -k 10 400 python -u -m pytest tests/test_gpu_fano.py tests/test_gpu_seq_fuzz.py -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/fab/pytest.log 2>&1 || { tail -20 gpurun_out/fab/pytest.log; exit 1; }
tail -2 gpurun_out/fab/pytest.log
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export CCV_CORE_LIB=libccv_core_r6base.so; else unset CCV_CORE_LIB; fi
    timeout -k 10 200 python bench.py --decoder fano --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/fab/soft_${v}_${rep}.log 2>&1 || exit 1
    timeout -k 10 200 python bench.py --decoder fano --channel bsc --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/fab/bsc_${v}_${rep}.log 2>&1 || exit 1
    echo "$v $rep soft $(grep -o '"value": [0-9.]*' gpurun_out/fab/soft_${v}_${rep}.log | head -1) iq $(grep -o '"fano_received_points": {"mbit_s": [0-9.]*' gpurun_out/fab/soft_${v}_${rep}.log | head -1 | grep -o '[0-9.]*$') bsc $(grep -o '"value": [0-9.]*' gpurun_out/fab/bsc_${v}_${rep}.log | head -1)"
  done
done

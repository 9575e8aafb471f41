#!/bin/bash
# Multi-process rehearsal on a one-GPU box (every rank on cuda:0, reductions over gloo -- RCCL
# refuses two ranks on one device): bench.py at N = 2 and 3 through its own torchrun self-launch,
# and the device-channel sweep at N = 1, 2, 3, whose counts must be equal.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/rehearsal; mkdir -p $O
for n in 2 3; do
  timeout -k 10 400 python bench.py --gpus $n --same-device --steps 5 --warmup 1 --no-cpu-baseline \
      --no-hbm-probe > $O/bench_n$n.log 2>&1 || { echo "bench n=$n failed"; tail -20 $O/bench_n$n.log; exit 1; }
  tail -1 $O/bench_n$n.log | cut -c1-260
done
for n in 1 2 3; do
  timeout -k 10 400 python -m ccviterbi.sim --code k7 --points 2:6 --device-channel --bits 100000000 \
      --gpus $n --same-device --backend gloo --out $O/sweep_n$n.json > $O/sweep_n$n.log 2>&1 \
      || { echo "sweep n=$n failed"; tail -20 $O/sweep_n$n.log; exit 1; }
done
python3 - <<'PY'
import json
runs = {n: json.load(open(f"gpurun_out/rehearsal/sweep_n{n}.json")) for n in (1, 2, 3)}
for k, p in enumerate(runs[1]):
    row = [(runs[n][k]["errors"], runs[n][k]["bits"], runs[n][k]["world_size"]) for n in (1, 2, 3)]
    print(p["ebn0_db"], row, "equal" if len({r[:2] for r in row}) == 1 else "DIFFER")
PY

#!/bin/bash
# Channel kernels with the decision storage forced (channel_lds_decisions 1 = LDS, 0 = HBM) and auto
# (-1): tools/chan_bench.py, two rounds, BSC and both noise modes. Run on the GPU box.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/chan; mkdir -p $O
for rep in 1 2; do
  for v in 1 0 -1; do
    timeout -k 10 200 python tools/chan_bench.py --code k7 k7:true code0 code3 --bsc 50000 --option channel_lds_decisions=$v --tag bsc_lds$v >> $O/opt.jsonl 2>>$O/opt.err || exit 1
    timeout -k 10 200 python tools/chan_bench.py --code k7 k7:true code0 --noise f64 f32 --option channel_lds_decisions=$v --tag soft_lds$v >> $O/opt.jsonl 2>>$O/opt.err || exit 1
  done
done

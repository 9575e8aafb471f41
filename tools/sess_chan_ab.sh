#!/bin/bash
# A/B of channel-kernel builds with tools/chan_bench.py, round-robin, two rounds. Usage (on the GPU
# box): bash tools/sess_chan_ab.sh "name:noises name:noises ..." [codes]; "cur" = the tree's own
# libraries, any other name = convolutional-codes_amd/build_ab/<name>/lib. noises: f64,f32 or "bsc".
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/chan; mkdir -p $O
CODES=${2:-k7 k7:true}
for rep in 1 2; do
  for spec in $1; do
    v=${spec%%:*}; nz=${spec#*:}
    if [ $v = cur ]; then unset CCV_LIB_DIR; else export CCV_LIB_DIR=$PWD/convolutional-codes_amd/build_ab/$v/lib; fi
    if [ "$nz" = bsc ]; then
      timeout -k 10 200 python tools/chan_bench.py --code $CODES --bsc 50000 --tag $v >> $O/ab.jsonl 2>> $O/ab.err || exit 1
    else
      timeout -k 10 200 python tools/chan_bench.py --code $CODES --noise ${nz//,/ } --tag $v >> $O/ab.jsonl 2>> $O/ab.err || exit 1
    fi
  done
done

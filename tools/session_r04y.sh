# Round 4: K = 9 decode rate against the launch size (bench.py 32 / 104 frames) and the sweep rate
# against the device-channel chunk (tools/sweep_chunk_probe.py).
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
for f in 32 104; do
  for c in k9 k9:true; do
    tag=$(echo $c | tr -d ':')_f$f
    timeout -k 10 300 python bench.py --code $c --frames $f --no-cpu-baseline --no-fused-channel > $O/bench_$tag.log 2>&1 || { tail -3 $O/bench_$tag.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/bench_$tag.log').read().strip().splitlines()[-1])
print('$c frames $f', d['value'], d['kernel_ms'])"
  done
done
timeout -k 10 300 python tools/sweep_chunk_probe.py k9 32 64 104 208 > $O/chunk_k9.log 2>&1; rc=$?; cat $O/chunk_k9.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/sweep_chunk_probe.py k9:true 32 64 104 208 > $O/chunk_k9true.log 2>&1; rc=$?; cat $O/chunk_k9true.log | tail -4; [ $rc -ne 0 ] && exit $rc
echo done

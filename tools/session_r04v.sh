# Round 4: the true-parity sweeps (K = 9 (561,753) and K = 7 (171,133)) with the on-device channel at
# 800 M bits per point, a kernel trace of the K = 9 true-parity point (frames + two-lane decode), and
# the stack decoder's rate against its batch size.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
for c in k9:true k7:true; do
  tag=$(echo $c | tr -d ':')
  timeout -k 10 300 python -m ccviterbi.sim --code $c --points 10:14 --device-channel > $O/sweep_$tag.log 2>&1 || { echo "sweep $c failed"; tail -3 $O/sweep_$tag.log; exit 1; }
  grep '^{' $O/sweep_$tag.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$c', d['ebn0_db'], d['errors'], d['bits'], d['mbit_s'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 -m ccviterbi.sim --code k9:true --points 14 --device-channel > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 -c "
import csv
for r in csv.reader(open('$O/prof/run_kernel_stats.csv')):
    print(r[0][:40], r[1:4])"
# stack decoder: batch size vs rate (the persistent rows' tail: waves live ~72 % of the 4-frame launch)
for f in 4 16 32; do
  for ch in awgn bsc; do
    timeout -k 10 300 python bench.py --decoder stack --channel $ch --frames $f --steps 5 --warmup 1 --no-cpu-baseline > $O/stack_${ch}_f$f.log 2>&1 || { echo "stack $f failed"; tail -3 $O/stack_${ch}_f$f.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/stack_${ch}_f$f.log').read().strip().splitlines()[-1])
print('stack $ch frames $f', d['value'], d['kernel_ms'])"
  done
done
echo done

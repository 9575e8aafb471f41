# Round 4: the two-lane K = 9 true-parity kernel with its cross phase through ds_swizzle
# (acs_multi2.hpp multi2_cross_swz) -- parity under CCV_K9_TRUE_LANES=2, then bench.py k9:true
# round-robin against the four-lane production kernel.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
CCV_K9_TRUE_LANES=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k9 or true" -x -q --timeout 200 --timeout-method thread > $O/pytest_two_lane.log 2>&1; rc=$?; tail -2 $O/pytest_two_lane.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for lanes in 4 2; do
    CCV_K9_TRUE_LANES=$lanes timeout -k 10 300 python bench.py --code k9:true --frames 32 --no-cpu-baseline --no-fused-channel > $O/k9t_l${lanes}_$rep.log 2>&1 || { echo "bench $lanes failed"; tail -3 $O/k9t_l${lanes}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/k9t_l${lanes}_$rep.log').read().strip().splitlines()[-1])
print('k9:true lanes=$lanes rep $rep', d['value'], d['kernel_ms'], d['ber']['errors'])"
  done
done
echo done

# Round 4: the two-lane K = 9 kernel with NO cross-lane VALU left (growth cross phase, argmin and
# traceback pair swaps through ds_swizzle) against the build that keeps DPP there
# (CCV_MULTI2_MISC_DPP=1, build_ab/miscdpp); parity incl. the lane-variant child-process test.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k9 or true or lane_variants" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for name in head miscdpp; do
    if [ $name = head ]; then dir=$PWD/convolutional-codes_amd/lib; else dir=$PWD/convolutional-codes_amd/build_ab/$name/lib; fi
    CCV_LIB_DIR=$dir timeout -k 10 300 python bench.py --code k9:true --frames 32 --no-cpu-baseline --no-fused-channel > $O/k9t_${name}_$rep.log 2>&1 || { echo "bench $name failed"; tail -3 $O/k9t_${name}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/k9t_${name}_$rep.log').read().strip().splitlines()[-1])
print('k9:true $name rep $rep', d['value'], d['kernel_ms'], d['ber']['errors'])"
  done
done
echo done

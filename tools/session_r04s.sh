# Round 4: tuning the two-lane K = 9 true-parity kernel -- scheduling groups of the in-lane phases
# (CCV_MULTI2_GROUP 8 / 16 / 32) and the swizzle chunk of the cross phase (CCV_MULTI2_XG 4 / 8 / 16),
# whole-library variants from tools/ab_variant.sh; parity of each, then bench.py k9:true round-robin.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
export CCV_K9_TRUE_LANES=2
for name in head g8 g32 xg4 xg16; do
  if [ $name = head ]; then dir=$PWD/convolutional-codes_amd/lib; else dir=$PWD/convolutional-codes_amd/build_ab/$name/lib; fi
  CCV_LIB_DIR=$dir timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "k9_wide_kernel and true" -x -q --timeout 200 --timeout-method thread > $O/pytest_$name.log 2>&1; rc=$?; echo "$name: $(tail -1 $O/pytest_$name.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for name in head g8 g32 xg4 xg16; do
    if [ $name = head ]; then dir=$PWD/convolutional-codes_amd/lib; else dir=$PWD/convolutional-codes_amd/build_ab/$name/lib; fi
    CCV_LIB_DIR=$dir timeout -k 10 300 python bench.py --code k9:true --frames 32 --no-cpu-baseline --no-fused-channel > $O/k9t_${name}_$rep.log 2>&1 || { echo "bench $name failed"; tail -3 $O/k9t_${name}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/k9t_${name}_$rep.log').read().strip().splitlines()[-1])
print('k9:true $name rep $rep', d['value'], d['kernel_ms'], d['ber']['errors'], d['variant'] if 'variant' in d else '')"
  done
done
echo done

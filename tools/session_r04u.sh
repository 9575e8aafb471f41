# Round 4: stack decoder, soft input -- the block's symbols read from global memory instead of LDS
# (CCV_STACK_SYMG=1 build, build_ab/symg: more resident waves, an L2 round trip in the chain);
# parity of the variant, then bench.py config 5 round-robin with the launch shape printed.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
SYMG=$PWD/convolutional-codes_amd/build_ab/symg/lib
CCV_LIB_DIR=$SYMG timeout -k 10 400 python -u -m pytest tests/test_gpu_stack.py -x -q --timeout 300 --timeout-method thread > $O/pytest_symg.log 2>&1; rc=$?; tail -1 $O/pytest_symg.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for name in head symg; do
    if [ $name = head ]; then dir=$PWD/convolutional-codes_amd/lib; else dir=$SYMG; fi
    CCV_STACK_DEBUG=1 CCV_LIB_DIR=$dir timeout -k 10 300 python bench.py --decoder stack --frames 4 --steps 5 --warmup 1 --no-cpu-baseline > $O/stack_${name}_$rep.log 2>&1 || { echo "bench $name failed"; tail -3 $O/stack_${name}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/stack_${name}_$rep.log').read().strip().splitlines()[-1])
print('stack $name rep $rep', d['value'], d['kernel_ms'])"
  done
done
grep -m2 "stack rows" $O/stack_head_1.log $O/stack_symg_1.log
echo done

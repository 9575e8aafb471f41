# Round 4: the stack decoder with the noisiest-first block order (soft input; CCV_STACK_ORDER=0 = the
# natural order) -- the stack parity tests, then bench.py round-robin at 4 and 16 frames.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stack.py -x -q --timeout 300 --timeout-method thread > $O/pytest_stack.log 2>&1; rc=$?; tail -1 $O/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
for f in 4 16; do
  for rep in 1 2; do
    for ord in 1 0; do
      CCV_STACK_ORDER=$ord timeout -k 10 300 python bench.py --decoder stack --frames $f --steps 5 --warmup 1 --no-cpu-baseline > $O/stack_f${f}_o${ord}_$rep.log 2>&1 || { echo "bench failed"; tail -3 $O/stack_f${f}_o${ord}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/stack_f${f}_o${ord}_$rep.log').read().strip().splitlines()[-1])
print('stack frames $f order $ord rep $rep', d['value'], d['kernel_ms'], d['ber'])"
    done
  done
done
echo done

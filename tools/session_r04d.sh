set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_stack.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_stack.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
CCV_STACK_DEBUG=1 TAG=stack bash tools/ab_bench.sh "--decoder stack --frames 4 --steps 5 --warmup 1" head r04pair || exit 1
grep -h "stack rows" gpurun_out/ab/stack_head_1.log gpurun_out/ab/stack_r04pair_1.log | head -2
TAG=stackbsc bash tools/ab_bench.sh "--decoder stack --channel bsc --frames 4 --steps 5 --warmup 1" head r04pair || exit 1
echo done

set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
bash tools/session_r04i.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_stack.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_stack.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
TAG=stack bash tools/ab_bench.sh "--decoder stack --frames 4 --steps 5 --warmup 1" head r04c || exit 1
TAG=stackbsc bash tools/ab_bench.sh "--decoder stack --channel bsc --frames 4 --steps 5 --warmup 1" head r04c || exit 1
echo done

set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k9 or multilane or resident or register_kernel_selected or true_parity" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k9.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k9.log; [ $rc -ne 0 ] && exit $rc
TAG=k9true bash tools/ab_bench.sh "--code k9:true --frames 32" head r04base || exit 1
timeout -k 10 300 python bench.py --code k9:true --frames 32 --no-fused-channel > gpurun_out/bench_k9_true.log 2>&1 || exit 1
bash tools/pmc_workload.sh --code k9:true --frames 32 > gpurun_out/pmc_k9true.log 2>&1 || exit 1

timeout -k 10 600 python -u -m pytest tests/test_gpu_ber.py tests/test_gpu_stack.py tests/test_gpu_fano.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_seq.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_seq.log; [ $rc -ne 0 ] && exit $rc
TAG=k9idiom bash tools/ab_bench.sh "--code k9 --frames 32" head r04base || exit 1

set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_stack.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_stack.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
CCV_STACK_DEBUG=1 TAG=stack bash tools/ab_bench.sh "--decoder stack --frames 4 --steps 5 --warmup 1" head r04pair || exit 1
grep -h "stack rows" gpurun_out/ab/stack_head_1.log gpurun_out/ab/stack_r04pair_1.log | head -2
TAG=stackbsc bash tools/ab_bench.sh "--decoder stack --channel bsc --frames 4 --steps 5 --warmup 1" head r04pair || exit 1

echo done

set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_stack.py tests/test_gpu_parity.py -k "stack or ownership" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_stack.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_stack.log; [ $rc -ne 0 ] && exit $rc
TAG=stack bash tools/ab_bench.sh "--decoder stack --frames 4 --steps 5 --warmup 1" head r04base || exit 1
TAG=stackbsc bash tools/ab_bench.sh "--decoder stack --channel bsc --frames 4 --steps 5 --warmup 1" head r04base || exit 1
bash tools/pmc_workload.sh --code k9:true --frames 32 > gpurun_out/pmc_k9true.log 2>&1 || exit 1
bash tools/pmc_workload.sh --code k7:true > gpurun_out/pmc_k7true.log 2>&1 || exit 1
bash tools/pmc_workload.sh --decoder stack --frames 4 > gpurun_out/pmc_stack.log 2>&1 || exit 1
bash tools/pmc_workload.sh --decoder fano --reps 2 > gpurun_out/pmc_fano.log 2>&1 || exit 1
echo done

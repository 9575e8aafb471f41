set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k9 or multilane or resident or register_kernel_selected or true_parity" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k9.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k9.log; [ $rc -ne 0 ] && exit $rc
CCV_K9_TRUE_LANES=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k9_wide_kernel and true" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k9_4.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k9_4.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in 2 4; do
    CCV_K9_TRUE_LANES=$v timeout -k 10 300 python bench.py --code k9:true --frames 32 --no-cpu-baseline --no-fused-channel > gpurun_out/k9true_l${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/k9true_l${v}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/k9true_l${v}_$rep.log').read().strip().splitlines()[-1])
print('lanes $v rep $rep', d['value'], d['kernel_ms'], d['config']['variant'])"
  done
done
bash tools/pmc_workload.sh --code k9:true --frames 32 > gpurun_out/pmc_k9true.log 2>&1 || exit 1
echo done

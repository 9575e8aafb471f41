set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
CCV_K9_TRUE_LANES=4 CCV_K9_SLOT_XSWZ=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k9_wide_kernel and true" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k9_swz.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k9_swz.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in "4 1"; do
    set -- $v
    CCV_K9_TRUE_LANES=$1 CCV_K9_SLOT_XSWZ=$2 timeout -k 10 300 python bench.py --code k9:true --frames 32 --no-cpu-baseline --no-fused-channel > gpurun_out/k9true_l$1x$2_$rep.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/k9true_l$1x$2_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/k9true_l$1x$2_$rep.log').read().strip().splitlines()[-1])
print('lanes $1 swz $2 rep $rep', d['value'], d['kernel_ms'])"
  done
done
CCV_K9_TRUE_LANES=4 CCV_K9_SLOT_XSWZ=1 bash tools/pmc_workload.sh --code k9:true --frames 32 > gpurun_out/pmc_k9true.log 2>&1 || exit 1
echo done

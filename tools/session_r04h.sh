set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
CCV_K9_TRUE_LANES=4 CCV_K9_SLOT_WAVES=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k9_wide_kernel and true" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k9_4w4.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k9_4w4.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in "2 3" "4 3" "4 4"; do
    set -- $v
    CCV_K9_TRUE_LANES=$1 CCV_K9_SLOT_WAVES=$2 timeout -k 10 300 python bench.py --code k9:true --frames 32 --no-cpu-baseline --no-fused-channel > gpurun_out/k9true_l$1w$2_$rep.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/k9true_l$1w$2_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/k9true_l$1w$2_$rep.log').read().strip().splitlines()[-1])
print('lanes $1 waves $2 rep $rep', d['value'], d['kernel_ms'])"
  done
done
CCV_K9_TRUE_LANES=4 CCV_K9_SLOT_WAVES=4 bash tools/pmc_workload.sh --code k9:true --frames 32 > gpurun_out/pmc_k9true.log 2>&1 || exit 1
echo done

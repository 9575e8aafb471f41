set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
CCV_PERSIST_STAGE=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "golden or full_frame or persist or resident or seeded or ragged or k7 or noiseless" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_direct.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_direct.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in 0 1; do
    CCV_PERSIST_STAGE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-fused-channel > gpurun_out/k7_d${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/k7_d${v}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/k7_d${v}_$rep.log').read().strip().splitlines()[-1])
print('k7 stage=$v rep $rep', d['value'], d['kernel_ms'], d['ber']['errors'])"
  done
done
for v in 0 1; do
  CCV_PERSIST_STAGE=$v timeout -k 10 300 python bench.py --code k7:true --no-cpu-baseline --no-fused-channel > gpurun_out/k7t_d$v.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/k7t_d$v.log').read().strip().splitlines()[-1])
print('k7:true stage=$v', d['value'], d['kernel_ms'], d['ber']['errors'])"
done
CCV_PERSIST_STAGE=1 bash tools/pmc_workload.sh > gpurun_out/pmc_k7stage.log 2>&1 || exit 1

timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "bsc or hard" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_hard.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_hard.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "frames_only" -x -q --timeout 100 --timeout-method thread > gpurun_out/pytest_frames.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_frames.log; [ $rc -ne 0 ] && exit $rc
TAG=bsc bash tools/ab_bench.sh "--channel bsc" head r04c || exit 1
echo done

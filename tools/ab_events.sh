export PYTHONPATH=$PWD/convolutional-codes_amd
mkdir -p gpurun_out/r06e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "reserved or k9_bsc" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1 || { tail -20 gpurun_out/r06e/pytest.log; exit 1; }
tail -2 gpurun_out/r06e/pytest.log
for rep in 1 2 3; do
  for ev in on off; do
    timeout -k 10 200 python bench.py --step-events $ev --no-cpu-baseline --no-hbm-probe --no-fused-channel --curve-frames 0 > gpurun_out/r06e/ev_${ev}_$rep.log 2>&1 || { tail -5 gpurun_out/r06e/ev_${ev}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06e/ev_${ev}_$rep.log').read().strip().splitlines()[-1])
print('$ev', $rep, d['value'], d['ms_per_step'], d['kernel_ms'], d['timed_steps_device_ms'])"
  done
done

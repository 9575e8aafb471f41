set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_fano.py -m gpu -q -p no:cacheprovider -k "seeded or golden" > gpurun_out/pt_fano3.log 2>&1
rc=$?; tail -2 gpurun_out/pt_fano3.log; [ $rc -ne 0 ] && exit $rc
for r in 0 1; do for db in 4 6; do
  CCV_FANO_ROWS=$r timeout -k 10 600 python bench.py --decoder fano --ebn0 $db --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bf_r${r}_$db.log 2>&1 || exit $?
  echo "rows=$r $db dB: $(tail -1 gpurun_out/bf_r${r}_$db.log | cut -c60-160)"
done; done

set -u
mkdir -p gpurun_out
for m in default 0 1; do
  if [ $m = default ]; then unset CCV_FANO_ROWS; else export CCV_FANO_ROWS=$m; fi
  timeout -k 10 600 python -m pytest tests/test_gpu_fano.py -m gpu -q -p no:cacheprovider -x > gpurun_out/pt_fano_m$m.log 2>&1
  rc=$?; echo "mode $m: $(tail -1 gpurun_out/pt_fano_m$m.log)"; [ $rc -ne 0 ] && exit $rc
done
unset CCV_FANO_ROWS
export CCV_FANO_DEBUG=1 CCV_FANO_COUNT_MOVES=1
timeout -k 10 500 python tools/fano_scaling.py 4 > gpurun_out/fscale_g.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/fscale_g.log | grep -v "lds "

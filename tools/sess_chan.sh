set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/chan; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "device_channel" -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -gt 1 ] && exit $rc
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export CCV_LIB_DIR=$PWD/convolutional-codes_amd/build_ab/base/lib; else unset CCV_LIB_DIR; fi
    timeout -k 10 200 python tools/chan_bench.py --code k7 k9 k7:true --tag $v >> $O/bench.jsonl 2>> $O/bench.err || exit 1
    timeout -k 10 200 python tools/chan_bench.py --code k7 k9 --bsc 50000 --tag $v >> $O/bench.jsonl 2>> $O/bench.err || exit 1
  done
done
cat $O/bench.jsonl

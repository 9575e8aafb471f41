# Fano decoder session: parity tests, search statistics, benches (soft 4/6 dB, BSC).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_fano.py -m gpu -q -p no:cacheprovider > gpurun_out/pt_fano2.log 2>&1
rc=$?; tail -3 gpurun_out/pt_fano2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/fano_stats.py k15 4 > gpurun_out/fstats.log 2>&1 || exit $?
cat gpurun_out/fstats.log
for db in 4 6; do
  timeout -k 10 600 python bench.py --decoder fano --ebn0 $db --steps 3 --warmup 1 > gpurun_out/bfano64_$db.log 2>&1 || exit $?
  tail -1 gpurun_out/bfano64_$db.log | cut -c1-200
done
timeout -k 10 600 python bench.py --decoder fano --channel bsc --steps 3 --warmup 1 > gpurun_out/bfano64_bsc.log 2>&1 || exit $?
tail -1 gpurun_out/bfano64_bsc.log | cut -c1-200

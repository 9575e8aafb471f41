set -u
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 ./tools/persist_bench > $O/persist_bench.txt 2>&1 || exit 1
head -4 $O/persist_bench.txt
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || exit 1
tail -1 $O/bench_default.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused-channel --channel bsc > $O/bench_bsc.log 2>&1 || exit 1
tail -1 $O/bench_bsc.log

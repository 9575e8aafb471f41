set -u
O=gpurun_out
timeout -k 10 300 ./tools/persist_bench > $O/persist_bench.txt 2>&1 || exit 1
cat $O/persist_bench.txt
TESTS_K="persistent or selected or dropped or ragged or golden_fixture" bash tools/gpu_ab.sh

set -u
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || exit 1
tail -1 $O/bench_default.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run -- python bench.py --no-cpu-baseline --no-fused-channel --steps 20 --warmup 5 > $O/prof2.log 2>&1 || exit 1
find $O/prof2 -name "*kernel_stats.csv" | head -3

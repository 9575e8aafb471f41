# Round 4: config 5 (stack decoder) at 16 frames per step -- PMC passes for the new workload keys and
# the two bench lines (with CPU baselines) as gpu_round.sh now runs them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
bash tools/pmc_workload.sh --decoder stack --frames 16 > $O/pmc_stack16.log 2>&1 || { tail -5 $O/pmc_stack16.log; exit 1; }
bash tools/pmc_workload.sh --decoder stack --channel bsc --frames 16 > $O/pmc_stack16_bsc.log 2>&1 || { tail -5 $O/pmc_stack16_bsc.log; exit 1; }
cp gpurun_out/pmc/pmc_workloads.json $O/pmc_workloads_stack16.json
timeout -k 10 300 python bench.py --decoder stack --frames 16 --steps 5 --warmup 1 > $O/bench_stack.log 2>&1 || { tail -3 $O/bench_stack.log; exit 1; }
timeout -k 10 300 python bench.py --decoder stack --channel bsc --frames 16 --steps 5 --warmup 1 > $O/bench_stack_bsc.log 2>&1 || { tail -3 $O/bench_stack_bsc.log; exit 1; }
for f in bench_stack bench_stack_bsc; do tail -1 $O/$f.log | cut -c1-200; done
echo done

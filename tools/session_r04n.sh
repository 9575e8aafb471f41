# Round 4: (1) Fano on the BSC -- received rows in LDS (default) or prefetched from global memory,
# expected-symbol table on / off, bench.py round-robin; (2) the K = 9 sweep's two kernels at 12 dB and
# 14 dB, one rocprof kernel trace per point (why 12 dB runs slower); (3) PMC passes.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
CCV_FANO_ROWS=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_fano.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "seeded or golden" > $O/pytest_fano_rows2.log 2>&1
rc=$?; tail -1 $O/pytest_fano_rows2.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for cfg in "1 1" "2 1" "1 0" "2 0"; do
    set -- $cfg
    tag=rows$1_tab$2_$rep
    CCV_FANO_ROWS=$1 CCV_FANO_SYMTAB=$2 timeout -k 10 300 python bench.py --decoder fano --channel bsc --steps 3 --warmup 1 --no-cpu-baseline > $O/fano_bsc_$tag.log 2>&1 || { echo "fano $tag failed"; tail -3 $O/fano_bsc_$tag.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/fano_bsc_$tag.log').read().strip().splitlines()[-1])
print('fano bsc $tag', d['value'], 'Mbit/s', d['kernel_ms'], 'ms')"
  done
done
for pt in 12 14; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$pt -o run -- python3 -m ccviterbi.sim --code k9 --points $pt --device-channel > $GRAFT_REPO_ROOT/$O/prof_$pt.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT && python3 -c "
import csv
for r in csv.reader(open('$O/prof_$pt/run_kernel_stats.csv')):
    print('$pt dB', r[0][:40], r[1:4])"
done
# (3) PMC passes (FETCH / WRITE / SQ / STALL) for the bench lines that have none yet
bash tools/pmc_workload.sh --code k7:true > $O/pmc_k7true.log 2>&1 || { tail -5 $O/pmc_k7true.log; exit 1; }
bash tools/pmc_workload.sh --code k9:true --frames 32 > $O/pmc_k9true.log 2>&1 || { tail -5 $O/pmc_k9true.log; exit 1; }
bash tools/pmc_workload.sh --decoder fano --reps 1 > $O/pmc_fano.log 2>&1 || { tail -5 $O/pmc_fano.log; exit 1; }
bash tools/pmc_workload.sh > $O/pmc_k7.log 2>&1 || { tail -5 $O/pmc_k7.log; exit 1; }
cp gpurun_out/pmc/pmc_workloads.json $O/pmc_workloads_new.json
echo done

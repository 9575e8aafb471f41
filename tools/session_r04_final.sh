# Round 4, end of round: the full gpu_round.sh (smoke, every GPU test, every bench line, rocprof of
# the headline), then the PMC pass of the two-lane K = 9 true-parity kernel (new default) and the
# Eb/N0 sweeps of configs 2 and 3 with the on-device channel (800 M bits per point, 0.2 s warm-up).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
bash tools/gpu_round.sh || exit $?
bash tools/pmc_workload.sh --code k9:true --frames 32 > gpurun_out/pmc_k9true2.log 2>&1 || { tail -5 gpurun_out/pmc_k9true2.log; exit 1; }
cp gpurun_out/pmc/pmc_workloads.json gpurun_out/pmc_workloads_final.json
for c in k9 k7; do
  timeout -k 10 300 python -m ccviterbi.sim --code $c --points 10:14 --device-channel > gpurun_out/sweep_${c}_final.log 2>&1 || { echo "sweep $c failed"; tail -3 gpurun_out/sweep_${c}_final.log; exit 1; }
  grep '^{' gpurun_out/sweep_${c}_final.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$c', d['ebn0_db'], d['errors'], d['bits'], d['mbit_s'])"
done
echo done

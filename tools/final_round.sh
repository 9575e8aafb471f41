#!/bin/bash
# Round-end GPU session: tools/gpu_round.sh (smoke, parity tests, benches, rocprof of the headline),
# then rocprofv3 kernel stats of the config-5 stack bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_round.sh || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stack -o run -- \
    python bench.py --decoder stack --frames 4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_stack.log 2>&1
rc=$?; echo "stack rocprof rc=$rc"; tail -1 gpurun_out/prof_stack.log | cut -c1-200
exit $rc

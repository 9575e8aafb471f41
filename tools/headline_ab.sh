#!/bin/bash
# Headline A/B on one box: this tree vs another built tree (AB_OLD, default .ab_old), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out
mkdir -p $O
OLD=${AB_OLD:-.ab_old}
for i in 1 2 3; do
  for tree in . $OLD; do
    (cd $tree && timeout -k 10 300 python bench.py --steps 50 --warmup 3 --no-cpu-baseline --no-fused-channel > $O/hab_${i}_$(basename $tree).log 2>&1) || exit 1
    python3 -c "
import json; d=json.loads(open('$O/hab_${i}_$(basename $tree).log').read().strip().splitlines()[-1])
print('run $i tree $tree', d['value'], d['kernel_ms'])"
  done
done

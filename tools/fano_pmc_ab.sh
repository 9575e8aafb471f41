#!/bin/bash
# PMC A/B for the Fano kernel at the bench size: received rows from global memory vs in LDS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CCV_FANO_ROWS=0 bash tools/pmc_kernel.sh fano_rows0 fano_decode --decoder fano --frames 32 --steps 1 --warmup 0 --no-cpu-baseline || exit $?
CCV_FANO_ROWS=1 bash tools/pmc_kernel.sh fano_rows1 fano_decode --decoder fano --frames 32 --steps 1 --warmup 0 --no-cpu-baseline || exit $?

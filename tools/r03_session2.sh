#!/bin/bash
# PMC (traffic, VALU issue, stall split) of every bench workload, then the BER curves again.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd
bash tools/pmc_workload.sh --code k7 --frames 104 || exit 1
bash tools/pmc_workload.sh --code k9 --frames 16 || exit 1
bash tools/pmc_workload.sh --code k7 --frames 104 --channel bsc || exit 1
bash tools/pmc_workload.sh --decoder stack --frames 4 || exit 1
bash tools/pmc_workload.sh --decoder stack --frames 4 --channel bsc || exit 1
bash tools/ber_curves.sh 1

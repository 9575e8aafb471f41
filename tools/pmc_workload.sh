#!/bin/bash
# PMC figures of one bench workload's dominant kernel, three rocprofv3 passes (one counter group
# each, kernel trace only -- gfx950 cannot hold FETCH_SIZE and WRITE_SIZE in one pass):
#   FETCH_SIZE | WRITE_SIZE | SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES
#                             SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU + GRBM_GUI_ACTIVE | stall split
# over tools/traffic_probe.py (a calibration copy + the bench decode), then tools/pmc_workload.py
# merges the per-launch figures into gpurun_out/pmc/pmc_workloads.json under the bench's workload key.
# Usage: tools/pmc_workload.sh [traffic_probe / bench.py workload args...]
# PMC_TAG=name keeps a variant's passes apart (gpurun_out/pmc/name_<args>/) and PMC_JSON=file sends
# its record to another JSON (A/B builds loaded with CCV_LIB_DIR).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS="$*"
TAG=$(echo "${ARGS:-default}" | tr -c 'A-Za-z0-9\n' '_')
OUT=gpurun_out/pmc/${PMC_TAG:+${PMC_TAG}_}$TAG
mkdir -p $OUT
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
      python tools/traffic_probe.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -20 $OUT/$name.log; exit 1; }
}
pass FETCH FETCH_SIZE
pass WRITE WRITE_SIZE
pass SQ SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass STALL SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES
python tools/pmc_workload.py $OUT ${PMC_JSON:-gpurun_out/pmc/pmc_workloads.json} $ARGS

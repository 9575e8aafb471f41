#!/bin/bash
# SQ counters of the Fano kernel (K=15, 4 dB, 16 frames, one pass) for two core-library builds:
# the park-capable kernel and the same source without the park/resume code (CCV_FANO_NO_PARK).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD/convolutional-codes_amd CCV_FANO_CAP=0
for lib in libccv_core.so libccv_core_nopark.so; do
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES"; do
    tag=$(echo $lib | tr -c 'a-z0-9\n' '_')_$(echo $set | cut -d' ' -f1)
    CCV_CORE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/fpmc/$tag -o run -- \
        python tools/traffic_probe.py --decoder fano --frames 16 --reps 1 > gpurun_out/fpmc_$tag.log 2>&1 || { tail gpurun_out/fpmc_$tag.log; exit 1; }
    python3 - gpurun_out/fpmc/$tag "$lib" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fano_decode" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], {k: f"{v:.4g}" for k, v in sorted(acc.items())})
PY
  done
done

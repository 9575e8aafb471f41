#!/bin/bash
# BER-vs-Eb/N0 curves of the benchmark codes on the GPU (python -m ccviterbi.sim, on-device channel,
# the reference's bit schedule AWGN-channel/main.c:202-211) -> gpurun_out/ber/<code>.json, then
# merged into gpurun_out/ber/ber_curves.json (copy to profiles/). Usage: tools/ber_curves.sh [GPUS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD/convolutional-codes_amd${PYTHONPATH:+:$PYTHONPATH}
OUT=gpurun_out/ber
mkdir -p $OUT
G=${1:-1}
for code in k7 k7:true k9 k9:true; do
  f=$OUT/$(echo $code | tr ':' '_').json
  timeout -k 10 600 python -m ccviterbi.sim --code $code --device-channel --gpus $G --out $f \
      > $OUT/$(echo $code | tr ':' '_').log 2>&1 || { tail -20 $OUT/*.log; exit 1; }
  tail -8 $OUT/$(echo $code | tr ':' '_').log | cut -c1-220
done
python - <<'PY'
import glob, json
pts = []
for f in sorted(glob.glob("gpurun_out/ber/k*.json")):
    pts += json.load(open(f))
json.dump({"generated_by": "tools/ber_curves.sh (python -m ccviterbi.sim --device-channel)",
           "schedule": "reference bits per point: AWGN-channel/main.c:202-211", "points": pts},
          open("gpurun_out/ber/ber_curves.json", "w"), indent=1)
print(len(pts), "points")
PY

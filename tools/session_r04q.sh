# Round 4: the constellation points as compile-time constants in the demapper and the encoder window
# shifted behind a real branch -- device-channel tests, then the K = 9 / K = 7 sweeps A/B against
# build_ab/cm2 (the tree before), plus a kernel trace of a K = 9 point.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd TMPDIR=/tmp
mkdir -p gpurun_out/r04q
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "device_channel" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04q/pytest_channel.log 2>&1; rc=$?; tail -2 gpurun_out/r04q/pytest_channel.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for name in head cm2; do
    if [ $name = head ]; then dir=$PWD/convolutional-codes_amd/lib; else dir=$PWD/convolutional-codes_amd/build_ab/$name/lib; fi
    CCV_LIB_DIR=$dir timeout -k 10 200 python -m ccviterbi.sim --code k9 --points 12:14 --device-channel > gpurun_out/r04q/sweep_k9_${name}_$rep.log 2>&1 || { echo "k9 $name failed"; tail -5 gpurun_out/r04q/sweep_k9_${name}_$rep.log; exit 1; }
    CCV_LIB_DIR=$dir timeout -k 10 200 python -m ccviterbi.sim --code k7 --points 12:14 --device-channel > gpurun_out/r04q/sweep_k7_${name}_$rep.log 2>&1 || { echo "k7 $name failed"; exit 1; }
    python3 - <<EOF
import json
for c in ("k9", "k7"):
    for l in open(f"gpurun_out/r04q/sweep_{c}_${name}_$rep.log"):
        if l.startswith("{"):
            d = json.loads(l); print(c, "${name}", $rep, d["ebn0_db"], d["errors"], d["mbit_s"])
EOF
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04q/prof --output-format csv -o run -- python3 -m ccviterbi.sim --code k9 --points 14 --device-channel > $GRAFT_REPO_ROOT/gpurun_out/r04q/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find gpurun_out/r04q/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04q/k9_sweep_kernel_stats.csv \;
echo done

# The unchanged reference AWGN driver (AWGN-channel/main.c) over the MI355X shim, code 0, all eight
# Eb/N0 points (~44 M blocks through decoder_input), then the published-table check.
set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
mkdir -p gpurun_out/refdriver
start=$(date +%s)
timeout -k 10 1040 oracle/_ref/awgn-simulation-ccv 0 > gpurun_out/refdriver/awgn_code0.log 2>&1
rc=$?
echo "driver rc=$rc after $(( $(date +%s) - start )) s"
[ $rc -ne 0 ] && exit $rc
python tools/ref_driver_check.py gpurun_out/refdriver/awgn_code0.log 0 gpurun_out/refdriver/awgn_code0_check.json

#!/bin/bash
# Fano benches at the bench size (64 frames): soft 4/6 dB, BSC; quick parity subset first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_fano.py -m gpu -q -p no:cacheprovider -k "seeded or golden" > gpurun_out/pt_fano3.log 2>&1
rc=$?; tail -2 gpurun_out/pt_fano3.log; [ $rc -ne 0 ] && exit $rc
for db in 4 6; do
  CCV_FANO_DEBUG=1 timeout -k 10 600 python bench.py --decoder fano --ebn0 $db --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bfano64_$db.log 2>&1 || exit $?
  grep "fano:" gpurun_out/bfano64_$db.log | sort | uniq -c | head -3
  echo "$db dB: $(tail -1 gpurun_out/bfano64_$db.log | cut -c60-150)"
done
timeout -k 10 600 python bench.py --decoder fano --channel bsc --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bfano64_bsc.log 2>&1 || exit $?
echo "bsc: $(tail -1 gpurun_out/bfano64_bsc.log | cut -c60-150)"

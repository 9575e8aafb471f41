set -u
export PYTHONPATH=$PWD/convolutional-codes_amd
# Fano soft at 4 dB: received rows after the move (0) vs both candidate rows prefetched (2), with the
# expected-symbol table or VALU parities
for v in "0 1" "2 1" "0 0" "2 0"; do
  set -- $v
  CCV_FANO_ROWS=$1 CCV_FANO_SYMTAB=$2 timeout -k 10 300 python bench.py --decoder fano --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/fano_rows$1_tab$2.log 2>&1 || { echo "fano $v failed"; tail -3 gpurun_out/fano_rows$1_tab$2.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/fano_rows$1_tab$2.log').read().strip().splitlines()[-1])
print('fano rows=$1 symtab=$2', d['value'], d['kernel_ms'])"
done
echo done

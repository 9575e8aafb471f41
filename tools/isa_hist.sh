#!/bin/bash
# Instruction histogram of one kernel in a built object: tools/isa_hist.sh OBJ KERNEL_REGEX [N]
# (unbundles the gfx950 code object, disassembles, prints the N most frequent mnemonics and the
# kernel's VGPR count). CPU only.
set -eu
OBJ=$1 RE=$2 N=${3:-25}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb $OBJ
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fb --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 $T/co > $T/s
L=$(grep -n -E "<${RE}>:$" $T/s | head -1 | cut -d: -f1)
[ -n "${DUMP:-}" ] && awk -v s=$L 'NR>s && /^0000/ {exit} NR>s' $T/s | cut -c1-90 > $DUMP
awk -v s=$L 'NR>s && /^0000/ {exit} NR>s {print $1}' $T/s | sort | uniq -c | sort -rn | head -$N
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/co | grep -E "\.name:|\.vgpr_count|\.vgpr_spill" | paste - - - | grep -E "${RE}" | head -1 | grep -oE "vgpr_count: +[0-9]+|vgpr_spill_count: +[0-9]+"
rm -rf $T
# DUMP=file also writes the kernel's disassembly there

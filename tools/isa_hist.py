#!/usr/bin/env python3
"""Instruction histogram of the kernels in a hipcc -S (gfx950) assembly file.

usage: isa_hist.py FILE.s [SUBSTRING] [--top N]
Prints, per kernel whose mangled name contains SUBSTRING: VGPR count, scratch, total instructions,
VALU / SALU / memory / branch split and the N most frequent opcodes. Static counts (straight-line
kernels: static = dynamic per group).
"""
import re
import sys
from collections import Counter


def kernels(path):
    cur, body = None, []
    with open(path) as f:
        for line in f:
            m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
            if m:
                cur, body = m.group(1), []
                continue
            if cur is None:
                continue
            if line.startswith(".Lfunc_end") or line.strip().startswith(".section"):
                yield cur, body
                cur = None
                continue
            body.append(line)


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_barrier"):
        return "sync"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 25
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
        args = [a for a in args if a != str(top)]
    path = args[0]
    sub = args[1] if len(args) > 1 else ""
    for name, body in kernels(path):
        if sub not in name:
            continue
        ops = Counter()
        for line in body:
            s = line.strip()
            if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
                continue
            ops[s.split()[0]] += 1
        cls = Counter()
        for op, c in ops.items():
            cls[classify(op)] += c
        print(f"== {name[:150]}")
        print("   total", sum(ops.values()), dict(cls))
        for op, c in ops.most_common(top):
            print(f"   {c:7d} {op}")


if __name__ == "__main__":
    main()

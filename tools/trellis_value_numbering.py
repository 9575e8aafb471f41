"""Value numbering of an x86-idiom trellis (tools/; not part of the product).

The x86 generator idiom makes many branches emit the same symbol, so many path metrics are equal
as expressions: a straight-line kernel's common-subexpression elimination only computes the distinct
adds / mins (and the decisions of distinct min pairs). This script symbolically runs the ACS of
AWGN-channel/viterbi-decoder.c:108-141 from generic initial metrics and counts, per steady-state step:

* K=7 (171,133): distinct adds, mins and decision pairs, and the classes of states sharing a decision;
* K=9 (561,753): the same for the whole block, and per lane of the 4-lane register kernel for every
  choice of the two physical state bits that are lane bits (acs_multi.hpp uses bits 6, 7).

usage: python3 tools/trellis_value_numbering.py
"""
import itertools


def parity(v):
    return bin(v).count("1") & 1


def gen_bit(v):   # trellis.hpp gen_bit, GEN_REF_X86
    return parity(v) & (parity(v & 0x1010101010101010) ^ 1)


def make_expected(K, polys):
    def e(s, i):
        sr = (s << (64 - K)) | (i << 63)
        r = 0
        for p in polys:
            r = (r << 1) | gen_bit(sr & p)
        return r
    return e


def block_counts(K, polys, steps=12):
    e = make_expected(K, polys)
    S, H = 1 << (K - 1), 1 << (K - 2)
    M = [("x", s) for s in range(S)]
    for t in range(steps):
        adds, mins, classes, N = set(), set(), {}, [None] * S
        for j in range(H):
            for i in (0, 1):
                a0 = ("add", M[2 * j], t, e(2 * j, i))
                a1 = ("add", M[2 * j + 1], t, e(2 * j + 1, i))
                adds.update((a0, a1))
                N[j + i * H] = ("min", a0, a1)
                mins.add(N[j + i * H])
                classes.setdefault(repr((a0, a1)), []).append(j + i * H)
        M = N
    return len(adds), len(mins), [c for c in classes.values() if len(c) > 1]


def lane_counts(K, polys, lanebits, steps=32):
    """Per-lane distinct adds / mins of the multilane kernel: an instruction computes register r for
    all lanes at once, so it is shared only when the whole per-lane vector of operands repeats."""
    e = make_expected(K, polys)
    n, S, H = K - 1, 1 << (K - 1), 1 << (K - 2)
    L = 1 << len(lanebits)
    regbits = [b for b in range(n) if b not in lanebits]

    def phys(q, r):
        x = 0
        for k, b in enumerate(lanebits):
            x |= ((q >> k) & 1) << b
        for k, b in enumerate(regbits):
            x |= ((r >> k) & 1) << b
        return x

    def rotr(x, p):
        p %= n
        return x if p == 0 else ((x >> p) | (x << (n - p))) & (S - 1)

    vid = {}

    def V(key):
        return vid.setdefault(key, len(vid))

    M = {s: V(("x", s)) for s in range(S)}
    tot = []
    for t in range(steps):
        p = t % n
        expr = {}
        for ns in range(S):
            i, j = ns >> (n - 1), ns & (H - 1)
            expr[ns] = ((M[2 * j], e(2 * j, i)), (M[2 * j + 1], e(2 * j + 1, i)))
        newM = {ns: V(("min",) + expr[ns]) for ns in range(S)}
        adds, mins = set(), set()
        for r in range(S // L):
            lanes = [rotr(phys(q, r), p + 1) for q in range(L)]
            adds.add(tuple(V(("add",) + expr[s][0]) for s in lanes))
            adds.add(tuple(V(("add",) + expr[s][1]) for s in lanes))
            mins.add(tuple(newM[s] for s in lanes))
        M = newM
        tot.append((len(adds), len(mins)))
    last = tot[-n:]
    return sum(a for a, _ in last) / n, sum(m for _, m in last) / n


if __name__ == "__main__":
    k7 = (0xF2 << 56, 0xB6 << 56)
    adds, mins, classes = block_counts(7, k7)
    print(f"K=7 (171,133) idiom: {adds} adds, {mins} distinct metrics/decisions per step")
    print("  states sharing a decision:", classes)
    k9 = (13294626099997704192, 17690139336311308288)
    adds, mins, _ = block_counts(9, k9)
    print(f"K=9 (561,753) idiom, whole block: {adds} adds, {mins} mins per step")
    for lb in itertools.combinations(range(8), 2):
        a, m = lane_counts(9, k9, list(lb))
        print(f"  lane bits {lb}: {a:.2f} adds, {m:.2f} mins per lane per step")

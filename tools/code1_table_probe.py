#!/usr/bin/env python3
"""Which decoder made results/binary_symmetric_channel.m:7 (codebook code 1 on the BSC)? CPU only.

Builds tools/code1_table_probe.c against oracle/build/libccoracle.so into /tmp, decodes the same Philox
BSC frames (libccv_sim) with four variants of the reference hard Viterbi -- the x86-idiom and the
true-parity generator, strict < ties, traceback from the argmin (the shipped decoder) or from state 0 --
and applies tests/test_gpu_ber.py's acceptance rule (burst factor B = blen, 3.29 sigma, half the print
resolution) against the table's 800 M-bit points. Writes profiles/r04_code1_table_probe.json.
"""
import ctypes
import json
import math
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "convolutional-codes_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
BLOCKS = int(os.environ.get("PROBE_BLOCKS", 1000000))


def main():
    import oracle_ctypes as O
    from ccviterbi import channel as ch
    from ccviterbi.code import get_code
    O.lib()
    so = "/tmp/code1_table_probe.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-I", os.path.join(REPO, "oracle"), "-o", so,
                    os.path.join(REPO, "tools", "code1_table_probe.c"),
                    os.path.join(REPO, "oracle", "build", "libccoracle.so"),
                    "-Wl,-rpath," + os.path.join(REPO, "oracle", "build")], check=True)
    L = ctypes.CDLL(so)
    L.var_hard.restype = ctypes.c_uint64
    L.var_hard.argtypes = [ctypes.POINTER(O.CcoCode), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                           ctypes.c_int, ctypes.c_int]
    pub = json.load(open(os.path.join(REPO, "tests", "golden", "published_ber.json")))
    curve = next(c for c in pub["curves"] if c["codebook_index"] == 1 and c["channel"] == "bsc"
                 and c["decoder"] == "viterbi")
    res = pub["print_resolution"]["bsc"]
    n_ref = 800e6
    rows = []
    for p, p_ref in zip(pub["bsc_p"], curve["ber"]):
        if p < 0.003 or p > 0.35:
            continue   # below: too few errors in 40 M bits to discriminate; above: saturated
        ppm = round(p * 1e6)
        for gm, gname in ((0, "ref-x86"), (1, "true-parity")):
            code = get_code(1).with_(gen_mode=gm)
            oc = O.code(code.n, code.K, code.blen, code.polys, code.gen_mode)
            info, syms = ch.bsc_blocks(code, BLOCKS, ppm, 0x7AB1E + ppm, threads=8)
            for zero in (0, 1):
                e = L.var_hard(ctypes.byref(oc), syms.ctypes.data, info.ctypes.data, BLOCKS, 0, zero)
                n = BLOCKS * code.blen
                ber = e / n
                q = (e + p_ref * n_ref) / (n + n_ref)
                tol = 3.29 * math.sqrt(code.blen * q * (1 - q) * (1 / n + 1 / n_ref)) + res / 2
                rows.append({"p": p, "generator": gname, "traceback_from": "state 0" if zero else "argmin",
                             "ber": ber, "table": p_ref, "tolerance": tol, "passes": abs(ber - p_ref) <= tol})
                print(rows[-1], flush=True)
    summary = {}
    for r in rows:
        k = f"{r['generator']}, traceback from {r['traceback_from']}"
        s = summary.setdefault(k, {"points": 0, "pass": 0})
        s["points"] += 1
        s["pass"] += r["passes"]
    doc = {"generated_by": "tools/code1_table_probe.py", "bits_per_point": BLOCKS * 40, "summary": summary,
           "rows": rows}
    with open(os.path.join(REPO, "profiles", "r04_code1_table_probe.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()

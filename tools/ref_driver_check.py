"""Check the stdout of the UNCHANGED reference AWGN driver (AWGN-channel/main.c built against the
MI355X shim libccv_awgn.so as oracle/_ref/awgn-simulation-ccv, oracle/Makefile:84-88) against the
published table results/awgn_channel.m (tests/golden/published_ber.json), point by point, with the
acceptance rule of tests/test_gpu_ber.py (z = 3.29, burst factor B = blen, both runs' variances,
half the print resolution).

The driver seeds glibc rand() from time(NULL) (main.c:147), so only the statistics can agree.

usage: python tools/ref_driver_check.py <driver stdout> <code index> <out.json>
"""
import json
import math
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "convolutional-codes_amd"))
from ccviterbi import CODEBOOK, sim  # noqa: E402

Z = 3.29


def parse(text):
    """(Eb/N0, BER) pairs in the order the driver prints them (main.c:196-236)."""
    text = text.replace("\r", "\n")
    snr = [float(x) for x in re.findall(r"Eb/N0: ([-0-9.]+)dB", text)]
    ber = [float(x) for x in re.findall(r"Overall transmission error rate: ([0-9.eE+-]+)", text)]
    return list(zip(snr, ber))


def main():
    log, idx, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    pub = json.load(open(os.path.join(REPO, "tests", "golden", "published_ber.json")))
    (curve,) = [c for c in pub["curves"] if c["channel"] == "awgn" and c["decoder"] == "viterbi"
                and c["codebook_index"] == idx and not c["hard_demap"]]
    blen = CODEBOOK[idx].blen
    rows, bad = [], 0
    for k, (snr, p) in enumerate(parse(open(log, errors="replace").read())):
        assert abs(snr - pub["awgn_ebn0_db"][k]) < 1e-6
        n = sim.reference_awgn_bits(snr, blen)           # the driver's own bit count per point
        p_r = curve["ber"][k]
        q = (p * n + p_r * n) / (2 * n)
        tol = Z * math.sqrt(blen * q * (1 - q) * (2.0 / n)) + 1e-8 / 2 + 1e-8 / 2
        ok = abs(p - p_r) <= tol
        bad += not ok
        rows.append({"ebn0_db": snr, "bits": n, "ber_driver_on_mi355x": p, "ber_published": p_r,
                     "tolerance": tol, "ok": ok})
        print(f"{snr:5.1f} dB  driver {p:.8f}  published {p_r:.8f}  +- {tol:.3g}  {'ok' if ok else 'OUT'}")
    res = {"driver": "AWGN-channel/main.c unchanged, linked to libccv_awgn.so (oracle/_ref/awgn-simulation-ccv)",
           "code_index": idx, "curve": curve["name"], "points": rows, "all_within": bad == 0 and len(rows) == 8}
    json.dump(res, open(out, "w"), indent=1)
    print("points", len(rows), "outside", bad)
    sys.exit(0 if res["all_within"] else 1)


if __name__ == "__main__":
    main()

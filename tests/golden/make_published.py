#!/usr/bin/env python3
"""Writes tests/golden/published_ber.json: the reference's published BER tables as data.

Source: /root/reference/results/awgn_channel.m and results/binary_symmetric_channel.m (Octave result
tables of the reference's own simulation runs; run here, in the container that holds the reference --
the GPU box reads only the JSON). Each `ber_coded_<x>[h][_stack|_fano] = [...]` row becomes one curve:
x = a..e are codebook codes 0, 1, 2, 3, 5 (the polynomials in the comment above each row match
common/codebook.c:14-54), f = the WSPR K=32 code (codebook index 4); `h` = the hard demapper
(common/hard-demapper.c, CMakeLists.txt:41); the suffix names the decoder. Abscissae: SNR (Eb/N0 dB,
awgn_channel.m:1) and ber_uncoded (p, binary_symmetric_channel.m:1). The bit counts per point are the
schedules the files state in their comments.
"""
import json
import os
import re

SRC = "/root/reference/results"
CODE_OF = {"a": 0, "b": 1, "c": 2, "d": 3, "e": 5, "f": 4}


def rows(path):
    text = open(path).read()
    out = {}
    for m in re.finditer(r"^\s*(\w+)\s*=\s*\[([^\]]*)\];", text, flags=re.M):
        if not re.fullmatch(r"[\d.eE+\-,\s]*", m.group(2)):
            continue
        out[m.group(1)] = ([float(v) for v in m.group(2).replace(",", " ").split()], text[:m.start()].count("\n") + 1)
    return out


def curves(path, channel):
    r = rows(path)
    res = []
    for name, (vals, line) in r.items():
        m = re.fullmatch(r"ber_coded_([a-f])(h?)(?:_(stack|fano))?", name)
        if not m:
            continue
        res.append({"name": name, "source": f"results/{os.path.basename(path)}:{line}",
                    "codebook_index": CODE_OF[m.group(1)], "channel": channel,
                    "hard_demap": bool(m.group(2)), "decoder": m.group(3) or "viterbi", "ber": vals})
    return r, res


def main():
    awgn_rows, awgn = curves(os.path.join(SRC, "awgn_channel.m"), "awgn")
    bsc_rows, bsc = curves(os.path.join(SRC, "binary_symmetric_channel.m"), "bsc")
    doc = {
        "generated_by": "tests/golden/make_published.py",
        "awgn_ebn0_db": awgn_rows["SNR"][0],
        "bsc_p": bsc_rows["ber_uncoded"][0],
        "bits_schedule": {
            "awgn": "800,000 bits for Eb/N0 <= 4 dB, 8 M <= 6 dB, 80 M <= 10 dB, 800 M above "
                    "(awgn_channel.m:9-13, AWGN-channel/main.c:202-211)",
            "bsc_viterbi_stack": "800 M bits per point (binary_symmetric_channel.m:3); the driver divides "
                                 "the blocks by 10 above p = 12500, 50000 and 200000 ppm "
                                 "(binary-symmetric-channel/main.c:145-156); WSPR stack: 800 M for "
                                 "p <= 0.025, 80 M above",
            "bsc_fano": "800 M bits for p <= 0.0125, 80 M <= 0.05, 8 M <= 0.2, 800 k above",
        },
        "print_resolution": {"awgn": 1e-8, "bsc": 1e-6, "bsc_8digit": 1e-8},
        "curves": awgn + bsc,
    }
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "published_ber.json")
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"{out}: {len(doc['curves'])} curves")


if __name__ == "__main__":
    main()

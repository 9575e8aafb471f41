#!/usr/bin/env python3
"""Writes tests/golden/reference_ber.json: BER of the reference decoder as it stands, run here.

results/binary_symmetric_channel.m:7 (code 1 = codebook.c code b, BSC Viterbi) lies 2-4 % below what
the reference's own sources produce today -- oracle/_ref/ref_harness_bsc (the unmodified
binary-symmetric-channel/viterbi-decoder.c, encoder.c and the driver's rand() flips) gives 0.1157 at
p = 0.1 where the table says 0.1126, far outside the Monte-Carlo spread of 800 M bits -- so that curve
was made by a different build of the decoder than the one in the repository. This script runs the
compiled reference (oracle/Makefile `ref`) at several crossover probabilities and records errors and
bits, so the GPU's statistics are checked against the code the reference ships (test_gpu_ber.py).
Container-only: needs /root/reference built into oracle/_ref.
"""
import json
import os
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness_bsc")
CASES = [(1, p) for p in (3125, 12500, 25000, 50000, 100000, 200000, 300000)]
BLOCKS = 500000
SEEDS = (101, 102)


def main():
    out = []
    with tempfile.TemporaryDirectory() as tmp:
        for cb, p in CASES:
            errors = bits = 0
            for seed in SEEDS:
                prefix = os.path.join(tmp, f"cb{cb}_{p}_{seed}")
                subprocess.run([HARNESS, prefix, str(seed), str(BLOCKS), str(p), f"cb:{cb}"], check=True,
                               stdout=subprocess.DEVNULL)
                meta = dict(line.split() for line in open(prefix + ".meta"))
                errors += int(meta["errors"])
                bits += int(meta["blocks_decoded"]) * int(meta["blen"])
                os.remove(prefix + ".out")
            out.append({"codebook_index": cb, "channel": "bsc", "decoder": "viterbi", "p_ppm": p,
                        "errors": errors, "bits": bits, "ber": errors / bits,
                        "seeds": list(SEEDS), "blocks_per_seed": BLOCKS})
            print(out[-1])
    doc = {"generated_by": "tests/golden/make_reference_ber.py (oracle/_ref/ref_harness_bsc, the compiled "
                           "unmodified reference decoder, encoder and BSC driver logic)",
           "points": out}
    with open(os.path.join(REPO, "tests", "golden", "reference_ber.json"), "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()

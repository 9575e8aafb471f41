#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the UNMODIFIED reference.

Runs only where /root/reference exists (the build container): `make -C oracle ref` compiles the
reference sources in place into oracle/_ref/ref_harness_{awgn,bsc} (driver logic: oracle/ref_harness.c),
and this script runs them with fixed seeds and packs what crossed the decoder boundary into one .npz
per case (plain arrays, loaded with allow_pickle=False). The GPU box never runs this script.

    python tests/golden/make_golden.py [--stack-only | --hd-only | --fano-only]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")

# AWGN-channel/main.c:157-161 (stored there as float).
SCALING = {0: "0.707106781186548", 2: "0.561674881261479", 4: "0.446154216921401",
           6: "0.354392891541971", 8: "0.281504279937367"}

K7 = "2:7:{blen}:F200000000000000:B600000000000000"      # (171,133)_8
K8 = "2:8:{blen}:F900000000000000:A700000000000000"      # (371,247)_8
# Longest block the reference encoder supports: its uint8_t output counter (common/encoder.c:15-16)
# limits T = blen + K - 1 to 255, so blen <= 249 at K = 7.

# (name, channel, code spec, seed, nblocks, channel parameter)
CASES = [
    ("bsc_cb0_p25000", "bsc", "cb:0", 101, 250, "25000"),
    ("bsc_cb0_p100000", "bsc", "cb:0", 102, 250, "100000"),
    ("bsc_cb0_p300000", "bsc", "cb:0", 103, 250, "300000"),
    ("bsc_cb1_p50000", "bsc", "cb:1", 104, 100, "50000"),
    ("bsc_cb2_p50000", "bsc", "cb:2", 105, 100, "50000"),
    ("bsc_cb3_p50000", "bsc", "cb:3", 106, 100, "50000"),
    ("bsc_cb5_p50000", "bsc", "cb:5", 107, 100, "50000"),
    ("bsc_k7_p50000", "bsc", K7.format(blen=40), 108, 200, "50000"),
    ("bsc_k7_p150000", "bsc", K7.format(blen=40), 109, 200, "150000"),
    ("bsc_k8_blen200_p20000", "bsc", K8.format(blen=200), 110, 20, "20000"),
    ("awgn_cb0_0dB", "awgn", "cb:0", 201, 200, SCALING[0]),
    ("awgn_cb0_4dB", "awgn", "cb:0", 202, 200, SCALING[4]),
    ("awgn_cb0_8dB", "awgn", "cb:0", 203, 200, SCALING[8]),
    ("awgn_cb1_2dB", "awgn", "cb:1", 204, 100, SCALING[2]),
    ("awgn_cb2_2dB", "awgn", "cb:2", 205, 100, SCALING[2]),
    ("awgn_cb3_2dB", "awgn", "cb:3", 206, 200, SCALING[2]),
    ("awgn_cb3_4dB", "awgn", "cb:3", 207, 200, SCALING[4]),
    ("awgn_cb5_2dB", "awgn", "cb:5", 208, 100, SCALING[2]),
    ("awgn_k7_2dB", "awgn", K7.format(blen=40), 209, 100, SCALING[2]),
    ("awgn_k7_4dB", "awgn", K7.format(blen=40), 210, 100, SCALING[4]),
    ("awgn_k8_blen200_2dB", "awgn", K8.format(blen=200), 211, 20, SCALING[2]),
    ("awgn_k7_blen249_4dB", "awgn", K7.format(blen=249), 212, 10, SCALING[4]),
    ("awgn_k3_blen1_2dB", "awgn", "2:3:1:A000000000000000:6000000000000000", 213, 50, SCALING[2]),
    ("awgn_k3_blen7_2dB", "awgn", "2:3:7:A000000000000000:6000000000000000", 214, 50, SCALING[2]),
    ("awgn_k2_2dB", "awgn", "2:2:40:C000000000000000:8000000000000000", 215, 50, SCALING[2]),
    ("awgn_n1k3_4dB", "awgn", "1:3:40:E000000000000000", 216, 50, SCALING[4]),
]

# AWGN through the reference's hard demapper (common/hard-demapper.c linked instead of demapper.c):
# (name, channel, code spec, seed, nblocks, channel parameter); manifest entries carry demapper "hard"
HD_CASES = [
    ("awgn_hd_cb0_4dB", "awgn", "cb:0", 501, 200, SCALING[4]),
    ("awgn_hd_cb5_6dB", "awgn", "cb:5", 502, 100, SCALING[6]),
    ("awgn_hd_k7_4dB", "awgn", K7.format(blen=40), 503, 100, SCALING[4]),
]

# K=15 r=1/2 (46321,51271)_8 for BASELINE config 5 (the codebook has no K=15 code); the metric weight
# is the codebook's long-code (WSPR, K=32) value, codebook.c:71-73.
K15 = "2:15:{blen}:" + "%016X:%016X" % (0o46321 << 49, 0o51271 << 49)

# Stack-decoder cases (manifest_stack.json): (name, channel, code spec, seed, nblocks, channel
# parameter, metrics override or None = the codebook's)
STACK_CASES = [
    ("stack_awgn_cb0_4dB", "awgn", "cb:0", 301, 200, SCALING[4], None),
    ("stack_awgn_cb0_8dB", "awgn", "cb:0", 302, 200, SCALING[8], None),
    ("stack_awgn_cb3_2dB", "awgn", "cb:3", 303, 100, SCALING[2], None),
    ("stack_awgn_cb4_4dB", "awgn", "cb:4", 304, 60, SCALING[4], None),
    ("stack_awgn_cb5_4dB", "awgn", "cb:5", 305, 100, SCALING[4], None),
    ("stack_awgn_k15_4dB", "awgn", K15.format(blen=40), 306, 100, SCALING[4], "-7.0"),
    ("stack_awgn_k15_2dB", "awgn", K15.format(blen=40), 307, 60, SCALING[2], "-7.0"),
    ("stack_awgn_k7_blen200_4dB", "awgn", K7.format(blen=200), 308, 20, SCALING[4], "-10.0"),
    ("stack_bsc_cb0_p25000", "bsc", "cb:0", 401, 200, "25000", None),
    ("stack_bsc_cb2_p50000", "bsc", "cb:2", 402, 100, "50000", None),
    ("stack_bsc_cb4_p20000", "bsc", "cb:4", 403, 60, "20000", None),
    ("stack_bsc_k15_p30000", "bsc", K15.format(blen=40), 404, 100, "30000", "1,-11"),
]


# Fano-decoder cases (manifest_fano.json), same fields as STACK_CASES
FANO_CASES = [
    ("fano_awgn_cb0_4dB", "awgn", "cb:0", 601, 200, SCALING[4], None),
    ("fano_awgn_cb0_8dB", "awgn", "cb:0", 602, 200, SCALING[8], None),
    ("fano_awgn_cb3_4dB", "awgn", "cb:3", 603, 100, SCALING[4], None),
    ("fano_awgn_cb4_6dB", "awgn", "cb:4", 604, 60, SCALING[6], None),
    ("fano_awgn_cb5_4dB", "awgn", "cb:5", 605, 100, SCALING[4], None),
    ("fano_awgn_k15_4dB", "awgn", K15.format(blen=40), 606, 100, SCALING[4], "-11.0"),
    ("fano_awgn_k7_blen200_6dB", "awgn", K7.format(blen=200), 607, 20, SCALING[6], "-110.0"),
    ("fano_bsc_cb0_p10000", "bsc", "cb:0", 701, 200, "10000", None),
    ("fano_bsc_cb2_p30000", "bsc", "cb:2", 702, 100, "30000", None),
    ("fano_bsc_cb4_p20000", "bsc", "cb:4", 703, 60, "20000", None),
    ("fano_bsc_k15_p30000", "bsc", K15.format(blen=40), 704, 100, "30000", "1,-11"),
]


def run_case(name, channel, spec, seed, nblocks, param, tmp, decoder="viterbi", metrics=None,
             demapper="soft"):
    suffix = ("" if decoder == "viterbi" else "_" + decoder) + ("_hd" if demapper == "hard" else "")
    exe = os.path.join(REF_DIR, f"ref_harness_{channel}{suffix}")
    prefix = os.path.join(tmp, name)
    cmd = [exe, prefix, str(seed), str(nblocks), param, spec] + ([metrics] if metrics else [])
    subprocess.run(cmd, check=True, timeout=600)
    meta = {}
    with open(prefix + ".meta") as f:
        for line in f:
            k, v = line.split()
            meta[k] = v
    n, K, blen = int(meta["n"]), int(meta["K"]), int(meta["blen"])
    polys = np.array([int(meta[f"poly{k}"], 16) for k in range(n)], dtype=np.uint64)
    T = blen + K - 1
    IB, OB = (blen + 7) // 8, (T + 7) // 8
    arrays = {
        "info": np.fromfile(prefix + ".info", dtype=np.uint8).reshape(nblocks, IB),
        "out": np.fromfile(prefix + ".out", dtype=np.uint8).reshape(nblocks, OB),
        "n": np.int32(n), "K": np.int32(K), "blen": np.int32(blen), "polys": polys,
        "seed": np.uint32(seed), "errors": np.uint64(int(meta["errors"])),
    }
    if channel == "awgn":
        arrays["rx"] = np.fromfile(prefix + ".rx", dtype=np.float32).reshape(nblocks, T, 1 << n)
        arrays["scaling"] = np.float32(float(param))
    else:
        arrays["rx"] = np.fromfile(prefix + ".rx", dtype=np.uint8).reshape(nblocks, T)
        arrays["p_ppm"] = np.int32(int(param))
        arrays["path_metric"] = np.fromfile(prefix + ".pm", dtype=np.int32).reshape(nblocks)
    if decoder == "stack":
        arrays["metric_weight"] = np.float32(float(meta["metric_weight"]))
        arrays["bit_metrics"] = np.array([int(meta["bit_metric0"]), int(meta["bit_metric1"])], np.int32)
    if decoder == "fano":
        arrays["fano_metric_weight"] = np.float32(float(meta["fano_metric_weight"]))
        arrays["fano_bit_metrics"] = np.array([int(meta["fano_bit_metric0"]), int(meta["fano_bit_metric1"])],
                                              np.int32)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    entry = {"name": name, "channel": channel, "spec": spec, "seed": seed, "nblocks": nblocks,
             "param": param, "errors": int(meta["errors"])}
    if decoder in ("stack", "fano"):
        entry.update(decoder=decoder, metrics=metrics)
    if demapper == "hard":
        entry.update(demapper="hard")
    return entry


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_golden.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    manifest = []
    only_new = any(a in sys.argv for a in ("--stack-only", "--hd-only", "--fano-only"))
    with tempfile.TemporaryDirectory() as tmp:
        for case in ([] if only_new else CASES):
            manifest.append(run_case(*case, tmp))
            print(manifest[-1])
        if "--stack-only" not in sys.argv and "--fano-only" not in sys.argv:
            if only_new:   # append to the existing manifest without rewriting the other fixtures
                with open(os.path.join(HERE, "manifest.json")) as f:
                    manifest = [m for m in json.load(f) if m.get("demapper") != "hard"]
            for case in HD_CASES:
                manifest.append(run_case(*case, tmp, demapper="hard"))
                print(manifest[-1])
    if manifest:
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1)
    if "--hd-only" in sys.argv:
        return
    if "--fano-only" in sys.argv or "--stack-only" not in sys.argv:
        fano = []
        with tempfile.TemporaryDirectory() as tmp:
            for name, channel, spec, seed, nb, param, metrics in FANO_CASES:
                fano.append(run_case(name, channel, spec, seed, nb, param, tmp, "fano", metrics))
                print(fano[-1])
        with open(os.path.join(HERE, "manifest_fano.json"), "w") as f:
            json.dump(fano, f, indent=1)
        if "--fano-only" in sys.argv:
            return
    stack = []
    with tempfile.TemporaryDirectory() as tmp:
        for name, channel, spec, seed, nb, param, metrics in STACK_CASES:
            stack.append(run_case(name, channel, spec, seed, nb, param, tmp, "stack", metrics))
            print(stack[-1])
    with open(os.path.join(HERE, "manifest_stack.json"), "w") as f:
        json.dump(stack, f, indent=1)


if __name__ == "__main__":
    main()

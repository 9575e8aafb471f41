"""Consecutive headline decodes on one stream vs alternated over two streams (one plan and one output
buffer per stream), round-robin repeats on one box: does the next batch's launch fill the previous
launch's tail (the last ~4 % of a launch has SIMDs with one wave or none)?

  python tools/overlap_probe.py [--frames 104] [--steps 40] [--reps 5] [--code k7] [--channel soft|bsc]

Prints one JSON line per (mode, rep) and a summary; checks the outputs and error counts of every
stream equal the one-stream decode's.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "convolutional-codes_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ccviterbi import HARD, K7, K9, SOFT, Plan, channel as ch  # noqa: E402

FRAME = 25000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=104)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--code", default="k7")
    ap.add_argument("--channel", default="soft")
    ap.add_argument("--streams", type=int, default=2)
    args = ap.parse_args()
    code = {"k7": K7, "k9": K9}[args.code]
    hard = args.channel == "bsc"
    nb = args.frames * FRAME
    if hard:
        info, rx = ch.bsc_blocks(code, nb, 50000, 1)
    else:
        info, rx = ch.awgn_blocks(code, nb, ch.noise_scaling(4.0), 1)
    d_rx = torch.from_numpy(rx).cuda()
    d_info = torch.from_numpy(info).cuda()
    S = args.streams
    streams = [torch.cuda.Stream() for _ in range(S)]
    plans = [Plan(code, HARD if hard else SOFT) for _ in range(S)]
    for p in plans:
        p.reserve(nb)
    outs = [torch.empty((nb, code.out_bytes), dtype=torch.uint8, device="cuda") for _ in range(S)]
    errs = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(S)]

    def run(mode, steps):
        ns = 1 if mode == "one" else S
        for e in errs:
            e.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            i = k % ns
            with torch.cuda.stream(streams[i]):
                plans[i].decode_device(d_rx, nb, outs[i], d_info=d_info, d_errors=errs[i], stream=streams[i])
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    # clock warm-up
    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        run("two", 10)
    res = {"one": [], "two": []}
    for rep in range(args.reps):
        for mode in ("one", "two"):
            w = run(mode, args.steps)
            ms = w * 1e3 / args.steps
            res[mode].append(ms)
            print(json.dumps({"mode": mode, "rep": rep, "ms_per_step": round(ms, 4),
                              "gbit_s": round(nb * code.blen / (ms * 1e-3) / 1e9, 2)}), flush=True)
    # exactness: every stream's output and count equal the one-stream decode's
    run("one", 1)
    ref, ref_err = outs[0].clone(), int(errs[0].item())
    run("two", S)
    for i in range(S):
        assert torch.equal(outs[i], ref) and int(errs[i].item()) == ref_err, i
    one, two = np.median(res["one"]), np.median(res["two"])
    print(json.dumps({"summary": True, "code": args.code, "channel": args.channel, "frames": args.frames,
                      "streams": S, "one_ms": round(float(one), 4), "two_ms": round(float(two), 4),
                      "ratio": round(float(two / one), 4), "exact": True}))


if __name__ == "__main__":
    main()

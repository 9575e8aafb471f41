#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC traffic passes (tools/pmc_traffic.sh): a calibration copy with a
known byte count, then the bench decode (same code, frames and layout as bench.py)."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "convolutional-codes_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="k7")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--layout", choices=("block", "step"), default="block")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from ccviterbi import SOFT, Plan, channel as ch, named_code
    from ccviterbi.decoder import FLAG_STEP_MAJOR
    code = named_code(args.code)
    nb = args.frames * 25000
    info, rx = ch.awgn_blocks(code, nb, ch.noise_scaling(4.0), 0xC0DE)
    host_in = rx if args.layout == "block" else np.ascontiguousarray(rx.transpose(1, 0, 2))
    d_rx = torch.from_numpy(host_in).to("cuda")
    d_info = torch.from_numpy(info).to("cuda")
    # calibration: a plain device copy of the same number of bytes (reads and writes known exactly)
    dst = torch.empty_like(d_rx)
    for _ in range(args.reps):
        dst.copy_(d_rx)
    torch.cuda.synchronize()
    d_out = torch.empty((nb, code.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    plan = Plan(code, SOFT, FLAG_STEP_MAJOR if args.layout == "step" else 0)
    plan.reserve(nb)
    for _ in range(args.reps):
        plan.decode_device(d_rx, nb, d_out, d_info=d_info, d_errors=d_err,
                           stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    print("copy_bytes", d_rx.numel() * 4, "nblocks", nb)


if __name__ == "__main__":
    main()

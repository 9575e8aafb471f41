#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC passes (tools/pmc_workload.sh): a calibration copy with a known
byte count, then REPS decodes of the bench workload (same code, frames, layout, channel and decoder as
bench.py, same seeds). Prints `copy_bytes N nblocks N`."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "convolutional-codes_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default=None)
    ap.add_argument("--frames", type=int, default=104)
    ap.add_argument("--layout", choices=("block", "step"), default="block")
    ap.add_argument("--channel", choices=("awgn", "bsc"), default="awgn")
    ap.add_argument("--decoder", choices=("viterbi", "stack", "fano"), default="viterbi")
    ap.add_argument("--ebn0", type=float, default=4.0)
    ap.add_argument("--p-ppm", type=int, default=50000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0xC0DE)
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--iq", action="store_true",
                    help="Fano, soft: the frames as received points from the on-device channel, decoded "
                         "with option fano_input 1 (bench.py fano_received_points)")
    args = ap.parse_args()
    import torch

    from ccviterbi import HARD, SOFT, FanoPlan, Plan, StackPlan, channel as ch, named_code
    from ccviterbi.decoder import FLAG_STEP_MAJOR
    code = named_code(args.code or ("k7" if args.decoder == "viterbi" else "k15"))
    nb = args.frames * 25000
    hard = args.channel == "bsc"
    if hard:
        info, rx = ch.bsc_blocks(code, nb, args.p_ppm, args.seed)
    else:
        info, rx = ch.awgn_blocks(code, nb, ch.noise_scaling(args.ebn0), args.seed)
    host_in = rx if args.layout == "block" else np.ascontiguousarray(rx.transpose(1, 0, 2))
    d_rx = torch.from_numpy(host_in).to("cuda")
    d_info = torch.from_numpy(info).to("cuda")
    # calibration: a plain device copy of the same number of bytes (reads and writes known exactly)
    dst = torch.empty_like(d_rx)
    for _ in range(args.reps):
        dst.copy_(d_rx)
    torch.cuda.synchronize()
    copy_bytes = d_rx.numel() * d_rx.element_size()
    del dst
    d_out = torch.empty((nb, code.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    chan = HARD if hard else SOFT
    if args.decoder == "stack":
        plan = StackPlan(code, chan)
    elif args.decoder == "fano":
        plan = FanoPlan(code, chan)
    else:
        plan = Plan(code, chan, FLAG_STEP_MAJOR if args.layout == "step" else 0)
    for opt in args.option:
        name, value = opt.split("=", 1)
        plan.set_option(name, int(value))
    if args.iq:   # the same Philox frames, as received points
        plan.set_option("fano_input", 1)
        d_rx = torch.empty((nb, code.steps, 2), dtype=torch.float32, device="cuda")
        plan.simulate_frames(args.seed, 0, nb, ch.noise_scaling(args.ebn0), d_rx, d_info=d_info, iq=True)
    plan.reserve(nb)
    for _ in range(args.reps):
        plan.decode_device(d_rx, nb, d_out, d_info=d_info, d_errors=d_err, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    print("copy_bytes", copy_bytes, "nblocks", nb)


if __name__ == "__main__":
    main()

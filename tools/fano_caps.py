#!/usr/bin/env python3
"""Fano two-pass schedule sweep: search-length percentiles of the bench workload (K=15, 104 frames)
and the decode time for several park caps (plan option fano_cap; 0 = one pass), interleaved repeats.
usage: fano_caps.py [--ebn0 4] [--channel awgn|bsc] [--frames 104] caps..."""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "convolutional-codes_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ebn0", type=float, default=4.0)
    ap.add_argument("--channel", default="awgn")
    ap.add_argument("--p-ppm", type=int, default=50000)
    ap.add_argument("--frames", type=int, default=104)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("caps", nargs="*", default=["0", "54000", "162000", "324000"])
    args = ap.parse_args()
    import torch
    from ccviterbi import HARD, K15, SOFT, FanoPlan, channel as ch
    c, nb = K15, args.frames * 25000
    hard = args.channel == "bsc"
    if hard:
        info, rx = ch.bsc_blocks(c, nb, args.p_ppm, 0xC0DE)
    else:
        info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(args.ebn0), 0xC0DE)
    d_rx = torch.from_numpy(rx).cuda()
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_it = torch.zeros(nb, dtype=torch.int32, device="cuda")
    plan = FanoPlan(c, HARD if hard else SOFT)
    plan.set_option("fano_cap", 0)
    plan.decode_fano_device(d_rx, nb, d_out, d_iterations=d_it)
    torch.cuda.synchronize()
    it = d_it.cpu().numpy()
    qs = [50, 75, 90, 95, 97, 98, 99, 99.5, 99.9]
    print(f"{args.channel} {args.ebn0 if not hard else args.p_ppm}: search length (outer ticks) mean {it.mean():.0f}, "
          + ", ".join(f"p{q} {np.percentile(it, q):.0f}" for q in qs) + f", timeouts {(it == 10000 * c.steps).mean():.4f}")
    ref = d_out.cpu().numpy().copy()
    times = {cap: [] for cap in args.caps}
    for _ in range(args.reps):
        for cap in args.caps:
            plan.set_option("fano_cap", int(cap))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            plan.decode_fano_device(d_rx, nb, d_out)
            torch.cuda.synchronize()
            times[cap].append(time.perf_counter() - t0)
            assert np.array_equal(d_out.cpu().numpy(), ref), cap
    for cap in args.caps:
        t = min(times[cap])
        print(f"  cap {cap:>8s}: {t * 1e3:8.1f} ms  {nb * c.blen / t / 1e6:7.1f} Mbit/s", flush=True)


if __name__ == "__main__":
    main()

"""Throughput of the fused on-device channel + decoder (ccv_simulate_device), the kernel behind the
Eb/N0 sweeps: `python tools/chan_bench.py [--code k7 k9 ...] [--noise f64 f32] [--ebn0 12]`.
Per (code, noise): 0.3 s warm-up, then REPS timed runs of 8 chunks of 2.6 M blocks (832 M info bits at
blen 40, the sweep's point size); prints best and median Gbit/s. CCV_LIB_DIR selects an A/B build.
"""
import argparse
import json
import statistics
import time

from ccviterbi import HARD, SOFT, named_code
from ccviterbi.sim import DeviceChannelDecoder


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", nargs="+", default=["k7", "k9"])
    ap.add_argument("--noise", nargs="+", default=["f64", "f32"])
    ap.add_argument("--ebn0", type=float, default=12.0)
    ap.add_argument("--bsc", type=int, default=None, help="BSC at this p_ppm instead of AWGN")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunks", type=int, default=8)
    ap.add_argument("--tag", default="")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="plan option (ccv_plan_set_option), e.g. channel_lds_decisions=0")
    args = ap.parse_args()
    import torch
    for name in args.code:
        code = named_code(name)
        channel, point = (HARD, args.bsc) if args.bsc is not None else (SOFT, args.ebn0)
        for nz in (["-"] if channel == HARD else args.noise):
            dev = DeviceChannelDecoder(code, channel, 25000, 0xC0DE, noise_f32=nz == "f32")
            for opt in args.option:
                oname, value = opt.split("=")
                dev.plan.set_option(oname, int(value))
            dev.warm_up(0.3, point)
            nb = dev.chunk * args.chunks
            rates = []
            for r in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dev(point, r * nb, nb)   # syncs (reads the error count)
                rates.append(nb * code.blen / (time.perf_counter() - t0) / 1e9)
            print(json.dumps({"tag": args.tag, "options": args.option, "code": name, "noise": nz, "point": point,
                              "bits": nb * code.blen, "best_gbit_s": round(max(rates), 2),
                              "median_gbit_s": round(statistics.median(rates), 2)}), flush=True)


if __name__ == "__main__":
    main()

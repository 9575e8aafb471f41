"""Batched BER sweep: the counterpart of the reference drivers (AWGN-channel/main.c:146-242,
binary-symmetric-channel/main.c:100-183) built for throughput.

The reference streams one block at a time through encoder -> channel -> decoder callbacks and counts
errors in the decoded callback. Here a sweep point is a set of FRAMES (frame_blocks independent
blocks each); block b of frame f at point p draws its randomness from the Philox stream
(seed, p << 40 | f * frame_blocks + b), so results do not depend on how frames are spread over
processes. Rank r of a world of W processes (one per GPU) takes the contiguous frame range
[r*F/W, (r+1)*F/W) of the point's F frames; each frame is produced on the host (libccv_sim) or on the
GPU (ccv_simulate_device), decoded on the GPU with the bit-error count fused into the traceback, and at the end ONE all-reduce (sum, int64) of the (errors, bits) counters goes over
torch.distributed (RCCL over xGMI with the nccl backend, gloo on CPU).
"""
import math
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import channel as ch
from .code import HARD, SOFT, Code


@dataclass
class BerPoint:
    param: float          # Eb/N0 in dB (AWGN) or crossover probability in ppm (BSC)
    errors: int
    bits: int

    @property
    def ber(self):
        return self.errors / self.bits if self.bits else float("nan")


def reference_awgn_bits(ebn0_db: float, blen: int) -> int:
    """Bits the reference simulates per AWGN point (AWGN-channel/main.c:202-211)."""
    nb = 800000000 // blen
    if ebn0_db <= 4.0:
        nb //= 10
    if ebn0_db <= 6.0:
        nb //= 10
    if ebn0_db <= 10.0:
        nb //= 10
    return nb * blen


def reference_bsc_bits(p_ppm: int, blen: int) -> int:
    """Bits the reference simulates per BSC point (binary-symmetric-channel/main.c:145-156)."""
    nb = 20000000
    if p_ppm > 12500:
        nb //= 10
    if p_ppm > 50000:
        nb //= 10
    if p_ppm > 200000:
        nb //= 10
    return nb * blen


DECODERS = ("viterbi", "stack", "fano")


def _make_plan(code: Code, channel: int, decoder: str):
    from .decoder import FanoPlan, Plan, StackPlan
    return {"viterbi": Plan, "stack": StackPlan, "fano": FanoPlan}[decoder](code, channel)


class GpuFrameDecoder:
    """Decodes one host frame on the current GPU and returns its bit-error count (Viterbi, or the
    stack / Fano decoder: AWGN-channel/{viterbi,stack,fano}-decoder.c and their BSC twins)."""

    def __init__(self, code: Code, channel: int, frame_blocks: int, device=None, decoder: str = "viterbi"):
        import torch

        self.torch = torch
        self.device = torch.device(device if device is not None else "cuda")
        self.plan = _make_plan(code, channel, decoder)
        self.plan.reserve(frame_blocks)
        self.code, self.channel = code, channel
        in_elems = code.steps * ((1 << code.n) if channel == SOFT else 1)
        dt = torch.float32 if channel == SOFT else torch.uint8
        self.d_in = torch.empty((frame_blocks, in_elems), dtype=dt, device=self.device)
        self.d_info = torch.empty((frame_blocks, code.info_bytes), dtype=torch.uint8, device=self.device)
        self.d_out = torch.empty((frame_blocks, code.out_bytes), dtype=torch.uint8, device=self.device)
        self.d_pm = torch.empty(frame_blocks, dtype=torch.int32, device=self.device)
        self.d_err = torch.zeros(1, dtype=torch.int64, device=self.device)

    def __call__(self, info: np.ndarray, data: np.ndarray) -> int:
        torch = self.torch
        nb = info.shape[0]
        self.d_in[:nb].copy_(torch.from_numpy(data.reshape(nb, -1)))
        self.d_info[:nb].copy_(torch.from_numpy(info))
        self.d_err.zero_()
        stream = torch.cuda.current_stream(self.device)
        self.plan.decode_device(self.d_in, nb, self.d_out,
                                d_path_metric=self.d_pm if self.channel == HARD else None,
                                d_info=self.d_info, d_errors=self.d_err, stream=stream)
        return int(self.d_err.item())


class DeviceChannelDecoder:
    """Frames generated AND decoded on the current GPU (ccv_simulate_device): the same Philox frames
    as the host producers, no host generation and no input traffic. A rank's frames are contiguous
    blocks of the point's Philox stream, so they go to the device in chunks of `chunk_blocks` (104
    frames for the Viterbi kernels: enough groups for every resident wave). For the stack / Fano
    decoders the on-device channel writes its output (the demapped floats or the BSC symbols) into one
    HBM chunk buffer that the sequential decoder then reads, with its error count fused (frames only:
    no Viterbi plan and no decode of the chunk beside the sequential one)."""

    def __init__(self, code: Code, channel: int, frame_blocks: int, seed: int, device=None,
                 hard_demap=False, decoder: str = "viterbi", chunk_blocks: Optional[int] = None,
                 noise_f32: bool = False, fano_iq: Optional[bool] = None):
        import torch

        from .decoder import Plan
        self.torch = torch
        self.device = torch.device(device if device is not None else "cuda")
        if chunk_blocks is None:
            # stack: 32 frames per launch, where the persistent rows' tail of long searches weighs
            # little (568 Mbit/s at 4 frames, 863 at 32)
            per_launch = {"viterbi": 2_600_000, "stack": 800_000}.get(decoder, 200_000)
            chunk_blocks = frame_blocks * max(1, per_launch // frame_blocks)
        self.chunk = chunk_blocks
        # Viterbi: one plan generates and decodes (fused); stack / Fano: the sequential plan itself
        # generates the frames (CCV_CHANNEL_FRAMES_ONLY, no Viterbi plan, any K) and then decodes them
        self.seq = None if decoder == "viterbi" else _make_plan(code, channel, decoder)
        self.plan = Plan(code, channel) if self.seq is None else self.seq
        self.plan.reserve(self.chunk)
        self.channel, self.frame_blocks, self.seed = channel, frame_blocks, seed
        self.hard_demap = hard_demap
        self.noise_f32 = noise_f32
        self.d_err = torch.zeros(1, dtype=torch.int64, device=self.device)
        # Fano, soft rate 1/2: the channel writes the received points and the decoder demaps them
        # (CCV_CHANNEL_IQ + option fano_input 1: half the bytes per node, the same decoder input)
        if fano_iq is None:
            fano_iq = decoder == "fano" and channel == SOFT and code.n == 2 and code.K <= 32
        self.iq = bool(fano_iq) and decoder == "fano"
        if self.iq:
            self.seq.set_option("fano_input", 1)
        if self.seq is not None:
            self.seq.reserve(self.chunk)
            per_block = code.steps * (2 if self.iq else (1 << code.n) if channel == SOFT else 1)
            dt = torch.float32 if channel == SOFT else torch.uint8
            self.d_ch = torch.empty((self.chunk, per_block), dtype=dt, device=self.device)
            self.d_info = torch.empty((self.chunk, code.info_bytes), dtype=torch.uint8, device=self.device)
            self.d_out = torch.empty((self.chunk, code.out_bytes), dtype=torch.uint8, device=self.device)
            self.d_pm = torch.empty(self.chunk, dtype=torch.int32, device=self.device)

    def warm_up(self, seconds: float, point: Optional[float] = None) -> int:
        """Decode throw-away slices (blocks 2^62.., a Philox range no point uses) until `seconds` have
        passed: the GPU's clock ramp (~35 ms of load) and the first launches then stay
        out of the first point's time. A Viterbi slice is one whole chunk (the launch size of the
        points: small launches leave the chip below the power state the points run at, and the first
        points of a sweep came out 10-25 % slow); the stack / Fano decoders run one
        frame per slice, so the limit is kept to within one slice. The Viterbi kernels run at `point`
        (the sweep's first point; their time does not depend on the noise); the sequential decoders
        at a low-noise point (10 dB / 1,000 ppm), where no search runs into its timeout. Returns the
        slices run."""
        import time
        seq = self.seq is not None
        if seq or point is None:
            point = (10.0 if seq else 4.0) if self.channel == SOFT else (1000 if seq else 50000)
        nb = min(self.chunk, self.frame_blocks) if seq else self.chunk
        n, t0 = 0, time.perf_counter()
        while n == 0 or time.perf_counter() - t0 < seconds:
            self(point, 1 << 62, nb)
            n += 1
        return n

    def __call__(self, point: float, first_block: int, nblocks: int) -> int:
        """Bit errors of blocks first_block .. first_block + nblocks - 1 at Eb/N0 (dB) or p_ppm `point`."""
        param = ch.noise_scaling(point) if self.channel == SOFT else int(point)
        self.d_err.zero_()
        stream = self.torch.cuda.current_stream(self.device)
        for first in range(first_block, first_block + nblocks, self.chunk):
            nb = min(self.chunk, first_block + nblocks - first)
            if self.seq is None:
                self.plan.simulate_device(self.seed, first, nb, param, d_errors=self.d_err,
                                          stream=stream, hard_demap=self.hard_demap, noise_f32=self.noise_f32)
                continue
            self.seq.simulate_frames(self.seed, first, nb, param, self.d_ch, d_info=self.d_info,
                                     stream=stream, hard_demap=self.hard_demap, noise_f32=self.noise_f32,
                                     iq=self.iq)
            self.seq.decode_device(self.d_ch, nb, self.d_out,
                                   d_path_metric=self.d_pm if self.channel == HARD else None,
                                   d_info=self.d_info, d_errors=self.d_err, stream=stream)
        return int(self.d_err.item())


def shard(nframes: int, rank: int, world: int) -> range:
    """Rank r's frames: a contiguous range (the per-block Philox stream makes the totals independent
    of how frames are spread; contiguous ranges let the on-device channel take them in one call)."""
    return range(nframes * rank // world, nframes * (rank + 1) // world)


def ber_sweep(code: Code, points: Sequence[float], channel: int = SOFT,
              bits_per_point: Optional[Callable[[float], int]] = None, frame_blocks: int = 25000,
              seed: int = 0xC0DE, rank: int = 0, world: int = 1,
              decode: Optional[Callable[[np.ndarray, np.ndarray], int]] = None,
              threads: Optional[int] = None, reduce: bool = True,
              device_channel: bool = False, hard_demap: bool = False, noise_f32: bool = False,
              decoder: str = "viterbi", point_index: int = 0,
              device_decoder: Optional["DeviceChannelDecoder"] = None) -> List[BerPoint]:
    """BER at each point; `decode(info, data) -> errors` defaults to the GPU decoder. With
    device_channel the frames are generated on the GPU as well (DeviceChannelDecoder, or the one
    passed as `device_decoder`). Point k of `points` draws the Philox stream of point
    point_index + k, so a sweep split into calls gives the same frames."""
    if bits_per_point is None:
        if channel == SOFT:
            bits_per_point = lambda p: reference_awgn_bits(p, code.blen)   # noqa: E731
        else:
            bits_per_point = lambda p: reference_bsc_bits(int(p), code.blen)  # noqa: E731
    dev = device_decoder
    if dev is None and device_channel and decode is None:
        dev = DeviceChannelDecoder(code, channel, frame_blocks, seed, hard_demap=hard_demap, decoder=decoder,
                                   noise_f32=noise_f32)
    if noise_f32 and dev is None:
        raise ValueError("noise_f32 is an option of the on-device channel (device_channel=True)")
    if decode is None and dev is None:
        decode = GpuFrameDecoder(code, channel, frame_blocks, decoder=decoder)
    counters = np.zeros((len(points), 2), np.int64)
    for row, p in enumerate(points):
        pi = point_index + row   # the point's Philox stream: (seed, pi << 40 | block)
        nframes = max(1, math.ceil(bits_per_point(p) / (frame_blocks * code.blen)))
        mine = shard(nframes, rank, world)
        if dev is not None:
            if len(mine):
                counters[row, 0] += dev(p, (pi << 40) + mine.start * frame_blocks, len(mine) * frame_blocks)
            counters[row, 1] += len(mine) * frame_blocks * code.blen
            continue
        for f in mine:
            first = (pi << 40) + f * frame_blocks
            if channel == SOFT:
                info, data = ch.awgn_blocks(code, frame_blocks, ch.noise_scaling(p), seed,
                                            first_block=first, threads=threads, hard_demap=hard_demap)
            else:
                info, data = ch.bsc_blocks(code, frame_blocks, int(p), seed, first_block=first,
                                           threads=threads)
            counters[row, 0] += decode(info, data)
            counters[row, 1] += frame_blocks * code.blen
    if reduce and world > 1:
        counters = all_reduce_counters(counters)
    return [BerPoint(float(p), int(e), int(b)) for p, (e, b) in zip(points, counters)]


def all_reduce_counters(counters: np.ndarray) -> np.ndarray:
    """One sum all-reduce of the int64 counter table over the default process group."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.from_numpy(np.ascontiguousarray(counters, np.int64)).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def ber_interval(errors: int, bits: int, z: float = 3.29, burst: float = 1.0):
    """Two-sided interval for the BER behind `errors` of `bits`: Wilson's binomial score interval with
    the variance inflated by `burst` (decoder errors come in bursts inside a block, so the counts are
    over-dispersed against independent bits); z = 3.29 is 99.9 %."""
    if bits <= 0:
        return (0.0, 1.0)
    n = bits / burst
    p = errors / bits
    z2 = z * z
    den = 1.0 + z2 / n
    mid = (p + z2 / (2 * n)) / den
    half = z * math.sqrt(p * (1 - p) / n + z2 / (4 * n * n)) / den
    return (max(0.0, mid - half), min(1.0, mid + half))


def _parse_points(text: Optional[str], channel: int) -> List[float]:
    """Comma list, or an inclusive range start:stop[:step] (step 2, the reference's Eb/N0 spacing,
    AWGN-channel/main.c:193-197, when omitted)."""
    if not text:
        return list(ch.REFERENCE_EBN0_DB if channel == SOFT else ch.REFERENCE_P_PPM)
    if ":" in text:
        parts = [float(x) for x in text.split(":")]
        start, stop, step = parts[0], parts[1], parts[2] if len(parts) > 2 else 2.0
        if step <= 0 or len(parts) > 3:
            raise ValueError(f"bad point range {text!r}")
        n = int(math.floor((stop - start) / step + 1e-9)) + 1
        return [start + i * step for i in range(max(n, 0))]
    return [float(x) for x in text.split(",") if x.strip()]


def main(argv=None, decode=None):
    """Sharded BER sweep CLI: `python -m ccviterbi.sim [--gpus N] ...` prints one JSON line per point
    on rank 0 (the reference drivers print one BER line per point, AWGN-channel/main.c:233,
    binary-symmetric-channel/main.c:175). `decode(info, data) -> errors` replaces the GPU decoder
    (tests: the oracle under gloo)."""
    import argparse
    import json
    import os
    import sys
    import time

    from . import launch
    from .code import named_code

    ap = argparse.ArgumentParser(prog="python -m ccviterbi.sim", description=main.__doc__)
    ap.add_argument("--code", default="code0", help="k7, k9, code0..code5 / wspr, suffix :true = true parity")
    ap.add_argument("--channel", choices=("awgn", "bsc"), default="awgn")
    ap.add_argument("--decoder", choices=DECODERS, default="viterbi")
    ap.add_argument("--points", default=None,
                    help="comma-separated Eb/N0 dB (awgn) or p in ppm (bsc), or start:stop[:step] (step 2); "
                         "default the reference sweep "
                         "(AWGN-channel/main.c:150-161, binary-symmetric-channel/main.c:103-109)")
    ap.add_argument("--bits", type=float, default=None,
                    help="info bits per point (default: the reference's schedule, AWGN-channel/main.c:202-211, "
                         "binary-symmetric-channel/main.c:145-156)")
    ap.add_argument("--bits-scale", type=float, default=1.0, help="multiply the reference schedule")
    ap.add_argument("--frame-blocks", type=int, default=25000, help="blocks per frame (25,000 = 1 M bits)")
    ap.add_argument("--seed", type=int, default=0xC0DE)
    ap.add_argument("--device-channel", action="store_true",
                    help="generate the frames on the GPU (encoder, mapper, Philox AWGN / BSC, demapper)")
    ap.add_argument("--hard-demap", action="store_true", help="common/hard-demapper.c instead of demapper.c")
    ap.add_argument("--noise", choices=("f64", "f32"), default="f64",
                    help="on-device AWGN Box-Muller: f64 (default, the reference's double precision) or the "
                         "opt-in f32 from the hardware transcendentals (faster; the same BER statistics, "
                         "not the same samples)")
    ap.add_argument("--threads", type=int, default=None, help="host producer threads per rank")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); self-launches torchrun")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default=None,
                    help="process-group backend (default nccl = RCCL over xGMI)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on cuda:0, reductions over gloo")
    ap.add_argument("--out", default=None, help="also write the points as a JSON list (rank 0)")
    ap.add_argument("--warmup", type=float, default=0.2,
                    help="seconds of throw-away device-channel chunks before the first point (allocation, "
                         "clock ramp); 0 = none")
    ap.add_argument("--first-point-index", type=int, default=0,
                    help="Philox stream index of the first point (point k draws stream first + k): a sweep "
                         "split over several invocations reproduces the frames of one call when each part "
                         "passes the index its first point had there")
    args = ap.parse_args(argv)

    if launch.needs_launch(args.gpus):
        return launch.relaunch(args.gpus, "ccviterbi.sim", sys.argv[1:] if argv is None else list(argv),
                               module=True)
    rank, local_rank, world = launch.world_from_env()
    launch.check_world(args.gpus, world)
    code = named_code(args.code)
    channel = HARD if args.channel == "bsc" else SOFT
    if args.hard_demap and channel != SOFT:
        raise SystemExit("--hard-demap belongs to the AWGN channel")
    if args.noise == "f32" and (channel != SOFT or not args.device_channel):
        raise SystemExit("--noise f32 is an option of the on-device AWGN channel (--device-channel)")
    points = _parse_points(args.points, channel)
    # --same-device puts every rank on cuda:0, which RCCL refuses: gloo then, as in bench.py
    backend = args.backend or ("gloo" if decode is not None or args.same_device else "nccl")
    if args.same_device and backend == "nccl" and world > 1:
        raise SystemExit("--same-device runs every rank on cuda:0, which RCCL (nccl) refuses: use --backend gloo")

    import torch
    import torch.distributed as dist
    device_index = 0 if args.same_device else local_rank
    if backend == "nccl" or decode is None:
        torch.cuda.set_device(device_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device_index))
        else:
            dist.init_process_group("gloo")

    if args.bits is not None:
        bits_fn = lambda p: int(args.bits)   # noqa: E731
    elif channel == SOFT:
        bits_fn = lambda p: int(reference_awgn_bits(p, code.blen) * args.bits_scale)   # noqa: E731
    else:
        bits_fn = lambda p: int(reference_bsc_bits(int(p), code.blen) * args.bits_scale)   # noqa: E731

    # the decoder is built once; each point runs locally, then ONE all-reduce (sum) of the whole
    # [points][errors, bits] table and one MAX of the per-point times
    dev = gpu = None
    if decode is None:
        if args.device_channel:
            dev = DeviceChannelDecoder(code, channel, args.frame_blocks, args.seed,
                                       hard_demap=args.hard_demap, decoder=args.decoder,
                                       noise_f32=args.noise == "f32")
            if args.warmup > 0:
                dev.warm_up(args.warmup, points[0] if points else None)
        else:
            gpu = GpuFrameDecoder(code, channel, args.frame_blocks, decoder=args.decoder)
    counters = np.zeros((len(points), 2), np.int64)
    secs = np.zeros(len(points), np.float64)
    for k, p in enumerate(points):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        (pt,) = ber_sweep(code, [p], channel, bits_per_point=bits_fn, frame_blocks=args.frame_blocks,
                          seed=args.seed, rank=rank, world=world, decode=decode or gpu,
                          threads=args.threads, reduce=False, hard_demap=args.hard_demap,
                          decoder=args.decoder, point_index=args.first_point_index + k,
                          device_decoder=dev)
        secs[k] = time.perf_counter() - t0
        counters[k] = (pt.errors, pt.bits)
    if world > 1:
        counters = all_reduce_counters(counters)
        t = torch.from_numpy(secs).to("cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        secs = t.cpu().numpy()
    results = []
    for k, p in enumerate(points):
        errors, bits = int(counters[k, 0]), int(counters[k, 1])
        lo, hi = ber_interval(errors, bits)
        rec = {"code": code.name or args.code, "n": code.n, "K": code.K, "blen": code.blen,
               "generator": "ref-x86" if code.gen_mode == 0 else "true-parity",
               "channel": args.channel + ("-hard-demap" if args.hard_demap else ""),
               "noise": args.noise if channel == SOFT else None,
               "decoder": args.decoder, ("ebn0_db" if channel == SOFT else "p_ppm"): p,
               "errors": errors, "bits": bits, "ber": errors / bits if bits else None,
               "ber_99.9_binomial": [lo, hi], "seconds": round(float(secs[k]), 4),
               "mbit_s": round(bits / secs[k] / 1e6, 1) if secs[k] > 0 else None,
               "world_size": world, "device_channel": bool(args.device_channel),
               "point_index": args.first_point_index + k, "seed": args.seed,
               "warmup_s": args.warmup if dev is not None else 0.0}
        results.append(rec)
        if rank == 0:
            print(json.dumps(rec), flush=True)
    if rank == 0 and args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

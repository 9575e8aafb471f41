"""Batched BER sweep: the counterpart of the reference drivers (AWGN-channel/main.c:146-242,
binary-symmetric-channel/main.c:100-183) built for throughput.

The reference streams one block at a time through encoder -> channel -> decoder callbacks and counts
errors in the decoded callback. Here a sweep point is a set of FRAMES (frame_blocks independent
blocks each); block b of frame f at point p draws its randomness from the Philox stream
(seed, p << 40 | f * frame_blocks + b), so results do not depend on how frames are spread over
processes. Rank r of a world of W processes (one per GPU) takes frames f = r, r+W, ...; each frame is
produced on the host (libccv_sim), decoded on the GPU with the bit-error count fused into the
traceback, and at the end ONE all-reduce (sum, int64) of the (errors, bits) counters goes over
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
    """Bits the reference simulates per BSC point (binary-symmetric-channel/main.c:389-398)."""
    nb = 20000000
    if p_ppm > 12500:
        nb //= 10
    if p_ppm > 50000:
        nb //= 10
    if p_ppm > 200000:
        nb //= 10
    return nb * blen


class GpuFrameDecoder:
    """Decodes one host frame on the current GPU and returns its bit-error count."""

    def __init__(self, code: Code, channel: int, frame_blocks: int, device=None):
        import torch

        from .decoder import Plan
        self.torch = torch
        self.device = torch.device(device if device is not None else "cuda")
        self.plan = Plan(code, channel)
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
    as the host producers, no host generation and no input traffic."""

    def __init__(self, code: Code, channel: int, frame_blocks: int, seed: int, device=None,
                 hard_demap=False):
        import torch

        from .decoder import Plan
        self.torch = torch
        self.device = torch.device(device if device is not None else "cuda")
        self.plan = Plan(code, channel)
        self.plan.reserve(frame_blocks)
        self.channel, self.frame_blocks, self.seed = channel, frame_blocks, seed
        self.hard_demap = hard_demap
        self.d_err = torch.zeros(1, dtype=torch.int64, device=self.device)

    def __call__(self, point: float, first_blocks: Sequence[int]) -> int:
        """Bit errors of the frames starting at `first_blocks` at Eb/N0 (dB) or p_ppm `point`."""
        param = ch.noise_scaling(point) if self.channel == SOFT else int(point)
        self.d_err.zero_()
        stream = self.torch.cuda.current_stream(self.device)
        for first in first_blocks:
            self.plan.simulate_device(self.seed, first, self.frame_blocks, param, d_errors=self.d_err,
                                      stream=stream, hard_demap=self.hard_demap)
        return int(self.d_err.item())


def ber_sweep(code: Code, points: Sequence[float], channel: int = SOFT,
              bits_per_point: Optional[Callable[[float], int]] = None, frame_blocks: int = 25000,
              seed: int = 0xC0DE, rank: int = 0, world: int = 1,
              decode: Optional[Callable[[np.ndarray, np.ndarray], int]] = None,
              threads: Optional[int] = None, reduce: bool = True,
              device_channel: bool = False, hard_demap: bool = False) -> List[BerPoint]:
    """BER at each point; `decode(info, data) -> errors` defaults to the GPU decoder. With
    device_channel the frames are generated on the GPU as well (DeviceChannelDecoder)."""
    if bits_per_point is None:
        if channel == SOFT:
            bits_per_point = lambda p: reference_awgn_bits(p, code.blen)   # noqa: E731
        else:
            bits_per_point = lambda p: reference_bsc_bits(int(p), code.blen)  # noqa: E731
    dev = DeviceChannelDecoder(code, channel, frame_blocks, seed, hard_demap=hard_demap) \
        if device_channel else None
    if decode is None and dev is None:
        decode = GpuFrameDecoder(code, channel, frame_blocks)
    counters = np.zeros((len(points), 2), np.int64)
    for pi, p in enumerate(points):
        nframes = max(1, math.ceil(bits_per_point(p) / (frame_blocks * code.blen)))
        if dev is not None:
            mine = range(rank, nframes, world)
            counters[pi, 0] += dev(p, [(pi << 40) + f * frame_blocks for f in mine])
            counters[pi, 1] += len(mine) * frame_blocks * code.blen
            continue
        for f in range(rank, nframes, world):
            first = (pi << 40) + f * frame_blocks
            if channel == SOFT:
                info, data = ch.awgn_blocks(code, frame_blocks, ch.noise_scaling(p), seed,
                                            first_block=first, threads=threads, hard_demap=hard_demap)
            else:
                info, data = ch.bsc_blocks(code, frame_blocks, int(p), seed, first_block=first,
                                           threads=threads)
            counters[pi, 0] += decode(info, data)
            counters[pi, 1] += frame_blocks * code.blen
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

"""Fano kernel scaling probe (tools/ only): launch time vs number of blocks, and one lone block.

Prints, for each batch size, the kernel time, total moves (CCV_FANO_COUNT_MOVES) and the implied
chip-wide move rate; then the latency of the longest block decoded alone (one lane busy)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "convolutional-codes_amd")
from ccviterbi import FanoPlan, SOFT, channel as ch, named_code  # noqa: E402

code = named_code("k15")
db = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
nmax = 800000
info, rx = ch.awgn_blocks(code, nmax, ch.noise_scaling(db), 0xC0DE)
plan = FanoPlan(code, SOFT)
d_rx = torch.from_numpy(rx).cuda()
d_out = torch.empty((nmax, code.out_bytes), dtype=torch.uint8, device="cuda")
d_it = torch.zeros(nmax, dtype=torch.int32, device="cuda")


def run(nb, src=None):
    src = d_rx if src is None else src
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan.decode_fano_device(src, nb, d_out[:nb], d_iterations=d_it[:nb])
    torch.cuda.synchronize()
    return time.perf_counter() - t0


run(1000)
for nb in (25000, 100000, 200000, 400000, 800000):
    dt = run(nb)
    mv = d_it[:nb].cpu().numpy().astype(np.int64)
    print(f"rows={os.environ.get('CCV_FANO_ROWS', 'default')} {db} dB nb={nb}: {dt*1e3:.1f} ms, "
          f"moves {mv.sum():.3e} max {mv.max()} -> {mv.sum()/dt:.3e} moves/s, "
          f"{dt/mv.max()*1e9:.0f} ns per move of the longest block", flush=True)
b = int(np.argmax(d_it[:nmax].cpu().numpy()))
one = d_rx[b:b + 1].contiguous()
dt = run(1, one)
mv = int(d_it[0].item())
print(f"lone block {b}: {mv} moves in {dt*1e3:.1f} ms -> {dt/mv*1e9:.0f} ns per move", flush=True)

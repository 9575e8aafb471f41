"""Single-lane Fano search latency: decode one block that runs into the timeout (tools/ only)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "convolutional-codes_amd")
from ccviterbi import FanoPlan, SOFT, channel as ch, named_code  # noqa: E402

code = named_code("k15")
nb = 20000
info, rx = ch.awgn_blocks(code, nb, ch.noise_scaling(4.0), 0xC0DE)
plan = FanoPlan(code, SOFT)
d_rx = torch.from_numpy(rx).cuda()
d_out = torch.empty((nb, code.out_bytes), dtype=torch.uint8, device="cuda")
d_it = torch.zeros(nb, dtype=torch.int32, device="cuda")
plan.decode_fano_device(d_rx, nb, d_out, d_iterations=d_it)
torch.cuda.synchronize()
it = d_it.cpu().numpy()
b = int(np.argmax(it))
one = d_rx[b:b + 1].contiguous()
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan.decode_fano_device(one, 1, d_out[:1], d_iterations=d_it[:1])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
print(f"RXL={os.environ.get('CCV_FANO_RXL', 'default')}: block {b}, {int(it[b])} iterations, "
      f"{dt*1e3:.1f} ms -> {dt / it[b] * 1e9:.0f} ns per iteration (one lane)", flush=True)

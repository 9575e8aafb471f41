"""Eb/N0 sweep throughput against the device-channel chunk (frames per ccv_simulate_device launch):
one 800 M-bit point at 14 dB per chunk size, after the CLI's 0.2 s warm-up.
usage: python tools/sweep_chunk_probe.py CODE [frames per chunk ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "convolutional-codes_amd"))
import torch  # noqa: E402

from ccviterbi import SOFT, named_code, sim  # noqa: E402

code = named_code(sys.argv[1])
fb = 25000
for frames in [int(x) for x in sys.argv[2:]] or [32, 64, 104, 208]:
    dev = sim.DeviceChannelDecoder(code, SOFT, fb, 0xC0DE, chunk_blocks=frames * fb)
    dev.warm_up(0.2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    err = dev(14.0, 7 << 40, 800 * fb)
    dt = time.perf_counter() - t0
    print(f"{sys.argv[1]} chunk {frames} frames: {800 * fb * code.blen / dt / 1e9:.2f} Gbit/s, errors {err}", flush=True)
    del dev
    torch.cuda.empty_cache()

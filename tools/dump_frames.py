"""Write the bench's block-major AWGN frames (float32 [nb][T][4]) to a raw file for tools/kbench."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "convolutional-codes_amd"))
from ccviterbi import channel as ch, named_code  # noqa: E402

nb, path = int(sys.argv[1]), sys.argv[2]
ebn0 = float(sys.argv[3]) if len(sys.argv) > 3 else 4.0
code = named_code("k7")
_, rx = ch.awgn_blocks(code, nb, ch.noise_scaling(ebn0), 0xC0DE, threads=16)
rx.tofile(path)

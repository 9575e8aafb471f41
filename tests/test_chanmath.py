"""Host check of csrc/channel_math.hpp, the on-device AWGN channel's double-precision Box-Muller pieces
(-2 ln u, sqrt, sin / cos of 2 pi u), compiled with g++ by tools/chanmath_check.cpp with the hardware
rcp / rsq approximations emulated: error bounds in ulp against long double, and the fp32 channel
samples against the glibc-based ones the host producer (csrc/sim.cpp:150-170) writes."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import REPO


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_channel_math_vs_glibc(tmp_path):
    exe = str(tmp_path / "chanmath_check")
    subprocess.run(["g++", "-O2", "-std=c++20", "-o", exe, os.path.join(REPO, "tools", "chanmath_check.cpp")],
                   check=True, timeout=120)
    out = subprocess.run([exe, "2"], check=True, timeout=120, capture_output=True, text=True).stdout
    log_ulp = float(re.search(r"-2 ln u\s+channel_math ([0-9.]+)", out).group(1))
    sqrt_ulp = float(re.search(r"sqrt\s+channel_math ([0-9.]+)", out).group(1))
    sin_err, cos_err = map(float, re.search(r"channel_math ([0-9.e-]+) / ([0-9.e-]+)", out).groups())
    assert log_ulp <= 3.0 and sqrt_ulp <= 1.0, out
    assert sin_err <= 2.3e-16 and cos_err <= 2.3e-16, out
    for line in re.findall(r"differing from glibc's: (\d+) of (\d+)", out):
        bad, total = map(int, line)
        assert total > 4_000_000 and bad <= 2, out   # 268 M draws: <= 2.2e-8 (profiles/r04_chanmath_check.txt)

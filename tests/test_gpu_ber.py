"""The published BER curves (results/awgn_channel.m, results/binary_symmetric_channel.m) reproduced on
the GPU: Viterbi soft and hard-demapper AWGN curves of codebook codes 0/1/2/3/5, the BSC Viterbi
curves, and the stack and Fano decoder curves, each point checked statistically. Needs an MI355X.

The frames come from the on-device channel (ccv_simulate_device: Philox AWGN / BSC with the reference's
noise scaling, mapper and demapper), so the noise samples differ from the reference's glibc rand()
stream and only the statistics can agree (the decoders themselves are bit-exact: test_gpu_parity).

Acceptance per point, stated up front: with p_r the published BER over N_r bits (the reference's bit
schedule, tests/golden/published_ber.json) and p the BER here over N bits,

    |p - p_r| <= z * sqrt(B * q * (1 - q) * (1/N + 1/N_r)) + res / 2,     q = pooled BER,

z = 3.29 (99.9 % two-sided), res = the table's print resolution, and the BURST FACTOR B = blen: bit
errors of different blocks are independent, and a block holds at most blen erroneous bits, so the
variance of a block's error count is at most blen times its mean (measured dispersion: 1.2 to 27 for
these codes and Eb/N0, oracle runs of 200,000 blocks) -- B = blen bounds the over-dispersion of every
decoder here without a fitted constant. Both runs' variances count (the reference's table is itself a
Monte-Carlo estimate).
"""
import json
import math
import os

import numpy as np
import pytest

from ccviterbi import CODEBOOK, HARD, SOFT, sim
from conftest import REPO

pytestmark = pytest.mark.gpu
PUB = json.load(open(os.path.join(REPO, "tests", "golden", "published_ber.json")))
Z = 3.29


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


def _curve(name, channel):
    (c,) = [c for c in PUB["curves"] if c["name"] == name and c["channel"] == channel]
    return c


def _ref_bits(curve, k):
    """Bits behind the published point k (the schedules stated in the result files)."""
    code = CODEBOOK[curve["codebook_index"]]
    if curve["channel"] == "awgn":
        return sim.reference_awgn_bits(PUB["awgn_ebn0_db"][k], code.blen)
    p = PUB["bsc_p"][k]
    if curve["decoder"] == "fano":          # binary_symmetric_channel.m:30
        return 800_000_000 if p <= 0.0125 else 80_000_000 if p <= 0.05 else 8_000_000 if p <= 0.2 else 800_000
    if curve["codebook_index"] == 4:        # WSPR stack, binary_symmetric_channel.m:27
        return 800_000_000 if p <= 0.025 else 80_000_000
    return sim.reference_bsc_bits(int(round(p * 1e6)), code.blen)


def _resolution(curve, k):
    if curve["channel"] == "awgn":
        return 1e-8
    v = curve["ber"][k]
    # BSC Viterbi rows print 6 decimals; the Fano rows and the small WSPR entries 8
    return 1e-8 if curve["decoder"] == "fano" or (curve["codebook_index"] == 4 and v < 1e-4) else 1e-6


def _check(curve, k, errors, bits, blen):
    p_r, n_r = curve["ber"][k], _ref_bits(curve, k)
    p = errors / bits
    q = (errors + p_r * n_r) / (bits + n_r)
    tol = Z * math.sqrt(blen * q * (1 - q) * (1.0 / bits + 1.0 / n_r)) + _resolution(curve, k) / 2
    return abs(p - p_r) <= tol, f"{curve['name']} point {k}: {p:.4g} ({errors}/{bits}) vs {p_r:.4g} +- {tol:.3g}"


def _run(curve, ks, bits_of, decoder, noise="f64"):
    code = CODEBOOK[curve["codebook_index"]]
    soft = curve["channel"] == "awgn"
    pts = [PUB["awgn_ebn0_db"][k] if soft else round(PUB["bsc_p"][k] * 1e6) for k in ks]
    out, bad = [], []
    for k, pt in zip(ks, pts):
        (r,) = sim.ber_sweep(code, [pt], SOFT if soft else HARD, bits_per_point=lambda _p: bits_of(k),
                             seed=0xBE4 + k, device_channel=True, hard_demap=curve["hard_demap"],
                             decoder=decoder, point_index=k, noise_f32=noise == "f32")
        ok, msg = _check(curve, k, r.errors, r.bits, code.blen)
        out.append(msg)
        if not ok:
            bad.append(msg)
    print("\n".join(out))
    assert not bad, "\n".join(bad)


VITERBI_AWGN = [c["name"] for c in PUB["curves"] if c["channel"] == "awgn" and c["decoder"] == "viterbi"]


# The AWGN curves run twice: with the default double-precision Box-Muller (the reference's arithmetic)
# and with the opt-in fp32 one (CCV_CHANNEL_NOISE_F32; error bound: tools/chanmath_f32_check.hip).
NOISE = ["f64", "f32"]


@pytest.mark.parametrize("noise", NOISE)
@pytest.mark.parametrize("name", VITERBI_AWGN)
def test_viterbi_awgn_curve(torch_cuda, name, noise):
    """results/awgn_channel.m:15-28: every soft (code x) and hard-demapper (code xh) Viterbi curve,
    0-14 dB, four times the reference's bits per point (at least 8 M)."""
    curve = _curve(name, "awgn")
    _run(curve, range(8), lambda k: max(8_000_000, 4 * _ref_bits(curve, k)), "viterbi", noise)


# results/binary_symmetric_channel.m:7 (code 1) disagrees with the reference's own sources: the
# compiled, unmodified reference decoder + driver give a BER 2-4 % above the table at every point
# (tests/golden/make_reference_ber.py: 0.1159 at p = 0.1 over 40 M bits vs 0.1126), as does this GPU
# decoder -- that curve came from another build. Checked against the reference run instead
# (test_viterbi_bsc_code1_vs_reference_run); the table comparison is kept as a strict xfail.
PUBLISHED_MISMATCH = {"ber_coded_b": "results/binary_symmetric_channel.m:7 is 2-4 % below the compiled "
                                     "reference's own BER (tests/golden/reference_ber.json)"}
VITERBI_BSC = [pytest.param(c["name"], marks=pytest.mark.xfail(strict=True, reason=PUBLISHED_MISMATCH[c["name"]]))
               if c["name"] in PUBLISHED_MISMATCH else c["name"]
               for c in PUB["curves"] if c["channel"] == "bsc" and c["decoder"] == "viterbi"]
REFRUN = json.load(open(os.path.join(REPO, "tests", "golden", "reference_ber.json")))["points"]


def test_viterbi_bsc_code1_vs_reference_run(torch_cuda):
    """Code 1 on the BSC against the compiled reference's own BER (same acceptance rule, the run's
    bits in place of the table's schedule): 7 crossover probabilities, 40 M reference bits each."""
    bad, out = [], []
    for k, ref in enumerate(REFRUN):
        code = CODEBOOK[ref["codebook_index"]]
        (r,) = sim.ber_sweep(code, [ref["p_ppm"]], HARD, bits_per_point=lambda _p: 80_000_000,
                             seed=0xC1 + k, device_channel=True, point_index=k)
        q = (r.errors + ref["errors"]) / (r.bits + ref["bits"])
        tol = Z * math.sqrt(code.blen * q * (1 - q) * (1.0 / r.bits + 1.0 / ref["bits"]))
        msg = f"p={ref['p_ppm']}: {r.ber:.5g} vs reference run {ref['ber']:.5g} +- {tol:.3g}"
        out.append(msg)
        if abs(r.ber - ref["ber"]) > tol:
            bad.append(msg)
    print("\n".join(out))
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("name", VITERBI_BSC)
def test_viterbi_bsc_curve(torch_cuda, name):
    """results/binary_symmetric_channel.m:5-13: the BSC Viterbi curves of codes 0/1/2/3/5 at all 17
    crossover probabilities, the reference's bits per point."""
    curve = _curve(name, "bsc")
    _run(curve, range(17), lambda k: _ref_bits(curve, k), "viterbi")


SEQ_AWGN = [c["name"] for c in PUB["curves"] if c["channel"] == "awgn" and c["decoder"] != "viterbi"
            and c["codebook_index"] != 4]


@pytest.mark.parametrize("noise", NOISE)
@pytest.mark.parametrize("name", SEQ_AWGN)
def test_sequential_awgn_curve(torch_cuda, name, noise):
    """results/awgn_channel.m:30-78: stack and Fano curves (soft and hard demapper) of codes
    0/1/2/3/5, 0-10 dB at the reference's bits per point: the on-device channel writes its frames
    to HBM and the sequential decoder reads them."""
    curve = _curve(name, "awgn")
    _run(curve, range(6), lambda k: _ref_bits(curve, k), curve["decoder"], noise)


SEQ_BSC = [c["name"] for c in PUB["curves"] if c["channel"] == "bsc" and c["decoder"] != "viterbi"
           and c["codebook_index"] != 4]


@pytest.mark.parametrize("name", SEQ_BSC)
def test_sequential_bsc_curve(torch_cuda, name):
    """results/binary_symmetric_channel.m:15-40: BSC stack and Fano curves of codes 0/1/2/3/5 at the
    crossover probabilities from 0.0625 % up, at most 80 M bits per point."""
    curve = _curve(name, "bsc")
    ks = [k for k, p in enumerate(PUB["bsc_p"]) if p >= 0.000625]
    _run(curve, ks, lambda k: min(80_000_000, _ref_bits(curve, k)), curve["decoder"])


@pytest.mark.parametrize("name", ["ber_coded_f_stack", "ber_coded_fh_stack", "ber_coded_f_fano",
                                  "ber_coded_fh_fano"])
def test_wspr_awgn_curve_low_snr(torch_cuda, name):
    """results/awgn_channel.m:50-53,75-78: the WSPR K=32 code (blen 50) with the stack and Fano
    decoders at 0-4 dB (800,000 bits each; host-produced frames: the on-device channel is built for
    the register-trellis codes)."""
    curve = _curve(name, "awgn")
    code = CODEBOOK[4]
    bad, out = [], []
    for k in range(3):
        (r,) = sim.ber_sweep(code, [PUB["awgn_ebn0_db"][k]], SOFT, bits_per_point=lambda _p: 800_000,
                             frame_blocks=4000, seed=0x5A5 + k, hard_demap=curve["hard_demap"],
                             decoder=curve["decoder"], point_index=k)
        ok, msg = _check(curve, k, r.errors, r.bits, code.blen)
        out.append(msg)
        if not ok:
            bad.append(msg)
    print("\n".join(out))
    assert not bad, "\n".join(bad)


def test_interval_rejects_a_shifted_curve():
    """The acceptance rule has power: code 0's soft curve shifted by 1 dB (the published 2 dB value
    checked as if it were 4 dB's, and so on) fails at every point that has errors."""
    curve = dict(_curve("ber_coded_a", "awgn"))
    shifted = curve["ber"][1:] + [0.0]
    for k in range(5):
        bits = 4 * _ref_bits(curve, k)
        ok, _ = _check(curve, k, int(round(shifted[k] * bits)), bits, 40)
        assert not ok

"""Seeded random parity sweep of the sequential decoders (needs an MI355X): the stack decoder
(config 5's algorithm, stack_dev.hpp) and the Fano decoder (fano_dev.hpp) on random codes -- n 2 or
3, K 3..24 with random generator taps in both generator modes, block lengths 8..120 -- and channel
frames at random Eb/N0 (soft, the reference's demapper) or crossover probability (BSC), each decoded
through ccv_*_decode_host and compared bit for bit with the oracle restatements of stack-decoder.c /
fano-decoder.c (outputs, and path metrics for hard input). The draws are fixed by the seed. A stack
case whose search would make the reference read past its buffers (the oracle refuses it) is redrawn
with the next channel seed."""
import numpy as np
import pytest

import oracle_ctypes as O
from ccviterbi import GEN_REF_X86, GEN_TRUE_PARITY, HARD, SOFT, Code, FanoPlan, StackPlan, channel as ch

pytestmark = pytest.mark.gpu

N_STACK, N_FANO = 48, 32


def _code(rng, kmax):
    n = 2 if rng.random() < 0.75 else 3
    K = int(rng.integers(3, kmax + 1))
    polys = []
    for _ in range(n):
        taps = int(rng.integers(1, 1 << K)) | (1 << (K - 1))   # the current-input tap, as every codebook code
        polys.append(taps << (64 - K))
    gen = GEN_TRUE_PARITY if rng.random() < 0.4 else GEN_REF_X86
    blen = int(rng.integers(8, 121))
    return Code(n, K, blen, tuple(polys), gen)


def _frames(rng, c, channel, nb, seed):
    if channel == SOFT:
        db = float(rng.uniform(3.0, 8.0))
        return ch.awgn_blocks(c, nb, ch.noise_scaling(db), seed)
    return ch.bsc_blocks(c, nb, int(rng.integers(2000, 40000)), seed)


def _ocode(c):
    return O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)


@pytest.mark.parametrize("i", range(N_STACK))
def test_random_stack_vs_oracle(i):
    rng = np.random.default_rng(0x57AC + 104729 * i)
    c = _code(rng, 24)
    channel = HARD if rng.random() < 0.4 else SOFT
    nb = int(rng.integers(1, 200))
    for attempt in range(6):
        info, data = _frames(rng, c, channel, nb, 1000 * i + attempt)
        try:
            if channel == SOFT:
                ref = O.stack_soft(_ocode(c), c.metric_weight, data)
            else:
                ref, ref_pm = O.stack_hard(_ocode(c), c.bit_metrics, data)
            break
        except RuntimeError:   # the reference would read past its buffers on some block: redraw
            continue
    else:
        pytest.skip("no frame the reference decodes within its buffers")
    what = f"stack case {i}: n={c.n} K={c.K} blen={c.blen} gen={c.gen_mode} {'hard' if channel else 'soft'} nb={nb}"
    plan = StackPlan(c, channel)
    if channel == SOFT:
        assert np.array_equal(plan.decode_host(data), ref), what
    else:
        out, pm = plan.decode_host(data)
        assert np.array_equal(out, ref), what
        assert np.array_equal(pm, ref_pm), what


@pytest.mark.parametrize("i", range(N_FANO))
def test_random_fano_vs_oracle(i):
    rng = np.random.default_rng(0xFA40 + 7907 * i)
    c = _code(rng, 20)
    channel = HARD if rng.random() < 0.4 else SOFT
    nb = int(rng.integers(1, 200))
    info, data = _frames(rng, c, channel, nb, 77 + i)
    what = f"fano case {i}: n={c.n} K={c.K} blen={c.blen} gen={c.gen_mode} {'hard' if channel else 'soft'} nb={nb}"
    plan = FanoPlan(c, channel)
    if channel == SOFT:
        ref = O.fano_soft(_ocode(c), c.fano_metric_weight, data)
        assert np.array_equal(plan.decode_host(data), ref), what
    else:
        ref, ref_pm = O.fano_hard(_ocode(c), c.fano_bit_metrics, data)
        out, pm = plan.decode_host(data)
        assert np.array_equal(out, ref), what
        assert np.array_equal(pm, ref_pm), what

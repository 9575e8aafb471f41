"""Seeded random parity sweep over the plan space (needs an MI355X): random codes -- K 2..10, n 1..4,
random generator taps in both generator modes, block lengths 1..200 -- random batch sizes, soft and
hard input, and the plan flags that re-route a code (generic kernel, no persistent kernel, HBM
decisions, step-major input), each decoded through ccv_decode_host (step-major: ccv_decode_device)
and compared bit for bit with the oracle (outputs, and path metrics for hard input). Inputs are random demapper rows (positive fp32
distances, every fourth case small integers so ties are common) or random received symbols, so every
code is exercised whether or not the reference has a channel for its rate. The draws are fixed by the
seed: a failure names its case and reproduces."""
import numpy as np
import pytest

import oracle_ctypes as O
from ccviterbi import GEN_REF_X86, GEN_TRUE_PARITY, HARD, SOFT, Code, Plan
from ccviterbi.decoder import FLAG_GENERIC, FLAG_GLOBAL_DECISIONS, FLAG_NO_PERSISTENT, FLAG_STEP_MAJOR

pytestmark = pytest.mark.gpu

N_CASES = 200
# the benchmark codes, so the specialised kernels are drawn too (their blen is randomised below)
NAMED = [(2, 7, (0xF200000000000000, 0xB600000000000000)), (2, 9, (0xB880000000000000, 0xF580000000000000)),
         (2, 8, (0xF900000000000000, 0xA700000000000000)), (2, 3, (0xA000000000000000, 0x6000000000000000)),
         (3, 3, (0xA000000000000000, 0xC000000000000000, 0x2000000000000000))]


def _case(i):
    rng = np.random.default_rng(0xF022 + 7919 * i)
    if rng.random() < 0.35:
        n, K, polys = NAMED[int(rng.integers(len(NAMED)))]
        blen = 40 if rng.random() < 0.5 else int(rng.integers(1, 201))
    else:
        K = int(rng.integers(2, 11))
        n = int(rng.integers(1, 5))
        polys = []
        for _ in range(n):
            taps = int(rng.integers(1, 1 << K))
            polys.append(taps << (64 - K))
        polys = tuple(polys)
        blen = int(rng.integers(1, 201))
    blen = min(blen, 256 - K)   # T = blen + K - 1 <= 255 (the reference's uint8 counters)
    gen = GEN_TRUE_PARITY if rng.random() < 0.4 else GEN_REF_X86
    channel = HARD if rng.random() < 0.4 else SOFT
    flags = 0
    r = rng.random()
    if r < 0.15:
        flags = FLAG_GENERIC
    elif r < 0.3:
        flags = FLAG_NO_PERSISTENT
    elif r < 0.4:
        flags = FLAG_GLOBAL_DECISIONS
    elif r < 0.5 and channel == SOFT:
        flags = FLAG_STEP_MAJOR
    nb = int(rng.integers(1, 1500)) if rng.random() < 0.8 else int(rng.integers(1, 70))
    c = Code(n, K, blen, polys, gen)
    T = c.steps
    if channel == SOFT:
        if i % 4 == 3:
            data = rng.integers(0, 4, size=(nb, T, 1 << n)).astype(np.float32)
        else:
            data = (rng.random((nb, T, 1 << n), dtype=np.float32) * 4.0).astype(np.float32)
    else:
        data = rng.integers(0, 1 << n, size=(nb, T)).astype(np.uint8)
    return c, channel, flags, data


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_plan_vs_oracle(i):
    c, channel, flags, data = _case(i)
    oc = O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)
    try:
        plan = Plan(c, channel, flags)
    except Exception as e:   # a flag that does not apply to this code is refused at plan creation
        if flags in (FLAG_STEP_MAJOR, FLAG_GLOBAL_DECISIONS, FLAG_NO_PERSISTENT):
            plan = Plan(c, channel, 0)
            flags = 0
        else:
            raise AssertionError(f"case {i}: plan creation failed: {e}")
    what = f"case {i}: n={c.n} K={c.K} blen={c.blen} gen={c.gen_mode} {'hard' if channel else 'soft'} " \
           f"flags={flags} nb={data.shape[0]} variant={plan.variant}"
    if channel == SOFT:
        if flags == FLAG_STEP_MAJOR:   # a device-input layout ([T][nb][2^n]): ccv_decode_device
            import torch
            nb = data.shape[0]
            d_in = torch.from_numpy(np.ascontiguousarray(data.transpose(1, 0, 2))).to("cuda")
            d_out = torch.zeros((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
            plan.decode_device(d_in, nb, d_out)
            torch.cuda.synchronize()
            out = d_out.cpu().numpy()
        else:
            out = plan.decode_host(data)
        ref = O.viterbi_soft(oc, data)
        assert np.array_equal(out, ref), what
    else:
        out, pm = plan.decode_host(data)
        ref, ref_pm = O.viterbi_hard(oc, data)
        assert np.array_equal(out, ref), what
        assert np.array_equal(pm, ref_pm), what

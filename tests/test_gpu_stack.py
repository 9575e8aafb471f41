"""GPU parity of the stack (sequential) decoder (ccv_stack_plan_create / ccv_stack_decode_device,
convolutional-codes_amd/csrc/stack_dev.hpp) against

* the unmodified reference stack-decoder.c outputs (tests/golden/stack_*.npz, manifest_stack.json:
  codebook codes 0, 2, 3, 4 (WSPR K=32), 5 and the K=15 code of BASELINE config 5, AWGN and BSC),
* the oracle restatement (oracle/ccoracle.c cco_stack_*) on seeded channel frames,

plus the streaming context across calls (d_prev) and the fused error count.
"""
import numpy as np
import pytest

import oracle_ctypes as O
from ccviterbi import (CODEBOOK, GEN_REF_X86, GEN_TRUE_PARITY, HARD, K15, SOFT, Code, StackPlan,
                       channel as ch)
from conftest import golden_manifest

pytestmark = pytest.mark.gpu
STACK_CASES = golden_manifest("stack")


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


def _stack_code(g, gen=GEN_REF_X86):
    return Code(int(g["n"]), int(g["K"]), int(g["blen"]), tuple(int(p) for p in g["polys"]), gen,
                bit_metrics=tuple(int(x) for x in g["bit_metrics"]),
                metric_weight=float(g["metric_weight"]))


def _ocode(c: Code):
    return O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)


@pytest.mark.parametrize("case", STACK_CASES, ids=[c["name"] for c in STACK_CASES])
def test_stack_golden_fixture(case):
    g = O.load_golden(case["name"])
    c = _stack_code(g)
    channel = SOFT if case["channel"] == "awgn" else HARD
    plan = StackPlan(c, channel)
    assert plan.kernel == "stack"
    res = plan.decode_host(g["rx"])
    if channel == SOFT:
        out = res
    else:
        out, pm = res
        assert np.array_equal(pm, g["path_metric"])
    assert np.array_equal(out, g["out"])
    assert ch.count_bit_errors(c, g["info"], out) == int(g["errors"])


SEEDED = [
    ("k15_soft", K15, SOFT), ("k15_true_soft", K15.with_(gen_mode=GEN_TRUE_PARITY), SOFT),
    ("k15_hard", K15, HARD), ("k15_true_hard", K15.with_(gen_mode=GEN_TRUE_PARITY), HARD),
    ("code0_soft", CODEBOOK[0], SOFT), ("code3_hard", CODEBOOK[3], HARD),
    ("wspr_soft", CODEBOOK[4], SOFT), ("code5_soft", CODEBOOK[5], SOFT),
    ("k15_blen200_soft", K15.with_(blen=200), SOFT),
]


@pytest.mark.parametrize("name,c,channel", SEEDED, ids=[s[0] for s in SEEDED])
def test_stack_seeded_vs_oracle(name, c, channel):
    nb = 150 if c.blen <= 50 else 20
    for db, p_ppm in ((3.0, 40000), (6.0, 10000)):
        if channel == SOFT:
            info, data = ch.awgn_blocks(c, nb, ch.noise_scaling(db), 77 + c.K)
            ref = O.stack_soft(_ocode(c), c.metric_weight, data)
            assert np.array_equal(StackPlan(c, SOFT).decode_host(data), ref)
        else:
            info, data = ch.bsc_blocks(c, nb, p_ppm, 88 + c.K)
            ref, ref_pm = O.stack_hard(_ocode(c), c.bit_metrics, data)
            out, pm = StackPlan(c, HARD).decode_host(data)
            assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)


def test_stack_streaming_context_and_error_count(torch_cuda):
    """Two calls with d_prev = the last block of the first call decode exactly like one call (the
    reference keeps one input buffer across blocks); the fused error count matches the host count."""
    torch = torch_cuda
    c = CODEBOOK[3]                          # idiom K=6: twin paths and self-duplication happen
    nb = 400
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(2.0), 5)
    ref = O.stack_soft(_ocode(c), c.metric_weight, rx)
    plan = StackPlan(c, SOFT)
    d_rx = torch.from_numpy(rx).cuda()
    d_info = torch.from_numpy(info).cuda()
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_st = torch.full((nb,), -1, dtype=torch.int32, device="cuda")
    half = nb // 2
    plan.decode_stack_device(d_rx[:half], half, d_out[:half], d_info=d_info[:half], d_errors=d_err,
                             d_status=d_st[:half])
    plan.decode_stack_device(d_rx[half:], nb - half, d_out[half:], d_prev=d_rx[half - 1],
                             d_info=d_info[half:], d_errors=d_err, d_status=d_st[half:])
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert np.array_equal(out, ref)
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)
    assert not d_st.cpu().numpy().any()


@pytest.mark.parametrize("channel", [SOFT, HARD], ids=["soft", "hard"])
@pytest.mark.parametrize("c", [K15, CODEBOOK[3], CODEBOOK[0]], ids=["k15", "code3", "code0"])
def test_stack_rows_kernel_vs_wave_kernel(c, channel):
    """The four-searches-per-wave kernel (stack_decode_rows, persistent rows pulling blocks from a
    counter) decodes bit for bit like the one-search-per-wave kernel (option stack_kernel=1) and the
    oracle: fewer blocks than rows, a ragged batch, noise down to 0 dB (deep searches, full stacks,
    the idiom codes' self-duplication), with path metrics and per-block status."""
    plan = StackPlan(c, channel)
    wave_plan = StackPlan(c, channel).set_option("stack_kernel", 1)
    for nb, db, p_ppm, seed in ((1, 2.0, 60000, 1), (3, 0.0, 100000, 2), (517, 1.0, 80000, 3)):
        if channel == SOFT:
            _, data = ch.awgn_blocks(c, nb, ch.noise_scaling(db), seed)
        else:
            _, data = ch.bsc_blocks(c, nb, p_ppm, seed)
        rows = plan.decode_host(data)
        wave = wave_plan.decode_host(data)
        if channel == SOFT:
            assert np.array_equal(rows, wave)
            assert np.array_equal(rows, O.stack_soft(_ocode(c), c.metric_weight, data))
        else:
            assert np.array_equal(rows[0], wave[0]) and np.array_equal(rows[1], wave[1])
            ref, ref_pm = O.stack_hard(_ocode(c), c.bit_metrics, data)
            assert np.array_equal(rows[0], ref) and np.array_equal(rows[1], ref_pm)


K20 = Code(2, 20, 30, (0xB5A39 << 44, 0xE4C6D << 44), metric_weight=-7.0, bit_metrics=(1, -11),
           name="k20_custom")   # K in [17, 32], T = 49 <= 64: rows kernel WITHOUT the symbol table
ROWS_VARIANTS = [
    ("k20_notab_soft", K20, SOFT, {}),
    ("k20_notab_hard", K20, HARD, {}),
    ("k15_hard_unkeyed_rl8", K15, HARD, {"stack_keys": 0}),
    ("k15_hard_unkeyed_rl16", K15, HARD, {"stack_keys": 0, "stack_row_lanes": 16}),
    ("k15_hard_keyed_rl8", K15, HARD, {"stack_row_lanes": 8}),
    ("k15_soft_rl8", K15, SOFT, {"stack_row_lanes": 8}),
    ("k15_soft_parities", K15, SOFT, {"stack_symtab": 0}),
    # bit metrics too large for the 32-bit metric/index key: the unkeyed 8-lane default
    ("code3_hard_bigmetric", CODEBOOK[3].with_(bit_metrics=(1, -200000)), HARD, {}),
]


@pytest.mark.parametrize("name,c,channel,opts", ROWS_VARIANTS, ids=[v[0] for v in ROWS_VARIANTS])
def test_stack_rows_kernel_variants_vs_oracle(name, c, channel, opts):
    """Every rows-kernel variant the dispatcher can select (stack.hip launch_rows_t): no symbol table
    (17 <= K <= 32, lane_symbols in the kernel), unkeyed hard scans with the lo_sent sentinel at 8 and
    16 lanes per search, keyed at 8 lanes, soft at 8 lanes, per-iteration parities -- against the
    oracle and the one-search-per-wave kernel, with path metrics."""
    plan = StackPlan(c, channel)
    for k, v in opts.items():
        plan.set_option(k, v)
    wave_plan = StackPlan(c, channel).set_option("stack_kernel", 1)
    for nb, db, p_ppm, seed in ((1, 2.0, 60000, 11), (261, 1.0, 80000, 12)):
        if channel == SOFT:
            _, data = ch.awgn_blocks(c, nb, ch.noise_scaling(db), seed)
        else:
            _, data = ch.bsc_blocks(c, nb, p_ppm, seed)
        rows = plan.decode_host(data)
        wave = wave_plan.decode_host(data)
        if channel == SOFT:
            assert np.array_equal(rows, O.stack_soft(_ocode(c), c.metric_weight, data))
            assert np.array_equal(rows, wave)
        else:
            ref, ref_pm = O.stack_hard(_ocode(c), c.bit_metrics, data)
            assert np.array_equal(rows[0], ref) and np.array_equal(rows[1], ref_pm)
            assert np.array_equal(rows[0], wave[0]) and np.array_equal(rows[1], wave[1])


def test_stack_plan_limits():
    with pytest.raises(Exception, match="uint8_t"):
        StackPlan(K15.with_(blen=250), HARD)          # T = 264 > 255
    with pytest.raises(Exception):
        StackPlan(Code(2, 65, 40, (1 << 63, 1 << 62)), SOFT)


@pytest.mark.parametrize("case", STACK_CASES, ids=[c["name"] for c in STACK_CASES])
def test_reference_driver_with_mi355x_stack_decoder(case, tmp_path):
    """Drop-in check: oracle/ref_harness.c (the reference drivers' producer chain and callbacks,
    compiled against the reference's headers) linked to libccv_stack_{awgn,bsc}.so instead of
    stack-decoder.c reproduces the reference's output files byte for byte -- block after block
    through one decoder, callbacks inside decoder_input."""
    import os
    import subprocess
    from conftest import REPO
    exe = os.path.join(REPO, "oracle", "_ref", f"ref_harness_{case['channel']}_stack_ccv")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref drop-in harness not built (needs /root/reference at build time)")
    g = O.load_golden(case["name"])
    prefix = str(tmp_path / case["name"])
    cmd = [exe, prefix, str(case["seed"]), str(case["nblocks"]), case["param"], case["spec"]]
    subprocess.run(cmd + ([case["metrics"]] if case["metrics"] else []), check=True, timeout=300)
    out = np.fromfile(prefix + ".out", dtype=np.uint8).reshape(g["out"].shape)
    assert np.array_equal(out, g["out"])
    if case["channel"] == "bsc":
        assert np.array_equal(np.fromfile(prefix + ".pm", dtype=np.int32), g["path_metric"])
    meta = dict(line.split() for line in open(prefix + ".meta"))
    assert int(meta["errors"]) == case["errors"]

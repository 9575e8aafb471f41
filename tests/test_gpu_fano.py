"""GPU parity of the Fano decoder (ccv_fano_plan_create / ccv_fano_decode_device,
convolutional-codes_amd/csrc/fano_dev.hpp) against the unmodified reference fano-decoder.c outputs
(tests/golden/fano_*.npz, manifest_fano.json: codebook codes 0, 2, 3, 4 (WSPR K=32), 5, K=15, a
K=7 blen-200 case that runs into the timeout; AWGN and BSC) and the oracle restatement on seeded
frames, plus the per-block search length export and the fused error count."""
import numpy as np
import pytest

import oracle_ctypes as O
from ccviterbi import (CODEBOOK, GEN_REF_X86, GEN_TRUE_PARITY, HARD, K15, SOFT, Code, FanoPlan,
                       channel as ch)
from conftest import golden_manifest

pytestmark = pytest.mark.gpu
FANO_CASES = golden_manifest("fano")


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


def _fano_code(g, gen=GEN_REF_X86):
    return Code(int(g["n"]), int(g["K"]), int(g["blen"]), tuple(int(p) for p in g["polys"]), gen,
                fano_bit_metrics=tuple(int(x) for x in g["fano_bit_metrics"]),
                fano_metric_weight=float(g["fano_metric_weight"]))


def _ocode(c: Code):
    return O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)


@pytest.mark.parametrize("case", FANO_CASES, ids=[c["name"] for c in FANO_CASES])
def test_fano_golden_fixture(case):
    g = O.load_golden(case["name"])
    c = _fano_code(g)
    channel = SOFT if case["channel"] == "awgn" else HARD
    plan = FanoPlan(c, channel)
    assert plan.kernel == "fano"
    res = plan.decode_host(g["rx"])
    if channel == SOFT:
        out = res
    else:
        out, pm = res
        assert np.array_equal(pm, g["path_metric"])
    assert np.array_equal(out, g["out"])
    assert ch.count_bit_errors(c, g["info"], out) == int(g["errors"])


SEEDED = [
    ("code0_soft", CODEBOOK[0], SOFT), ("code0_hard", CODEBOOK[0], HARD),
    ("code3_soft", CODEBOOK[3], SOFT), ("code5_soft", CODEBOOK[5], SOFT),
    ("wspr_soft", CODEBOOK[4], SOFT), ("wspr_hard", CODEBOOK[4], HARD),
    ("k15_soft", K15, SOFT), ("k15_true_soft", K15.with_(gen_mode=GEN_TRUE_PARITY), SOFT),
    ("k15_hard", K15, HARD),
]


@pytest.mark.parametrize("name,c,channel", SEEDED, ids=[s[0] for s in SEEDED])
def test_fano_seeded_vs_oracle(name, c, channel):
    nb = 300
    for db, p_ppm in ((4.0, 30000), (7.0, 8000)):
        if channel == SOFT:
            info, data = ch.awgn_blocks(c, nb, ch.noise_scaling(db), 31 + c.K)
            ref = O.fano_soft(_ocode(c), c.fano_metric_weight, data)
            assert np.array_equal(FanoPlan(c, SOFT).decode_host(data), ref)
        else:
            info, data = ch.bsc_blocks(c, nb, p_ppm, 41 + c.K)
            ref, ref_pm = O.fano_hard(_ocode(c), c.fano_bit_metrics, data)
            out, pm = FanoPlan(c, HARD).decode_host(data)
            assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)


def test_fano_timeouts_iterations_and_error_count(torch_cuda):
    """A channel bad enough that some searches hit the reference's 10000*T timeout: outputs still
    bit-exact, the exported search length shows the timeouts, the fused error count matches."""
    torch = torch_cuda
    c = CODEBOOK[0]
    nb = 400
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(1.5), 3)
    ref = O.fano_soft(_ocode(c), c.fano_metric_weight, rx)
    plan = FanoPlan(c, SOFT)
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_it = torch.zeros(nb, dtype=torch.int32, device="cuda")
    plan.decode_fano_device(torch.from_numpy(rx).cuda(), nb, d_out, d_info=torch.from_numpy(info).cuda(),
                            d_errors=d_err, d_iterations=d_it)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert np.array_equal(out, ref)
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)
    it = d_it.cpu().numpy().astype(np.int64)
    assert (it >= c.steps).all()
    assert (it <= 10000 * c.steps).all()
    assert (it == 10000 * c.steps).any()          # some blocks timed out (the search gave up)
    assert (it < 10000 * c.steps).any()


@pytest.mark.parametrize("rows", [-1, 0, 2], ids=["rows_auto", "rows_direct", "rows_pair"])
@pytest.mark.parametrize("table", [1, 0])
def test_fano_queue_order_and_symbol_table_change_nothing(torch_cuda, table, rows):
    """The noisiest-first queue order (soft input), the expected-symbol table and the received-row
    access (after the move, or both candidates prefetched) only change
    the schedule and where the symbols come from: outputs, error count and every block's search
    length equal the natural-order run and the oracle (K=15, 2 dB: long searches and timeouts)."""
    torch = torch_cuda
    c = K15
    nb = 700
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(2.0), 11)
    ref = O.fano_soft(_ocode(c), c.fano_metric_weight, rx)
    plan = FanoPlan(c, SOFT).set_option("fano_symtab", table).set_option("fano_rows", rows)
    d_rx = torch.from_numpy(rx).cuda()
    d_info = torch.from_numpy(info).cuda()
    runs = []
    for order in (1, 0):
        plan.set_option("fano_order", order)
        d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
        d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
        d_it = torch.zeros(nb, dtype=torch.int32, device="cuda")
        plan.decode_fano_device(d_rx, nb, d_out, d_info=d_info, d_errors=d_err, d_iterations=d_it)
        torch.cuda.synchronize()
        runs.append((d_out.cpu().numpy(), int(d_err.item()), d_it.cpu().numpy()))
    (o1, e1, i1), (o0, e0, i0) = runs
    assert np.array_equal(o1, ref) and np.array_equal(o0, ref)
    assert e1 == e0 == ch.count_bit_errors(c, info, o1)
    assert np.array_equal(i1, i0)


_TWO_PASS = {}


def _two_pass_case(channel):
    """K=15 frames with long searches and timeouts, and the oracle's decode (computed once)."""
    if channel not in _TWO_PASS:
        c, nb = K15, 900
        if channel == SOFT:
            info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(2.0), 21)
            ref, ref_pm = O.fano_soft(_ocode(c), c.fano_metric_weight, rx), None
        else:
            info, rx = ch.bsc_blocks(c, nb, 90000, 21)
            ref, ref_pm = O.fano_hard(_ocode(c), c.fano_bit_metrics, rx)
        _TWO_PASS[channel] = (info, rx, ref, ref_pm)
    return _TWO_PASS[channel]


@pytest.mark.parametrize("rows", [-1, 0], ids=["rows_auto", "rows_direct"])
@pytest.mark.parametrize("channel", [SOFT, HARD], ids=["soft", "hard"])
@pytest.mark.parametrize("cap", [0, 7, 300, -1], ids=["cap0", "cap7", "cap300", "default"])
def test_fano_two_pass_park_and_resume_is_exact(torch_cuda, channel, cap, rows):
    """The two-pass schedule (fano_dev.hpp): searches parked after `fano_cap` moves and resumed in
    pass 2 -- after 7 moves nearly every search parks mid-flight (forward runs, look-backs, threshold
    relaxations), after 300 only the long ones -- give the one-pass (cap 0) outputs, path metrics,
    error count and per-block search lengths, and the oracle's outputs (K=15, timeouts included); with
    the default row access and rows read after the move."""
    torch = torch_cuda
    c = K15
    nb = 900
    info, rx, ref, ref_pm = _two_pass_case(channel)
    plan = FanoPlan(c, channel).set_option("fano_cap", cap).set_option("fano_rows", rows)
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_pm = torch.zeros(nb, dtype=torch.int32, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_it = torch.zeros(nb, dtype=torch.int32, device="cuda")
    plan.decode_fano_device(torch.from_numpy(rx).cuda(), nb, d_out,
                            d_path_metric=d_pm if channel == HARD else None,
                            d_info=torch.from_numpy(info).cuda(), d_errors=d_err, d_iterations=d_it)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert np.array_equal(out, ref)
    if channel == HARD:
        assert np.array_equal(d_pm.cpu().numpy(), ref_pm)
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)
    it = d_it.cpu().numpy()
    assert (it <= 10000 * c.steps).all()
    if channel == SOFT:
        assert (it == 10000 * c.steps).any()
    # the search lengths equal the one-pass run's
    plan.set_option("fano_cap", 0)
    d_it0 = torch.zeros(nb, dtype=torch.int32, device="cuda")
    plan.decode_fano_device(torch.from_numpy(rx).cuda(), nb, d_out,
                            d_path_metric=d_pm if channel == HARD else None, d_iterations=d_it0)
    torch.cuda.synchronize()
    assert np.array_equal(d_it0.cpu().numpy(), it)


def test_fano_plan_limits():
    with pytest.raises(Exception, match="uint8_t"):
        FanoPlan(K15.with_(blen=250), SOFT)           # T = 264 > 255


@pytest.mark.parametrize("case", FANO_CASES, ids=[c["name"] for c in FANO_CASES])
def test_reference_driver_with_mi355x_fano_decoder(case, tmp_path):
    """Drop-in check: oracle/ref_harness.c (the reference drivers' producer chain and callbacks)
    linked to libccv_fano_{awgn,bsc}.so instead of fano-decoder.c reproduces the reference's output
    files byte for byte."""
    import os
    import subprocess
    from conftest import REPO
    exe = os.path.join(REPO, "oracle", "_ref", f"ref_harness_{case['channel']}_fano_ccv")
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


@pytest.mark.parametrize("hard_demap", [False, True], ids=["demap", "hard_demap"])
@pytest.mark.parametrize("rows", [-1, 1], ids=["iq_global", "iq_lds"])
def test_fano_received_points_equal_distance_rows(torch_cuda, rows, hard_demap):
    """Device sweeps of the Fano decoder (round 6): the channel writes the received points (x, y)
    (CCV_CHANNEL_IQ) and the kernel demaps them with the demapper's exact fp32 operations (option
    fano_input 1; points prefetched from global memory, or in LDS with fano_rows 1). Same seed, same
    frames: the demapped points equal the channel's distance frames bit for bit (recomputed on the
    host in numpy fp32 as common/demapper.c:66-70), and the decode -- outputs, error count, every
    block's search length, two-pass parking included -- equals the distance-row decode (K = 15 at
    2 dB: long searches and timeouts)."""
    torch = torch_cuda
    c, nb, seed = K15, 1500, 77
    param = ch.noise_scaling(2.0)
    dist_plan = FanoPlan(c, SOFT)
    iq_plan = FanoPlan(c, SOFT).set_option("fano_input", 1).set_option("fano_rows", rows)
    d_dist = torch.empty((nb, c.steps, 4), dtype=torch.float32, device="cuda")
    d_iq = torch.empty((nb, c.steps, 2), dtype=torch.float32, device="cuda")
    d_info = torch.empty((nb, c.info_bytes), dtype=torch.uint8, device="cuda")
    d_info2 = torch.empty_like(d_info)
    dist_plan.simulate_frames(seed, 5 << 40, nb, param, d_dist, d_info=d_info, hard_demap=hard_demap)
    iq_plan.simulate_frames(seed, 5 << 40, nb, param, d_iq, d_info=d_info2, hard_demap=hard_demap, iq=True)
    torch.cuda.synchronize()
    assert torch.equal(d_info, d_info2)
    xy = d_iq.cpu().numpy()
    a = np.float32(0.707107)
    nd = np.float32(np.float32(a - (-a)) * np.float32(a - (-a)))   # (dx*dx) + (dy*dy) with dx = 0
    host = np.empty((nb, c.steps, 4), np.float32)
    for e in range(4):
        px = np.float32(-a if e & 2 else a)
        py = np.float32(-a if e & 1 else a)
        dx = xy[..., 0] - px
        dy = xy[..., 1] - py
        host[..., e] = ((dx * dx) + (dy * dy)) / nd
    assert np.array_equal(host.view(np.uint32), d_dist.cpu().numpy().view(np.uint32))
    runs = []
    for plan, d_in in ((dist_plan, d_dist), (iq_plan, d_iq)):
        d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
        d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
        d_it = torch.zeros(nb, dtype=torch.int32, device="cuda")
        plan.decode_fano_device(d_in, nb, d_out, d_info=d_info, d_errors=d_err, d_iterations=d_it)
        torch.cuda.synchronize()
        runs.append((d_out.cpu().numpy(), int(d_err.item()), d_it.cpu().numpy()))
    (o0, e0, i0), (o1, e1, i1) = runs
    assert np.array_equal(o0, o1) and e0 == e1 and np.array_equal(i0, i1)
    assert (i0 == 10000 * c.steps).any()   # timeouts in the batch
    assert e0 == ch.count_bit_errors(c, d_info.cpu().numpy(), o0)


def test_fano_received_points_option_limits():
    """fano_input 1 is for soft rate-1/2 Fano plans with K <= 32; received points belong to AWGN."""
    with pytest.raises(Exception, match="received points"):
        FanoPlan(K15, HARD).set_option("fano_input", 1)
    with pytest.raises(Exception, match="Fano"):
        from ccviterbi import Plan, K7
        Plan(K7, SOFT).set_option("fano_input", 1)

"""HIP-graph capture of the device decode (ccv_decode_device) and of the device channel. Needs an MI355X.

A plan reserved for the batch (ccv_plan_reserve) allocates and synchronises nothing inside a decode,
so the whole call -- the persistent kernels with their per-XCD group queue (acs_persist.hpp
GroupQueue), the K = 9 one-lane kernel with its decision slots, the ragged last group, the fused error
count -- records into a graph. The queue resets itself at the end of every launch (the last wave out
zeroes the heads), so every replay walks the whole batch again. Each replay here runs on NEW inputs
copied into the captured buffers and must equal the eager decode of those inputs, which the oracle
checks in turn (a queue left dirty by one launch would skip groups in the next and show up here).
"""
import numpy as np
import pytest

import oracle_ctypes as O
from ccviterbi import CODEBOOK, GEN_TRUE_PARITY, HARD, K7, K9, SOFT, Plan, channel as ch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


def _ocode(c):
    return O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)


def _inputs(c, channel, nb, seed):
    if channel == SOFT:
        return ch.awgn_blocks(c, nb, ch.noise_scaling(3.0), seed)
    return ch.bsc_blocks(c, nb, 60000, seed)


# (code, channel, blocks): K = 7 soft and BSC run the queue-scheduled persistent kernels over many
# groups per wave plus a ragged last group; K = 9 the one-lane kernel (idiom) and the two-lane kernel
# (true parity); code 0 (config 1) the static walk.
CASES = [
    ("k7_soft", K7, SOFT, 2048 * 64 + 2048 * 8 + 77),
    ("k7_bsc", K7, HARD, 3072 * 64 + 3072 * 8 + 13),
    ("k9_soft", K9, SOFT, 40_000 + 5),
    ("k9_true_soft", K9.with_(gen_mode=GEN_TRUE_PARITY), SOFT, 20_000 + 3),
    ("code0_bsc", CODEBOOK[0], HARD, 50_000 + 1),
]


@pytest.mark.parametrize("name,c,channel,nb", CASES, ids=[x[0] for x in CASES])
def test_decode_device_replays_in_a_hip_graph(torch_cuda, name, c, channel, nb):
    torch = torch_cuda
    runs = [_inputs(c, channel, nb, 900 + k) for k in range(2)]
    info0, rx0 = runs[0]
    d_in = torch.from_numpy(np.ascontiguousarray(rx0)).to("cuda")
    d_info = torch.from_numpy(np.ascontiguousarray(info0)).to("cuda")
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_pm = torch.empty(nb, dtype=torch.int32, device="cuda") if channel == HARD else None
    plan = Plan(c, channel)
    plan.reserve(nb)

    # eager decodes of both inputs (the expected results), on the stream the graph is captured from
    side = torch.cuda.Stream()
    expect = []
    with torch.cuda.stream(side):
        for info, rx in runs:
            d_in.copy_(torch.from_numpy(np.ascontiguousarray(rx)))
            d_info.copy_(torch.from_numpy(np.ascontiguousarray(info)))
            d_err.zero_()
            plan.decode_device(d_in, nb, d_out, d_path_metric=d_pm, d_info=d_info, d_errors=d_err,
                               stream=side)
            expect.append((d_out.clone(), int(d_err.item()), None if d_pm is None else d_pm.clone()))
    torch.cuda.synchronize()

    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        d_err.zero_()
        plan.decode_device(d_in, nb, d_out, d_path_metric=d_pm, d_info=d_info, d_errors=d_err,
                           stream=torch.cuda.current_stream())
    for k in (1, 0, 1):
        info, rx = runs[k]
        d_in.copy_(torch.from_numpy(np.ascontiguousarray(rx)))
        d_info.copy_(torch.from_numpy(np.ascontiguousarray(info)))
        d_out.fill_(0xA5)
        graph.replay()
        torch.cuda.synchronize()
        out, errors, pm = expect[k]
        assert torch.equal(d_out, out), f"{name}: replay {k} differs from the eager decode"
        assert int(d_err.item()) == errors
        if pm is not None:
            assert torch.equal(d_pm, pm)

    # the eager results against the oracle (whole batch) and the fused count against the host count
    for k, (info, rx) in enumerate(runs[:1]):
        out = expect[k][0].cpu().numpy()
        if channel == SOFT:
            ref = O.viterbi_soft(_ocode(c), rx)
        else:
            ref, ref_pm = O.viterbi_hard(_ocode(c), rx)
            assert np.array_equal(expect[k][2].cpu().numpy(), ref_pm)
        assert np.array_equal(out, ref)
        assert expect[k][1] == ch.count_bit_errors(c, info, out)


def test_simulate_device_replays_in_a_hip_graph(torch_cuda):
    """The fused channel + decode (ccv_simulate_device, K = 7 AWGN) captured once: replays draw the
    same Philox blocks, so every replay's error count equals the eager call's."""
    torch = torch_cuda
    c = K7
    nb = 64 * 1000 + 9
    plan = Plan(c, SOFT)
    plan.reserve(nb)
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    scaling = ch.noise_scaling(3.0)
    plan.simulate_device(7, 0, nb, scaling, d_errors=d_err, d_out=d_out)
    torch.cuda.synchronize()
    errors, out = int(d_err.item()), d_out.clone()
    assert errors > 0
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        d_err.zero_()
        plan.simulate_device(7, 0, nb, scaling, d_errors=d_err, d_out=d_out,
                             stream=torch.cuda.current_stream())
    for _ in range(3):
        d_out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert int(d_err.item()) == errors
        assert torch.equal(d_out, out)

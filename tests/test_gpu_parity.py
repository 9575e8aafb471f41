"""Parity of the HIP decoder (through the C ABI) with the reference and the oracle. Needs an MI355X.

* every golden fixture (reference outputs) on both kernels (code-specialised register trellis and the
  table-driven generic kernel), through ccv_* and through the reference-compatible decoder_* shims;
* seeded random inputs vs the oracle for codes the reference cannot run (K=9) or has no fixture for;
* edge cases: ragged batch sizes, empty batches, longest blocks, K=2 and K=12, n up to 8;
* BASELINE-size properties (1 M-bit frames): noiseless round trip, fused error count vs host count,
  exported decisions re-traced on the host, determinism.
Bit-exact comparisons throughout (the ACS is adds and compares only, fp32 as in the reference).
"""
import numpy as np
import pytest

import oracle_ctypes as O
from ccviterbi import (CODEBOOK, GEN_REF_X86, GEN_TRUE_PARITY, HARD, K7, K8, K9, SOFT, Code,
                       HardDecoder, Plan, SoftDecoder, channel as ch)
from ccviterbi import sim
from ccviterbi.decoder import FLAG_GENERIC, FLAG_GLOBAL_DECISIONS, FLAG_NO_PERSISTENT, FLAG_STEP_MAJOR
from conftest import golden_manifest

pytestmark = pytest.mark.gpu
CASES = golden_manifest()


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


def _code_of(g, gen=GEN_REF_X86):
    return Code(int(g["n"]), int(g["K"]), int(g["blen"]), tuple(int(p) for p in g["polys"]), gen)


def _ocode(c: Code):
    return O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)


def _oracle(c: Code, channel, data):
    if channel == SOFT:
        return O.viterbi_soft(_ocode(c), data), None
    return O.viterbi_hard(_ocode(c), data)


@pytest.mark.parametrize("flags", [0, FLAG_GLOBAL_DECISIONS, FLAG_GENERIC],
                         ids=["register", "register-hbm-decisions", "generic"])
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_fixture(case, flags):
    g = O.load_golden(case["name"])
    c = _code_of(g)
    channel = SOFT if case["channel"] == "awgn" else HARD
    plan = Plan(c, channel, flags)
    if flags & FLAG_GENERIC:
        assert plan.kernel == "generic"
    res = plan.decode_host(g["rx"])
    if channel == SOFT:
        out = res
    else:
        out, pm = res
        assert np.array_equal(pm, g["path_metric"])
    assert np.array_equal(out, g["out"])
    assert ch.count_bit_errors(c, g["info"], out) == int(g["errors"])


def test_register_kernel_selected_for_benchmark_codes():
    for c in (K7, K7.with_(gen_mode=GEN_TRUE_PARITY), CODEBOOK[0], CODEBOOK[3], CODEBOOK[5]):
        assert Plan(c, SOFT).kernel == "register"
        assert Plan(c, HARD).kernel == "register"
    for c in (K8, K9):
        for gen in (GEN_REF_X86, GEN_TRUE_PARITY):
            for channel in (SOFT, HARD):
                plan = Plan(c.with_(gen_mode=gen), channel)
                assert plan.kernel == "multilane" and plan.desc.lanes == 1 << (c.K - 7)
        assert Plan(c, SOFT, FLAG_GENERIC).kernel == "generic"
    # survivor decisions: VGPR-resident for the K<=7 benchmark codes at blen 40 (persistent kernels,
    # soft r = 1/2 and hard), for other soft r = 1/2 blocks up to T = 48 (viterbi_soft_regdec)
    for c in (K7, K7.with_(gen_mode=GEN_TRUE_PARITY), CODEBOOK[0], CODEBOOK[3]):
        for channel in (SOFT, HARD):
            assert Plan(c, channel).decisions == "registers"
            assert Plan(c, channel).variant == "persistent"
            assert Plan(c, channel, FLAG_GLOBAL_DECISIONS).decisions == "hbm"
        assert Plan(c, SOFT, FLAG_NO_PERSISTENT).variant == "register-regdec"
        assert Plan(c, HARD, FLAG_NO_PERSISTENT).decisions == "hbm"
    assert Plan(CODEBOOK[5], HARD).variant == "persistent"           # r = 1/3, hard
    assert Plan(K7.with_(blen=42), SOFT).decisions == "registers"   # T = 48
    assert Plan(K7.with_(blen=42), SOFT).variant == "register-regdec"
    assert Plan(K7.with_(blen=43), SOFT).decisions == "hbm"         # T = 49
    assert Plan(K7.with_(blen=42), HARD).decisions == "hbm"
    assert Plan(CODEBOOK[5], SOFT).decisions == "hbm"               # r = 1/3
    assert Plan(K7, SOFT, FLAG_GENERIC).decisions == "lds"          # acs_generic.hpp
    # K = 8, 9 (multilane kernel): register-resident up to T = 48 (K9) / 49 (K8), soft and hard
    for c in (K8, K9, K9.with_(gen_mode=GEN_TRUE_PARITY)):
        # the K = 9 x86-idiom code runs one lane per block with a per-wave decision slot (the
        # true-parity K = 9 code two lanes per block with a slot too, viterbi_multi2_slot); the BSC
        # at K = 9 runs the same kernels on Hamming-distance rows
        slot = "slot" if c.K == 9 else "registers"
        assert Plan(c, SOFT).decisions == slot and Plan(c, HARD).decisions == slot
        assert Plan(c, SOFT, FLAG_GLOBAL_DECISIONS).decisions == "hbm"
        assert Plan(c, SOFT, FLAG_NO_PERSISTENT).decisions == "registers"
    assert Plan(K9.with_(blen=41), SOFT).decisions == "hbm"           # T = 49
    assert Plan(K8.with_(blen=42), SOFT).decisions == "registers"     # T = 49
    # a K=9 code without an ahead-of-time kernel falls back to the table-driven kernel
    assert Plan(Code(2, 9, 40, (0xF080000000000000, 0xA980000000000000)), SOFT).kernel == "generic"


@pytest.mark.parametrize("case", [c for c in CASES if c["name"] in (
    "awgn_k7_4dB", "awgn_cb5_2dB", "bsc_k7_p50000", "bsc_cb0_p100000")], ids=lambda c: c["name"])
def test_reference_api_streaming(case):
    """decoder_create/init/register_callback/input exactly as the reference drivers use it: one
    trellis step per decoder_input call, the callback firing inside the call that completes a block."""
    g = O.load_golden(case["name"])
    c = _code_of(g)
    soft = case["channel"] == "awgn"
    dec = SoftDecoder() if soft else HardDecoder()
    got = []
    if soft:
        dec.register_callback(lambda data, n: got.append((data, n)))
    else:
        dec.register_callback(lambda data, n, pm: got.append((data, n, pm)))
    dec.init(c)
    nb = 12
    for b in range(nb):
        for t in range(c.steps):
            dec.input(g["rx"][b, t])
        assert len(got) == b + 1
    for b in range(nb):
        assert got[b][0] == g["out"][b].tobytes()
        assert got[b][1] == c.blen
        if not soft:
            assert got[b][2] == g["path_metric"][b]
    # batch extension: same callbacks, in order
    got.clear()
    dec.input_blocks(g["rx"][nb:2 * nb])
    assert [x[0] for x in got] == [g["out"][b].tobytes() for b in range(nb, 2 * nb)]
    # several steps per call, split at arbitrary step boundaries (len <= 255)
    got.clear()
    flat = g["rx"][2 * nb:3 * nb].reshape(-1) if soft else g["rx"][2 * nb:3 * nb].reshape(-1)
    step = (1 << c.n) if soft else 1
    pos = 0
    rng = np.random.default_rng(0)
    while pos < flat.size:
        k = int(rng.integers(1, 255 // step + 1)) * step
        dec.input(flat[pos:pos + k])
        pos += k
    assert [x[0] for x in got] == [g["out"][b].tobytes() for b in range(2 * nb, 3 * nb)]
    if soft:
        with pytest.raises(Exception):
            dec.input(np.zeros(3, np.float32))      # len % 2^n != 0 -> -1 (viterbi-decoder.c:226-228)
    dec.destroy()


@pytest.mark.parametrize("case", ["awgn_k7_4dB", "bsc_cb0_p100000"])
def test_reference_api_callback_takes_ownership(case):
    """A callback that returns 0 takes the output buffer (AWGN-channel/viterbi-decoder.c:92-106,
    binary-symmetric-channel/viterbi-decoder.c:98-112; api_shim.cpp emit_output_buffer): the decoder
    must allocate a fresh buffer for the next block and never touch the taken one again. Odd blocks
    are taken (kept until the end, then freed with free() as the new owner), even blocks are copied
    and handed back (-1), both through the streaming and the batch entry points: every taken buffer
    still holds its own block, all taken pointers differ, and the handed-back blocks are correct."""
    import ctypes
    import ctypes.util
    g = O.load_golden(case)
    c = _code_of(g)
    soft = case.startswith("awgn")
    dec = SoftDecoder() if soft else HardDecoder()
    dec.init(c)
    taken, copied, pms = [], [], []
    count = [0]

    def take(data, length, *rest):   # rest: (userdata,) soft / (path_metric, userdata) hard
        assert length == c.blen
        count[0] += 1
        if not soft:
            pms.append(int(rest[0]))
        if count[0] % 2 == 1:
            taken.append((count[0] - 1, ctypes.cast(data, ctypes.c_void_p).value))
            return 0
        copied.append((count[0] - 1, ctypes.string_at(data, c.out_bytes)))
        return -1

    from ccviterbi.decoder import _HARD_CB, _SOFT_CB
    cb = (_SOFT_CB if soft else _HARD_CB)(take)
    dec._lib.decoder_register_callback(dec._obj, ctypes.cast(cb, ctypes.c_void_p))
    nb = 10
    for b in range(nb):                                   # streaming: one step per call
        for t in range(c.steps):
            dec.input(g["rx"][b, t])
    dec.input_blocks(g["rx"][nb:2 * nb])                  # batch extension, same callbacks
    assert count[0] == 2 * nb
    assert len({p for _, p in taken}) == len(taken) == nb, "a taken buffer was reused"
    for b, p in taken:
        assert ctypes.string_at(p, c.out_bytes) == g["out"][b].tobytes(), b
    for b, data in copied:
        assert data == g["out"][b].tobytes(), b
    if not soft:
        assert pms == [int(x) for x in g["path_metric"][:2 * nb]]
    dec.destroy()
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.free.argtypes = [ctypes.c_void_p]
    for _, p in taken:
        libc.free(p)


def test_reference_api_generator_mode_true_parity():
    c = K7.with_(gen_mode=GEN_TRUE_PARITY)
    info, rx = ch.awgn_blocks(c, 300, ch.noise_scaling(3.0), 5)
    dec = SoftDecoder()
    dec.init(c)
    out = dec.decode_blocks(rx)
    assert np.array_equal(out, O.viterbi_soft(_ocode(c), rx))


def test_reference_api_k9_batches_and_streaming():
    """The reference decoder API (libccv_awgn.so) with the K = 9 code: a large batch through
    decode_blocks (the one-lane-per-block kernel) and single steps through decoder_input (the
    latency path) give the oracle's bytes; the callbacks fire in block order."""
    info, rx = ch.awgn_blocks(K9, 3000, ch.noise_scaling(3.0), 606)
    dec = SoftDecoder()
    dec.init(K9)
    out = dec.decode_blocks(rx)
    sample = np.arange(0, 3000, 10)
    assert np.array_equal(out[sample], O.viterbi_soft(_ocode(K9), rx[sample]))
    got = []
    dec.register_callback(lambda data, n: got.append(data))
    for b in range(3):
        for t in range(K9.steps):
            dec.input(rx[b, t])
    assert [bytes(x) for x in got] == [out[b].tobytes() for b in range(3)]


SEEDED = [
    ("k7_ref_soft", K7, SOFT), ("k7_true_soft", K7.with_(gen_mode=GEN_TRUE_PARITY), SOFT),
    ("k7_ref_hard", K7, HARD), ("k7_true_hard", K7.with_(gen_mode=GEN_TRUE_PARITY), HARD),
    ("k8_soft", K8, SOFT), ("k8_true_soft", K8.with_(gen_mode=GEN_TRUE_PARITY), SOFT),
    ("k8_hard", K8, HARD), ("k8_true_hard", K8.with_(gen_mode=GEN_TRUE_PARITY), HARD),
    ("k9_soft", K9, SOFT), ("k9_true_soft", K9.with_(gen_mode=GEN_TRUE_PARITY), SOFT),
    ("k9_hard", K9, HARD), ("k9_true_hard", K9.with_(gen_mode=GEN_TRUE_PARITY), HARD),
    ("code1_true_soft", CODEBOOK[1].with_(gen_mode=GEN_TRUE_PARITY), SOFT),
    ("code2_true_hard", CODEBOOK[2].with_(gen_mode=GEN_TRUE_PARITY), HARD),
    ("code3_true_soft", CODEBOOK[3].with_(gen_mode=GEN_TRUE_PARITY), SOFT),
    ("code5_hard", CODEBOOK[5], HARD),
]


@pytest.mark.parametrize("flags", [0, FLAG_GENERIC], ids=["auto", "generic"])
@pytest.mark.parametrize("name,c,channel", SEEDED, ids=[s[0] for s in SEEDED])
def test_seeded_vs_oracle(name, c, channel, flags):
    nb = 1000 if c.K <= 8 else 300
    for db, p_ppm in ((1.0, 120000), (4.0, 30000)):
        if channel == SOFT:
            info, data = ch.awgn_blocks(c, nb, ch.noise_scaling(db), 1234 + c.K)
        else:
            info, data = ch.bsc_blocks(c, nb, p_ppm, 4321 + c.K)
        res = Plan(c, channel, flags).decode_host(data)
        ref, ref_pm = _oracle(c, channel, data)
        if channel == SOFT:
            assert np.array_equal(res, ref)
        else:
            assert np.array_equal(res[0], ref) and np.array_equal(res[1], ref_pm)


# Register-resident decisions (viterbi_soft_regdec) cut a block into 8-step chunks ending at step T,
# padding the first one with 8*ceil(T/8) - T neutral steps: every padding 0..7, both sides of the
# T <= 48 limit, and T < 8 (one padded chunk only).
REGDEC_BLENS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 17, 33, 40, 41, 42, 43, 44]


@pytest.mark.parametrize("blen", REGDEC_BLENS)
@pytest.mark.parametrize("base", [K7, K7.with_(gen_mode=GEN_TRUE_PARITY), CODEBOOK[0], CODEBOOK[3]],
                         ids=["k7", "k7_true", "code0", "code3"])
def test_register_decisions_all_paddings(base, blen):
    c = base.with_(blen=blen)
    info, rx = ch.awgn_blocks(c, 333, ch.noise_scaling(2.0), 77 + blen)
    ref = O.viterbi_soft(_ocode(c), rx)
    for flags in (0, FLAG_GLOBAL_DECISIONS):
        assert np.array_equal(Plan(c, SOFT, flags).decode_host(rx), ref)
    tied = np.random.default_rng(blen).integers(-2, 3, size=rx.shape).astype(np.float32)
    assert np.array_equal(Plan(c, SOFT).decode_host(tied), O.viterbi_soft(_ocode(c), tied))


# Persistent K <= 7 kernels (acs_persist.hpp, blen 40): growth steps from the reset metrics, static
# chunks, waves walking 64-block groups with the next group's input prefetched. Checked against the
# oracle on ragged batches (partial last group; hard: the partial group on viterbi_hard_reg) and,
# for batches with many groups per resident wave, against the non-persistent kernels block for block.
PERSIST_CODES = [("k7", K7), ("k7_true", K7.with_(gen_mode=GEN_TRUE_PARITY)), ("code0", CODEBOOK[0]),
                 ("code1", CODEBOOK[1]), ("code2_true", CODEBOOK[2].with_(gen_mode=GEN_TRUE_PARITY)),
                 ("code3", CODEBOOK[3])]


@pytest.mark.parametrize("nb", [1, 63, 64, 65, 200, 1999])
@pytest.mark.parametrize("name,c", PERSIST_CODES, ids=[x[0] for x in PERSIST_CODES])
def test_persistent_kernels_vs_oracle(name, c, nb):
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(1.5), 300 + nb)
    plan = Plan(c, SOFT)
    assert plan.variant == "persistent"
    assert np.array_equal(plan.decode_host(rx), O.viterbi_soft(_ocode(c), rx))
    tied = np.random.default_rng(nb).integers(-3, 4, size=rx.shape).astype(np.float32)
    assert np.array_equal(plan.decode_host(tied), O.viterbi_soft(_ocode(c), tied))
    info, syms = ch.bsc_blocks(c, nb, 110000, 500 + nb)
    out, pm = Plan(c, HARD).decode_host(syms)
    ref, ref_pm = O.viterbi_hard(_ocode(c), syms)
    assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)


def test_persistent_hard_rate_one_third():
    c = CODEBOOK[5]
    for nb in (64, 1000):
        info, syms = ch.bsc_blocks(c, nb, 90000, nb)
        plan = Plan(c, HARD)
        assert plan.variant == "persistent"
        out, pm = plan.decode_host(syms)
        ref, ref_pm = O.viterbi_hard(_ocode(c), syms)
        assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)


@pytest.mark.parametrize("channel", [SOFT, HARD], ids=["soft", "hard"])
@pytest.mark.parametrize("gen", [GEN_REF_X86, GEN_TRUE_PARITY], ids=["ref", "true"])
def test_persistent_many_groups_per_wave(torch_cuda, gen, channel):
    """8 x 1 M-bit frames + 17 blocks: every resident wave walks several groups, so the cross-group
    prefetch and the per-group reset are exercised; the output, path metrics and fused error count
    must equal the non-persistent kernel's block for block (and the oracle's on a subsample)."""
    torch = torch_cuda
    c = K7.with_(gen_mode=gen)
    nb = 8 * FRAME + 17
    if channel == SOFT:
        info, data = ch.awgn_blocks(c, nb, ch.noise_scaling(3.0), 4242)
    else:
        info, data = ch.bsc_blocks(c, nb, 60000, 4242)
    d_in, d_info = _device(torch, data), _device(torch, info)
    res = []
    for flags in (0, FLAG_NO_PERSISTENT):
        plan = Plan(c, channel, flags)
        d_out = torch.zeros((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
        d_pm = torch.zeros(nb, dtype=torch.int32, device="cuda")
        d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
        plan.decode_device(d_in, nb, d_out, d_path_metric=d_pm if channel == HARD else None,
                           d_info=d_info, d_errors=d_err)
        torch.cuda.synchronize()
        res.append((d_out.cpu().numpy(), d_pm.cpu().numpy(), int(d_err.item())))
    (out, pm, err), (out2, pm2, err2) = res
    assert np.array_equal(out, out2) and np.array_equal(pm, pm2) and err == err2
    assert err == ch.count_bit_errors(c, info, out)
    idx = np.arange(0, nb, 211)
    ref, ref_pm = _oracle(c, channel, data[idx])
    assert np.array_equal(out[idx], ref)
    if channel == HARD:
        assert np.array_equal(pm[idx], ref_pm)


def test_persistent_grid_per_kernel(torch_cuda):
    """The resident-wave grid is cached per KERNEL (all persistent kernels share one C++ type): after
    K=7 soft, code 0 hard and K=9 soft decode in one process, in that order, each plan's launches use
    its own kernel's occupancy, not the first kernel's."""
    torch = torch_cuda
    plans = [(K7, SOFT), (CODEBOOK[0], HARD), (K9, SOFT)]
    for c, channel in plans:
        p = Plan(c, channel)
        assert p.variant == ("persistent-wide" if c is K9 else "persistent")
        nb = 3 * 64 + 5
        if channel == SOFT:
            info, data = ch.awgn_blocks(c, nb, ch.noise_scaling(3.0), 5)
        else:
            info, data = ch.bsc_blocks(c, nb, 40000, 5)
        out = p.decode_host(data)
        out = out[0] if channel == HARD else out
        assert np.array_equal(out, _oracle(c, channel, data)[0])
        cached, fresh = p.persistent_waves(), p.persistent_waves(fresh=True)
        assert cached > 0 and cached == fresh, (c.name, channel, cached, fresh)
    assert Plan(CODEBOOK[0], SOFT, FLAG_NO_PERSISTENT).persistent_waves() == 0


def test_dropped_plans_release_device_memory(torch_cuda):
    """Plan.__del__ destroys the plan: creating and dropping plans with large HBM decision scratch
    does not leak device memory (nor streams)."""
    import gc
    torch = torch_cuda
    # the first plans of a process load the code objects and the runtime's own pools (~150 MB when
    # this test runs first): one create/reserve/drop of each kind before the baseline
    for ch_ in (SOFT, HARD):
        with Plan(K7, ch_, FLAG_GLOBAL_DECISIONS) as plan:
            plan.reserve(1_600_000)
    torch.cuda.synchronize()
    gc.collect()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(12):
        plan = Plan(K7, SOFT, FLAG_GLOBAL_DECISIONS)
        plan.reserve(1_600_000)          # ~590 MB of decision scratch each
        del plan
    with Plan(K7, HARD, FLAG_GLOBAL_DECISIONS) as plan:
        plan.reserve(1_600_000)
    gc.collect()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free1 >= free0 - (64 << 20), (free0, free1)


@pytest.mark.parametrize("nb", [1, 2, 63, 64, 65, 127, 1000])
def test_ragged_batches(nb):
    info, rx = ch.awgn_blocks(K7, nb, ch.noise_scaling(2.0), nb)
    assert np.array_equal(Plan(K7, SOFT).decode_host(rx), O.viterbi_soft(_ocode(K7), rx))
    info, syms = ch.bsc_blocks(K7, nb, 80000, nb)
    out, pm = Plan(K7, HARD).decode_host(syms)
    ref, ref_pm = O.viterbi_hard(_ocode(K7), syms)
    assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)


MULTI_SHAPES = [(1, 40), (3, 1), (15, 7), (16, 8), (17, 9), (33, 249), (100, 255), (257, 23)]


@pytest.mark.parametrize("K", [8, 9])
@pytest.mark.parametrize("nb,blen", MULTI_SHAPES, ids=[f"nb{a}_blen{b}" for a, b in MULTI_SHAPES])
def test_multilane_shapes(K, nb, blen):
    """Multilane kernel: ragged batches (lane groups straddling waves) and every T mod (K-1) phase
    the final argmin and the traceback start from (T = blen + K - 1)."""
    c = (K8 if K == 8 else K9).with_(blen=blen)
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(2.0), nb * 7 + blen)
    info, syms = ch.bsc_blocks(c, nb, 90000, nb * 5 + blen)
    ref, ref_pm = O.viterbi_hard(_ocode(c), syms)
    for flags in (0, FLAG_GLOBAL_DECISIONS):   # register-resident (T <= 48/49) and HBM decisions
        plan = Plan(c, SOFT, flags)
        assert plan.kernel == "multilane"
        assert np.array_equal(plan.decode_host(rx), O.viterbi_soft(_ocode(c), rx))
        out, pm = Plan(c, HARD, flags).decode_host(syms)
        assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)


@pytest.mark.parametrize("gen", [GEN_REF_X86, GEN_TRUE_PARITY], ids=["idiom", "true"])
@pytest.mark.parametrize("nb", [1, 15, 16, 17, 63, 64, 65, 3 * 64 + 5, 150000])
def test_k9_wide_kernel(torch_cuda, nb, gen):
    """K = 9 soft at blen 40 runs a persistent kernel whose decisions go through a per-wave scratch
    slot: one lane per block for the x86-idiom code (acs_wide.hpp), two lanes per block with the main
    periods as a loop for the true-parity code (acs_multi2.hpp viterbi_multi2_slot). Ragged batches and
    more groups than resident waves (150,000 blocks: each wave decodes several groups through its one
    slot) decode exactly as the non-persistent four-lane kernel (FLAG_NO_PERSISTENT) and, on a
    sample, the oracle; the fused error count equals the host count."""
    torch = torch_cuda
    c = K9.with_(gen_mode=gen)
    plan = Plan(c, SOFT)
    assert plan.variant == ("persistent-wide" if gen == GEN_REF_X86 else "persistent-slot2")
    assert plan.decisions == "slot"
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(3.0), 4242 + nb)
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    plan.decode_device(_device(torch, rx), nb, d_out, d_info=_device(torch, info), d_errors=d_err)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)
    four_lane = Plan(c, SOFT, FLAG_NO_PERSISTENT)
    assert four_lane.variant.startswith("multilane")
    assert np.array_equal(out, four_lane.decode_host(rx))
    sample = np.unique(np.linspace(0, nb - 1, min(nb, 300)).astype(np.int64))
    assert np.array_equal(out[sample], O.viterbi_soft(_ocode(c), rx[sample]))




@pytest.mark.parametrize("gen", [GEN_REF_X86, GEN_TRUE_PARITY], ids=["ref", "true"])
def test_k9_bsc_through_the_persistent_kernels(torch_cuda, gen):
    """K = 9 BSC at blen 40 runs the soft persistent kernels on Hamming-distance rows (core.hip
    hard_rows; x86 idiom: one lane per block, true parity: two lanes): outputs and path metrics equal
    the oracle's and the multilane BSC kernel's, for ragged batches, from clean to p = 0.4 (where the
    0xFF00 saturation of the reference would show if it mattered)."""
    c = K9.with_(gen_mode=gen)
    plan = Plan(c, HARD)
    assert plan.variant == ("persistent-wide" if gen == GEN_REF_X86 else "persistent-slot2")
    multilane = Plan(c, HARD, FLAG_NO_PERSISTENT)
    assert multilane.variant.startswith("multilane")
    for nb, p_ppm in ((1, 0), (3 * 64 + 5, 50000), (2048 + 77, 400000)):
        _, syms = ch.bsc_blocks(c, nb, p_ppm, 1234 + nb)
        out, pm = plan.decode_host(syms)
        ref, ref_pm = O.viterbi_hard(_ocode(c), syms)
        assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)
        out2, pm2 = multilane.decode_host(syms)
        assert np.array_equal(out, out2) and np.array_equal(pm, pm2)


@pytest.mark.parametrize("gen", [GEN_REF_X86, GEN_TRUE_PARITY], ids=["ref", "true"])
def test_k9_bsc_reserved_plan_allocates_nothing_on_decode(torch_cuda, gen):
    """ccv_plan_reserve(max_blocks) sizes everything a decode of up to max_blocks needs -- for K = 9
    BSC also the Hamming-distance rows (16 B per step, core.hip hard_rows): the decode then
    runs no hipMalloc (free device memory unchanged), and the result is the unreserved plan's."""
    torch = torch_cuda
    c = K9.with_(gen_mode=gen)
    nb = 25000   # one 1 M-bit frame: 19.2 MB of rows, far above the allocation granularity
    _, syms = ch.bsc_blocks(c, nb, 50000, 4321)
    d_in = torch.from_numpy(syms).to("cuda")
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    # the runtime's own first-launch allocations (code object; the scratch of a kernel with a spill,
    # per HIP stream and sized by the grid) come from a throw-away plan's decode on the same stream
    Plan(c, HARD).decode_device(d_in, nb, d_out)
    plan = Plan(c, HARD)
    plan.reserve(nb)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    plan.decode_device(d_in, nb, d_out)
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info()[0] >= free0
    ref, _ = Plan(c, HARD).decode_host(syms)
    assert np.array_equal(d_out.cpu().numpy(), ref)


def test_k9_true_two_lane_kernel_ragged_groups(torch_cuda):
    """The true-parity K = 9 kernel (two lanes per block, acs_multi2.hpp) decodes a ragged batch of
    several rounds of 32-block groups over the resident waves identically to the oracle."""
    c = K9.with_(gen_mode=GEN_TRUE_PARITY)
    plan = Plan(c, SOFT)
    assert plan.variant == "persistent-slot2"
    nb = 3 * 2048 + 77
    _, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(2.0), 515)
    assert np.array_equal(plan.decode_host(rx), O.viterbi_soft(_ocode(c), rx))


def test_multilane_error_count_and_no_decision_export(torch_cuda):
    torch = torch_cuda
    c = K9.with_(gen_mode=GEN_TRUE_PARITY)
    nb = 2000
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(3.0), 99)
    plan = Plan(c, SOFT)
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    plan.decode_device(_device(torch, rx), nb, d_out, d_info=_device(torch, info), d_errors=d_err)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert np.array_equal(out, O.viterbi_soft(_ocode(c), rx))
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)
    d_dec = torch.empty((c.steps, 4 * nb + 64), dtype=torch.int64, device="cuda")
    with pytest.raises(Exception, match="single-lane"):
        plan.decode_device(_device(torch, rx), nb, d_out, d_decisions=d_dec)


def test_empty_batch_is_noop(torch_cuda):
    torch = torch_cuda
    plan = Plan(K7, SOFT)
    plan.decode_device(torch.empty(0, device="cuda"), 0, torch.empty(0, dtype=torch.uint8, device="cuda"))
    out = plan.decode_host(np.zeros((0, K7.steps, 4), np.float32))
    assert out.shape == (0, K7.out_bytes)


EDGE = [
    ("k7_blen255", K7.with_(blen=255), SOFT),            # T = 261 > the reference encoder's 255
    ("k7_blen1", K7.with_(blen=1), SOFT),
    ("k2", Code(2, 2, 40, (0xC000000000000000, 0x8000000000000000)), SOFT),
    ("k9_blen255", K9.with_(blen=255), SOFT),
    ("k8_blen255_hard", K8.with_(blen=255), HARD),
    ("k12", Code(2, 12, 60, (0xFFD0000000000000, 0xB970000000000000)), SOFT),
    ("k12_hard", Code(2, 12, 60, (0xFFD0000000000000, 0xB970000000000000)), HARD),
    ("n1_k5", Code(1, 5, 40, (0xF800000000000000,)), SOFT),
    ("n4_k4_hard", Code(4, 4, 40, (0xF000000000000000, 0xB000000000000000, 0xD000000000000000,
                                   0x9000000000000000)), HARD),
    ("n8_k3_hard", Code(8, 3, 40, tuple([0xE000000000000000, 0xA000000000000000, 0xC000000000000000,
                                          0x6000000000000000] * 2)), HARD),
    ("n4_k3_soft", Code(4, 3, 40, (0xE000000000000000, 0xA000000000000000, 0xC000000000000000,
                                   0x6000000000000000)), SOFT),
]


@pytest.mark.parametrize("name,c,channel", EDGE, ids=[e[0] for e in EDGE])
def test_edge_codes(name, c, channel):
    rng = np.random.default_rng(len(name))
    nb = 200 if c.K < 10 else 40
    if channel == SOFT:
        # arbitrary non-negative metrics (n may exceed the 3 bits a constellation exists for)
        data = rng.exponential(size=(nb, c.steps, 1 << c.n)).astype(np.float32)
    else:
        data = rng.integers(0, 256, size=(nb, c.steps), dtype=np.uint8)
    for flags in (0, FLAG_GENERIC):
        res = Plan(c, channel, flags).decode_host(data)
        ref, ref_pm = _oracle(c, channel, data)
        if channel == SOFT:
            assert np.array_equal(res, ref)
        else:
            assert np.array_equal(res[0], ref) and np.array_equal(res[1], ref_pm)


def test_negative_and_tied_soft_metrics():
    """General float inputs: negative metrics and exact ties follow the reference's strict '<'."""
    rng = np.random.default_rng(3)
    for c in (K7, CODEBOOK[0], K8, K9, K9.with_(gen_mode=GEN_TRUE_PARITY)):
        data = rng.integers(-3, 4, size=(300, c.steps, 4)).astype(np.float32)  # many exact ties
        for flags in (0, FLAG_GLOBAL_DECISIONS, FLAG_GENERIC):
            assert np.array_equal(Plan(c, SOFT, flags).decode_host(data), O.viterbi_soft(_ocode(c), data))


# --------------------------------------------------------------- BASELINE-size (1 M-bit frame) checks

FRAME = 25000   # blocks of 40 bits = 10^6 info bits


def _device(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).to("cuda")


@pytest.mark.parametrize("base", [K7, K9], ids=["k7", "k9"])
@pytest.mark.parametrize("gen", [GEN_REF_X86, GEN_TRUE_PARITY])
def test_full_frame_noiseless(torch_cuda, gen, base):
    """True parity: (171,133) is a proper non-catastrophic code, so a noiseless frame decodes with
    zero errors. The x86-idiom variant is not injective (some butterflies emit the same symbol for
    both inputs), so even noiseless frames keep errors -- there the check is equality with the oracle."""
    torch = torch_cuda
    c = base.with_(gen_mode=gen)
    info, rx = ch.awgn_blocks(c, FRAME, 0.0, 2024)
    plan = Plan(c, SOFT)
    d_out = torch.empty((FRAME, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    plan.decode_device(_device(torch, rx), FRAME, d_out, d_info=_device(torch, info), d_errors=d_err)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)
    if gen == GEN_TRUE_PARITY:
        assert int(d_err.item()) == 0
        bits = np.unpackbits(out, axis=1)
        assert np.array_equal(bits[:, :c.blen], np.unpackbits(info, axis=1)[:, :c.blen])
        assert not bits[:, c.blen:c.steps].any()   # the zero tail decodes as zeros
    # the whole frame against the oracle (round 6; a strided subsample before)
    assert np.array_equal(out, O.viterbi_soft(_ocode(c), rx))


def test_full_frame_error_count_decisions_and_determinism(torch_cuda):
    torch = torch_cuda
    c = K7
    info, rx = ch.awgn_blocks(c, FRAME, ch.noise_scaling(4.0), 77)
    plan = Plan(c, SOFT)
    d_rx, d_info = _device(torch, rx), _device(torch, info)
    d_out = torch.empty((FRAME, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_dec = torch.empty((c.steps, (FRAME + 63) // 64 * 64), dtype=torch.int64, device="cuda")
    plan.decode_device(d_rx, FRAME, d_out, d_info=d_info, d_errors=d_err, d_decisions=d_dec)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    # fused consumer == host consumer (AWGN-channel/main.c:129-141)
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)
    # the whole frame against the oracle (round 6; a strided subsample before)
    assert np.array_equal(out, O.viterbi_soft(_ocode(c), rx))
    idx = np.arange(0, FRAME, 97)
    # exported decisions re-traced on the host reproduce the output (host-traceback mode)
    dec = d_dec.cpu().numpy().view(np.uint64)
    S = c.states
    for b in idx[:40]:
        # final metrics are not exported: take the argmin state implied by the device's output,
        # i.e. check that walking back from the state the last K-1 output bits encode is consistent
        st = 0
        for t in range(c.steps - 1, c.steps - c.K, -1):
            bit = (out[b, t // 8] >> (7 - t % 8)) & 1
            st |= int(bit) << (c.K - 2 - (c.steps - 1 - t))
        bits = []
        for t in range(c.steps - 1, -1, -1):
            bits.append(st >> (c.K - 2))
            d = int(dec[t, b] >> np.uint64(st)) & 1
            st = ((st << 1) & (S - 1)) | d
        host = np.packbits(np.array(bits[::-1], np.uint8))
        assert np.array_equal(host[:c.out_bytes], out[b])
    # determinism: a second decode is identical
    d_out2 = torch.empty_like(d_out)
    plan.decode_device(d_rx, FRAME, d_out2)
    torch.cuda.synchronize()
    assert torch.equal(d_out, d_out2)


def test_full_frame_bsc_k7(torch_cuda):
    torch = torch_cuda
    info, syms = ch.bsc_blocks(K7, FRAME, 50000, 8)
    plan = Plan(K7, HARD)
    d_out = torch.empty((FRAME, K7.out_bytes), dtype=torch.uint8, device="cuda")
    d_pm = torch.empty(FRAME, dtype=torch.int32, device="cuda")
    plan.decode_device(_device(torch, syms), FRAME, d_out, d_path_metric=d_pm)
    torch.cuda.synchronize()
    ref, ref_pm = O.viterbi_hard(_ocode(K7), syms)   # the whole frame (round 6)
    assert np.array_equal(d_out.cpu().numpy(), ref)
    assert np.array_equal(d_pm.cpu().numpy(), ref_pm)
    # path metric = Hamming distance between the survivor path re-encoded from the zero state (all T
    # decided inputs, tail decisions included: the traceback is not forced to end in state 0) and
    # the received symbols
    out = d_out.cpu().numpy()
    full = K7.with_(blen=K7.steps)                  # encode T input bits, keep the first T symbols
    recoded = ch.encode(full, out)[:, :K7.steps]
    dist = np.unpackbits((recoded ^ syms)[..., None], axis=-1)[..., -2:].sum(axis=(1, 2))
    assert np.array_equal(dist, d_pm.cpu().numpy())


def test_statistical_ber_code0_matches_published(torch_cuda):
    """results/awgn_channel.m:15, code 0 soft Viterbi: BER at 4 dB and 6 dB within tolerance."""
    from ccviterbi import sim
    pts = sim.ber_sweep(CODEBOOK[0], [4.0, 6.0], bits_per_point=lambda p: 2_000_000, frame_blocks=25000,
                        seed=31)
    assert abs(pts[0].ber - 0.05668375) / 0.05668375 < 0.05
    assert abs(pts[1].ber - 0.00545587) / 0.00545587 < 0.1


@pytest.mark.parametrize("c", [K7, K7.with_(gen_mode=GEN_TRUE_PARITY), CODEBOOK[0], CODEBOOK[5]],
                         ids=["k7", "k7_true", "code0", "code5"])
def test_step_major_layout_matches(torch_cuda, c):
    """CCV_FLAG_STEP_MAJOR: the same frames transposed to [T][nb][2^n] decode identically."""
    from ccviterbi.decoder import FLAG_STEP_MAJOR
    torch = torch_cuda
    nb = 3001
    info, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(3.0), 17)
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    Plan(c, SOFT, FLAG_STEP_MAJOR).decode_device(_device(torch, rx.transpose(1, 0, 2)), nb, d_out,
                                                  d_info=_device(torch, info), d_errors=d_err)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert np.array_equal(out, O.viterbi_soft(_ocode(c), rx))
    assert int(d_err.item()) == ch.count_bit_errors(c, info, out)


DROPIN_CASES = [c for c in CASES if c["name"] in (
    "awgn_cb0_4dB", "awgn_k7_2dB", "awgn_cb5_2dB", "awgn_k3_blen7_2dB", "bsc_cb0_p100000", "bsc_k7_p50000")]


@pytest.mark.parametrize("case", DROPIN_CASES, ids=lambda c: c["name"])
def test_reference_driver_with_mi355x_decoder(case, tmp_path):
    """Drop-in check: oracle/ref_harness.c -- the reference drivers' producer chain and callback
    logic, compiled against the reference's own headers -- linked to libccv_{awgn,bsc}.so instead of
    the reference decoder, reproduces the reference's output files byte for byte."""
    import os
    import subprocess
    from conftest import REPO
    exe = os.path.join(REPO, "oracle", "_ref", f"ref_harness_{case['channel']}_ccv")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref drop-in harness not built (needs /root/reference at build time)")
    g = O.load_golden(case["name"])
    prefix = str(tmp_path / case["name"])
    subprocess.run([exe, prefix, str(case["seed"]), str(case["nblocks"]), case["param"], case["spec"]],
                   check=True, timeout=300)
    out = np.fromfile(prefix + ".out", dtype=np.uint8).reshape(g["out"].shape)
    assert np.array_equal(out, g["out"])
    if case["channel"] == "bsc":
        assert np.array_equal(np.fromfile(prefix + ".pm", dtype=np.int32), g["path_metric"])
    meta = dict(line.split() for line in open(prefix + ".meta"))
    assert int(meta["errors"]) == case["errors"]


@pytest.mark.parametrize("channel", [SOFT, HARD], ids=["soft", "hard"])
def test_streaming_service_kernel(channel, monkeypatch):
    """The resident streaming service (acs_generic.hpp viterbi_service, ccv_decode_host with <= 4
    blocks): many single-block calls, 1-4-block calls, pauses past the kernel's 20 ms idle exit (so it
    is relaunched) and the launch-per-call and staged paths (CCV_HOST_LATENCY=1 / 0) all give the
    oracle's output and path metrics."""
    import time
    c = K7 if channel == SOFT else CODEBOOK[0]
    nb = 120
    if channel == SOFT:
        _, data = ch.awgn_blocks(c, nb, ch.noise_scaling(3.0), 77)
    else:
        _, data = ch.bsc_blocks(c, nb, 80000, 77)
    ref, ref_pm = _oracle(c, channel, data)
    for mode in ("2", "1", "0"):
        monkeypatch.setenv("CCV_HOST_LATENCY", mode)
        plan = Plan(c, channel)
        k = 0
        sizes = [1] * 40 + [2, 3, 4, 1, 4, 3, 2] * 4
        for i, n in enumerate(sizes):
            if k + n > nb:
                break
            if i in (10, 41):
                time.sleep(0.05)   # past the service's idle exit: the next call relaunches it
            res = plan.decode_host(data[k:k + n])
            out = res if channel == SOFT else res[0]
            assert np.array_equal(out, ref[k:k + n]), (mode, i)
            if channel == HARD:
                assert np.array_equal(res[1], ref_pm[k:k + n]), (mode, i)
            k += n
        plan.close()   # stops a service kernel that is still polling


# The one-wave latency kernel (acs_latency.hpp) has two shapes: register exchange for T <= 64 and
# decision masks + a traceback beyond; every K it serves (2..7), both sides of T = 64, tied inputs.
K2 = Code(2, 2, 40, (0xC000000000000000, 0x8000000000000000), GEN_REF_X86)
LATENCY_CODES = [("k2", K2), ("code0", CODEBOOK[0]), ("code1", CODEBOOK[1]), ("code2", CODEBOOK[2]),
                 ("code3", CODEBOOK[3]), ("code5_r13", CODEBOOK[5]), ("k7", K7),
                 ("k7_true", K7.with_(gen_mode=GEN_TRUE_PARITY))]
LATENCY_BLENS = [1, 5, 40, 57, 58, 59, 100, 255]   # K=7: T = 7, 11, 46, 63, 64, 65, 106, 261


@pytest.mark.parametrize("blen", LATENCY_BLENS)
@pytest.mark.parametrize("name,base", LATENCY_CODES, ids=[x[0] for x in LATENCY_CODES])
def test_latency_kernel_shapes(name, base, blen, monkeypatch):
    c = base.with_(blen=blen)
    monkeypatch.setenv("CCV_HOST_LATENCY", "1")            # one launch per call, one wave per block
    nb = 48
    _, rx = ch.awgn_blocks(c, nb, ch.noise_scaling(2.0), 31 + blen)
    tied = np.random.default_rng(blen).integers(-2, 3, size=rx.shape).astype(np.float32)
    _, syms = ch.bsc_blocks(c, nb, 90000, 31 + blen)
    plan_s, plan_h = Plan(c, SOFT), Plan(c, HARD)
    for data in (rx, tied):
        assert np.array_equal(plan_s.decode_host(data), O.viterbi_soft(_ocode(c), data))
    out, pm = plan_h.decode_host(syms)
    ref, ref_pm = O.viterbi_hard(_ocode(c), syms)
    assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)
    monkeypatch.setenv("CCV_HOST_LATENCY", "2")            # the resident service, <= 4 blocks a call
    plan_s2 = Plan(c, SOFT)
    for k in range(0, 12, 3):
        assert np.array_equal(plan_s2.decode_host(tied[k:k + 3]), O.viterbi_soft(_ocode(c), tied[k:k + 3]))
    plan_s2.close()
    plan_s.close()
    plan_h.close()


def test_streaming_shim_latency_config1(tmp_path):
    """Config 1 (BSC K=3 code 0, 10 k bits = 250 blocks) through the reference drivers' call pattern
    (one decoder_input() per trellis step, oracle/ref_harness.c linked to libccv_bsc.so): output equal
    to the reference decoder's on the same stream, and the time spent inside decoder_input() reported
    (.meta decoder_seconds) -- each completed block is decoded by the resident service kernel
    (INTEGRATION.md states the measured microseconds per block)."""
    import os
    import subprocess
    from conftest import REPO
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness_bsc_ccv")
    ref_exe = os.path.join(REPO, "oracle", "_ref", "ref_harness_bsc")
    if not (os.path.exists(exe) and os.path.exists(ref_exe)):
        pytest.skip("oracle/_ref harnesses not built (needs /root/reference at build time)")
    outs, secs = [], []
    for e in (exe, ref_exe):
        prefix = str(tmp_path / os.path.basename(e))
        subprocess.run([e, prefix, "5", "250", "25000", "cb:0"], check=True, timeout=300)
        meta = dict(line.split() for line in open(prefix + ".meta"))
        assert int(meta["blocks_decoded"]) == 250
        secs.append(float(meta["decoder_seconds"]))
        outs.append(open(prefix + ".out", "rb").read())
    assert outs[0] == outs[1]
    per_block_us = secs[0] / 250 * 1e6
    print(f"decoder_input: {per_block_us:.1f} us per block on the MI355X shim, "
          f"{secs[1] / 250 * 1e6:.2f} us in the reference decoder")
    assert 0 < per_block_us < 2000


# --------------------------------------------------------------- on-device channel (ccv_simulate_device)

def _simulate(torch, plan, c, seed, first, nb, param, hard_demap=False, noise_f32=False):
    hard = plan.channel == HARD
    d_info = torch.empty((nb, c.info_bytes), dtype=torch.uint8, device="cuda")
    d_out = torch.empty((nb, c.out_bytes), dtype=torch.uint8, device="cuda")
    d_pm = torch.empty(nb, dtype=torch.int32, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    shape = (nb, c.steps) if hard else (nb, c.steps, 1 << c.n)
    d_ch = torch.empty(shape, dtype=torch.uint8 if hard else torch.float32, device="cuda")
    plan.simulate_device(seed, first, nb, param, d_errors=d_err, d_info=d_info, d_out=d_out,
                         d_path_metric=d_pm if hard else None, d_channel=d_ch, hard_demap=hard_demap,
                         noise_f32=noise_f32)
    torch.cuda.synchronize()
    return (d_info.cpu().numpy(), d_ch.cpu().numpy(), d_out.cpu().numpy(), d_pm.cpu().numpy(),
            int(d_err.item()))


CHANNEL_CODES = [("k7", K7), ("k7_true", K7.with_(gen_mode=GEN_TRUE_PARITY)), ("code0", CODEBOOK[0]),
                 ("code5_r13", CODEBOOK[5]), ("k8", K8), ("k9", K9), ("k9_true", K9.with_(gen_mode=GEN_TRUE_PARITY)),
                 ("k9_blen255", K9.with_(blen=255)), ("k7_blen1", K7.with_(blen=1)),
                 # longer blocks (and the LDS-decision kernel's limit: code3 = K=6 at blen 80 fits
                 # its 20 KiB column, K=7 at blen 100 does not)
                 ("code3_blen80", CODEBOOK[3].with_(blen=80)), ("k7_blen100", K7.with_(blen=100))]


@pytest.mark.parametrize("name,c", CHANNEL_CODES, ids=[x[0] for x in CHANNEL_CODES])
def test_device_channel_bsc_bit_exact(torch_cuda, name, c):
    """BSC frames generated on the GPU: info, received symbols, decode, path metrics and error
    count are identical to the host Philox producer followed by the oracle decoder."""
    for nb, first, p_ppm in ((1, 0, 100000), (200, 12345, 60000)):
        info, syms, out, pm, err = _simulate(torch_cuda, Plan(c, HARD), c, 77, first, nb, p_ppm)
        h_info, h_syms = ch.bsc_blocks(c, nb, p_ppm, 77, first_block=first)
        assert np.array_equal(info, h_info)
        assert np.array_equal(syms, h_syms)
        ref, ref_pm = O.viterbi_hard(_ocode(c), syms)
        assert np.array_equal(out, ref) and np.array_equal(pm, ref_pm)
        assert err == ch.count_bit_errors(c, info, out)


# The device channel's double log / sqrt / sincos (channel_math.hpp) against glibc's: the host
# checker with the hardware approximations emulated measures 0 - 2.2e-8 of the fp32 samples differing
# (tools/chanmath_check.cpp, profiles/r04_chanmath_check.txt), i.e. ~0.001 expected at these test
# sizes. Allow 2, so a device-only precision loss (v_rsq_f64 / v_rcp_f64 less exact than emulated)
# fails here instead of hiding under a 0.1 % gate.
MAX_CHANNEL_DIFFS = 2


def _assert_samples_match(rx, h_rx, hard_demap=False):
    diff = np.any(rx != h_rx, axis=2) if hard_demap else (rx != h_rx)
    assert int(np.count_nonzero(diff)) <= MAX_CHANNEL_DIFFS, (int(np.count_nonzero(diff)), diff.size)
    if not hard_demap:
        assert np.allclose(rx, h_rx, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name,c", CHANNEL_CODES, ids=[x[0] for x in CHANNEL_CODES])
def test_device_channel_awgn(torch_cuda, name, c):
    """AWGN frames generated on the GPU: info bits identical to the host Philox producer; the
    demapped samples agree with the host's except where the device and glibc double log/sin/cos
    round differently (tolerance below); the decode of the device's own samples is bit-exact."""
    nb, first = 300, 999
    scaling = ch.noise_scaling(2.0)
    info, rx, out, _, err = _simulate(torch_cuda, Plan(c, SOFT), c, 5, first, nb, scaling)
    h_info, h_rx = ch.awgn_blocks(c, nb, scaling, 5, first_block=first)
    assert np.array_equal(info, h_info)
    _assert_samples_match(rx, h_rx)
    assert np.array_equal(out, O.viterbi_soft(_ocode(c), rx))
    assert err == ch.count_bit_errors(c, info, out)


@pytest.mark.parametrize("name,c", CHANNEL_CODES[:5], ids=[x[0] for x in CHANNEL_CODES[:5]])
def test_device_channel_awgn_hard_demapper(torch_cuda, name, c):
    """The reference's hard demapper (common/hard-demapper.c) on the device: decoder input equal to
    the host producer's (both snap to the nearest point; a sample may land on the other side of a
    decision boundary only where device and glibc libm round differently), decode bit-exact."""
    nb = 300
    scaling = ch.noise_scaling(3.0)
    info, rx, out, _, err = _simulate(torch_cuda, Plan(c, SOFT), c, 9, 4321, nb, scaling, hard_demap=True)
    h_info, h_rx = ch.awgn_blocks(c, nb, scaling, 9, first_block=4321, hard_demap=True)
    assert np.array_equal(info, h_info)
    _assert_samples_match(rx, h_rx, hard_demap=True)
    assert np.array_equal(out, O.viterbi_soft(_ocode(c), rx))
    assert err == ch.count_bit_errors(c, info, out)


# The opt-in fp32 Box-Muller (CCV_CHANNEL_NOISE_F32) draws the same uniforms as the double-precision
# path, so its samples track the default's to within the fp32 error of R * (cos, sin): at most
# F32_NOISE_ABS times the noise scaling over every (k1, k2) (tools/chanmath_f32_check.hip,
# profiles/r05_noise/chanmath_f32_check.txt), plus the fp32 roundings of the sample and the demapper.
F32_NOISE_ABS = 4e-6   # measured: 2.38e-6
F32_CODES = [("k7", K7), ("k9", K9), ("code0", CODEBOOK[0]), ("code5_r13", CODEBOOK[5]),
             ("k9_true", K9.with_(gen_mode=GEN_TRUE_PARITY))]


@pytest.mark.parametrize("hard_demap", [False, True], ids=["demap", "hard_demap"])
@pytest.mark.parametrize("name,c", F32_CODES, ids=[x[0] for x in F32_CODES])
def test_device_channel_awgn_f32_noise(torch_cuda, name, c, hard_demap):
    """CCV_CHANNEL_NOISE_F32: info bits identical to the double-precision channel's; soft decoder
    input within the fp32 error bound of it (hard-demapped input: equal except for samples within
    that bound of a decision boundary); the decode of the fp32 samples bit-exact against the oracle;
    error counts within a handful of the default's."""
    nb, first = 400, 31337
    scaling = ch.noise_scaling(2.0)
    f64 = _simulate(torch_cuda, Plan(c, SOFT), c, 13, first, nb, scaling, hard_demap=hard_demap)
    f32 = _simulate(torch_cuda, Plan(c, SOFT), c, 13, first, nb, scaling, hard_demap=hard_demap, noise_f32=True)
    assert np.array_equal(f32[0], f64[0])
    rx, rx64 = f32[1], f64[1]
    if hard_demap:
        diff = int(np.count_nonzero(np.any(rx != rx64, axis=2)))
        assert diff <= max(4, rx.shape[0] * rx.shape[1] // 10000), diff
    else:
        # demapper.c: squared distance / ndist; a sample error e moves it by <= 2 |x - a| e / ndist + e^2
        eps = 2 * F32_NOISE_ABS * scaling + 2 ** -22 * (1 + 8 * scaling)
        assert np.max(np.abs(rx - rx64)) <= 8 * eps * (1 + np.max(np.abs(rx64))), np.max(np.abs(rx - rx64))
    assert np.array_equal(f32[2], O.viterbi_soft(_ocode(c), rx))
    assert f32[4] == ch.count_bit_errors(c, f32[0], f32[2])
    assert abs(f32[4] - f64[4]) <= max(8, f64[4] // 100), (f32[4], f64[4])


def test_device_channel_f32_noise_frames_only_and_rejections(torch_cuda):
    """The fp32 noise in the frames-only producer (stack / Fano sweeps) tracks the default the same
    way; a BSC plan refuses the flag."""
    from ccviterbi import K15, StackPlan
    c, nb, s = K15, 200, ch.noise_scaling(3.0)
    plan = StackPlan(c, SOFT)
    rxs = []
    for f32 in (False, True):
        d_ch = torch_cuda.empty((nb, c.steps, 1 << c.n), dtype=torch_cuda.float32, device="cuda")
        plan.simulate_frames(5, 77, nb, s, d_ch, noise_f32=f32)
        torch_cuda.cuda.synchronize()
        rxs.append(d_ch.cpu().numpy())
    eps = 2 * F32_NOISE_ABS * s + 2 ** -22 * (1 + 8 * s)
    assert np.max(np.abs(rxs[1] - rxs[0])) <= 8 * eps * (1 + np.max(np.abs(rxs[0])))
    plan.close()
    d_ch = torch_cuda.empty((4, K7.steps), dtype=torch_cuda.uint8, device="cuda")
    with pytest.raises(Exception, match="AWGN"):
        Plan(K7, HARD).simulate_frames(1, 0, 4, 50000, d_ch, noise_f32=True)


def test_device_channel_ber_sweep_matches_host(torch_cuda):
    """The whole-sweep driver: device-generated BSC frames give the host path's exact counts."""
    for channel, points, c in ((HARD, [40000, 100000], K7), (SOFT, [3.0], CODEBOOK[0])):
        kw = dict(channel=channel, bits_per_point=lambda p: 3 * 500 * c.blen, frame_blocks=500, seed=11)
        dev = sim.ber_sweep(c, points, device_channel=True, **kw)
        host = sim.ber_sweep(c, points, **kw)
        for d, h in zip(dev, host):
            assert d.bits == h.bits
            if channel == HARD:
                assert d.errors == h.errors
            else:
                assert abs(d.errors - h.errors) <= max(2, h.errors // 1000)


@pytest.mark.parametrize("decoder,c,channel", [("viterbi", K7, SOFT), ("viterbi", K9, SOFT),
                                               ("stack", CODEBOOK[0], HARD)], ids=["k7", "k9", "stack"])
def test_device_channel_warm_up_changes_nothing(torch_cuda, decoder, c, channel):
    """The sweep CLI's warm-up (DeviceChannelDecoder.warm_up: throw-away chunks from block 2^62 on)
    leaves the counts of the points after it unchanged."""
    point = 3.0 if channel == SOFT else 60000
    fresh = sim.DeviceChannelDecoder(c, channel, 1000, 7, decoder=decoder, chunk_blocks=4000)
    want = fresh(point, 5 << 40, 9000)
    warm = sim.DeviceChannelDecoder(c, channel, 1000, 7, decoder=decoder, chunk_blocks=4000)
    assert warm.warm_up(0.01) >= 1
    assert warm(point, 5 << 40, 9000) == want


@pytest.mark.parametrize("noise_f32", [False, True], ids=["f64", "f32"])
@pytest.mark.parametrize("gen", [GEN_REF_X86, GEN_TRUE_PARITY], ids=["ref", "true"])
def test_device_channel_k9_frames_path_equals_fused(torch_cuda, gen, noise_f32):
    """K = 9 soft at blen 40: ccv_simulate_device writes the frames (channel_frames) and decodes them
    with the persistent kernel (x86 idiom: one lane per block; true parity: two lanes); the fused
    multilane channel kernel (option channel_fused=1) draws the same frames -- info, decoder input,
    output and error count are identical, with and without the hard demapper, for ragged batches,
    in both noise modes."""
    c = K9.with_(gen_mode=gen)
    for nb, hard_demap in ((1, False), (200, False), (3 * 64 + 5, True)):
        runs = []
        for fused in (0, 1):
            runs.append(_simulate(torch_cuda, Plan(c, SOFT).set_option("channel_fused", fused), c, 21,
                                  7000 + nb, nb, ch.noise_scaling(2.0), hard_demap=hard_demap,
                                  noise_f32=noise_f32))
        a, b = runs
        for k in (0, 1, 2):
            assert np.array_equal(a[k], b[k])
        assert a[4] == b[4]


def _frames_only_plans():
    from ccviterbi import K15, FanoPlan, StackPlan
    return [("viterbi_k7", Plan, K7), ("viterbi_code5_r13", Plan, CODEBOOK[5]),
            ("stack_k15", StackPlan, K15), ("stack_k15_true", StackPlan, K15.with_(gen_mode=GEN_TRUE_PARITY)),
            ("stack_wspr", StackPlan, CODEBOOK[4]), ("fano_k15", FanoPlan, K15),
            ("stack_k15_blen200", StackPlan, K15.with_(blen=200))]


@pytest.mark.parametrize("idx", range(7), ids=[p[0] for p in _frames_only_plans()])
@pytest.mark.parametrize("channel", [SOFT, HARD])
def test_device_channel_frames_only(torch_cuda, idx, channel):
    """CCV_CHANNEL_FRAMES_ONLY (the producer of the stack / Fano device sweeps, any K <= 32): info
    bytes and decoder input from the run-time-code encoder equal the host Philox producer's
    (BSC bit-exact; AWGN within the libm tolerance of test_device_channel_awgn), ragged counts,
    first_block offsets, and the hard demapper on AWGN."""
    name, cls, c = _frames_only_plans()[idx]
    plan = cls(c, channel)
    for nb, first, demap in ((1, 0, False), (333, 123456, False), (70, 99, channel == SOFT)):
        shape = (nb, c.steps) if channel == HARD else (nb, c.steps, 1 << c.n)
        d_ch = torch_cuda.empty(shape, dtype=torch_cuda.uint8 if channel == HARD else torch_cuda.float32,
                                device="cuda")
        d_info = torch_cuda.empty((nb, c.info_bytes), dtype=torch_cuda.uint8, device="cuda")
        if channel == HARD:
            plan.simulate_frames(41, first, nb, 80000, d_ch, d_info=d_info)
            h_info, h_rx = ch.bsc_blocks(c, nb, 80000, 41, first_block=first)
        else:
            s = ch.noise_scaling(2.5)
            plan.simulate_frames(41, first, nb, s, d_ch, d_info=d_info, hard_demap=demap)
            h_info, h_rx = ch.awgn_blocks(c, nb, s, 41, first_block=first, hard_demap=demap)
        torch_cuda.cuda.synchronize()
        info, rx = d_info.cpu().numpy(), d_ch.cpu().numpy()
        assert np.array_equal(info, h_info)
        if channel == HARD:
            assert np.array_equal(rx, h_rx)
        else:
            _assert_samples_match(rx, h_rx, hard_demap=demap)
    plan.close()


@pytest.mark.parametrize("channel,noise_f32", [(SOFT, False), (SOFT, True), (HARD, False)],
                         ids=["soft", "soft_f32", "hard"])
def test_device_channel_lds_vs_hbm_decisions(torch_cuda, channel, noise_f32):
    """The LDS-decision channel kernel (option channel_lds_decisions=1) and the HBM-scratch one (=0;
    -1, the default, picks by occupancy) decode the same device-generated frames identically
    (outputs, path metrics, error counts), in both noise modes."""
    param = 70000 if channel == HARD else ch.noise_scaling(1.0)
    for c in (K7, CODEBOOK[0], CODEBOOK[3].with_(blen=80), K7.with_(blen=1)):
        runs = []
        for forced in (1, 0):
            plan = Plan(c, channel).set_option("channel_lds_decisions", forced)
            runs.append(_simulate(torch_cuda, plan, c, 3, 5000, 777, param, noise_f32=noise_f32))
        a, b = runs
        for x, y in zip(a[:4], b[:4]):
            if channel == SOFT and x is a[3]:
                continue   # path metrics are hard-decision only
            assert np.array_equal(x, y)
        assert a[4] == b[4]


def test_plan_options_validate(torch_cuda):
    """ccv_plan_set_option: unknown names, out-of-range values and options of another decoder fail
    with a message; valid ones return the plan."""
    from ccviterbi import K15, FanoPlan, StackPlan
    plan = Plan(K7, SOFT)
    assert plan.set_option("channel_lds_decisions", -1) is plan
    for name, value, match in (("no_such_option", 1, "unknown option"), ("channel_fused", 2, "0 / 1"),
                               ("stack_keys", 0, "stack-decoder plan"), ("fano_rows", 3, "Fano-decoder plan")):
        with pytest.raises(Exception, match=match):
            plan.set_option(name, value)
    with pytest.raises(Exception, match="8 or 16"):
        StackPlan(K15, HARD).set_option("stack_row_lanes", 4)
    with pytest.raises(Exception, match="0..2"):
        FanoPlan(K15, SOFT).set_option("fano_rows", 3)


def test_device_channel_rejects_huge_noise(torch_cuda):
    plan = Plan(K7, SOFT)
    with pytest.raises(Exception, match="2\\^28"):
        plan.simulate_device(1, 0, 10, 3.0e8)


def test_device_channel_frames_only_rejects_step_major(torch_cuda):
    """Frames-only output is block-major: a step-major plan would decode it as scrambled input
    (ADVICE r04), so ccv_simulate_device refuses it."""
    plan = Plan(K7, SOFT, FLAG_STEP_MAJOR)
    d_ch = torch_cuda.empty((4, K7.steps, 4), dtype=torch_cuda.float32, device="cuda")
    with pytest.raises(Exception, match="step-major"):
        plan.simulate_frames(1, 0, 4, ch.noise_scaling(3.0), d_ch)


def test_device_channel_rejects_generic_codes(torch_cuda):
    plan = Plan(K9, SOFT, FLAG_GENERIC)
    with pytest.raises(Exception, match="register-trellis"):
        plan.simulate_device(1, 0, 10, 0.5)


@pytest.mark.parametrize("channel", [SOFT, HARD], ids=["soft", "hard"])
def test_group_queue_boundaries_one_plan(torch_cuda, channel):
    """The K = 7 persistent kernels take their groups from the per-XCD queue (acs_persist.hpp
    GroupQueue): every wave starts on one static group, then dequeues from eight heads over contiguous
    eighths of the rest and steals from the other heads when its own is empty. Batch sizes around the
    grid -- fewer groups than waves, exactly the grid, one group more, fewer extra groups than heads,
    two grids less one, each with and without a ragged last group -- decoded back to back by ONE plan
    (so every launch starts from the queue the previous one reset) equal the non-persistent kernel's
    outputs, path metrics and fused error counts block for block."""
    torch = torch_cuda
    c = K7
    plan = Plan(c, channel)
    ref_plan = Plan(c, channel, FLAG_NO_PERSISTENT)
    g = plan.persistent_waves()
    assert g > 0
    groups = [g // 2, g - 1, g, g + 1, g + 5, g + 8, 2 * g - 1, 2 * g + 9]
    sizes = [64 * n + r for n in groups for r in (0, 37)]
    nmax = max(sizes)
    if channel == SOFT:
        info, data = ch.awgn_blocks(c, nmax, ch.noise_scaling(2.5), 777)
    else:
        info, data = ch.bsc_blocks(c, nmax, 70000, 777)
    d_in, d_info = _device(torch, data), _device(torch, info)
    for nb in sizes:
        res = []
        for p in (plan, ref_plan):
            d_out = torch.full((nb, c.out_bytes), 0xA5, dtype=torch.uint8, device="cuda")
            d_pm = torch.full((nb,), -7, dtype=torch.int32, device="cuda")
            d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
            p.decode_device(d_in, nb, d_out, d_path_metric=d_pm if channel == HARD else None,
                            d_info=d_info, d_errors=d_err)
            torch.cuda.synchronize()
            res.append((d_out, d_pm, int(d_err.item())))
        (out, pm, err), (out2, pm2, err2) = res
        assert torch.equal(out, out2), (channel, nb)
        assert err == err2, (channel, nb)
        if channel == HARD:
            assert torch.equal(pm, pm2), (channel, nb)
    # the last (largest) batch against the oracle on a subsample
    idx = np.arange(0, nmax, 97)
    ref, ref_pm = _oracle(c, channel, data[idx])
    assert np.array_equal(out.cpu().numpy()[idx], ref)

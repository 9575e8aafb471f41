"""Host-side product logic on CPU: producers (libccv_sim), code tables, the BER driver's sharding
and counter reduction, and the C ABI surface. No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_ctypes as O
from ccviterbi import CODEBOOK, K7, K9, Code, channel as ch, code as code_mod, sim
from ccviterbi import _native
from conftest import REPO, golden_manifest

CASES = golden_manifest()


def _code_of(g, gen=code_mod.GEN_REF_X86):
    return Code(int(g["n"]), int(g["K"]), int(g["blen"]), tuple(int(p) for p in g["polys"]), gen)


def _ocode(c: Code):
    return O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_producers_reproduce_reference_inputs(case):
    """CCV_RNG_GLIBC reproduces the reference driver's decoder input bit for bit."""
    g = O.load_golden(case["name"])
    c = _code_of(g)
    nb = g["info"].shape[0]
    if case["channel"] == "awgn":
        info, rx = ch.awgn_blocks(c, nb, float(g["scaling"]), int(g["seed"]), rng=ch.RNG_GLIBC,
                                  hard_demap=case.get("demapper") == "hard")
        assert np.array_equal(rx.view(np.uint32), g["rx"].view(np.uint32))
    else:
        info, syms = ch.bsc_blocks(c, nb, int(g["p_ppm"]), int(g["seed"]), rng=ch.RNG_GLIBC)
        assert np.array_equal(syms, g["rx"])
    assert np.array_equal(info, g["info"])


ALL_CODES = [c for c in CODEBOOK if c.K <= 12] + [K7, K9]


@pytest.mark.parametrize("gen", [code_mod.GEN_REF_X86, code_mod.GEN_TRUE_PARITY])
@pytest.mark.parametrize("c", ALL_CODES, ids=[c.name for c in ALL_CODES])
def test_encoder_matches_oracle(c, gen):
    c = c.with_(gen_mode=gen)
    rng = np.random.default_rng(c.K * 10 + gen)
    info = rng.integers(0, 256, size=(64, c.info_bytes), dtype=np.uint8)
    syms = ch.encode(c, info)
    for b in range(info.shape[0]):
        assert np.array_equal(syms[b], O.encode_block(_ocode(c), info[b]))


@pytest.mark.parametrize("n", [1, 2, 3])
def test_demapper_matches_oracle(n):
    rng = np.random.default_rng(n)
    iq = rng.normal(size=(500, 2)).astype(np.float32)
    rx = ch.demap(n, iq)
    for k in range(iq.shape[0]):
        ref = np.zeros(1 << n, np.float32)
        O.lib().cco_demap(n, float(iq[k, 0]), float(iq[k, 1]), ref.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(rx[k].view(np.uint32), ref.view(np.uint32))


def test_philox_frames_independent_of_threads_and_sharding():
    a_info, a_rx = ch.awgn_blocks(K7, 1000, ch.noise_scaling(4.0), 99, threads=1)
    b_info, b_rx = ch.awgn_blocks(K7, 1000, ch.noise_scaling(4.0), 99, threads=7)
    assert np.array_equal(a_info, b_info) and np.array_equal(a_rx, b_rx)
    c_info, c_rx = ch.awgn_blocks(K7, 400, ch.noise_scaling(4.0), 99, first_block=600, threads=3)
    assert np.array_equal(c_info, a_info[600:]) and np.array_equal(c_rx, a_rx[600:])
    d_info, d_syms = ch.bsc_blocks(K7, 300, 50000, 5, threads=4)
    e_info, e_syms = ch.bsc_blocks(K7, 100, 50000, 5, first_block=200, threads=1)
    assert np.array_equal(e_syms, d_syms[200:]) and np.array_equal(e_info, d_info[200:])


def test_philox_channel_statistics():
    """Noise power and BSC flip rate of the fast source match the requested channel."""
    c = CODEBOOK[0]
    info, syms = ch.bsc_blocks(c, 20000, 100000, 3)
    clean = ch.encode(c, info)
    flips = np.unpackbits((syms ^ clean)[..., None], axis=-1)[..., -2:].mean()
    assert abs(flips - 0.1) < 0.003
    s = ch.noise_scaling(0.0)
    a_info, rx = ch.awgn_blocks(c, 5000, s, 4)
    # demapped distance to the transmitted point has mean 2*s^2/ndist for QPSK, ndist = 2
    clean_syms = ch.encode(c, a_info)
    d_tx = np.take_along_axis(rx, clean_syms[..., None].astype(np.int64), axis=-1)
    assert abs(d_tx.mean() - s * s) < 0.01


def test_noise_scaling_table():
    for db, s in zip(ch.REFERENCE_EBN0_DB, ch.REFERENCE_SCALING):
        assert ch.noise_scaling(db) == float(np.float32(s))
        assert abs(_native.sim().ccv_sim_noise_scaling(db) - s) < 1e-12


def test_codebook_matches_reference_fixtures():
    for case in CASES:
        if not case["spec"].startswith("cb:"):
            continue
        g = O.load_golden(case["name"])
        c = CODEBOOK[int(case["spec"][3:])]
        assert (c.n, c.K, c.blen) == (int(g["n"]), int(g["K"]), int(g["blen"]))
        assert tuple(c.polys) == tuple(int(p) for p in g["polys"])


def test_code_param_abi_layout():
    """struct code_param offsets on x86-64 (common/include/code.h:9-19)."""
    P = code_mod.CodeParam
    assert (P.symlen_out.offset, P.constr_len.offset, P.block_len.offset) == (0, 1, 2)
    assert P.polynomials.offset == 8 and P.bit_metrics.offset == 16
    assert P.fano_bit_metrics.offset == 24 and P.metric_weight.offset == 32
    assert P.fano_metric_weight.offset == 36 and P.userdata.offset == 40
    assert ctypes.sizeof(P) == 48


def _header_functions(path):
    text = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    text = re.sub(r"^\s*typedef[^;]*;", "", text, flags=re.M)
    return set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\**\s*\b(\w+)\s*\([^;{]*\)\s*;", text, flags=re.M))


@pytest.mark.parametrize("header,lib", [("ccv.h", "libccv_core.so"), ("decoder_awgn.h", "libccv_awgn.so"),
                                        ("decoder_bsc.h", "libccv_bsc.so"), ("ccv_sim.h", "libccv_sim.so")])
def test_library_exports_every_header_symbol(header, lib):
    names = _header_functions(os.path.join(REPO, "include", header))
    assert len(names) >= 5
    so = ctypes.CDLL(os.path.join(_native.LIB_DIR, lib), mode=ctypes.RTLD_LOCAL)
    missing = [n for n in sorted(names) if not hasattr(so, n)]
    assert not missing, f"{lib} lacks {missing}"


def test_reference_symbols_in_shims():
    """The six reference entry points (AWGN-channel/include/decoder.h:17-26) exist in both shims."""
    for lib in ("libccv_awgn.so", "libccv_bsc.so"):
        so = ctypes.CDLL(os.path.join(_native.LIB_DIR, lib), mode=ctypes.RTLD_LOCAL)
        for n in ("decoder_create", "decoder_destroy", "decoder_init", "decoder_register_callback",
                  "decoder_reset", "decoder_input"):
            assert hasattr(so, n)


def test_decoder_create_destroy_without_gpu_compute():
    L = _native.awgn()
    obj = ctypes.c_void_p(L.decoder_create())
    assert obj
    L.decoder_destroy(ctypes.byref(obj))
    assert not obj
    L.decoder_destroy(ctypes.byref(obj))   # destroying a NULL handle is a no-op


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, "LIB_DIR", str(tmp_path))
    monkeypatch.setattr(_native, "_cache", {})
    with pytest.raises(_native.NativeLibraryError):
        _native.core()


# ------------------------------------------------------------------------- BER driver (oracle-fed)

def _oracle_decoder(c: Code, soft: bool):
    oc = _ocode(c)

    def decode(info, data):
        out = O.viterbi_soft(oc, data) if soft else O.viterbi_hard(oc, data)[0]
        return O.count_errors(oc, info, out)
    return decode


def test_ber_sweep_sharding_is_world_size_invariant():
    c = CODEBOOK[0]
    bits = lambda p: 3 * 500 * c.blen   # noqa: E731  three frames of 500 blocks
    dec = _oracle_decoder(c, True)
    full = sim.ber_sweep(c, [2.0, 4.0], bits_per_point=bits, frame_blocks=500, decode=dec, seed=11)
    parts = [sim.ber_sweep(c, [2.0, 4.0], bits_per_point=bits, frame_blocks=500, decode=dec, seed=11,
                           rank=r, world=2, reduce=False) for r in range(2)]
    for i, p in enumerate(full):
        assert p.errors == parts[0][i].errors + parts[1][i].errors
        assert p.bits == parts[0][i].bits + parts[1][i].bits == 3 * 500 * c.blen
    assert full[0].ber > full[1].ber > 0


def test_reference_bit_schedule():
    assert sim.reference_awgn_bits(0.0, 40) == 800000
    assert sim.reference_awgn_bits(6.0, 40) == 8000000
    assert sim.reference_awgn_bits(8.0, 40) == 80000000
    assert sim.reference_awgn_bits(12.0, 40) == 800000000
    assert sim.reference_bsc_bits(1, 40) == 800000000
    assert sim.reference_bsc_bits(400000, 40) == 800000

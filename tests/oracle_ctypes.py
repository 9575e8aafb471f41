"""ctypes view of oracle/build/libccoracle.so -- the CPU restatement used as the parity CHECKER.

Test infrastructure only (imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg). Nothing in convolutional-codes_amd/ imports this module.
"""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
GEN_REF_X86, GEN_TRUE_PARITY = 0, 1


class CcoCode(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("K", ctypes.c_int), ("blen", ctypes.c_int),
                ("poly", ctypes.c_uint64 * 8), ("gen_mode", ctypes.c_int)]


class CcoRng(ctypes.Structure):
    _fields_ = [("s", ctypes.c_uint32 * 31), ("f", ctypes.c_int), ("r", ctypes.c_int),
                ("R", ctypes.c_double), ("T", ctypes.c_double), ("phase", ctypes.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "build", "libccoracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", ORACLE_DIR, "oracle"], check=True, capture_output=True)
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        L.cco_srand.argtypes = [P(CcoRng), ctypes.c_uint32]
        L.cco_rand.argtypes = [P(CcoRng)]
        L.cco_rand.restype = ctypes.c_int32
        L.cco_gengauss.argtypes = [P(CcoRng)]
        L.cco_gengauss.restype = ctypes.c_double
        L.cco_gen_bit.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.cco_gen_bit.restype = ctypes.c_int
        L.cco_trellis.argtypes = [P(CcoCode), ctypes.c_void_p]
        L.cco_encode_block.argtypes = [P(CcoCode), ctypes.c_void_p, ctypes.c_void_p]
        L.cco_demap.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        L.cco_awgn_blocks.argtypes = [P(CcoCode), ctypes.c_uint32, ctypes.c_float, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.cco_awgn_blocks_demap.argtypes = [P(CcoCode), ctypes.c_uint32, ctypes.c_float, ctypes.c_size_t,
                                            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.cco_bsc_blocks.argtypes = [P(CcoCode), ctypes.c_uint32, ctypes.c_int32, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.cco_viterbi_soft.argtypes = [P(CcoCode), ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.cco_viterbi_hard.argtypes = [P(CcoCode), ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_void_p]
        L.cco_stack_soft.argtypes = [P(CcoCode), ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p]
        L.cco_stack_hard.argtypes = [P(CcoCode), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.cco_fano_soft.argtypes = [P(CcoCode), ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p]
        L.cco_fano_hard.argtypes = [P(CcoCode), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.cco_count_errors.argtypes = [P(CcoCode), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.cco_count_errors.restype = ctypes.c_uint64
        _lib = L
    return _lib


def code(n, K, blen, polys, gen_mode=GEN_REF_X86):
    c = CcoCode()
    c.n, c.K, c.blen, c.gen_mode = int(n), int(K), int(blen), int(gen_mode)
    for k, p in enumerate(polys):
        c.poly[k] = int(p)
    return c


def dims(c):
    T = c.blen + c.K - 1
    return T, (c.blen + 7) // 8, (T + 7) // 8


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def trellis(c):
    out = np.zeros((1 << (c.K - 1), 2), dtype=np.uint8)
    lib().cco_trellis(ctypes.byref(c), _ptr(out))
    return out


def awgn_blocks(c, seed, scaling, nblocks, hard_demap=False):
    T, IB, _ = dims(c)
    info = np.zeros((nblocks, IB), np.uint8)
    rx = np.zeros((nblocks, T, 1 << c.n), np.float32)
    lib().cco_awgn_blocks_demap(ctypes.byref(c), seed, scaling, nblocks, 1 if hard_demap else 0,
                                _ptr(info), _ptr(rx))
    return info, rx


def bsc_blocks(c, seed, p_ppm, nblocks):
    T, IB, _ = dims(c)
    info = np.zeros((nblocks, IB), np.uint8)
    syms = np.zeros((nblocks, T), np.uint8)
    lib().cco_bsc_blocks(ctypes.byref(c), seed, p_ppm, nblocks, _ptr(info), _ptr(syms))
    return info, syms


def viterbi_soft(c, rx):
    rx = np.ascontiguousarray(rx, dtype=np.float32)
    _, _, OB = dims(c)
    out = np.zeros((rx.shape[0], OB), np.uint8)
    lib().cco_viterbi_soft(ctypes.byref(c), _ptr(rx), rx.shape[0], _ptr(out))
    return out


def viterbi_hard(c, syms):
    syms = np.ascontiguousarray(syms, dtype=np.uint8)
    _, _, OB = dims(c)
    out = np.zeros((syms.shape[0], OB), np.uint8)
    pm = np.zeros(syms.shape[0], np.int32)
    lib().cco_viterbi_hard(ctypes.byref(c), _ptr(syms), syms.shape[0], _ptr(out), _ptr(pm))
    return out, pm


def stack_soft(c, metric_weight, rx):
    """Stack decoder restatement (AWGN-channel/stack-decoder.c)."""
    rx = np.ascontiguousarray(rx, dtype=np.float32)
    _, _, OB = dims(c)
    out = np.zeros((rx.shape[0], OB), np.uint8)
    if lib().cco_stack_soft(ctypes.byref(c), float(metric_weight), _ptr(rx), rx.shape[0], _ptr(out)):
        raise RuntimeError("the reference would read past its buffers on some block")
    return out


def stack_hard(c, bit_metrics, syms):
    """Stack decoder restatement (binary-symmetric-channel/stack-decoder.c); (out, path metric)."""
    syms = np.ascontiguousarray(syms, dtype=np.uint8)
    bm = np.ascontiguousarray(bit_metrics, dtype=np.int32)
    _, _, OB = dims(c)
    out = np.zeros((syms.shape[0], OB), np.uint8)
    pm = np.zeros(syms.shape[0], np.int32)
    if lib().cco_stack_hard(ctypes.byref(c), _ptr(bm), _ptr(syms), syms.shape[0], _ptr(out), _ptr(pm)):
        raise RuntimeError("the reference would read past its buffers on some block")
    return out, pm


def fano_soft(c, fano_metric_weight, rx):
    """Fano decoder restatement (AWGN-channel/fano-decoder.c)."""
    rx = np.ascontiguousarray(rx, dtype=np.float32)
    _, _, OB = dims(c)
    out = np.zeros((rx.shape[0], OB), np.uint8)
    lib().cco_fano_soft(ctypes.byref(c), float(fano_metric_weight), _ptr(rx), rx.shape[0], _ptr(out))
    return out


def fano_hard(c, fano_bit_metrics, syms):
    """Fano decoder restatement (binary-symmetric-channel/fano-decoder.c); (out, path metric)."""
    syms = np.ascontiguousarray(syms, dtype=np.uint8)
    bm = np.ascontiguousarray(fano_bit_metrics, dtype=np.int32)
    _, _, OB = dims(c)
    out = np.zeros((syms.shape[0], OB), np.uint8)
    pm = np.zeros(syms.shape[0], np.int32)
    lib().cco_fano_hard(ctypes.byref(c), _ptr(bm), _ptr(syms), syms.shape[0], _ptr(out), _ptr(pm))
    return out, pm


_fast = None


def fast_viterbi(c, data, hard=False, threads=1):
    """oracle/ccfast.c: the optimised (table-driven, AVX2, pthreads) CPU Viterbi of bench.py's second
    CPU baseline. Returns (seconds, out[, path metrics])."""
    global _fast
    if _fast is None:
        path = os.path.join(ORACLE_DIR, "build", "libccfast.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", ORACLE_DIR, "oracle"], check=True, capture_output=True)
        L = ctypes.CDLL(path)
        L.ccfast_viterbi.argtypes = [ctypes.POINTER(CcoCode), ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.ccfast_viterbi.restype = ctypes.c_double
        _fast = L
    data = np.ascontiguousarray(data, dtype=np.uint8 if hard else np.float32)
    nb = data.shape[0]
    _, _, OB = dims(c)
    out = np.zeros((nb, OB), np.uint8)
    pm = np.zeros(nb, np.int32)
    t = _fast.ccfast_viterbi(ctypes.byref(c), 1 if hard else 0, _ptr(data), nb, _ptr(out), _ptr(pm), threads)
    if t < 0:
        raise ValueError("ccfast_viterbi: unsupported code")
    return (t, out, pm) if hard else (t, out)


def count_errors(c, info, out):
    info = np.ascontiguousarray(info, np.uint8)
    out = np.ascontiguousarray(out, np.uint8)
    return int(lib().cco_count_errors(ctypes.byref(c), _ptr(info), _ptr(out), info.shape[0]))


def encode_block(c, info_bytes):
    T, _, _ = dims(c)
    info_bytes = np.ascontiguousarray(info_bytes, np.uint8)
    syms = np.zeros(T, np.uint8)
    lib().cco_encode_block(ctypes.byref(c), _ptr(info_bytes), _ptr(syms))
    return syms


def load_golden(name):
    path = os.path.join(REPO, "tests", "golden", name + ".npz")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_code(g, gen_mode=GEN_REF_X86):
    return code(int(g["n"]), int(g["K"]), int(g["blen"]), [int(p) for p in g["polys"]], gen_mode)

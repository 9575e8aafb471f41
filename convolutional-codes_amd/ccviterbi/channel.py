"""CPU producers of the decoder input (libccv_sim.so, include/ccv_sim.h): the reference's
encoder -> mapper -> channel -> demapper chain, batched over independent blocks."""
import os

import numpy as np

from . import _native
from .code import Code

RNG_GLIBC = 0    # reproduces the reference drivers' rand() stream from srand(seed), sequential
RNG_PHILOX = 1   # counter-based per block: any thread count / sharding gives the same frames

# AWGN-channel/main.c:150-161 (Eb/N0 points of the reference sweep and their float scalings)
REFERENCE_EBN0_DB = (0.0, 2.0, 4.0, 6.0, 8.0, 10.0, 12.0, 14.0)
REFERENCE_SCALING = (0.707106781186548, 0.561674881261479, 0.446154216921401, 0.354392891541971,
                     0.281504279937367, 0.223606797749979, 0.177617192929090, 0.141086351316046)
# binary-symmetric-channel/main.c:103-109 (crossover probabilities in ppm)
REFERENCE_P_PPM = (1, 5, 25, 125, 625, 3125, 6250, 12500, 15625, 25000, 50000, 78125, 100000,
                   200000, 300000, 390625, 400000)


def default_threads():
    return max(1, min(16, os.cpu_count() or 1))


def noise_scaling(ebn0_db: float) -> float:
    """1/sqrt(2) * 10^(-Eb/N0 / 20), computed like the reference's table (float)."""
    for db, s in zip(REFERENCE_EBN0_DB, REFERENCE_SCALING):
        if abs(db - ebn0_db) < 1e-12:
            return float(np.float32(s))
    return float(np.float32(_native.sim().ccv_sim_noise_scaling(float(ebn0_db))))


def encode(code: Code, info: np.ndarray) -> np.ndarray:
    info = np.ascontiguousarray(info, np.uint8).reshape(-1, code.info_bytes)
    syms = np.zeros((info.shape[0], code.steps), np.uint8)
    polys = code.poly_array()
    if _native.sim().ccv_sim_encode(code.n, code.K, code.blen, polys, code.gen_mode, info.ctypes.data,
                                    info.shape[0], syms.ctypes.data) != 0:
        raise ValueError("ccv_sim_encode failed")
    return syms


def demap(n: int, iq: np.ndarray) -> np.ndarray:
    iq = np.ascontiguousarray(iq, np.float32).reshape(-1, 2)
    rx = np.zeros((iq.shape[0], 1 << n), np.float32)
    if _native.sim().ccv_sim_demap(n, iq.ctypes.data, iq.shape[0], rx.ctypes.data) != 0:
        raise ValueError("ccv_sim_demap failed")
    return rx


DEMAP_HARD = 0x100   # CCV_DEMAP_HARD: common/hard-demapper.c instead of common/demapper.c


def awgn_blocks(code: Code, nblocks: int, scaling: float, seed: int, rng: int = RNG_PHILOX,
                first_block: int = 0, threads: int = None, info=None, rx=None, hard_demap=False):
    """(info uint8 [nb, IB], rx float32 [nb, T, 2^n]); `info`/`rx` may be preallocated views."""
    if hard_demap:
        rng |= DEMAP_HARD
    if info is None:
        info = np.empty((nblocks, code.info_bytes), np.uint8)
    if rx is None:
        rx = np.empty((nblocks, code.steps, 1 << code.n), np.float32)
    polys = code.poly_array()
    if _native.sim().ccv_sim_awgn(code.n, code.K, code.blen, polys, code.gen_mode, rng, seed,
                                  scaling, first_block, nblocks, info.ctypes.data, rx.ctypes.data,
                                  threads or default_threads()) != 0:
        raise ValueError("ccv_sim_awgn failed")
    return info, rx


def bsc_blocks(code: Code, nblocks: int, p_ppm: int, seed: int, rng: int = RNG_PHILOX,
               first_block: int = 0, threads: int = None, info=None, syms=None):
    """(info uint8 [nb, IB], syms uint8 [nb, T])."""
    if info is None:
        info = np.empty((nblocks, code.info_bytes), np.uint8)
    if syms is None:
        syms = np.empty((nblocks, code.steps), np.uint8)
    polys = code.poly_array()
    if _native.sim().ccv_sim_bsc(code.n, code.K, code.blen, polys, code.gen_mode, rng, seed,
                                 int(p_ppm), first_block, nblocks, info.ctypes.data, syms.ctypes.data,
                                 threads or default_threads()) != 0:
        raise ValueError("ccv_sim_bsc failed")
    return info, syms


def count_bit_errors(code: Code, info: np.ndarray, out: np.ndarray) -> int:
    """Host consumer (AWGN-channel/main.c:129-141): errors over the first blen bits per block."""
    a = np.unpackbits(np.ascontiguousarray(info, np.uint8).reshape(-1, code.info_bytes), axis=1)
    d = np.unpackbits(np.ascontiguousarray(out, np.uint8).reshape(-1, code.out_bytes), axis=1)
    return int(np.count_nonzero(a[:, :code.blen] != d[:, :code.blen]))

"""ccviterbi -- MI355X-native Viterbi decoder for the thomas-emig/convolutional-codes BER simulator.

The hot path (branch metric + add-compare-select + traceback) runs as hand-written HIP kernels for
gfx950 in libccv_core.so; libccv_awgn.so / libccv_bsc.so export the reference's decoder_* C ABI;
libccv_sim.so holds the CPU-side producers. This package is the Python host mirror.
"""
from .code import (CODEBOOK, GEN_REF_X86, GEN_TRUE_PARITY, HARD, K7, K8, K9, K15, SOFT, STANDARD, Code,
                   CodeParam, get_code, named_code)
from .decoder import DecoderError, FanoPlan, HardDecoder, Plan, SoftDecoder, StackPlan, device_count
from ._native import NativeLibraryError

__all__ = [
    "CODEBOOK", "GEN_REF_X86", "GEN_TRUE_PARITY", "HARD", "K7", "K8", "K9", "K15", "SOFT", "STANDARD",
    "Code", "CodeParam", "get_code", "named_code", "DecoderError", "HardDecoder", "Plan",
    "SoftDecoder", "StackPlan", "FanoPlan", "device_count", "NativeLibraryError",
]

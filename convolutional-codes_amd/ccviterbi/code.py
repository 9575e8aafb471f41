"""Code parameters: the reference's struct code_param (common/include/code.h:9-19) and codebook
(common/codebook.c:14-120), plus the benchmark codes BASELINE.json names but the codebook lacks."""
import ctypes
from dataclasses import dataclass, field
from typing import Sequence, Tuple

GEN_REF_X86 = 0       # generator bit as the reference computes it on x86 (default, bit-exact parity)
GEN_TRUE_PARITY = 1   # textbook parity

SOFT, HARD = 0, 1


class CodeParam(ctypes.Structure):
    """ABI mirror of struct code_param (include/code.h)."""
    _fields_ = [("symlen_out", ctypes.c_uint8), ("constr_len", ctypes.c_uint8),
                ("block_len", ctypes.c_uint8), ("polynomials", ctypes.POINTER(ctypes.c_uint64)),
                ("bit_metrics", ctypes.POINTER(ctypes.c_int32)),
                ("fano_bit_metrics", ctypes.POINTER(ctypes.c_int32)),
                ("metric_weight", ctypes.c_float), ("fano_metric_weight", ctypes.c_float),
                ("userdata", ctypes.c_void_p)]


@dataclass(frozen=True)
class Code:
    n: int                       # symlen_out
    K: int                       # constr_len
    blen: int                    # block_len
    polys: Tuple[int, ...]       # MSB-aligned generators
    gen_mode: int = GEN_REF_X86
    bit_metrics: Tuple[int, int] = (1, -15)
    fano_bit_metrics: Tuple[int, int] = (1, -20)
    metric_weight: float = -15.0
    fano_metric_weight: float = -200.0
    name: str = field(default="", compare=False)

    @property
    def steps(self):       # T
        return self.blen + self.K - 1

    @property
    def states(self):      # S
        return 1 << (self.K - 1)

    @property
    def info_bytes(self):  # IB
        return (self.blen + 7) // 8

    @property
    def out_bytes(self):   # OB
        return (self.steps + 7) // 8

    def with_(self, **kw):
        d = dict(self.__dict__)
        d.update(kw)
        return Code(**d)

    def poly_array(self):
        return (ctypes.c_uint64 * len(self.polys))(*self.polys)

    def to_param(self):
        """(CodeParam, keep-alive tuple). The decoder borrows the polynomial array, as the
        reference does (AWGN-channel/viterbi-decoder.c:169), so keep the second item alive."""
        polys = self.poly_array()
        bm = (ctypes.c_int32 * 2)(*self.bit_metrics)
        fbm = (ctypes.c_int32 * 2)(*self.fano_bit_metrics)
        p = CodeParam(self.n, self.K, self.blen, polys, bm, fbm, self.metric_weight,
                      self.fano_metric_weight, None)
        return p, (polys, bm, fbm)


def _octal_to_msb(octal: int, K: int) -> int:
    """Generator given in octal with the current-input tap as its most significant bit."""
    return int(octal) << (64 - K)


# common/codebook.c:14-79, indexed like get_code() (codebook.c:110-120)
CODEBOOK: Sequence[Code] = (
    Code(2, 3, 40, (0xA000000000000000, 0x6000000000000000), GEN_REF_X86, (1, -15), (1, -20), -15.0, -200.0, "code0"),
    Code(2, 4, 40, (0xB000000000000000, 0xE000000000000000), GEN_REF_X86, (1, -25), (1, -45), -15.0, -150.0, "code1"),
    Code(2, 5, 40, (0xA800000000000000, 0xF000000000000000), GEN_REF_X86, (1, -30), (1, -48), -20.0, -130.0, "code2"),
    Code(2, 6, 40, (0xB400000000000000, 0xE800000000000000), GEN_REF_X86, (1, -39), (1, -55), -16.0, -110.0, "code3"),
    Code(2, 32, 50, (0x8ACA0B4F00000000, 0xE23C862700000000), GEN_REF_X86, (1, -27), (1, -38), -7.0, -11.0, "wspr"),
    Code(3, 3, 40, (0xA000000000000000, 0xC000000000000000, 0x2000000000000000), GEN_REF_X86, (1, -9), (1, -30), -7.0, -70.0, "code5"),
)


def get_code(index: int) -> Code:
    """common/codebook.c:110-120"""
    return CODEBOOK[index]


# Codes named by BASELINE.json that the codebook lacks.
K7 = Code(2, 7, 40, (_octal_to_msb(0o171, 7), _octal_to_msb(0o133, 7)), name="k7_171_133")
K9 = Code(2, 9, 40, (_octal_to_msb(0o561, 9), _octal_to_msb(0o753, 9)), name="k9_561_753")
K8 = Code(2, 8, 40, (_octal_to_msb(0o371, 8), _octal_to_msb(0o247, 8)), name="k8_371_247")

# BASELINE config 5: K=15 r=1/2 (46321,51271)_8 for the stack decoder; the codebook has no K=15 code,
# so its stack metrics borrow the codebook's long-code (WSPR K=32) weight (codebook.c:71-73).
K15 = Code(2, 15, 40, (_octal_to_msb(0o46321, 15), _octal_to_msb(0o51271, 15)), metric_weight=-7.0,
           bit_metrics=(1, -11), fano_metric_weight=-11.0, fano_bit_metrics=(1, -11),
           name="k15_46321_51271")
STANDARD = {"k7": K7, "k8": K8, "k9": K9, "k15": K15}


def named_code(name: str) -> Code:
    """'k7', 'k9', 'code0'..'code5' / 'cb0'..'cb5', optionally suffixed ':true' for true parity."""
    base, _, mode = name.partition(":")
    if base in STANDARD:
        c = STANDARD[base]
    elif base.startswith("cb") or base.startswith("code"):
        c = get_code(int(base.lstrip("cbode")))
    else:
        raise KeyError(name)
    if mode in ("true", "true_parity"):
        c = c.with_(gen_mode=GEN_TRUE_PARITY)
    return c

"""Host-side mirror of the reference decoder interface over the MI355X libraries.

* `SoftDecoder` / `HardDecoder` wrap libccv_awgn.so / libccv_bsc.so, whose C ABI is the reference's
  decoder_* API (AWGN-channel/include/decoder.h:9-26, binary-symmetric-channel/include/decoder.h:9-26):
  create, init, register_callback, reset, input (streaming, callback per block), destroy, plus the
  batch extension (input_blocks, decode_blocks, decode_device).
* `Plan` wraps libccv_core.so's ccv_* API directly: the device-resident batched decode with the fused
  bit-error count that the BER driver and bench.py use.
Every call goes to the HIP kernels; a missing library or a failing call raises.
"""
import ctypes

import numpy as np

from . import _native
from .code import GEN_REF_X86, HARD, SOFT, Code

KERNEL_REGISTER, KERNEL_GENERIC, KERNEL_MULTILANE, KERNEL_STACK, KERNEL_FANO = 1, 2, 3, 4, 5
FLAG_GENERIC = 1
FLAG_STEP_MAJOR = 2
FLAG_GLOBAL_DECISIONS = 4   # survivor decisions through an HBM scratch array (A/B vs register-resident)
FLAG_NO_PERSISTENT = 8      # skip the persistent K <= 7 kernels (A/B)


CHANNEL_HARD_DEMAP = 1     # include/ccv.h CCV_CHANNEL_HARD_DEMAP
CHANNEL_FRAMES_ONLY = 2    # include/ccv.h CCV_CHANNEL_FRAMES_ONLY
CHANNEL_NOISE_F32 = 4      # include/ccv.h CCV_CHANNEL_NOISE_F32 (opt-in fp32 Box-Muller)
CHANNEL_IQ = 8             # include/ccv.h CCV_CHANNEL_IQ (frames only: received points, not distances)


class DecoderError(RuntimeError):
    pass


def _ptr(x):
    """Address of a numpy array, a torch tensor, or an int (already a device pointer)."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    raise TypeError(f"cannot take the address of {type(x)}")


def _stream_handle(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream   # torch.cuda.Stream


def device_count() -> int:
    return _native.core().ccv_device_count()


class Plan:
    """A code bound to the current HIP device (ccv_plan_create, include/ccv.h)."""

    def __init__(self, code: Code, channel: int = SOFT, flags: int = 0):
        self.code = code
        self.channel = channel
        self._lib = _native.core()
        self._polys = code.poly_array()
        h = ctypes.c_void_p()
        if self._lib.ccv_plan_create(ctypes.byref(h), channel, code.n, code.K, code.blen,
                                     self._polys, code.gen_mode, flags) != 0:
            raise DecoderError(f"ccv_plan_create: {_native.last_error()}")
        self._h = h
        self.desc = _native.CcvPlanDesc()
        self._lib.ccv_plan_describe(self._h, ctypes.byref(self.desc))

    @property
    def kernel(self):
        return {KERNEL_REGISTER: "register", KERNEL_GENERIC: "generic",
                KERNEL_MULTILANE: "multilane", KERNEL_STACK: "stack",
                KERNEL_FANO: "fano"}[self.desc.kernel]

    @property
    def decisions(self):
        """Where survivor decisions live during a decode: "none", "hbm", "registers", "lds" or "slot"
        (a per-wave scratch slot, include/ccv.h CCV_DECISIONS_SLOT)."""
        return {0: "none", 1: "hbm", 2: "registers", 3: "lds", 4: "slot"}[self._lib.ccv_plan_decision_storage(self._h)]

    @property
    def variant(self):
        """The kernel a decode without decision export runs (ccv_plan_kernel_variant)."""
        return self._lib.ccv_plan_kernel_variant(self._h).decode()

    def persistent_waves(self, fresh: bool = False) -> int:
        """Grid of the plan's persistent kernel (0 = none); fresh bypasses the per-kernel cache."""
        w = self._lib.ccv_plan_persistent_waves(self._h, 1 if fresh else 0)
        if w < 0:
            raise DecoderError(f"ccv_plan_persistent_waves: {_native.last_error()}")
        return w

    def trellis(self) -> np.ndarray:
        out = np.zeros((self.desc.states, 2), np.uint8)
        self._lib.ccv_plan_trellis(self._h, out.ctypes.data)
        return out

    def set_option(self, name: str, value: int):
        """ccv_plan_set_option: a per-plan kernel A/B switch (include/ccv.h lists them); returns self."""
        if self._lib.ccv_plan_set_option(self._h, name.encode(), int(value)) != 0:
            raise DecoderError(f"ccv_plan_set_option: {_native.last_error()}")
        return self

    def reserve(self, max_blocks: int):
        if self._lib.ccv_plan_reserve(self._h, max_blocks) != 0:
            raise DecoderError(f"ccv_plan_reserve: {_native.last_error()}")

    def decode_device(self, d_in, nblocks, d_out, d_path_metric=None, d_info=None, d_errors=None,
                      d_decisions=None, stream=None):
        """Asynchronous decode of device-resident blocks (torch tensors or raw device pointers)."""
        rc = self._lib.ccv_decode_device(self._h, _ptr(d_in), int(nblocks), _ptr(d_out),
                                         _ptr(d_path_metric), _ptr(d_info), _ptr(d_errors),
                                         _ptr(d_decisions), _stream_handle(stream))
        if rc != 0:
            raise DecoderError(f"ccv_decode_device: {_native.last_error()}")

    def simulate_device(self, seed, first_block, nblocks, channel_param, d_errors=None, d_info=None,
                        d_out=None, d_path_metric=None, d_channel=None, stream=None, hard_demap=False,
                        noise_f32=False):
        """On-device channel + decode (ccv_simulate_device): blocks first_block.. of the Philox stream
        `seed`; channel_param = AWGN noise scaling (soft plan) or BSC p_ppm (hard plan); hard_demap
        selects the reference's hard demapper (common/hard-demapper.c); noise_f32 the opt-in fp32
        Box-Muller (statistically, not bit-, equal to the double-precision default)."""
        flags = (CHANNEL_HARD_DEMAP if hard_demap else 0) | (CHANNEL_NOISE_F32 if noise_f32 else 0)
        rc = self._lib.ccv_simulate_device(self._h, int(seed), int(first_block), int(nblocks),
                                           float(channel_param), flags,
                                           _ptr(d_info), _ptr(d_out),
                                           _ptr(d_path_metric), _ptr(d_errors), _ptr(d_channel),
                                           _stream_handle(stream))
        if rc != 0:
            raise DecoderError(f"ccv_simulate_device: {_native.last_error()}")

    def simulate_frames(self, seed, first_block, nblocks, channel_param, d_channel, d_info=None,
                        stream=None, hard_demap=False, noise_f32=False, iq=False):
        """The on-device channel's frames only (ccv_simulate_device with CCV_CHANNEL_FRAMES_ONLY):
        info bytes into d_info and the decoder input into d_channel, no decode; any plan (Viterbi,
        stack, Fano), any code with n <= 3. iq: the received points (float [nb][T][2]) instead of
        the demapper's distances (CCV_CHANNEL_IQ; a Fano plan decodes them with fano_input 1)."""
        flags = (CHANNEL_FRAMES_ONLY | (CHANNEL_HARD_DEMAP if hard_demap else 0) |
                 (CHANNEL_NOISE_F32 if noise_f32 else 0) | (CHANNEL_IQ if iq else 0))
        rc = self._lib.ccv_simulate_device(self._h, int(seed), int(first_block), int(nblocks),
                                           float(channel_param), flags, _ptr(d_info), None, None, None,
                                           _ptr(d_channel), _stream_handle(stream))
        if rc != 0:
            raise DecoderError(f"ccv_simulate_device: {_native.last_error()}")

    def decode_host(self, data: np.ndarray):
        """Synchronous decode of host blocks; returns out [nb, OB] (and path metrics for HARD)."""
        dt = np.float32 if self.channel == SOFT else np.uint8
        data = np.ascontiguousarray(data, dtype=dt)
        per_block = self.desc.steps * (self.desc.in_step_bytes // data.itemsize)
        nb = data.size // per_block
        if nb * per_block != data.size:
            raise ValueError("input is not a whole number of blocks")
        out = np.zeros((nb, self.desc.out_bytes), np.uint8)
        pm = np.zeros(nb, np.int32) if self.channel == HARD else None
        if self._lib.ccv_decode_host(self._h, data.ctypes.data, nb, out.ctypes.data,
                                     None if pm is None else pm.ctypes.data) != 0:
            raise DecoderError(f"ccv_decode_host: {_native.last_error()}")
        return out if pm is None else (out, pm)

    def close(self):
        """Release the plan's stream and device scratch (also done when the plan is collected)."""
        if getattr(self, "_h", None):
            self._lib.ccv_plan_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StackPlan(Plan):
    """Stack (sequential) decoder plan (ccv_stack_plan_create): AWGN-channel/stack-decoder.c or
    binary-symmetric-channel/stack-decoder.c, metrics from the code (code_param.metric_weight /
    bit_metrics). decode_host / decode_device behave as one fresh decoder fed the blocks in order."""

    def __init__(self, code: Code, channel: int = SOFT):
        self.code = code
        self.channel = channel
        self._lib = _native.core()
        self._polys = code.poly_array()
        self._bm = (ctypes.c_int32 * 2)(*code.bit_metrics)
        h = ctypes.c_void_p()
        if self._lib.ccv_stack_plan_create(ctypes.byref(h), channel, code.n, code.K, code.blen,
                                           self._polys, code.gen_mode, float(code.metric_weight),
                                           self._bm) != 0:
            raise DecoderError(f"ccv_stack_plan_create: {_native.last_error()}")
        self._h = h
        self.desc = _native.CcvPlanDesc()
        self._lib.ccv_plan_describe(self._h, ctypes.byref(self.desc))

    def decode_stack_device(self, d_in, nblocks, d_out, d_prev=None, d_path_metric=None, d_info=None,
                            d_errors=None, d_status=None, stream=None):
        """ccv_stack_decode_device: d_prev = the block the decoder saw before block 0 (None = fresh);
        d_status[nb] flags blocks whose search would make the reference read past its buffers."""
        rc = self._lib.ccv_stack_decode_device(self._h, _ptr(d_in), int(nblocks), _ptr(d_prev),
                                               _ptr(d_out), _ptr(d_path_metric), _ptr(d_info),
                                               _ptr(d_errors), _ptr(d_status), _stream_handle(stream))
        if rc != 0:
            raise DecoderError(f"ccv_stack_decode_device: {_native.last_error()}")


class FanoPlan(Plan):
    """Fano decoder plan (ccv_fano_plan_create): AWGN-channel/fano-decoder.c or
    binary-symmetric-channel/fano-decoder.c with the code's fano_metric_weight / fano_bit_metrics."""

    def __init__(self, code: Code, channel: int = SOFT):
        self.code = code
        self.channel = channel
        self._lib = _native.core()
        self._polys = code.poly_array()
        self._bm = (ctypes.c_int32 * 2)(*code.fano_bit_metrics)
        h = ctypes.c_void_p()
        if self._lib.ccv_fano_plan_create(ctypes.byref(h), channel, code.n, code.K, code.blen,
                                          self._polys, code.gen_mode, float(code.fano_metric_weight),
                                          self._bm) != 0:
            raise DecoderError(f"ccv_fano_plan_create: {_native.last_error()}")
        self._h = h
        self.desc = _native.CcvPlanDesc()
        self._lib.ccv_plan_describe(self._h, ctypes.byref(self.desc))

    def decode_fano_device(self, d_in, nblocks, d_out, d_path_metric=None, d_info=None, d_errors=None,
                           d_iterations=None, stream=None):
        """ccv_fano_decode_device; d_iterations[nb] = search iterations (10000 * T = timeout)."""
        rc = self._lib.ccv_fano_decode_device(self._h, _ptr(d_in), int(nblocks), _ptr(d_out),
                                              _ptr(d_path_metric), _ptr(d_info), _ptr(d_errors),
                                              _ptr(d_iterations), _stream_handle(stream))
        if rc != 0:
            raise DecoderError(f"ccv_fano_decode_device: {_native.last_error()}")


_SOFT_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint8, ctypes.c_void_p)
_HARD_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint8,
                            ctypes.c_int32, ctypes.c_void_p)


class _ViterbiDecoder:
    """decoder_create / init / register_callback / reset / input / destroy."""
    _soft = True

    def __init__(self):
        self._lib = _native.awgn() if self._soft else _native.bsc()
        self._obj = ctypes.c_void_p(self._lib.decoder_create())
        if not self._obj:
            raise DecoderError("decoder_create failed")
        self._keep = None
        self._cb = None
        self.code = None

    def _check(self, rc, what):
        if rc != 0:
            raise DecoderError(f"{what}: {self._lib.decoder_last_error().decode(errors='replace')}")

    def set_generator_mode(self, mode: int):
        self._check(self._lib.decoder_set_generator_mode(self._obj, mode), "decoder_set_generator_mode")

    def init(self, code: Code):
        """decoder_init. The generator mode is taken from code.gen_mode."""
        self.set_generator_mode(code.gen_mode)
        param, keep = code.to_param()
        self._keep = (param, keep)
        self._check(self._lib.decoder_init(self._obj, ctypes.byref(param)), "decoder_init")
        self.code = code

    def register_callback(self, fn):
        """fn(bits: bytes, len_bits: int[, path_metric: int]). The decoded buffer is copied out for
        fn and the trampoline returns -1, so the decoder keeps (and reuses) its buffer."""
        if self._soft:
            def tramp(data, length, _ud):
                if fn:
                    fn(ctypes.string_at(data, self.code.out_bytes), int(length))
                return -1
            self._cb = _SOFT_CB(tramp)
        else:
            def tramp(data, length, pm, _ud):
                if fn:
                    fn(ctypes.string_at(data, self.code.out_bytes), int(length), int(pm))
                return -1
            self._cb = _HARD_CB(tramp)
        self._lib.decoder_register_callback(self._obj, ctypes.cast(self._cb, ctypes.c_void_p))

    def reset(self):
        self._lib.decoder_reset(self._obj)

    def _as_input(self, data):
        dt = np.float32 if self._soft else np.uint8
        return np.ascontiguousarray(data, dtype=dt)

    def input(self, data):
        """decoder_input; len (floats or symbols) must fit the reference's uint8_t."""
        arr = self._as_input(data).ravel()
        if arr.size > 255:
            raise ValueError("decoder_input takes at most 255 elements per call (uint8_t len)")
        self._check(self._lib.decoder_input(self._obj, arr.ctypes.data, arr.size), "decoder_input")

    def input_blocks(self, data):
        arr = self._as_input(data)
        nb = arr.size // (self.code.steps * ((1 << self.code.n) if self._soft else 1))
        self._check(self._lib.decoder_input_blocks(self._obj, arr.ctypes.data, nb), "decoder_input_blocks")

    def destroy(self):
        if self._obj:
            self._lib.decoder_destroy(ctypes.byref(self._obj))
            self._obj = ctypes.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class SoftDecoder(_ViterbiDecoder):
    """AWGN soft-decision decoder (include/decoder_awgn.h)."""
    _soft = True

    def decode_blocks(self, data):
        arr = self._as_input(data)
        nb = arr.size // (self.code.steps << self.code.n)
        out = np.zeros((nb, self.code.out_bytes), np.uint8)
        self._check(self._lib.decoder_decode_blocks(self._obj, arr.ctypes.data, nb, out.ctypes.data),
                    "decoder_decode_blocks")
        return out

    def decode_device(self, d_in, nblocks, d_out, stream=None):
        self._check(self._lib.decoder_decode_device(self._obj, _ptr(d_in), int(nblocks), _ptr(d_out),
                                                    _stream_handle(stream)), "decoder_decode_device")


class HardDecoder(_ViterbiDecoder):
    """BSC hard-decision decoder (include/decoder_bsc.h)."""
    _soft = False

    def decode_blocks(self, data):
        arr = self._as_input(data)
        nb = arr.size // self.code.steps
        out = np.zeros((nb, self.code.out_bytes), np.uint8)
        pm = np.zeros(nb, np.int32)
        self._check(self._lib.decoder_decode_blocks(self._obj, arr.ctypes.data, nb, out.ctypes.data,
                                                    pm.ctypes.data), "decoder_decode_blocks")
        return out, pm

    def decode_device(self, d_in, nblocks, d_out, d_path_metrics=None, stream=None):
        self._check(self._lib.decoder_decode_device(self._obj, _ptr(d_in), int(nblocks), _ptr(d_out),
                                                    _ptr(d_path_metrics), _stream_handle(stream)),
                    "decoder_decode_device")

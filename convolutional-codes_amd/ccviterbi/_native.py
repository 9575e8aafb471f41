"""Loading of the in-tree native libraries (lib/*.so built by `make -C convolutional-codes_amd`).

There is no fallback: if a library is missing or fails to load, every entry point raises
NativeLibraryError. The decoder is the HIP path or nothing.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)            # convolutional-codes_amd/
# CCV_LIB_DIR: load another in-tree build of the same libraries instead (A/B timing of two builds in
# one session, tools/ab_build.sh); still native code, never a fallback
LIB_DIR = os.environ.get("CCV_LIB_DIR") or os.path.join(ROOT_DIR, "lib")

_P = ctypes.POINTER
_vp, _sz, _i, _u, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint, ctypes.c_uint64


class NativeLibraryError(RuntimeError):
    pass


def _share_torch_hip_runtime():
    """PyTorch-ROCm ships its own libamdhip64 with the same SONAME (libamdhip64.so.7) as the
    system ROCm our libraries link. Whichever loads first serves the whole process, and PyTorch sees
    no device if the system runtime came first. Importing torch (when installed) before our
    libraries makes its runtime the shared one; without torch the system runtime is used."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


class CcvPlanDesc(ctypes.Structure):
    """ccv_plan_desc (include/ccv.h)."""
    _fields_ = [(name, ctypes.c_int) for name in (
        "channel", "n", "K", "blen", "gen_mode", "steps", "states", "info_bytes", "out_bytes",
        "in_step_bytes", "kernel", "decision_word_bytes", "device", "lanes")]


_cache = {}


def _load(name):
    if name in _cache:
        return _cache[name]
    _share_torch_hip_runtime()
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"{path} is missing: build it with `make -C {ROOT_DIR}` (or __graft_entry__.build())")
    try:
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    except OSError as e:
        raise NativeLibraryError(f"cannot load {path}: {e}") from e
    _cache[name] = lib
    return lib


def core():
    """libccv_core.so: the HIP decoder (include/ccv.h)."""
    if "core" in _cache:
        return _cache["core"]
    # CCV_CORE_LIB: an alternative build of the core library in lib/ (kernel A/B builds, tools/)
    L = _load(os.environ.get("CCV_CORE_LIB", "libccv_core.so"))
    L.ccv_plan_create.argtypes = [_P(_vp), _i, _i, _i, _i, _P(_u64), _i, _u]
    L.ccv_plan_create.restype = _i
    L.ccv_plan_destroy.argtypes = [_vp]
    L.ccv_plan_destroy.restype = None
    L.ccv_plan_describe.argtypes = [_vp, _P(CcvPlanDesc)]
    L.ccv_plan_describe.restype = _i
    L.ccv_plan_trellis.argtypes = [_vp, _vp]
    L.ccv_plan_trellis.restype = _i
    L.ccv_plan_decision_storage.argtypes = [_vp]
    L.ccv_plan_decision_storage.restype = _i
    L.ccv_plan_kernel_variant.argtypes = [_vp]
    L.ccv_plan_kernel_variant.restype = ctypes.c_char_p
    L.ccv_plan_persistent_waves.argtypes = [_vp, _i]
    L.ccv_plan_persistent_waves.restype = _i
    L.ccv_plan_reserve.argtypes = [_vp, _sz]
    L.ccv_plan_reserve.restype = _i
    L.ccv_decode_device.argtypes = [_vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]
    L.ccv_decode_device.restype = _i
    L.ccv_simulate_device.argtypes = [_vp, _u64, _u64, _sz, ctypes.c_double, _u, _vp, _vp, _vp, _vp,
                                      _vp, _vp]
    L.ccv_simulate_device.restype = _i
    L.ccv_stack_plan_create.argtypes = [_P(_vp), _i, _i, _i, _i, _P(_u64), _i, ctypes.c_float, _vp]
    L.ccv_stack_plan_create.restype = _i
    L.ccv_stack_decode_device.argtypes = [_vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.ccv_stack_decode_device.restype = _i
    L.ccv_fano_plan_create.argtypes = [_P(_vp), _i, _i, _i, _i, _P(_u64), _i, ctypes.c_float, _vp]
    L.ccv_fano_plan_create.restype = _i
    L.ccv_fano_decode_device.argtypes = [_vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]
    L.ccv_fano_decode_device.restype = _i
    L.ccv_decode_host.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.ccv_decode_host.restype = _i
    # entry points added in round 5: bound where present, so the libraries of an older revision
    # (whole-build A/B, tools/ab_build.sh) still load; calling one that is absent raises
    if hasattr(L, "ccv_plan_set_option"):
        L.ccv_plan_set_option.argtypes = [_vp, ctypes.c_char_p, ctypes.c_longlong]
        L.ccv_plan_set_option.restype = _i
    if hasattr(L, "ccv_hbm_probe"):
        L.ccv_hbm_probe.argtypes = [_i, _vp, _vp, _sz, _vp, _vp]
        L.ccv_hbm_probe.restype = _i
    L.ccv_device_count.argtypes = []
    L.ccv_device_count.restype = _i
    L.ccv_last_error.argtypes = []
    L.ccv_last_error.restype = ctypes.c_char_p
    _cache["core"] = L
    return L


def _shim(name, soft):
    key = "shim_" + name
    if key in _cache:
        return _cache[key]
    L = _load(name)
    in_t = _vp
    L.decoder_create.argtypes = []
    L.decoder_create.restype = _vp
    L.decoder_destroy.argtypes = [_P(_vp)]
    L.decoder_destroy.restype = None
    L.decoder_init.argtypes = [_vp, _vp]
    L.decoder_init.restype = _i
    L.decoder_register_callback.argtypes = [_vp, _vp]
    L.decoder_register_callback.restype = None
    L.decoder_reset.argtypes = [_vp]
    L.decoder_reset.restype = None
    L.decoder_input.argtypes = [_vp, in_t, ctypes.c_uint8]
    L.decoder_input.restype = _i
    L.decoder_set_generator_mode.argtypes = [_vp, _i]
    L.decoder_set_generator_mode.restype = _i
    L.decoder_input_blocks.argtypes = [_vp, in_t, _sz]
    L.decoder_input_blocks.restype = _i
    if soft:
        L.decoder_decode_blocks.argtypes = [_vp, in_t, _sz, _vp]
        L.decoder_decode_device.argtypes = [_vp, _vp, _sz, _vp, _vp]
    else:
        L.decoder_decode_blocks.argtypes = [_vp, in_t, _sz, _vp, _vp]
        L.decoder_decode_device.argtypes = [_vp, _vp, _sz, _vp, _vp, _vp]
    L.decoder_decode_blocks.restype = _i
    L.decoder_decode_device.restype = _i
    L.decoder_last_error.argtypes = []
    L.decoder_last_error.restype = ctypes.c_char_p
    _cache[key] = L
    return L


def awgn():
    """libccv_awgn.so: reference-compatible soft decoder (include/decoder_awgn.h)."""
    return _shim("libccv_awgn.so", soft=True)


def bsc():
    """libccv_bsc.so: reference-compatible hard decoder (include/decoder_bsc.h)."""
    return _shim("libccv_bsc.so", soft=False)


def sim():
    """libccv_sim.so: CPU producers (include/ccv_sim.h)."""
    if "sim" in _cache:
        return _cache["sim"]
    L = _load("libccv_sim.so")
    L.ccv_sim_encode.argtypes = [_i, _i, _i, _P(_u64), _i, _vp, _sz, _vp]
    L.ccv_sim_encode.restype = _i
    L.ccv_sim_demap.argtypes = [_i, _vp, _sz, _vp]
    L.ccv_sim_demap.restype = _i
    L.ccv_sim_noise_scaling.argtypes = [ctypes.c_double]
    L.ccv_sim_noise_scaling.restype = ctypes.c_double
    L.ccv_sim_awgn.argtypes = [_i, _i, _i, _P(_u64), _i, _i, _u64, ctypes.c_float, _sz, _sz, _vp, _vp, _i]
    L.ccv_sim_awgn.restype = _i
    L.ccv_sim_bsc.argtypes = [_i, _i, _i, _P(_u64), _i, _i, _u64, ctypes.c_int32, _sz, _sz, _vp, _vp, _i]
    L.ccv_sim_bsc.restype = _i
    _cache["sim"] = L
    return L


def last_error():
    return core().ccv_last_error().decode(errors="replace")

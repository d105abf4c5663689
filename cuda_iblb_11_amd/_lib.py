"""ctypes binding of include/iblb.h (the C ABI of libiblb.so).

The shared library is built in-tree (``make`` -> cuda_iblb_11_amd/lib/libiblb.so).  There is
no CPU fallback: if the library is missing, or no HIP device is visible, every compute
entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(_HERE)
# IBLB_LIB: another build of the same library (A/B measurements of kernel builds only)
LIB_PATH = os.environ.get("IBLB_LIB") or os.path.join(_HERE, "lib", "libiblb.so")
HEADER = os.path.join(REPO, "include", "iblb.h")

IBLB_OK = 0
IBLB_ERR_ARG = -1
IBLB_ERR_HIP = -2
IBLB_ERR_STATE = -3
IBLB_ERR_COMM = -4
IBLB_ERR_NOMEM = -5
IBLB_ERR_UNSUPPORTED = -6
IBLB_ERR_NODEVICE = -7
PREC_F64 = 0
PREC_F32 = 1
UNIQUE_ID_BYTES = 128

_ERRNAMES = {
    IBLB_ERR_ARG: "IBLB_ERR_ARG", IBLB_ERR_HIP: "IBLB_ERR_HIP", IBLB_ERR_STATE: "IBLB_ERR_STATE",
    IBLB_ERR_COMM: "IBLB_ERR_COMM", IBLB_ERR_NOMEM: "IBLB_ERR_NOMEM",
    IBLB_ERR_UNSUPPORTED: "IBLB_ERR_UNSUPPORTED", IBLB_ERR_NODEVICE: "IBLB_ERR_NODEVICE",
}


class IblbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class Config(C.Structure):
    """struct iblb_config (include/iblb.h)."""
    _fields_ = [
        ("nx", C.c_int), ("ny", C.c_int),
        ("tau", C.c_double), ("tau2", C.c_double),
        ("precision", C.c_int),
        ("body_force", C.c_double * 2),
        ("flux_norm", C.c_double),
        ("flux_column", C.c_int),
        ("device", C.c_int),
        ("x_begin", C.c_int), ("x_count", C.c_int),
        ("max_points", C.c_int),
    ]


class Timing(C.Structure):
    """struct iblb_timing (include/iblb.h)."""
    _fields_ = [
        ("steps", C.c_longlong), ("fused_launches", C.c_longlong),
        ("fused_ms", C.c_double), ("ib_ms", C.c_double), ("halo_ms", C.c_double),
        ("fused_bytes", C.c_double), ("cells", C.c_longlong), ("fused_cells", C.c_longlong),
        ("sweep_launches", C.c_longlong), ("sweep_ms", C.c_double), ("sweep_cells", C.c_longlong),
        ("sweepk_launches", C.c_longlong), ("sweepk_ms", C.c_double), ("sweepk_cells", C.c_longlong), ("sweepk_depth", C.c_longlong),
        ("band_cycles", C.c_longlong), ("band_merged_cycles", C.c_longlong), ("band_par_cycles", C.c_longlong),
        ("deep_launches", C.c_longlong), ("deep_iterations", C.c_longlong),
        ("dev_wait_launches", C.c_longlong),
        ("deep_mode", C.c_longlong), ("deep_vs", C.c_longlong), ("deep_waves_per_simd", C.c_longlong),
        ("deep_vgprs", C.c_longlong),
    ]


class Cilia(C.Structure):
    """struct iblb_cilia (include/iblb.h)."""
    _fields_ = [("c_num", C.c_int), ("c_space", C.c_double), ("T", C.c_int), ("p_step", C.c_int)]


_vp = C.c_void_p
_SIGS = {
    # (1) reference-shaped kernels: device pointers + stream
    "iblb_equilibrium": ([_vp, _vp, _vp, _vp, _vp, C.c_int, C.c_int, C.c_double, _vp], C.c_int),
    "iblb_collision": ([_vp, _vp, _vp, _vp, C.c_double, C.c_double, C.c_int, C.c_int, C.c_int, _vp], C.c_int),
    "iblb_streaming": ([_vp, _vp, C.c_int, C.c_int, _vp], C.c_int),
    "iblb_macro": ([_vp, _vp, _vp, C.c_int, C.c_int, _vp], C.c_int),
    "iblb_interpolate": ([_vp, _vp, C.c_int, _vp, _vp, _vp, C.c_int, C.c_int, _vp], C.c_int),
    "iblb_spread": ([_vp, _vp, _vp, C.c_int, _vp, _vp, _vp, _vp, C.c_int, _vp, _vp, _vp], C.c_int),
    "iblb_spread_ex": ([_vp, _vp, _vp, C.c_int, _vp, _vp, _vp, _vp, C.c_int, C.c_int, _vp, _vp, C.c_int,
                        C.c_double, _vp], C.c_int),
    "iblb_delta": ([C.c_int, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "iblb_define_filament": ([C.c_int, C.c_int, C.c_double, C.c_int, C.c_double, _vp, _vp, _vp, _vp], C.c_int),
    "iblb_boundary_check": ([C.c_double, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp], C.c_int),
    # (2) context API
    "iblb_config_default": ([C.POINTER(Config)], C.c_int),
    "iblb_create": ([C.POINTER(Config), C.POINTER(_vp)], C.c_int),
    "iblb_destroy": ([_vp], None),
    "iblb_last_error": ([_vp], C.c_char_p),
    "iblb_version": ([], C.c_char_p),
    "iblb_abi_version": ([], C.c_int),
    "iblb_device_count": ([C.POINTER(C.c_int)], C.c_int),
    "iblb_set_state": ([_vp, _vp, _vp, _vp, _vp], C.c_int),
    "iblb_set_lagrangian": ([_vp, C.c_int, _vp, _vp, _vp], C.c_int),
    "iblb_set_lagrangian_steps": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "iblb_set_cilia": ([_vp, C.POINTER(Cilia)], C.c_int),
    "iblb_get_lagrangian": ([_vp, _vp, _vp, _vp], C.c_int),
    "iblb_step": ([_vp, C.c_int], C.c_int),
    "iblb_get_macro": ([_vp, _vp, _vp], C.c_int),
    "iblb_get_populations": ([_vp, _vp], C.c_int),
    "iblb_get_force": ([_vp, _vp], C.c_int),
    "iblb_get_lagrangian_force": ([_vp, _vp], C.c_int),
    "iblb_get_flux": ([_vp, C.POINTER(C.c_double)], C.c_int),
    "iblb_get_step": ([_vp, C.POINTER(C.c_longlong)], C.c_int),
    "iblb_count_nonfinite": ([_vp, C.POINTER(C.c_longlong)], C.c_int),
    "iblb_set_profiling": ([_vp, C.c_int], C.c_int),
    "iblb_get_timing": ([_vp, C.POINTER(Timing), C.c_int], C.c_int),
    "iblb_get_timing_ex": ([_vp, C.POINTER(Timing), C.c_ulong, C.c_int], C.c_int),
    "iblb_get_stream": ([_vp, C.POINTER(_vp)], C.c_int),
    "iblb_synchronize": ([_vp], C.c_int),
    "iblb_link_local": ([C.POINTER(_vp), C.c_int], C.c_int),
    "iblb_group_step": ([C.POINTER(_vp), C.c_int, C.c_int], C.c_int),
    "iblb_rccl_unique_id": ([C.c_char_p], C.c_int),
    "iblb_attach_rccl": ([_vp, C.c_char_p, C.c_int, C.c_int], C.c_int),
    "iblb_set_wait_timeout": ([_vp, C.c_double], C.c_int),
    "iblb_gather_macro": ([_vp, C.c_int, _vp, _vp], C.c_int),
    "iblb_save_checkpoint": ([_vp, C.c_char_p], C.c_int),
    "iblb_load_checkpoint": ([_vp, C.c_char_p], C.c_int),
}

_lib = None


def header_functions() -> list[str]:
    """Names of every function declared in include/iblb.h."""
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(iblb_[a-z_]+)\s*\(", text)))


def configure(lib: C.CDLL) -> C.CDLL:
    """Attach the include/iblb.h signatures to a loaded library."""
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


def load_from(path: str) -> C.CDLL:
    """Load another build of the C ABI (e.g. the mock-RCCL test build) without torch."""
    return configure(C.CDLL(path))


def load() -> C.CDLL:
    """Load libiblb.so (raises if it was not built; there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `make` (hipcc, gfx950); there is no CPU fallback")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 / librccl.so.1.  If torch
    # is importable, load it first so libiblb binds to the same runtime (same SONAMEs) instead of
    # a second copy from /opt/rocm, which would leave torch without devices.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    _lib = configure(C.CDLL(LIB_PATH))
    return _lib


def check(rc: int, ctx=None, lib: C.CDLL | None = None) -> None:
    if rc != IBLB_OK:
        msg = (lib or load()).iblb_last_error(ctx)
        raise IblbError(rc, msg.decode() if msg else "")


def device_count() -> int:
    n = C.c_int(0)
    load().iblb_device_count(C.byref(n))
    return n.value

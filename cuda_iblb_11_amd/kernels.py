"""Reference-named kernel entry points on device tensors (include/iblb.h, part 1).

Same names, argument order and layouts as the reference kernels (LatticeBoltzmann.cuh:4-10,
ImmersedBoundary.cuh:4-8); each call launches the HIP kernel through libiblb.so on the
current torch stream.  torch is only the device-memory/stream plumbing here.
"""
from __future__ import annotations

import ctypes as C

from . import _lib as L


def _dev(t, dtype=None):
    import torch
    if t is None:
        return None
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError("expected a device (HIP) tensor; the HIP kernels have no CPU path")
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"expected {dtype}, got {t.dtype}")
    return C.c_void_p(t.data_ptr())


def _stream(stream=None):
    import torch
    s = torch.cuda.current_stream() if stream is None else stream
    return C.c_void_p(s.cuda_stream)


def _f64():
    import torch
    return torch.float64


def _f32():
    import torch
    return torch.float32


def _i32():
    import torch
    return torch.int32


def equilibrium(u, rho, f0, force, F, XDIM, YDIM, TAU, stream=None):
    d = _f64()
    L.check(L.load().iblb_equilibrium(_dev(u, d), _dev(rho, d), _dev(f0, d), _dev(force, d), _dev(F, d),
                                      int(XDIM), int(YDIM), float(TAU), _stream(stream)))


def collision(f0, f, f1, F, TAU, TAU2, XDIM, YDIM, it=0, stream=None):
    d = _f64()
    L.check(L.load().iblb_collision(_dev(f0, d), _dev(f, d), _dev(f1, d), _dev(F, d), float(TAU), float(TAU2),
                                    int(XDIM), int(YDIM), int(it), _stream(stream)))


def streaming(f1, f, XDIM, YDIM, stream=None):
    d = _f64()
    L.check(L.load().iblb_streaming(_dev(f1, d), _dev(f, d), int(XDIM), int(YDIM), _stream(stream)))


def macro(f, u, rho, XDIM, YDIM, stream=None):
    d = _f64()
    L.check(L.load().iblb_macro(_dev(f, d), _dev(u, d), _dev(rho, d), int(XDIM), int(YDIM), _stream(stream)))


def interpolate(rho, u, Ns, u_s, F_s, s, XDIM, YDIM, stream=None):
    d, fl = _f64(), _f32()
    L.check(L.load().iblb_interpolate(_dev(rho, d), _dev(u, d), int(Ns), _dev(u_s, fl), _dev(F_s, fl), _dev(s, fl),
                                      int(XDIM), int(YDIM), _stream(stream)))


def spread(rho, u, f, Ns, u_s, F_s, force, s, XDIM, Q, epsilon, YDIM=None, flux_column=None, flux_norm=192.0,
           stream=None):
    """ImmersedBoundary.cu:138.  YDIM=None keeps the reference's hard-coded 192."""
    d, fl, i = _f64(), _f32(), _i32()
    lib = L.load()
    if YDIM is None and flux_column is None and flux_norm == 192.0:
        L.check(lib.iblb_spread(_dev(rho, d), _dev(u, d), _dev(f, d), int(Ns), _dev(u_s, fl), _dev(F_s, fl),
                                _dev(force, d), _dev(s, fl), int(XDIM), _dev(Q, d), _dev(epsilon, i), _stream(stream)))
        return
    yd = 192 if YDIM is None else int(YDIM)
    fc = int(XDIM) - 5 if flux_column is None else int(flux_column)
    L.check(lib.iblb_spread_ex(_dev(rho, d), _dev(u, d), _dev(f, d), int(Ns), _dev(u_s, fl), _dev(F_s, fl),
                               _dev(force, d), _dev(s, fl), int(XDIM), yd, _dev(Q, d), _dev(epsilon, i), fc,
                               float(flux_norm), _stream(stream)))


def define_filament(T, it, c_space, p_step, c_num, s, lasts, b_points, stream=None):
    """main.cu:77: s = d_boundary [5*9600*c_num], lasts [2*9600*c_num], b_points [5*96*c_num]."""
    fl = _f32()
    L.check(L.load().iblb_define_filament(int(T), int(it), float(c_space), int(p_step), float(c_num), _dev(s, fl),
                                          _dev(lasts, fl), _dev(b_points, fl), _stream(stream)))


def boundary_check(c_space, c_num, XDIM, it, b_points, s, u_s, epsilon, stream=None):
    """main.cu:176: Lagrangian s [2*96*c_num], u_s, epsilon [96*c_num] from b_points."""
    fl, i = _f32(), _i32()
    L.check(L.load().iblb_boundary_check(float(c_space), int(c_num), int(XDIM), int(it), _dev(b_points, fl),
                                         _dev(s, fl), _dev(u_s, fl), _dev(epsilon, i), _stream(stream)))


def d_delta(xs, ys, x, y, out, stream=None):
    fl, i = _f32(), _i32()
    L.check(L.load().iblb_delta(int(xs.numel()), _dev(xs, fl), _dev(ys, fl), _dev(x, i), _dev(y, i), _dev(out, fl),
                                _stream(stream)))

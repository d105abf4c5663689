"""ctypes/numpy front end of the CPU oracle (oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product package (cuda_iblb_11_amd) never does.

Parity status: the restatement is UNPINNED against the reference binary (the reference's
CUDA sources cannot be built in this image); it is pinned by analytic known-answer tests
and by the reference's nominal outputs (see oracle.h).

Functions carry the reference kernel names and argument order
(LatticeBoltzmann.cuh:4-10, ImmersedBoundary.cuh:4-8) and operate on numpy arrays in the
reference layouts: f/f0/f1/F AoS [9*j+i], u/force SoA [a*size+j], rho [size],
Lagrangian s/u_s/F_s interleaved float32 [2*Ns], epsilon int32 [Ns]; j = y*XDIM + x.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None

# LatticeBoltzmann.cu:11-27
C_S = 0.57735
C_L = np.array([[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]], dtype=np.int64)
W = np.array([4 / 9] + [1 / 9] * 4 + [1 / 36] * 4)

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_fp = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


class _State(C.Structure):
    _fields_ = [
        ("XDIM", C.c_int), ("YDIM", C.c_int), ("TAU", C.c_double), ("TAU2", C.c_double),
        ("f", C.c_void_p), ("f0", C.c_void_p), ("f1", C.c_void_p), ("F", C.c_void_p),
        ("rho", C.c_void_p), ("u", C.c_void_p), ("force", C.c_void_p), ("Q", C.c_void_p),
        ("Ns", C.c_int), ("s", C.c_void_p), ("u_s", C.c_void_p), ("F_s", C.c_void_p),
        ("epsilon", C.c_void_p), ("body_force", C.c_double * 2), ("flux_column", C.c_int),
        ("flux_norm", C.c_double), ("point_spread", C.c_int),
    ]


def lib_path(native: bool = False) -> str:
    return os.path.join(_HERE, "liboracle_native.so" if native else "liboracle.so")


def build(native: bool = False) -> str:
    """Compile the oracle with make (gcc).  Returns the library path."""
    target = ["native"] if native else []
    subprocess.run(["make", "-s", "-C", _HERE] + target, check=True)
    return lib_path(native)


def load(native: bool | None = None):
    """Load the oracle (portable build by default; native=True switches every wrapper below to
    the -march=native build, compiling it first if needed)."""
    global _lib
    if _lib is not None and native is None:
        return _lib
    native = bool(native)
    path = lib_path(native)
    if not os.path.exists(path):
        build(native)
    lib = C.CDLL(path)
    lib.oracle_equilibrium.argtypes = [_dp, _dp, _dp, _dp, _dp, C.c_int, C.c_int, C.c_double]
    lib.oracle_collision.argtypes = [_dp, _dp, _dp, _dp, C.c_double, C.c_double, C.c_int, C.c_int, C.c_int]
    lib.oracle_streaming.argtypes = [_dp, _dp, C.c_int, C.c_int]
    lib.oracle_macro.argtypes = [_dp, _dp, _dp, C.c_int, C.c_int]
    lib.oracle_d_delta.argtypes = [C.c_float, C.c_float, C.c_int, C.c_int]
    lib.oracle_d_delta.restype = C.c_float
    lib.oracle_interpolate.argtypes = [_dp, _dp, C.c_int, _fp, _fp, _fp, C.c_int, C.c_int]
    for name in ("oracle_spread", "oracle_spread_points"):
        getattr(lib, name).argtypes = [_dp, _dp, _dp, C.c_int, _fp, _fp, _dp, _fp, C.c_int, C.c_int,
                                       _dp, _ip, C.c_int, C.c_double]
    lib.oracle_define_filament.argtypes = [C.c_int, C.c_int, C.c_double, C.c_int, C.c_double, _fp, _fp, _fp]
    lib.oracle_boundary_check.argtypes = [C.c_double, C.c_int, C.c_int, C.c_int, _fp, _fp, _fp, _ip]
    lib.oracle_step.argtypes = [C.POINTER(_State), C.c_int]
    lib.oracle_run.argtypes = [C.POINTER(_State), C.c_int, C.c_int]
    lib.oracle_set_threads.argtypes = [C.c_int]
    lib.oracle_get_threads.restype = C.c_int
    _lib = lib
    return lib


def set_threads(n: int) -> None:
    load().oracle_set_threads(int(n))


# ---- kernel-level restatements (same names/argument order as the reference) --------

def equilibrium(u, rho, f0, force, F, XDIM, YDIM, TAU):
    load().oracle_equilibrium(u, rho, f0, force, F, XDIM, YDIM, TAU)


def collision(f0, f, f1, F, TAU, TAU2, XDIM, YDIM, it=0):
    load().oracle_collision(f0, f, f1, F, TAU, TAU2, XDIM, YDIM, it)


def streaming(f1, f, XDIM, YDIM):
    load().oracle_streaming(f1, f, XDIM, YDIM)


def macro(f, u, rho, XDIM, YDIM):
    load().oracle_macro(f, u, rho, XDIM, YDIM)


def d_delta(xs, ys, x, y) -> float:
    return float(load().oracle_d_delta(xs, ys, x, y))


def interpolate(rho, u, Ns, u_s, F_s, s, XDIM, YDIM):
    load().oracle_interpolate(rho, u, Ns, u_s, F_s, s, XDIM, YDIM)


def spread(rho, u, f, Ns, u_s, F_s, force, s, XDIM, Q, epsilon, YDIM=192, flux_column=None,
           flux_norm=192.0, point_centric=False):
    fc = XDIM - 5 if flux_column is None else flux_column
    fn = load().oracle_spread_points if point_centric else load().oracle_spread
    fn(rho, u, f, Ns, u_s, F_s, force, s, XDIM, YDIM, Q, epsilon, fc, flux_norm)


def define_filament(T, it, c_space, p_step, c_num, s, lasts, b_points):
    load().oracle_define_filament(int(T), int(it), float(c_space), int(p_step), float(c_num), s, lasts, b_points)


def boundary_check(c_space, c_num, XDIM, it, b_points, s, u_s, epsilon):
    load().oracle_boundary_check(float(c_space), int(c_num), int(XDIM), int(it), b_points, s, u_s, epsilon)


class Cilia:
    """The reference's Lagrangian source (main.cu:822-841) on host arrays: call points(it) once
    per iteration, in order (define_filament keeps the previous positions in `lasts`)."""

    def __init__(self, c_num, c_space, T, p_step, XDIM):
        self.c_num, self.c_space, self.T, self.p_step, self.XDIM = int(c_num), float(c_space), int(T), int(p_step), int(XDIM)
        nk = 9600 * self.c_num
        self.samples = np.zeros(5 * nk, dtype=np.float32)   # d_boundary
        self.lasts = np.zeros(2 * nk, dtype=np.float32)
        self.b_points = np.zeros(5 * 96 * self.c_num, dtype=np.float32)
        self.s = np.zeros(2 * 96 * self.c_num, dtype=np.float32)
        self.u_s = np.zeros_like(self.s)
        self.epsilon = np.ones(96 * self.c_num, dtype=np.int32)

    def points(self, it):
        define_filament(self.T, it, self.c_space, self.p_step, self.c_num, self.samples, self.lasts, self.b_points)
        boundary_check(self.c_space, self.c_num, self.XDIM, it, self.b_points, self.s, self.u_s, self.epsilon)
        return self.s, self.u_s, self.epsilon


# ---- whole-step driver ----------------------------------------------------------------

def feq(rho: np.ndarray, u: np.ndarray, XDIM: int, YDIM: int, TAU: float = 1.0) -> np.ndarray:
    """Initial populations exactly as main.cu:720-754 (one `equilibrium` launch, f = f0)."""
    size = XDIM * YDIM
    f0 = np.zeros(9 * size)
    F = np.zeros(9 * size)
    equilibrium(np.ascontiguousarray(u, dtype=np.float64), np.ascontiguousarray(rho, dtype=np.float64),
                f0, np.zeros(2 * size), F, XDIM, YDIM, TAU)
    return f0


class Simulation:
    """Host-array state + oracle_step (main.cu:852-909).  Arrays in reference layouts."""

    def __init__(self, XDIM, YDIM, TAU, TAU2, rho=None, u=None, f=None, force=None, body_force=(0.0, 0.0),
                 flux_column=None, flux_norm=192.0, point_spread=True, threads=None):
        self.XDIM, self.YDIM = int(XDIM), int(YDIM)
        size = self.XDIM * self.YDIM
        self.size = size
        self.rho = np.ones(size) if rho is None else np.array(rho, dtype=np.float64)
        self.u = np.zeros(2 * size) if u is None else np.array(u, dtype=np.float64)
        # force^0: the given array (reference: zeros, main.cu:642-643) plus the uniform body force
        # (extension; the body force acts in every iteration including the first)
        self.force = np.zeros(2 * size) if force is None else np.array(force, dtype=np.float64)
        self.force[:size] += float(body_force[0])
        self.force[size:] += float(body_force[1])
        self.f = feq(self.rho, self.u, self.XDIM, self.YDIM, TAU) if f is None else np.array(f, dtype=np.float64)
        self.f0 = np.zeros(9 * size)
        self.f1 = np.zeros(9 * size)
        self.F = np.zeros(9 * size)
        self.Q = np.zeros(1)
        self.it = 0
        self._pts = None
        self.F_s = np.zeros(0, dtype=np.float32)
        st = _State()
        st.XDIM, st.YDIM, st.TAU, st.TAU2 = self.XDIM, self.YDIM, float(TAU), float(TAU2)
        st.body_force[0], st.body_force[1] = float(body_force[0]), float(body_force[1])
        st.flux_column = self.XDIM - 5 if flux_column is None else int(flux_column)
        st.flux_norm = float(flux_norm)
        st.point_spread = 1 if point_spread else 0
        st.Ns = 0
        self._st = st
        self._bind()
        if threads is not None:
            set_threads(threads)

    def _bind(self):
        st = self._st
        for name in ("f", "f0", "f1", "F", "rho", "u", "force", "Q"):
            setattr(st, name, getattr(self, name).ctypes.data)

    def set_lagrangian(self, s, u_s, epsilon=None):
        s = np.ascontiguousarray(s, dtype=np.float32)
        u_s = np.ascontiguousarray(u_s, dtype=np.float32)
        ns = s.size // 2
        eps = np.ones(ns, dtype=np.int32) if epsilon is None else np.ascontiguousarray(epsilon, dtype=np.int32)
        if self.F_s.size != 2 * ns:
            self.F_s = np.zeros(2 * ns, dtype=np.float32)
        self._pts = (s, u_s, eps)
        st = self._st
        st.Ns = ns
        st.s, st.u_s, st.F_s, st.epsilon = s.ctypes.data, u_s.ctypes.data, self.F_s.ctypes.data, eps.ctypes.data

    def step(self, n: int = 1):
        load().oracle_run(C.byref(self._st), self.it, int(n))
        self.it += int(n)

    @property
    def flux(self) -> float:
        return float(self.Q[0])

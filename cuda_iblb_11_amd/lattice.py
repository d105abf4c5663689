"""Host-side mirror of the fused context API (include/iblb.h, part 2).

`Lattice` owns one x-slab of a D2Q9 channel on one GPU and advances the reference time step
(main.cu:852-909: equilibrium -> collision -> streaming -> macro -> interpolate -> spread).
Arrays crossing this boundary are numpy arrays in the reference layouts restricted to the
slab: rho[N], u[2N] (u_x block then u_y block), force[2N], f[9N] AoS (f[9*j+i]),
j = y * x_count + (x - x_begin); Lagrangian s/u_s interleaved float32 xy, epsilon int32.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass

import numpy as np

from . import _lib as L


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ---- reference parameter derivation (main.cu:296-321) -------------------------------------

C_S_DRIVER = 0.577  # main.cu:27 (the kernels use 0.57735, LatticeBoltzmann.cu:11)
LENGTH = 96         # main.cu:279
YDIM_REF = 192      # main.cu:271


@dataclass
class RefParams:
    """Derived run parameters of the reference driver for its 10 positional arguments."""
    c_fraction: int
    c_num: int
    c_space: int
    Re: float
    T_num: float
    T_pow: int
    I_pow: float
    P_num: int
    ShARC: bool
    BigData: bool

    @property
    def XDIM(self) -> int:  # main.cu:298
        return self.c_num * self.c_space

    @property
    def YDIM(self) -> int:
        return YDIM_REF

    @property
    def T(self) -> int:  # main.cu:299
        return int(np.rint(np.float32(self.T_num) * 10.0 ** self.T_pow))

    @property
    def ITERATIONS(self) -> int:  # main.cu:300 (unsigned int = T * float I_pow, truncated)
        return int(self.T * np.float32(self.I_pow))

    @property
    def INTERVAL(self) -> int:  # main.cu:301
        return self.ITERATIONS // self.P_num

    @property
    def SPEED(self) -> float:  # main.cu:314
        return 0.8 * 1000 / self.T

    @property
    def TAU(self) -> float:  # main.cu:320
        return (self.SPEED * LENGTH) / (self.Re * C_S_DRIVER * C_S_DRIVER) + 1. / 2.

    @property
    def TAU2(self) -> float:  # main.cu:321
        return 1. / (12. * (self.TAU - (1. / 2.))) + (1. / 2.)


def reference_taus(Re: float = 1.0, T: int = 100000) -> tuple[float, float]:
    """TAU, TAU2 of main.cu:314-321 for a Reynolds number and beat period."""
    speed = 0.8 * 1000 / T
    tau = (speed * LENGTH) / (Re * C_S_DRIVER * C_S_DRIVER) + 0.5
    return tau, 1. / (12. * (tau - 0.5)) + 0.5


def plan_slabs(nx: int, n: int) -> list[tuple[int, int]]:
    """x-slab decomposition: n contiguous column ranges covering [0, nx) in order."""
    if n < 1 or n > nx:
        raise ValueError(f"cannot split {nx} columns into {n} slabs")
    edges = [(r * nx) // n for r in range(n + 1)]
    return [(edges[r], edges[r + 1] - edges[r]) for r in range(n)]


class Lattice:
    """One slab (or the whole lattice) on one GPU, behind the C ABI."""

    def __init__(self, nx: int, ny: int, tau: float | None = None, tau2: float | None = None, *,
                 precision: str = "f64", body_force=(0.0, 0.0), flux_norm: float = 192.0,
                 flux_column: int | None = None, device: int = 0, x_begin: int = 0, x_count: int = 0,
                 max_points: int = 0, lib=None):
        lib = lib or L.load()
        self._lib = lib
        cfg = L.Config()
        L.check(lib.iblb_config_default(C.byref(cfg)))
        if tau is None:
            tau, tau2 = reference_taus()
        cfg.nx, cfg.ny = int(nx), int(ny)
        cfg.tau, cfg.tau2 = float(tau), float(tau2)
        if precision not in ("f64", "f32"):
            raise ValueError("precision must be 'f64' or 'f32'")
        cfg.precision = L.PREC_F64 if precision == "f64" else L.PREC_F32
        cfg.body_force[0], cfg.body_force[1] = float(body_force[0]), float(body_force[1])
        cfg.flux_norm = float(flux_norm)
        cfg.flux_column = int(nx) - 5 if flux_column is None else int(flux_column)
        cfg.device = int(device)
        cfg.x_begin, cfg.x_count = int(x_begin), int(x_count)
        cfg.max_points = int(max_points)
        h = C.c_void_p()
        rc = lib.iblb_create(C.byref(cfg), C.byref(h))
        L.check(rc, None, lib)
        self._h = h
        self.nx, self.ny = int(nx), int(ny)
        self.x_begin = int(x_begin) if x_count > 0 else 0
        self.x_count = int(x_count) if x_count > 0 else int(nx)
        self.N = self.x_count * self.ny
        self.precision = precision
        self.max_points = int(max_points)
        self.ns = 0

    # -- lifecycle ------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.iblb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int) -> None:
        L.check(rc, self._h, self._lib)

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # -- state ------------------------------------------------------------------------------
    def set_state(self, rho=None, u=None, f=None, force=None) -> None:
        def arr(a, n):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=np.float64)
            if a.size != n:
                raise ValueError(f"expected {n} values, got {a.size}")
            return a
        rho, u = arr(rho, self.N), arr(u, 2 * self.N)
        f, force = arr(f, 9 * self.N), arr(force, 2 * self.N)
        if (rho is None) != (u is None):
            rho = np.ones(self.N) if rho is None else rho
            u = np.zeros(2 * self.N) if u is None else u
        self._check(self._lib.iblb_set_state(self._h, _ptr(rho), _ptr(u), _ptr(f), _ptr(force)))

    def set_lagrangian(self, s, u_s, epsilon=None) -> None:
        s = np.ascontiguousarray(s, dtype=np.float32).ravel()
        u_s = np.ascontiguousarray(u_s, dtype=np.float32).ravel()
        ns = s.size // 2
        if u_s.size != 2 * ns:
            raise ValueError("s and u_s must both hold 2*Ns values")
        eps = None if epsilon is None else np.ascontiguousarray(epsilon, dtype=np.int32).ravel()
        self._check(self._lib.iblb_set_lagrangian(self._h, ns, _ptr(s), _ptr(u_s), _ptr(eps)))
        self.ns = ns

    def set_lagrangian_steps(self, s, u_s, epsilon=None) -> None:
        """Points of the next n iterations given ahead (iblb_set_lagrangian_steps): s, u_s of
        shape (n, 2*Ns) (float32 xy), epsilon (n, Ns) or None; iteration steps+i uses row i."""
        s = np.ascontiguousarray(s, dtype=np.float32)
        u_s = np.ascontiguousarray(u_s, dtype=np.float32)
        if s.ndim != 2 or s.shape != u_s.shape or s.shape[1] % 2:
            raise ValueError("s and u_s must both have shape (nsteps, 2*Ns)")
        n, ns = s.shape[0], s.shape[1] // 2
        eps = None
        if epsilon is not None:
            eps = np.ascontiguousarray(epsilon, dtype=np.int32)
            if eps.shape != (n, ns):
                raise ValueError("epsilon must have shape (nsteps, Ns)")
        self._check(self._lib.iblb_set_lagrangian_steps(self._h, n, ns, _ptr(s), _ptr(u_s), _ptr(eps)))
        self.ns = ns

    def set_cilia(self, c_num: int, c_space: float, T: int, p_step: int) -> None:
        """Run the reference's cilia kinematics on the device every iteration (main.cu:822-841);
        c_num = 0 switches it off.  Needs max_points >= 96 * c_num."""
        k = L.Cilia(int(c_num), float(c_space), int(T), int(p_step))
        self._check(self._lib.iblb_set_cilia(self._h, C.byref(k)))
        self.ns = 96 * int(c_num) if c_num > 0 else 0

    def lagrangian(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Current Lagrangian points: s [2Ns], u_s [2Ns] (float32), epsilon [Ns] (int32)."""
        s = np.zeros(2 * self.ns, dtype=np.float32)
        us = np.zeros(2 * self.ns, dtype=np.float32)
        eps = np.zeros(self.ns, dtype=np.int32)
        self._check(self._lib.iblb_get_lagrangian(self._h, _ptr(s), _ptr(us), _ptr(eps)))
        return s, us, eps

    def step(self, n: int = 1) -> None:
        self._check(self._lib.iblb_step(self._h, int(n)))

    # -- readers ----------------------------------------------------------------------------
    def macro(self) -> tuple[np.ndarray, np.ndarray]:
        rho = np.empty(self.N)
        u = np.empty(2 * self.N)
        self._check(self._lib.iblb_get_macro(self._h, _ptr(rho), _ptr(u)))
        return rho, u

    def populations(self) -> np.ndarray:
        f = np.empty(9 * self.N)
        self._check(self._lib.iblb_get_populations(self._h, _ptr(f)))
        return f

    def force(self) -> np.ndarray:
        out = np.empty(2 * self.N)
        self._check(self._lib.iblb_get_force(self._h, _ptr(out)))
        return out

    def lagrangian_force(self) -> np.ndarray:
        out = np.zeros(2 * self.ns, dtype=np.float32)
        self._check(self._lib.iblb_get_lagrangian_force(self._h, _ptr(out)))
        return out

    @property
    def flux(self) -> float:
        q = C.c_double(0.0)
        self._check(self._lib.iblb_get_flux(self._h, C.byref(q)))
        return q.value

    @property
    def steps(self) -> int:
        n = C.c_longlong(0)
        self._check(self._lib.iblb_get_step(self._h, C.byref(n)))
        return n.value

    def count_nonfinite(self) -> int:
        """NaN / Inf stored populations of the current state (whole lattice; collective in an
        RCCL group)."""
        n = C.c_longlong(0)
        self._check(self._lib.iblb_count_nonfinite(self._h, C.byref(n)))
        return n.value

    # -- timing -----------------------------------------------------------------------------
    def set_profiling(self, on=True) -> None:
        """True / 1: events around every launch; 2: only the deep launches, by their own signals
        (include/iblb.h iblb_set_profiling); False / 0: off."""
        mode = 2 if (not isinstance(on, bool) and on == 2) else (1 if on else 0)
        self._check(self._lib.iblb_set_profiling(self._h, mode))

    def timing(self, reset: bool = False) -> dict:
        t = L.Timing()
        self._check(self._lib.iblb_get_timing_ex(self._h, C.byref(t), C.sizeof(t), 1 if reset else 0))
        return {k: getattr(t, k) for k, _ in L.Timing._fields_}

    @property
    def stream(self) -> int:
        s = C.c_void_p()
        self._check(self._lib.iblb_get_stream(self._h, C.byref(s)))
        return s.value or 0

    def synchronize(self) -> None:
        self._check(self._lib.iblb_synchronize(self._h))

    # -- checkpoint / restart -------------------------------------------------------------------
    def save_checkpoint(self, path) -> None:
        self._check(self._lib.iblb_save_checkpoint(self._h, os.fsencode(path)))

    def load_checkpoint(self, path) -> None:
        self._check(self._lib.iblb_load_checkpoint(self._h, os.fsencode(path)))
        self.ns = int(np.fromfile(path, dtype=np.int64, count=9, offset=8)[7])

    # -- RCCL group ---------------------------------------------------------------------------
    def attach_rccl(self, unique_id: bytes, nranks: int, rank: int) -> None:
        if len(unique_id) != L.UNIQUE_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        self._check(self._lib.iblb_attach_rccl(self._h, unique_id, int(nranks), int(rank)))
        self.rank = int(rank)

    def set_wait_timeout(self, seconds: float) -> None:
        """Bound of the group's device-side waits (include/iblb.h iblb_set_wait_timeout; default
        600 s): a neighbour late by less changes nothing, a longer stall fails the call."""
        self._check(self._lib.iblb_set_wait_timeout(self._h, float(seconds)))

    def gather_macro(self, root: int = 0):
        """Whole-lattice rho [nx*ny], u [2*nx*ny] on rank `root` (None elsewhere); collective."""
        n = self.nx * self.ny
        rho, u = np.empty(n), np.empty(2 * n)
        self._check(self._lib.iblb_gather_macro(self._h, int(root), _ptr(rho), _ptr(u)))
        return (rho, u) if getattr(self, "rank", 0) == int(root) else (None, None)


def rccl_unique_id(lib=None) -> bytes:
    lib = lib or L.load()
    buf = C.create_string_buffer(L.UNIQUE_ID_BYTES)
    L.check(lib.iblb_rccl_unique_id(buf), None, lib)
    return buf.raw


class LocalGroup:
    """Slabs of one process linked left to right (synchronous transport, for testing)."""

    def __init__(self, slabs: list[Lattice]):
        self.slabs = list(slabs)
        self._lib = self.slabs[0]._lib
        self._arr = (C.c_void_p * len(self.slabs))(*[s.handle for s in self.slabs])
        L.check(self._lib.iblb_link_local(self._arr, len(self.slabs)), self.slabs[0].handle, self._lib)

    def step(self, n: int = 1) -> None:
        rc = self._lib.iblb_group_step(self._arr, len(self.slabs), int(n))
        if rc != L.IBLB_OK:
            for s in self.slabs:
                msg = self._lib.iblb_last_error(s.handle)
                if msg:
                    raise L.IblbError(rc, msg.decode())
            L.check(rc, None, self._lib)

    def gather_macro(self) -> tuple[np.ndarray, np.ndarray]:
        """rho[N], u[2N] of the whole lattice in the reference layout."""
        ny = self.slabs[0].ny
        nx = self.slabs[0].nx
        rho = np.empty((ny, nx))
        u = np.empty((2, ny, nx))
        for s in self.slabs:
            r, uu = s.macro()
            rho[:, s.x_begin:s.x_begin + s.x_count] = r.reshape(ny, s.x_count)
            u[:, :, s.x_begin:s.x_begin + s.x_count] = uu.reshape(2, ny, s.x_count)
        return rho.ravel(), u.reshape(2, -1).ravel()

    @property
    def flux(self) -> float:
        return math.fsum(s.flux for s in self.slabs)


def split_state(arr: np.ndarray, ncomp: int, nx: int, ny: int, x_begin: int, x_count: int) -> np.ndarray:
    """Slice a whole-lattice reference-layout field (SoA with ncomp blocks) to one slab."""
    a = np.asarray(arr).reshape(ncomp, ny, nx)[:, :, x_begin:x_begin + x_count]
    return np.ascontiguousarray(a).ravel()


def split_populations(f: np.ndarray, nx: int, ny: int, x_begin: int, x_count: int) -> np.ndarray:
    """Slice whole-lattice AoS populations f[9*j+i] to one slab."""
    a = np.asarray(f).reshape(ny, nx, 9)[:, x_begin:x_begin + x_count, :]
    return np.ascontiguousarray(a).ravel()

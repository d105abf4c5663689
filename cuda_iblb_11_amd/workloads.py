"""Synthetic workloads of BASELINE.json / SURVEY.md §8(d), shared by tests and bench.py.

Channel = the reference boundary set (periodic x, half-way bounce-back at y=0, same-cell
mirror at y=YDIM-1), x fastest in the reference layout.  Relaxation times are the
reference defaults (Re=1, T=1e5: TAU=2.806798, TAU2=0.536125, main.cu:314-321).
"""
from __future__ import annotations

import numpy as np

from .lattice import reference_taus

TAU, TAU2 = reference_taus()
SEED = 12345
BODY_FORCE = (1e-6, 0.0)

CONFIGS = {
    # name: (nx, ny, precision, ib)
    "K1": (128, 128, "f64", False),
    "K2": (2048, 2048, "f64", False),
    "K3": (2048, 2048, "f64", True),
    "K4": (8192, 2048, "f64", False),
    "K5": (8192, 2048, "f32", True),
    "M": (4096, 4096, "f64", False),
}


def perturbed_state(nx: int, ny: int, seed: int = SEED, amp: float = 1e-3):
    """rho = 1 + amp*xi, u = amp*(xi_x, xi_y), xi ~ U(-1, 1); reference layout."""
    rng = np.random.default_rng(seed)
    n = nx * ny
    rho = 1.0 + amp * rng.uniform(-1.0, 1.0, n)
    u = amp * rng.uniform(-1.0, 1.0, 2 * n)
    return rho, u


def column_state(nx: int, ny: int, seed: int = SEED, amp: float = 1e-3):
    """x-uniform perturbed state (every column identical): used for size-independent checks."""
    rng = np.random.default_rng(seed)
    r = 1.0 + amp * rng.uniform(-1.0, 1.0, ny)
    ux = amp * rng.uniform(-1.0, 1.0, ny)
    uy = amp * rng.uniform(-1.0, 1.0, ny)
    rho = np.repeat(r, nx)
    u = np.concatenate([np.repeat(ux, nx), np.repeat(uy, nx)])
    return rho, u


def filament(it: int, n_points: int = 256, x0: float = 1024.0, y0: float = 1.0, dy: float = 1.0,
             U0: float = 1e-3, period: int = 1000, sway: float = 0.0):
    """Single prescribed filament (config K3): a vertical line of points at x0 (+ sway), spacing dy,
    velocity u_s = (U0 * (k/(n-1)) * sin(2 pi it/period), 0), epsilon = 1.
    dy = 1 is the reference's own discretisation (96 points per 96-cell cilium, main.cu:158-170);
    at dy = 0.5 the reference's penalty forcing (F_s = 2 delta rho (u_s - u)) over-corrects and
    the run diverges within ~100 steps (checked with the oracle)."""
    k = np.arange(n_points, dtype=np.float64)
    ph = 2.0 * np.pi * it / period
    xs = x0 + sway * (k / max(n_points - 1, 1)) * np.sin(ph)
    ys = y0 + dy * k
    s = np.empty(2 * n_points, dtype=np.float32)
    s[0::2], s[1::2] = xs, ys
    us = np.zeros(2 * n_points, dtype=np.float32)
    us[0::2] = U0 * (k / max(n_points - 1, 1)) * np.sin(ph)
    eps = np.ones(n_points, dtype=np.int32)
    return s, us, eps


def filament_array(it: int, nx: int, n_fil: int = 64, pts: int = 96, dy: float = 1.0, U0: float = 1e-3,
                   period: int = 1000, x_offset: float = 0.5):
    """Array of n_fil prescribed filaments evenly spaced in x with a metachronal phase lag
    (config K5 stand-in for the reference's cilia; 64 x 96 = 6144 points).  Filament m stands at
    x = (m + x_offset) * nx / n_fil and tilts by up to 8 columns; x_offset = 0 (config K5 as
    BASELINE.json states it, "filaments spanning slab boundaries") puts one on every edge of an
    x-slab decomposition into 1, 2, 4 or 8 slabs (x = 0 included), and positions are wrapped into
    [0, XDIM) like the reference's boundary_check (main.cu:193-196)."""
    s_all, u_all = [], []
    space = nx / n_fil
    for m in range(n_fil):
        k = np.arange(pts, dtype=np.float64)
        ph = 2.0 * np.pi * (it + m * period / n_fil) / period
        tilt = (k / pts) ** 2 * 8.0 * np.sin(ph)
        xs = np.mod((m + x_offset) * space + tilt, nx)
        ys = 1.0 + dy * k
        s = np.empty(2 * pts)
        s[0::2], s[1::2] = xs, ys
        us = np.zeros(2 * pts)
        us[0::2] = U0 * (k / pts) ** 2 * np.cos(ph)
        s_all.append(s)
        u_all.append(us)
    s = np.concatenate(s_all).astype(np.float32)
    us = np.concatenate(u_all).astype(np.float32)
    return s, us, np.ones(s.size // 2, dtype=np.int32)

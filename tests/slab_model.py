"""Numpy model of the slab-decomposed step the HIP path implements (pull streaming with
one-column halos; with IB a three-column halo so that every slab computes the nodes of the
points that spread into it by itself; spread clipped to owned columns).
TEST INFRASTRUCTURE: used by the CPU tests to check (a) that the pull form equals the
reference's push streaming and (b) that the x-slab decomposition with the halo and IB
exchange schedule of iblb_ctx.hip reproduces the single-domain reference step bit for bit.
Per-cell arithmetic is delegated to the oracle's C kernels so that only the data movement
is modelled here.
"""
from __future__ import annotations

import numpy as np

C_L = np.array([[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]])
LEFT_PLANES = (1, 5, 8)   # cx = +1: come from the left neighbour's last column
RIGHT_PLANES = (3, 6, 7)  # cx = -1: come from the right neighbour's first column
BOUNCE = {2: 4, 5: 7, 6: 8}   # y = 0:      f[k] <- g[same cell, BOUNCE[k]]
MIRROR = {4: 2, 8: 5, 7: 6}   # y = Y - 1:  f[k] <- g[same cell, MIRROR[k]]


def pull(g: np.ndarray, halo_left: np.ndarray, halo_right: np.ndarray) -> np.ndarray:
    """g: (ny, ncol, 9) post-collision populations of a slab; halo_left (ny, 3) = planes
    (1,5,8) of column -1; halo_right (ny, 3) = planes (3,6,7) of column ncol.
    Returns post-stream f (ny, ncol, 9)."""
    ny, ncol, _ = g.shape
    f = np.empty_like(g)
    for k in range(9):
        cx, cy = C_L[k]
        left = halo_left[:, LEFT_PLANES.index(k)] if k in LEFT_PLANES else np.zeros(ny)
        right = halo_right[:, RIGHT_PLANES.index(k)] if k in RIGHT_PLANES else np.zeros(ny)
        ext = np.concatenate([left[:, None], g[:, :, k], right[:, None]], axis=1)
        src = ext[:, 1 - cx:1 - cx + ncol]
        out = np.empty((ny, ncol))
        if cy == 0:
            out[:] = src
        elif cy == 1:
            out[1:] = src[:-1]
            out[0] = g[0, :, BOUNCE[k]]
        else:
            out[:-1] = src[1:]
            out[-1] = g[ny - 1, :, MIRROR[k]]
        f[:, :, k] = out
    return f


def periodic_halos(g: np.ndarray):
    return g[:, -1, list(LEFT_PLANES)], g[:, 0, list(RIGHT_PLANES)]


def pull_periodic(g_aos: np.ndarray, nx: int, ny: int) -> np.ndarray:
    g = g_aos.reshape(ny, nx, 9)
    hl, hr = periodic_halos(g)
    return pull(g, hl, hr).ravel()


class SlabRank:
    """One rank of the decomposed step.  `exchange(send_right, send_left)` must return
    (halo_left, halo_right) from the neighbours; `allreduce(x)` sums over ranks."""

    def __init__(self, O, nx, ny, x_begin, x_count, tau, tau2, rho, u, body_force=(0.0, 0.0),
                 flux_column=None, flux_norm=192.0):
        self.O = O
        self.nx, self.ny, self.xb, self.nc = nx, ny, x_begin, x_count
        self.tau, self.tau2 = tau, tau2
        n = x_count * ny
        self.n = n
        self.bf = body_force
        self.rho = np.array(rho, dtype=np.float64)
        self.u = np.array(u, dtype=np.float64)
        self.force = np.zeros(2 * n)
        self.force[:n] += body_force[0]
        self.force[n:] += body_force[1]
        self.f = O.feq(self.rho, self.u, x_count, ny, tau)
        self.g = np.zeros(9 * n)
        self.Q = 0.0
        self.fc = (nx - 5 if flux_column is None else flux_column) - x_begin
        self.flux_norm = flux_norm

    def collide(self):
        O, n = self.O, self.n
        f0, F = np.zeros(9 * n), np.zeros(9 * n)
        O.equilibrium(self.u, self.rho, f0, self.force, F, self.nc, self.ny, self.tau)
        O.collision(f0, self.f, self.g, F, self.tau, self.tau2, self.nc, self.ny, 0)

    def boundary(self):
        g = self.g.reshape(self.ny, self.nc, 9)
        return g[:, -1, list(LEFT_PLANES)].copy(), g[:, 0, list(RIGHT_PLANES)].copy()

    def stream_macro(self, halo_left, halo_right):
        O, n = self.O, self.n
        self.f = pull(self.g.reshape(self.ny, self.nc, 9), halo_left, halo_right).ravel()
        O.macro(self.f, self.u, self.rho, self.nc, self.ny)

    # -- IB halo: columns -3..-1 and ncol..ncol+2 of g from the neighbours -------------------
    def boundary_ext(self):
        """(to the right neighbour, to the left neighbour): my last / first three columns of g
        (ny, 3, 9).  The HIP path sends only the 21 planes of them that are read."""
        g = self.g.reshape(self.ny, self.nc, 9)
        return g[:, -3:, :].copy(), g[:, :3, :].copy()

    def stream_macro_ext(self, left3, right3):
        """Post-stream f and macro of the own columns (as stream_macro) plus rho, u_raw of
        the node columns -2..ncol+1 (self.ext_rho / self.ext_u, column index + 2)."""
        g = self.g.reshape(self.ny, self.nc, 9)
        ext = np.concatenate([left3, g, right3], axis=1)          # columns -3 .. ncol+2
        z = np.zeros((self.ny, 3))
        fe = pull(ext, z, z)[:, 1:-1, :]                           # valid: columns -2 .. ncol+1
        self.f = np.ascontiguousarray(fe[:, 2:2 + self.nc, :]).ravel()
        self.O.macro(self.f, self.u, self.rho, self.nc, self.ny)
        ne = self.nc + 4
        self.ext_rho, self.ext_u = np.zeros(ne * self.ny), np.zeros(2 * ne * self.ny)
        self.O.macro(np.ascontiguousarray(fe).ravel(), self.ext_u, self.ext_rho, ne, self.ny)

    def processes(self, s, k) -> bool:
        """Does point k spread into this slab (its 3x3 columns, clipped to the lattice)?"""
        x0 = int(np.rint(np.float64(s[2 * k])))
        return any(0 <= x < self.nx and self.xb <= x < self.xb + self.nc for x in (x0 - 1, x0, x0 + 1))

    def owns(self, s, k) -> bool:
        """The slab holding column min(x0, nx-1) reports F_s of point k (every point spreads
        there, given the reference's invariant 0 <= x0 <= XDIM)."""
        x = min(int(np.rint(np.float64(s[2 * k]))), self.nx - 1)
        return self.xb <= x < self.xb + self.nc

    def node_values(self, s):
        """(rho, u_x, u_y) at the 3x3 nodes of every point this slab processes, from the
        node columns of the IB halo; zeros for the other points."""
        ns = s.size // 2
        nv = np.zeros((ns, 9, 3))
        size = self.nx * self.ny
        ne = self.nc + 4
        for k in range(ns):
            if not self.processes(s, k):
                continue
            x0, y0 = int(np.rint(np.float64(s[2 * k]))), int(np.rint(np.float64(s[2 * k + 1])))
            for i in range(9):
                j = (y0 + C_L[i, 1]) * self.nx + (x0 + C_L[i, 0])
                if j < 0 or j >= size:
                    continue
                xj, yj = j % self.nx, j // self.nx
                xl = xj - self.xb       # flat-index node -> slab-local column, periodic
                if xl < -2:
                    xl += self.nx
                elif xl > self.nc + 1:
                    xl -= self.nx
                assert -2 <= xl <= self.nc + 1
                je = yj * ne + xl + 2
                nv[k, i] = (self.ext_rho[je], self.ext_u[je], self.ext_u[ne * self.ny + je])
        return nv

    def interp(self, s, u_s, nv):
        """ImmersedBoundary.cu:104-129 from the summed node values (float accumulation)."""
        ns = s.size // 2
        F_s = np.zeros(2 * ns, dtype=np.float32)
        size = self.nx * self.ny
        for k in range(ns):
            x0, y0 = int(np.rint(np.float64(s[2 * k]))), int(np.rint(np.float64(s[2 * k + 1])))
            fx, fy = np.float32(0), np.float32(0)
            for i in range(9):
                x, y = x0 + C_L[i, 0], y0 + C_L[i, 1]
                if not (0 <= y * self.nx + x < size):
                    continue
                d = np.float64(self.O.d_delta(float(s[2 * k]), float(s[2 * k + 1]), int(x), int(y)))
                r, ux, uy = nv[k, i]
                fx = np.float32(np.float64(fx) + 2.0 * (1.0 * 1.0 * d) * r * (np.float64(u_s[2 * k]) - ux))
                fy = np.float32(np.float64(fy) + 2.0 * (1.0 * 1.0 * d) * r * (np.float64(u_s[2 * k + 1]) - uy))
            F_s[2 * k], F_s[2 * k + 1] = fx, fy
        return F_s

    def spread(self, s, F_s, eps):
        """Point-centric spread clipped to the owned columns, then u correction and flux."""
        n, nc = self.n, self.nc
        force = np.zeros(2 * n)
        for k in range(s.size // 2):
            x0, y0 = int(np.rint(np.float64(s[2 * k]))), int(np.rint(np.float64(s[2 * k + 1])))
            for i in range(9):
                x, y = x0 + C_L[i, 0], y0 + C_L[i, 1]
                if x < 0 or x >= self.nx or y < 0 or y >= self.ny or not (self.xb <= x < self.xb + nc):
                    continue
                d = np.float32(self.O.d_delta(float(s[2 * k]), float(s[2 * k + 1]), int(x), int(y)))
                if d == 0:
                    continue
                jl = y * nc + (x - self.xb)
                force[jl] += np.float64(np.float32(F_s[2 * k] * d)) * 1.0 * eps[k]
                force[n + jl] += np.float64(np.float32(F_s[2 * k + 1] * d)) * 1.0 * eps[k]
        force[:n] += self.bf[0]
        force[n:] += self.bf[1]
        self.force = force
        self.correct_u()

    def no_ib(self):
        n = self.n
        self.force = np.zeros(2 * n)
        self.force[:n] = self.bf[0]
        self.force[n:] = self.bf[1]
        self.correct_u()

    def correct_u(self):
        """ImmersedBoundary.cu:249-264 (same term order as the restatement) + flux."""
        f = self.f.reshape(-1, 9)
        n = self.n
        ux = (0.0 * f[:, 0] + 1.0 * f[:, 1] + 0.0 * f[:, 2] + -1.0 * f[:, 3] + 0.0 * f[:, 4] + 1.0 * f[:, 5]
              + -1.0 * f[:, 6] + -1.0 * f[:, 7] + 1.0 * f[:, 8] + 0.5 * self.force[:n]) / self.rho
        uy = (0.0 * f[:, 1] + 0.0 * f[:, 1] + 1.0 * f[:, 2] + 0.0 * f[:, 3] + -1.0 * f[:, 4] + 1.0 * f[:, 5]
              + 1.0 * f[:, 6] + -1.0 * f[:, 7] + -1.0 * f[:, 8] + 0.5 * self.force[n:]) / self.rho
        self.u[:n], self.u[n:] = ux, uy
        if 0 <= self.fc < self.nc:
            for y in range(self.ny):
                self.Q += self.u[y * self.nc + self.fc] / self.flux_norm

"""A plain float32 restatement of the no-IB channel iteration (test infrastructure): the f32
accuracy floor the GPU's f32 path is judged against.

The oracle's step (oracle/oracle.c oracle_step: equilibrium, TRT collision, push streaming with
the reference's boundary flags, macro + u correction; LatticeBoltzmann.cu:30-411,
ImmersedBoundary.cu:249-255) written in numpy with every array in float32 and the populations
stored as deviations h = f - w_i, the storage the GPU's f32 path uses.  It shares no code and no
operation order with the kernels; its distance from the f64 oracle after n iterations is what an
f32 implementation of the reference algorithm gets, so a GPU f32 error of the same size is the
precision's floor, not a defect.
"""
from __future__ import annotations

import numpy as np

C_S = np.float32(0.57735)  # LatticeBoltzmann.cu:11
CX = np.array([0, 1, 0, -1, 0, 1, -1, -1, 1])
CY = np.array([0, 0, 1, 0, -1, 1, 1, -1, -1])
W = np.array([4 / 9] + [1 / 9] * 4 + [1 / 36] * 4, dtype=np.float32)
PAIRS = ((1, 3), (2, 4), (5, 7), (6, 8))


class F32Channel:
    """State in the reference layout (x fastest): h[i, y, x] deviations, rho, u, force."""

    def __init__(self, nx, ny, tau, tau2, rho, u, body_force):
        f32 = np.float32
        self.nx, self.ny = nx, ny
        self.op, self.om = f32(1 / tau), f32(1 / tau2)
        self.kg = f32(1.0 - 1.0 / (2.0 * tau))
        n = nx * ny
        rho = np.asarray(rho, dtype=np.float64).reshape(ny, nx)
        u = np.asarray(u, dtype=np.float64)
        self.drho = (rho - 1.0).astype(f32)
        self.rho = rho.astype(f32)
        self.ux = u[:n].reshape(ny, nx).astype(f32)
        self.uy = u[n:].reshape(ny, nx).astype(f32)
        self.Fx, self.Fy = f32(body_force[0]), f32(body_force[1])
        self.h = self._feq_dev()  # main.cu:720-754: f = f0 of the initial state

    def _feq_dev(self):
        cs2 = C_S * C_S
        usq = self.ux * self.ux + self.uy * self.uy
        h = np.empty((9, self.ny, self.nx), dtype=np.float32)
        for i in range(9):
            cu = self.ux * np.float32(CX[i]) + self.uy * np.float32(CY[i])
            shape = cu / cs2 + cu * cu / (np.float32(2) * cs2 * cs2) - usq / (np.float32(2) * cs2)
            h[i] = W[i] * (self.drho + self.rho * shape)  # rho w (1 + shape) - w
        return h

    def _guo(self):
        cs2 = C_S * C_S
        F = np.empty((9, self.ny, self.nx), dtype=np.float32)
        for i in range(9):
            cx, cy = np.float32(CX[i]), np.float32(CY[i])
            cu = cx * self.ux + cy * self.uy
            vx = (cx - self.ux) / cs2 + cu / (cs2 * cs2) * cx
            vy = (cy - self.uy) / cs2 + cu / (cs2 * cs2) * cy
            F[i] = self.kg * W[i] * (vx * self.Fx + vy * self.Fy)
        return F

    def step(self, n=1):
        half = np.float32(0.5)
        for _ in range(n):
            h0, F, h = self._feq_dev(), self._guo(), self.h
            h1 = np.empty_like(h)
            h1[0] = h[0] - self.op * (h[0] - h0[0])
            for a, b in PAIRS:
                hp, hm = (h[a] + h[b]) * half, (h[a] - h[b]) * half
                gp, gm = (h0[a] + h0[b]) * half, (h0[a] - h0[b]) * half
                h1[a] = h[a] - self.op * (hp - gp) - self.om * (hm - gm) + F[a]
                h1[b] = h[b] - self.op * (hp - gp) + self.om * (hm - gm) + F[b]
            # push streaming: periodic x, bounce-back at y = 0, same-cell mirror at y = ny-1
            hn = np.empty_like(h)
            for i in range(9):
                src = np.roll(h1[i], CX[i], axis=1)
                if CY[i] == 0:
                    hn[i] = src
                elif CY[i] == 1:
                    hn[i, 1:] = src[:-1]
                else:
                    hn[i, :-1] = src[1:]
            for i, k in ((4, 2), (7, 5), (8, 6)):
                hn[k, 0] = h1[i, 0]
            for i, k in ((2, 4), (5, 8), (6, 7)):
                hn[k, -1] = h1[i, -1]
            self.h = hn
            self.drho = hn.sum(axis=0, dtype=np.float32)
            self.rho = np.float32(1) + self.drho
            mx = hn[1] - hn[3] + hn[5] - hn[6] - hn[7] + hn[8]
            my = hn[2] - hn[4] + hn[5] + hn[6] - hn[7] - hn[8]
            self.ux = (mx + half * self.Fx) / self.rho
            self.uy = (my + half * self.Fy) / self.rho

    def macro(self):
        # rho = 1 + (rho - 1): the deviation sum carries the density's digits (as on the GPU)
        return (1.0 + self.drho.astype(np.float64).ravel(),
                np.concatenate([self.ux.ravel(), self.uy.ravel()]).astype(np.float64))

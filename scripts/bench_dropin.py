#!/usr/bin/env python3
"""The reference's own unfused step on the MI355X: the drop-in kernels (iblb_equilibrium,
iblb_collision, iblb_streaming, iblb_macro + the u correction of iblb_spread with Ns = 0), launched
in the reference's order (main.cu:852-909) on AoS arrays, against the fused context on the same
lattice.  Shows what a kernel-by-kernel port would reach; one JSON line per path.

usage: bench_dropin.py [--nx 4096 --ny 4096 --steps 50]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--ny", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import torch
    import cuda_iblb_11_amd as P
    from cuda_iblb_11_amd import kernels as K
    from cuda_iblb_11_amd import workloads as W

    nx, ny, N = a.nx, a.ny, a.nx * a.ny
    dev = torch.device("cuda", 0)
    rho_h, u_h = W.perturbed_state(nx, ny, W.SEED)
    rho = torch.tensor(rho_h, device=dev)
    u = torch.tensor(u_h, device=dev)
    force = torch.zeros(2 * N, dtype=torch.float64, device=dev)
    force[:N] = W.BODY_FORCE[0]
    f0 = torch.empty(9 * N, dtype=torch.float64, device=dev)
    F = torch.empty_like(f0)
    f1 = torch.empty_like(f0)
    f = torch.empty_like(f0)
    Q = torch.zeros(1, dtype=torch.float64, device=dev)
    fs = torch.zeros(2, dtype=torch.float32, device=dev)
    eps = torch.ones(1, dtype=torch.int32, device=dev)
    K.equilibrium(u, rho, f, torch.zeros_like(force), F, nx, ny, W.TAU)

    def step():
        K.equilibrium(u, rho, f0, force, F, nx, ny, W.TAU)
        K.collision(f0, f, f1, F, W.TAU, W.TAU2, nx, ny)
        K.streaming(f1, f, nx, ny)
        K.macro(f, u, rho, nx, ny)
        # spread with no points: force = 0 + ... the reference zeroes force; keep the body force
        K.spread(rho, u, f, 0, fs, fs, force, fs, nx, Q, eps, YDIM=ny)
        force[:N] = W.BODY_FORCE[0]

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"path": "reference kernel sequence (drop-in, AoS, 6 launches + fill)", "nx": nx, "ny": ny,
                      "ms_per_step": dt * 1e3, "mlups": N / dt / 1e6}), flush=True)

    lat = P.Lattice(nx, ny, W.TAU, W.TAU2, body_force=W.BODY_FORCE)
    lat.set_state(rho_h, u_h)
    lat.step(10)
    lat.synchronize()
    t0 = time.perf_counter()
    lat.step(a.steps)
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"path": "fused context (1 launch)", "nx": nx, "ny": ny, "ms_per_step": dt * 1e3,
                      "mlups": N / dt / 1e6}), flush=True)


if __name__ == "__main__":
    main()

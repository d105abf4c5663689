#!/usr/bin/env python3
"""Diagnostic: the reference cilia scenario on the GPU (device kinematics and host-fed points)
against the oracle, step by step; prints the first iteration where they part."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cuda_iblb_11_amd as P  # noqa: E402
from cuda_iblb_11_amd import workloads as W  # noqa: E402
from oracle import oracle as O  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def main(T, steps):
    c_num, c_space = 6, 48.0
    nx, ny = 288, 192
    p_step = T // c_num
    sim = O.Simulation(nx, ny, W.TAU, W.TAU2)
    cil = O.Cilia(c_num, c_space, T, p_step, nx)
    dev = P.Lattice(nx, ny, W.TAU, W.TAU2, max_points=576)
    dev.set_state()
    dev.set_cilia(c_num, c_space, T, p_step)
    host = P.Lattice(nx, ny, W.TAU, W.TAU2, max_points=576)
    host.set_state()
    for it in range(steps):
        s, us, eps = cil.points(it)
        sim.set_lagrangian(s, us, eps)
        sim.step(1)
        host.set_lagrangian(s, us, eps)
        host.step(1)
        dev.step(1)
        sd, usd, ed = dev.lagrangian()
        rd, ud = dev.macro()
        rh, uh = host.macro()
        fd, fh = dev.force(), host.force()
        print(f"T={T} it={it} |u|max={np.abs(sim.u).max():.3e} pts_equal={np.array_equal(sd, s) and np.array_equal(usd, us)}"
              f" dev-vs-oracle u {rel(ud, sim.u):.2e} host-vs-oracle u {rel(uh, sim.u):.2e}"
              f" dev-vs-host u {rel(ud, uh):.2e} force dev/host {rel(fd, fh):.2e} host/oracle {rel(fh, sim.force):.2e}",
              flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]))

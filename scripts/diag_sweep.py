#!/usr/bin/env python3
"""Where does the two-iteration sweep differ from two one-step launches?  Prints the mismatching
(plane, x, y) cells after boot + one sweep (diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nx, ny, prec, env, steps):
    import cuda_iblb_11_amd as P
    from cuda_iblb_11_amd import workloads as W
    for k, v in env.items():
        os.environ[k] = v
    rho, u = W.perturbed_state(nx, ny, 6)
    lat = P.Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, body_force=(1e-6, 3e-7))
    lat.set_state(rho, u)
    lat.step(steps)
    f = lat.populations().reshape(ny, nx, 9)  # j = y*nx + x, [9j+i]
    lat.close()
    return f


def main():
    nx, ny = int(sys.argv[1]), int(sys.argv[2])
    prec = sys.argv[3] if len(sys.argv) > 3 else "f64"
    env = dict(kv.split("=") for kv in sys.argv[4:])
    for steps in (3, 5):
        ref = run(nx, ny, prec, {"IBLB_SWEEP": "0"}, steps)
        got = run(nx, ny, prec, dict(env, IBLB_SWEEP="1"), steps)
        d = np.abs(got - ref)
        bad = np.argwhere(d > 0)
        print(f"steps={steps} mismatches={len(bad)} of {d.size}, max {d.max():.3e}")
        ys = sorted(set(bad[:, 0].tolist()))
        xs = sorted(set(bad[:, 1].tolist()))
        ks = sorted(set(bad[:, 2].tolist()))
        print("  rows:", ys[:40], "..." if len(ys) > 40 else "")
        print("  cols:", xs[:40], "..." if len(xs) > 40 else "")
        print("  planes:", ks)
        for y, x, k in bad[:12]:
            print(f"   y={y} x={x} k={k} got={got[y, x, k]:.10f} ref={ref[y, x, k]:.10f}")


if __name__ == "__main__":
    main()

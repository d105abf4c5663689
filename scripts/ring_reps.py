#!/usr/bin/env python3
"""Repeatability of the slab cycle inside ONE process: a slab (optionally the
RCCL self ring, optionally with the K5 filament array) primed once, then REPS timed regions of
STEPS iterations each; prints one JSON line with the ms/iteration of every repetition and the
spread (max/min - 1).

usage: scripts/ring_reps.py NX NY PRECISION [--ring] [--k5 OFFSET] [--reps 7] [--steps 420] [--same-phase]

--same-phase (with --k5): every timed region gets the points of the same STEPS iterations of the
beat (the lattice state goes on), so the regions do the same work; without it the regions follow
the beat, whose filament tilt (up to 8 columns) changes the band plans from region to region.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("nx", type=int)
    p.add_argument("ny", type=int)
    p.add_argument("precision")
    p.add_argument("--ring", action="store_true")
    p.add_argument("--k5", type=float, default=None, help="K5 filaments (8 per 1024 columns) at this offset")
    p.add_argument("--reps", type=int, default=7)
    p.add_argument("--steps", type=int, default=420)
    p.add_argument("--same-phase", action="store_true")
    a = p.parse_args()
    import cuda_iblb_11_amd as P
    from cuda_iblb_11_amd import workloads as W
    pts = None
    ns = 0
    if a.k5 is not None:
        nf = max(1, round(64 * a.nx / 8192))
        pts = lambda it: W.filament_array(it, a.nx, n_fil=nf, pts=96, period=1000, x_offset=a.k5)
        ns = nf * 96
    lat = P.Lattice(a.nx, a.ny, W.TAU, W.TAU2, precision=a.precision, body_force=W.BODY_FORCE, max_points=ns)
    rho, u = W.perturbed_state(a.nx, a.ny, W.SEED)
    lat.set_state(rho, u)
    if a.ring:
        os.environ["IBLB_RCCL_SELF"] = "1"
        lat.attach_rccl(P.rccl_unique_id(), 1, 0)
    t = [0]

    def stage(n, t0=None):
        if pts is None:
            return
        t0 = t[0] if t0 is None else t0
        e = [pts(it) for it in range(t0, t0 + n)]
        lat.set_lagrangian_steps(np.stack([x[0] for x in e]), np.stack([x[1] for x in e]), np.stack([x[2] for x in e]))

    def run(n):
        stage(n)
        lat.step(n)
        t[0] += n

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:  # prime: the clock settles under load
        run(50)
    reps = []
    phase0 = t[0]
    for _ in range(a.reps):
        stage(a.steps, phase0 if a.same_phase else None)  # the points given ahead outside the timed region
        lat.synchronize()
        ts = time.perf_counter()
        lat.step(a.steps)
        t[0] += a.steps
        lat.synchronize()
        reps.append((time.perf_counter() - ts) / a.steps * 1e3)
    tm = lat.timing()
    print(json.dumps({"nx": a.nx, "ny": a.ny, "precision": a.precision, "ring": a.ring, "k5": a.k5,
                      "same_phase": a.same_phase,
                      "ms_per_iter": [round(r, 5) for r in reps], "min": round(min(reps), 5),
                      "median": round(float(np.median(reps)), 5), "spread": round(max(reps) / min(reps) - 1, 4),
                      "band_cycles": tm["band_cycles"], "band_merged_cycles": tm["band_merged_cycles"]}), flush=True)
    lat.close()


if __name__ == "__main__":
    main()

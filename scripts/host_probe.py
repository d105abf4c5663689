#!/usr/bin/env python3
"""Host-side cost of iblb_step (GPU-side diagnostics): for a workload, time the return of
lat.step(n) (host submission) and the completion after synchronize, per iteration.  If the
submission time is close to the total, the run is host-bound.

usage: host_probe.py NX NY PRECISION WORKLOAD(K3/K5/none) [frozen] [rccl-self]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import cuda_iblb_11_amd as P  # noqa: E402
from cuda_iblb_11_amd import workloads as W  # noqa: E402


def main():
    nx, ny, prec, wl = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    frozen = "frozen" in sys.argv[5:]
    ring = "rccl-self" in sys.argv[5:]
    kind = {"K3": "filament", "K5": "array"}.get(wl)
    points = bench.workload_points(kind, nx) if kind else None
    ns = 0 if points is None else points(0)[0].size // 2
    lat = P.Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, body_force=W.BODY_FORCE, max_points=ns)
    rho, u = W.perturbed_state(nx, ny, W.SEED)
    lat.set_state(rho, u)
    if ring:
        os.environ["IBLB_RCCL_SELF"] = "1"
        lat.attach_rccl(P.rccl_unique_id(), 1, 0)
    drv = bench.Driver(lat, points, frozen)
    for _ in range(20):
        drv.run(50)
    lat.synchronize()
    for n in (100, 500):
        drv.stage(n)
        t0 = time.perf_counter()
        drv.run(n, staged=True)
        t1 = time.perf_counter()
        lat.synchronize()
        t2 = time.perf_counter()
        print(f"{nx}x{ny} {prec} {wl} frozen={frozen} ring={ring} n={n}: submit {(t1 - t0) / n * 1e3:.4f} ms/it, "
              f"total {(t2 - t0) / n * 1e3:.4f} ms/it", flush=True)
    lat.close()


if __name__ == "__main__":
    main()

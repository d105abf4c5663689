#!/usr/bin/env python3
"""On-device cilia (the reference's kinematics, main.cu:822-841) per iteration: band cycle
(kinematics run ahead as a schedule) vs one fused launch per iteration (IBLB_IB_BAND=0) vs the
same lattice without IB.  The reference scenario's penalty IB diverges after ~40 iterations
(DESIGN.md §9); the timing does not depend on the values.  usage: r03_cilia.py c_num c_space ny steps"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (one HIP runtime per process)
import cuda_iblb_11_amd as P
from cuda_iblb_11_amd import workloads as W

c_num, c_space, ny, steps = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
prec = sys.argv[5] if len(sys.argv) > 5 else "f64"
nx, T = int(c_num * c_space), 100000
res = {"c_num": c_num, "c_space": c_space, "nx": nx, "ny": ny, "steps": steps, "precision": prec}
for name, band, cilia in (("band", "1", True), ("one_step", "0", True), ("no_ib", "1", False)):
    os.environ["IBLB_IB_BAND"] = band
    lat = P.Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, max_points=96 * c_num, body_force=W.BODY_FORCE)
    lat.set_state()
    if cilia:
        lat.set_cilia(c_num, c_space, T, T // c_num)
    lat.step(50)  # warm-up (and the clock ramp)
    t0 = time.perf_counter()
    lat.step(steps)
    dt = (time.perf_counter() - t0) / steps
    lat.set_profiling(True)  # launch counts of 20 more iterations (not timed)
    lat.step(20)
    tm = lat.timing()
    res[name] = {"ms_per_iteration": round(dt * 1e3, 5), "mlups": round(nx * ny / dt / 1e6),
                 "sweepk_launches": tm["sweepk_launches"], "fused_launches": tm["fused_launches"]}
    lat.close()
    print(name, res[name], flush=True)
print(json.dumps(res))

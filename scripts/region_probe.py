#!/usr/bin/env python3
"""Fixed cost of a short timed region (the driver's `bench.py --steps 20`): M 4096^2 f64, regions
of N iterations timed on the host (synchronize on both sides) against the summed deep-launch time
from HIP events, with profiling events on / off and with / without an idle gap before the region.
usage: scripts/region_probe.py [--precision f64] [--reps 8]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="f64")
    p.add_argument("--reps", type=int, default=8)
    a = p.parse_args()
    import torch
    import cuda_iblb_11_amd as P
    from cuda_iblb_11_amd import workloads as W
    n = 4096
    lat = P.Lattice(n, n, W.TAU, W.TAU2, precision=a.precision, body_force=W.BODY_FORCE)
    rho, u = W.perturbed_state(n, n, W.SEED)
    lat.set_state(rho, u)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        lat.step(30)
    out = {}
    for steps in (20, 60, 240):
        for prof in (True, False):
            for idle in (0.0, 0.002):
                host, dev = [], []
                for _ in range(a.reps):
                    lat.step(5)
                    lat.synchronize()
                    lat.set_profiling(prof)
                    lat.timing(reset=True)
                    torch.cuda.synchronize()
                    if idle:
                        time.sleep(idle)
                    ts = time.perf_counter()
                    lat.step(steps)
                    lat.synchronize()
                    torch.cuda.synchronize()
                    host.append((time.perf_counter() - ts) * 1e3)
                    tm = lat.timing(reset=True)
                    dev.append(tm["sweepk_ms"])
                host.sort()
                key = f"{steps} steps, events {'on' if prof else 'off'}, idle {idle * 1e3:.0f} ms"
                med = host[len(host) // 2]
                out[key] = {"host_ms_median": round(med, 4), "host_ms_min": round(host[0], 4),
                            "launch_ms_sum_median": round(sorted(dev)[len(dev) // 2], 4) if prof else None,
                            "overhead_ms": round(med - sorted(dev)[len(dev) // 2], 4) if prof else None}
                print(key, json.dumps(out[key]), flush=True)
    lat.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: BASELINE configs 4 and 5 decomposed at their REAL size (8192 x 2048) over
N ranks of the RCCL slab path (mock-RCCL build, ranks as threads on one GPU), against the lone
slab of the same build and against the oracle (the reference restated, one iteration at a time).

usage: run_full.py NRANKS WORKLOAD(K4|K5) [STEPS]

K4: f64 channel, no IB, the group advanced in bulk calls (deep slab cycles with the K-column
    halo); must be bit-identical to the lone slab and <= 1e-9 vs the oracle.
K5: f32 channel + 64 filaments x 96 points (workloads.filament_array, x_offset = 0: one on every
    slab edge of 2, 4 or 8 slabs, x = 0 included) moving every iteration, points given ahead
    (iblb_set_lagrangian_steps): the IB band cycle with ghost-column trapezoids must run on every
    rank; <= 1e-4 vs the oracle on rho - 1, u_x, u_y (each normalised by its own max) and <= 1e-5
    vs the lone slab.  The JSON line reports, per rank, the band cycles run and how many of them
    ran the merged chain (the chained chain is what a 4096-column f32 slab selects).

Reference: ImmersedBoundary.cu:138-267 (every point spreads wherever its 3x3 nodes fall),
main.cu:193-194 (positions wrapped into [0, XDIM): straddling points are the normal case).
"""
import json
import os
import sys
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from cuda_iblb_11_amd import _lib as L  # noqa: E402
from cuda_iblb_11_amd import workloads as W  # noqa: E402
from cuda_iblb_11_amd.lattice import Lattice, plan_slabs, rccl_unique_id, split_state  # noqa: E402

NX, NY = 8192, 2048


def main():
    n, kind = int(sys.argv[1]), sys.argv[2]
    K = int(os.environ.get("IBLB_SWEEP_DEPTH", "7"))  # the library's deep-sweep depth
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1 + 4 * K
    ib = kind == "K5"
    prec = "f32" if ib else "f64"
    chunks = [1, 2 * K, steps - 1 - 2 * K] if steps > 1 + 2 * K else [1, steps - 1]
    lib = L.load_from(os.path.join(HERE, "libiblb_mockrccl.so"))
    rho, u = W.perturbed_state(NX, NY, 29)
    pts = (lambda it: W.filament_array(it, NX, n_fil=64, pts=96, period=200, x_offset=0.0)) if ib else None
    ns = 64 * 96 if ib else 0

    def sched(t0, k):
        e = [pts(it) for it in range(t0, t0 + k)]
        return np.stack([x[0] for x in e]), np.stack([x[1] for x in e]), np.stack([x[2] for x in e])

    def advance(lat):
        t = 0
        for k in chunks:
            if ib:
                lat.set_lagrangian_steps(*sched(t, k))
            lat.step(k)
            t += k

    # the lone slab (whole lattice, one context of the same build)
    single = Lattice(NX, NY, W.TAU, W.TAU2, precision=prec, body_force=W.BODY_FORCE, max_points=ns, lib=lib)
    single.set_state(rho, u)
    single.set_profiling(True)
    advance(single)
    r1, u1 = single.macro()
    q1 = single.flux
    t1 = single.timing()
    single.close()

    uid = rccl_unique_id(lib)
    out = [None] * n
    errors = []

    def worker(r):
        try:
            xb, xc = plan_slabs(NX, n)[r]
            lat = Lattice(NX, NY, W.TAU, W.TAU2, precision=prec, body_force=W.BODY_FORCE, max_points=ns,
                          x_begin=xb, x_count=xc, lib=lib)
            lat.set_state(split_state(rho, 1, NX, NY, xb, xc), split_state(u, 2, NX, NY, xb, xc))
            lat.attach_rccl(uid, n, r)
            lat.set_profiling(True)
            advance(lat)
            rs, us = lat.macro()
            out[r] = (xb, xc, rs, us, lat.flux, lat.timing())
            lat.close()
        except Exception as e:  # a failed rank would leave the others waiting: report and exit hard
            errors.append(f"rank {r}: {e!r}")
            print(json.dumps({"ok": False, "errors": errors}), flush=True)
            os._exit(2)

    th = [threading.Thread(target=worker, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    R = np.empty((NY, NX))
    U = np.empty((2, NY, NX))
    for xb, xc, rs, us, _, _ in out:
        R[:, xb:xb + xc] = rs.reshape(NY, xc)
        U[:, :, xb:xb + xc] = us.reshape(2, NY, xc)
    R, U = R.ravel(), U.reshape(2, -1).ravel()

    # the restatement of the reference, one iteration at a time
    from oracle import oracle as O
    O.load()
    O.set_threads(min(16, os.cpu_count() or 1))
    sim = O.Simulation(NX, NY, W.TAU, W.TAU2, rho=rho, u=u, body_force=W.BODY_FORCE)
    if ib:
        for it in range(steps):
            sim.set_lagrangian(*pts(it))
            sim.step(1)
    else:
        sim.step(steps)
    ro, uo = np.asarray(sim.rho), np.asarray(sim.u)
    N = NX * NY

    def vs(rr, uu, ra, ua):  # rho - 1 and u, each normalised by its own max
        return {"rho-1": float(np.max(np.abs(rr - ra)) / np.max(np.abs(ra - 1))),
                "ux": float(np.max(np.abs(uu[:N] - ua[:N])) / np.max(np.abs(ua[:N]))),
                "uy": float(np.max(np.abs(uu[N:] - ua[N:])) / np.max(np.abs(ua[N:])))}

    d_oracle = vs(R, U, ro, uo)
    d_oracle["flux"] = float(abs(out[0][4] - sim.flux) / max(abs(sim.flux), 1e-300))
    d_single = vs(R, U, r1, u1)
    d_single_oracle = vs(r1, u1, ro, uo)
    exact = bool(np.array_equal(R, r1) and np.array_equal(U, u1))
    fluxes = [o[4] for o in out]
    d_q = float(max(abs(q - q1) for q in fluxes) / max(abs(q1), 1e-300))
    ranks = [{"x": [o[0], o[1]], "band_cycles": o[5]["band_cycles"], "band_merged_cycles": o[5]["band_merged_cycles"],
              "sweepk_launches": o[5]["sweepk_launches"]} for o in out]
    if ib:
        ok = max(d_oracle.values()) <= 1e-4 and max(d_single.values()) <= 1e-5 and d_q <= 1e-5
        # the band cycle ran on every rank, as many cycles as on the lone slab
        ok = ok and t1["band_cycles"] > 0 and all(rk["band_cycles"] == t1["band_cycles"] for rk in ranks)
    else:
        ok = exact and max(d_oracle.values()) <= 1e-9 and d_q <= 1e-12
        ok = ok and all(rk["sweepk_launches"] >= (steps - 1) // K for rk in ranks)
    print(json.dumps({"ok": bool(ok), "n": n, "workload": kind, "steps": steps, "exact": exact,
                      "d_oracle": d_oracle, "d_single": d_single, "d_single_oracle": d_single_oracle,
                      "d_flux_single": d_q, "single_band_cycles": t1["band_cycles"],
                      "single_band_merged_cycles": t1["band_merged_cycles"], "ranks": ranks,
                      "band_merge_env": os.environ.get("IBLB_BAND_MERGE")}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: run the RCCL slab path of libiblb (iblb_attach_rccl + collective
iblb_step / readers) with N ranks as threads on one GPU, through the mock-RCCL build
(tests/mock_rccl/libiblb_mockrccl.so), and compare with a single-slab context of the same
build.  Prints one JSON line; exit status 0 = match.

usage: run_group.py NRANKS NX NY STEPS WITH_IB(0/1) PRECISION(f64/f32)
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


def main():
    n, nx, ny, steps, with_ib, prec = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]),
                                        sys.argv[5] == "1", sys.argv[6])
    lib = L.load_from(os.path.join(HERE, "libiblb_mockrccl.so"))
    rho, u = W.perturbed_state(nx, ny, 31)
    bf = (1e-6, 2e-7)
    edge = plan_slabs(nx, n)[0][1] - 0.4  # filament straddling the slab 0 | slab 1 edge
    pts = lambda it: W.filament(it, n_points=40, x0=edge, y0=1.0, U0=2e-3, period=30, sway=2.0)
    mp = 64 if with_ib else 0

    single = Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, body_force=bf, max_points=mp, lib=lib)
    single.set_state(rho, u)
    for it in range(steps):
        if with_ib:
            single.set_lagrangian(*pts(it))
        single.step(1)
    r1, u1 = single.macro()
    q1 = single.flux

    uid = rccl_unique_id(lib)
    out = [None] * n
    errors = []

    def worker(r):
        try:
            xb, xc = plan_slabs(nx, n)[r]
            lat = Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, body_force=bf, max_points=mp, x_begin=xb,
                          x_count=xc, lib=lib)
            lat.set_state(split_state(rho, 1, nx, ny, xb, xc), split_state(u, 2, nx, ny, xb, xc))
            lat.attach_rccl(uid, n, r)
            for it in range(steps):
                if with_ib:
                    lat.set_lagrangian(*pts(it))
                lat.step(1)
            rs, us = lat.macro()
            out[r] = (xb, xc, rs, us, lat.flux)
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
    R = np.empty((ny, nx))
    U = np.empty((2, ny, nx))
    for xb, xc, rs, us, _ in out:
        R[:, xb:xb + xc] = rs.reshape(ny, xc)
        U[:, :, xb:xb + xc] = us.reshape(2, ny, xc)
    R, U = R.ravel(), U.reshape(2, -1).ravel()
    d_rho = float(np.max(np.abs(R - r1)) / np.max(np.abs(r1)))
    d_u = float(np.max(np.abs(U - u1)) / np.max(np.abs(u1)))
    fluxes = [o[4] for o in out]
    d_q = float(max(abs(q - q1) for q in fluxes) / max(abs(q1), 1e-300))
    exact = bool(np.array_equal(R, r1) and np.array_equal(U, u1))
    tol = 1e-12 if prec == "f64" else 1e-5
    ok = d_rho <= tol and d_u <= tol and d_q <= 1e-12
    if not with_ib:  # same per-cell arithmetic, halos carry identical values: bit-identical
        ok = ok and exact
    print(json.dumps({"ok": bool(ok), "exact": exact, "d_rho": d_rho, "d_u": d_u, "d_flux": d_q, "n": n,
                      "with_ib": with_ib, "precision": prec}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

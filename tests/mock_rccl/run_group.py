#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: run the RCCL slab path of libiblb (iblb_attach_rccl + collective
iblb_step / readers) with N ranks as threads on one GPU, through the mock-RCCL build
(tests/mock_rccl/libiblb_mockrccl.so), and compare with a single-slab context of the same
build.  Prints one JSON line; exit status 0 = match.

usage: run_group.py NRANKS NX NY STEPS WITH_IB(0/1/2/3) PRECISION(f64/f32) [BULK(0/1)]

BULK=1 (no IB): the group advances in multi-step calls (two-iteration sweeps with the 2-step
halo, one-step launches for odd remainders) instead of one iteration per call.
"""
import json
import os
import sys
import tempfile
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from cuda_iblb_11_amd import _lib as L  # noqa: E402
from cuda_iblb_11_amd import workloads as W  # noqa: E402
from cuda_iblb_11_amd.lattice import Lattice, plan_slabs, rccl_unique_id, split_state  # noqa: E402


def main():
    n, nx, ny, steps, with_ib, prec = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]),
                                        sys.argv[5] in ("1", "2", "3"), sys.argv[6])
    # IB mode "2": one filament moving inside each slab, points given ahead (iblb_set_lagrangian_steps)
    # and stepped in bulk: the IB band cycle of slab groups.  Mode "3": one moving filament across
    # EVERY slab edge (x = 0 included, wrapped into [0, XDIM) like boundary_check, main.cu:193-196):
    # the band cycle with ghost-column trapezoids on every rank, also checked against the oracle
    band = sys.argv[5] in ("2", "3")
    straddle = sys.argv[5] == "3"
    bulk = len(sys.argv) > 7 and sys.argv[7] == "1" and (not with_ib or band)
    lib = L.load_from(os.path.join(HERE, "libiblb_mockrccl.so"))
    rho, u = W.perturbed_state(nx, ny, 31)
    bf = (1e-6, 2e-7)
    edge = plan_slabs(nx, n)[0][1] - 0.4  # filament straddling the slab 0 | slab 1 edge

    mid = plan_slabs(nx, n)[0][1] / 2 + 0.2  # inner points of slab 0 (IB without the halo)

    def pts(it):  # plus one at x = XDIM (nodes wrap to column 0 of the next row)
        a = W.filament(it, n_points=40, x0=edge, y0=1.0, U0=2e-3, period=30, sway=2.0)
        b = W.filament(it, n_points=20, x0=nx - 0.3, y0=50.0, U0=2e-3, period=30, sway=0.5)
        c = W.filament(it, n_points=16, x0=mid, y0=80.0, U0=2e-3, period=30, sway=1.0)
        return tuple(np.concatenate([p, q, r]) for p, q, r in zip(a, b, c))
    mp = 96 if with_ib else 0
    if band:
        def pts(it):
            parts = []
            for xb_, xc_ in plan_slabs(nx, n):
                ph = 2 * np.pi * it / 20
                parts.append(W.filament(it, n_points=12, x0=xb_ + xc_ / 2 + 0.3 + np.sin(ph), y0=10.0, U0=2e-3,
                                        period=20, sway=0.8))
            return tuple(np.concatenate(q) for q in zip(*parts))

    if straddle:
        def pts(it):
            parts = []
            for r, (xb_, xc_) in enumerate(plan_slabs(nx, n)):
                ph = 2 * np.pi * (it + 3 * r) / 20
                f = W.filament(it, n_points=12, x0=xb_ + 0.3 + 1.5 * np.sin(ph), y0=10.0 + 7 * r, U0=2e-3,
                               period=20, sway=1.2)
                f[0][0::2] = np.mod(f[0][0::2], nx)  # wrapped into [0, XDIM)
                parts.append(f)
            return tuple(np.concatenate(q) for q in zip(*parts))

    def sched(t0, k):
        e = [pts(it) for it in range(t0, t0 + k)]
        return np.stack([x[0] for x in e]), np.stack([x[1] for x in e]), np.stack([x[2] for x in e])

    fcol = int(os.environ.get("RUN_GROUP_FLUX_COLUMN", nx - 5))  # (diagnostics: another flux column)
    single = Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, body_force=bf, max_points=mp, lib=lib, flux_column=fcol)
    single.set_state(rho, u)
    trace = os.environ.get("RUN_GROUP_TRACE") == "1"  # diagnostics: flux after every call
    q_single = {}
    for it in range(steps):
        if with_ib:
            single.set_lagrangian(*pts(it))
        single.step(1)
        if trace:
            q_single[it + 1] = single.flux
    # (mode 2: the reference run takes the points per iteration, the slabs get them ahead)
    r1, u1 = single.macro()
    q1 = single.flux
    f1 = single.lagrangian_force() if with_ib else None
    d_oracle = None
    if straddle:  # the restatement of the reference, one iteration at a time
        from oracle import oracle as O
        O.load()
        sim = O.Simulation(nx, ny, W.TAU, W.TAU2, rho=rho, u=u, body_force=bf, flux_column=fcol)
        for it in range(steps):
            sim.set_lagrangian(*pts(it))
            sim.step(1)
        ro, uo = np.asarray(sim.rho).copy(), np.asarray(sim.u).copy()

    def vs_oracle(rr, uu):  # each field normalised by its own max (rho - 1, not rho ~ 1)
        N = nx * ny
        return {"rho-1": float(np.max(np.abs((rr - 1) - (ro - 1))) / np.max(np.abs(ro - 1))),
                "ux": float(np.max(np.abs(uu[:N] - uo[:N])) / np.max(np.abs(uo[:N]))),
                "uy": float(np.max(np.abs(uu[N:] - uo[N:])) / np.max(np.abs(uo[N:])))}

    uid = rccl_unique_id(lib)
    out = [None] * n
    par = [0] * n
    gathered = [None] * n
    restarted = [None] * n
    errors = []
    half = steps // 2
    tmp = tempfile.mkdtemp(prefix="iblb_ck_")
    ck = lambda r: os.path.join(tmp, f"ck.rank{r}")

    def guarded(fn):
        def run(r):
            try:
                fn(r)
            except Exception as e:  # a failed rank would leave the others waiting: report and exit hard
                errors.append(f"rank {r}: {e!r}")
                print(json.dumps({"ok": False, "errors": errors}), flush=True)
                os._exit(2)
        return run

    @guarded
    def worker(r):
        xb, xc = plan_slabs(nx, n)[r]
        lat = Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, body_force=bf, max_points=mp, x_begin=xb,
                      x_count=xc, lib=lib, flux_column=fcol)
        lat.set_state(split_state(rho, 1, nx, ny, xb, xc), split_state(u, 2, nx, ny, xb, xc))
        lat.attach_rccl(uid, n, r)
        if band:
            lat.set_lagrangian_steps(*sched(0, steps))
            lat.set_profiling(True)
        if bulk:  # calls of 3, 1, 2, ... steps up to the checkpoint, the rest in one call
            t = 0
            for k in (3, 1, 2, 4):
                if t + k <= half:
                    lat.step(k)
                    t += k
                    if trace:
                        q = lat.flux
                        if r == 0:
                            print("trace", t, q, q_single[t], flush=True)
            lat.step(half - t)
            if trace:
                q = lat.flux
                if r == 0:
                    print("trace", half, q, q_single[half], flush=True)
            lat.save_checkpoint(ck(r))
            if trace:
                for k in ([5, 5, 3] if steps - half == 13 else [steps - half]):
                    lat.step(k)
                    t2 = lat.steps
                    q = lat.flux
                    if r == 0:
                        print("trace", t2, q, q_single[t2], flush=True)
            else:
                lat.step(steps - half)
        for it in range(0 if not bulk else steps, steps):
            if it == half:
                lat.save_checkpoint(ck(r))
            if with_ib:
                lat.set_lagrangian(*pts(it))
            lat.step(1)
        if band:
            tm = lat.timing()
            if tm["sweepk_launches"] == 0:
                raise RuntimeError(f"rank {r}: the band cycle did not run")
            par[r] = tm["band_par_cycles"]
        rs, us = lat.macro()
        out[r] = (xb, xc, rs, us, lat.flux, lat.lagrangian_force() if with_ib else None)  # collective
        gathered[r] = lat.gather_macro(0)  # collective output gather to rank 0
        lat.close()

    uid2 = rccl_unique_id(lib)

    @guarded
    def resume(r):  # fresh contexts: attach, restore the mid-run checkpoint, finish the run
        xb, xc = plan_slabs(nx, n)[r]
        lat = Lattice(nx, ny, W.TAU, W.TAU2, precision=prec, body_force=bf, max_points=mp, x_begin=xb,
                      x_count=xc, lib=lib, flux_column=fcol)
        lat.attach_rccl(uid2, n, r)
        lat.load_checkpoint(ck(r))
        if band:  # the checkpoint holds the points of iteration half-1; the rest given ahead again
            lat.set_lagrangian_steps(*sched(half, steps - half))
        if bulk:
            lat.step(steps - half)
        for it in range(half if not bulk else steps, steps):
            if with_ib:
                lat.set_lagrangian(*pts(it))
            lat.step(1)
        rs, us = lat.macro()
        restarted[r] = (rs, us, lat.flux, lat.steps)
        lat.close()

    for fn in (worker, resume):
        th = [threading.Thread(target=fn, args=(r,)) for r in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    R = np.empty((ny, nx))
    U = np.empty((2, ny, nx))
    for xb, xc, rs, us, _, _ in out:
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
    # the gather reproduces the assembled slabs on rank 0 only
    g_ok = bool(np.array_equal(gathered[0][0], R) and np.array_equal(gathered[0][1], U)
                and all(g == (None, None) for g in gathered[1:]))
    # restart: same steps, same fields as the uninterrupted run (bit-identical without IB; the
    # IB spread's atomic summation order may differ in the last bit)
    rs_ok = all(restarted[r][3] == steps for r in range(n))
    d_re = 0.0
    for r in range(n):
        a, b = out[r], restarted[r]
        d_re = max(d_re, float(np.max(np.abs(a[2] - b[0]))), float(np.max(np.abs(a[3] - b[1]))))
        rs_ok = rs_ok and abs(a[4] - b[2]) <= 1e-12 * max(abs(a[4]), 1e-300)
    rs_ok = rs_ok and (d_re == 0.0 if not with_ib else d_re <= 1e-12)
    ok = ok and g_ok and rs_ok
    d_fs = 0.0
    if with_ib:  # every rank reports the whole F_s (summed over the slabs that hold it)
        d_fs = max(float(np.max(np.abs(o[5] - f1)) / np.max(np.abs(f1))) for o in out)
        ok = ok and d_fs <= 1e-5
    if straddle:  # the group (band cycles across every slab edge) against the restatement
        d_oracle = vs_oracle(R, U)
        d_oracle["flux"] = float(abs(fluxes[0] - sim.flux) / max(abs(sim.flux), 1e-300))
        d_oracle["flux_single"] = float(abs(q1 - sim.flux) / max(abs(sim.flux), 1e-300))
        ok = ok and max(d_oracle.values()) <= (1e-9 if prec == "f64" else 1e-4)
    print(json.dumps({"ok": bool(ok), "exact": exact, "d_rho": d_rho, "d_u": d_u, "d_flux": d_q, "n": n,
                      "gather_ok": g_ok, "restart_ok": bool(rs_ok), "d_restart": d_re, "d_F_s": d_fs,
                      "with_ib": with_ib, "precision": prec, "d_oracle": d_oracle, "band_par_cycles": par}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

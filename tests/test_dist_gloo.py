"""N>1 path on CPU: world_size 2 and 3 over torch.distributed (gloo) run the x-slab
decomposition the HIP path uses — slab plan from cuda_iblb_11_amd.plan_slabs, halo planes
{1,5,8} rightward / {3,6,7} leftward every step; with IB a three-column halo from which each
rank computes the nodes of every point spreading into it (no collective), spread clipped to
owned columns; flux owned by the slab holding column XDIM-5 — with the oracle
kernels doing the per-cell arithmetic, and must reproduce the single-domain reference step
bit for bit."""
import os
import socket

import numpy as np
import pytest


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _points(it, nx, world):
    from cuda_iblb_11_amd import workloads as W
    from cuda_iblb_11_amd.lattice import plan_slabs
    if world < 3:
        x0, sway = plan_slabs(nx, world)[0][1] - 0.6, 1.5
    else:
        x0, sway = nx - 0.3, 0.5
    return W.filament(it, n_points=30, x0=x0, y0=2.0, dy=1.0, U0=2e-3, period=20, sway=sway)


def _worker(rank, world, port, nx, ny, steps, with_ib, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from cuda_iblb_11_amd.lattice import plan_slabs
    from cuda_iblb_11_amd import workloads as W
    import slab_model as SM

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    xb, xc = plan_slabs(nx, world)[rank]
    rho, u = W.perturbed_state(nx, ny, 17)
    from cuda_iblb_11_amd.lattice import split_state
    bf = (1e-6, 2e-7)
    rk = SM.SlabRank(O, nx, ny, xb, xc, W.TAU, W.TAU2, split_state(rho, 1, nx, ny, xb, xc),
                     split_state(u, 2, nx, ny, xb, xc), body_force=bf)
    left, right = (rank - 1) % world, (rank + 1) % world
    # the same points on every rank: straddling the edge between slab 0 and slab 1, or (3 ranks)
    # at x = XDIM where the nodes wrap to column 0 of the next row
    pts = lambda it: _points(it, nx, world)
    rk.collide()  # iteration 0's equilibrium + collision from rho^0, u^0, force^0
    F_all = []
    for it in range(steps):
        send_r, send_l = rk.boundary_ext() if with_ib else rk.boundary()
        hl = torch.empty(send_r.shape, dtype=torch.float64)
        hr = torch.empty(send_l.shape, dtype=torch.float64)
        reqs = [dist.isend(torch.from_numpy(send_r), right, tag=0), dist.isend(torch.from_numpy(send_l), left, tag=1),
                dist.irecv(hl, left, tag=0), dist.irecv(hr, right, tag=1)]
        for r in reqs:
            r.wait()
        if with_ib:
            rk.stream_macro_ext(hl.numpy(), hr.numpy())
            s, us, eps = pts(it)
            F_s = rk.interp(s, us, rk.node_values(s))
            rk.spread(s, F_s, eps)
            mine = np.array([rk.owns(s, k) for k in range(s.size // 2)])
            F_all.append(np.where(np.repeat(mine, 2), F_s, np.float32(0)))
        else:
            rk.stream_macro(hl.numpy(), hr.numpy())
            rk.no_ib()
        if it < steps - 1:
            rk.collide()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), rho=rk.rho, u=rk.u, Q=rk.Q, xb=xb, xc=xc,
             F_s=np.array(F_all, dtype=np.float32))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,with_ib", [(2, False), (2, True), (3, False), (3, True)])
def test_slab_decomposition_gloo(tmp_path, oracle, world, with_ib):
    import torch.multiprocessing as mp
    nx, ny, steps = 30, 24 if not with_ib else 30, 12
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, world, port, nx, ny, steps, with_ib, str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    from cuda_iblb_11_amd import workloads as W
    from cuda_iblb_11_amd.lattice import plan_slabs
    rho, u = W.perturbed_state(nx, ny, 17)
    sim = oracle.Simulation(nx, ny, W.TAU, W.TAU2, rho=rho, u=u, body_force=(1e-6, 2e-7))
    F_ref = []
    for it in range(steps):
        if with_ib:
            s, us, eps = _points(it, nx, world)
            sim.set_lagrangian(s, us, eps)
        sim.step(1)
        if with_ib:
            F_ref.append(sim.F_s.copy())
    R = np.empty((ny, nx))
    U = np.empty((2, ny, nx))
    Q = 0.0
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        xb, xc = int(d["xb"]), int(d["xc"])
        R[:, xb:xb + xc] = d["rho"].reshape(ny, xc)
        U[:, :, xb:xb + xc] = d["u"].reshape(2, ny, xc)
        Q += float(d["Q"])
    assert np.array_equal(R.ravel(), sim.rho)
    assert np.array_equal(U.reshape(2, -1).ravel(), sim.u)
    assert Q == sim.flux
    if with_ib:  # every point's F_s reported by exactly one rank, equal to the reference's
        F = sum(np.load(tmp_path / f"rank{r}.npz")["F_s"] for r in range(world))
        assert np.array_equal(F, np.array(F_ref, dtype=np.float32))

#!/usr/bin/env python3
"""Benchmark of the MI355X IB-LBM hot path: BASELINE.json metric
"MLUPS and achieved-HBM-GB/s, 4096^2 D2Q9 channel, 1/2/4/8 MI355X".

One step = one reference iteration (main.cu:852-909) over the whole 4096 x 4096 channel
(periodic x, bounce-back / mirror walls, TRT + Guo forcing, uniform body force, no IB): one
deep sweep launch (pull-stream + collide K = 7 times, intermediate states in registers,
lbm_sweep_impl.h) per seven steps and slab (K - 1 = 6 where a call's length needs it).  N > 1: x-slab decomposition of the SAME 4096^2
lattice (strong scaling), one process per GPU; per K-iteration cycle a K-column ghost exchange
via RCCL and the boundary sweeps run on a comm stream beside the interior sweep; `--scaling weak`
gives every rank the configured width instead ((nx*N) x ny).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--precision f64|f32] [--nx 4096 --ny 4096]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints ONE JSON line.  `roofline.achieved` = algorithmic bytes of the collide-stream
kernel (18 populations x 8 B = 144 B per cell in f64) x cells per launch / mean launch time
measured with HIP events on the stream the kernel runs on (N = 1: inside the timed region;
N > 1: in a follow-up phase, so the events' cost stays out of `value`); `roofline.traffic` = HBM bytes
per launch from rocprofv3 PMC counters (profiles/pmc_traffic.json, FETCH_SIZE doubled per
MI355X_MICROARCH.md §HBM) when a matching profile exists.  `cpu_baseline` = the oracle
(reference kernels restated in C, unfused AoS sequence) on the host cores, rank 0 at N=1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "MLUPS and achieved-HBM-GB/s, 4096² D2Q9 channel, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# BASELINE.json configs: (nx, ny, precision, Lagrangian points or None, description)
WORKLOADS = {
    "M": (4096, 4096, "f64", None, "M: 4096x4096 D2Q9 channel, no IB"),
    "K2": (2048, 2048, "f64", None, "K2: 2048x2048 D2Q9 channel, no IB"),
    "K3": (2048, 2048, "f64", "filament", "K3: 2048x2048 channel + one 256-point filament"),
    "K4": (8192, 2048, "f64", None, "K4: 8192x2048 channel, no IB"),
    "K5": (8192, 2048, "f32", "array", "K5: 8192x2048 channel + 64 filaments x 96 points"),
}


def workload_points(kind, nx, offset=0.0):
    """Lagrangian points of iteration `it` (a function), IB evaluated every iteration:
    K3: one 256-point filament at x = nx/2, u_s = (U0 (k/255) sin(2 pi it/T), 0)
    changing every iteration; K5: 64 filaments x 96 points (W.filament_array) whose points move
    every iteration (tilt up to 8 columns over the period T = 1000), standing at m * 128: one on
    every slab edge of 1, 2, 4 or 8 slabs, x = 0 included (they cross it while they tilt)."""
    from cuda_iblb_11_amd import workloads as W
    if kind == "filament":
        return lambda it: W.filament(it, n_points=256, x0=nx / 2 + 0.3, y0=1.0, dy=1.0, U0=1e-3, period=1000)
    if kind == "array":  # 64 filaments per 8192 columns, one on every slab edge (BASELINE config 5)
        nf = max(1, round(64 * nx / 8192))
        return lambda it: W.filament_array(it, nx, n_fil=nf, pts=96, period=1000, x_offset=offset)
    return None


class Driver:
    """lat.step(n) with the workload's points of those n iterations given ahead
    (iblb_set_lagrangian_steps: staged in HBM before the launches, like the reference's
    per-iteration cilia positions that its kinematics kernels write to the device); --frozen:
    the points of iteration 250 for the whole run (round-1 workload)."""

    def __init__(self, lat, points, frozen):
        self.lat, self.points, self.frozen, self.t = lat, points, frozen, 0
        if points is not None and frozen:
            lat.set_lagrangian(*points(250))

    def stage(self, n):
        if self.points is None or self.frozen:
            return
        ent = [self.points(it) for it in range(self.t, self.t + n)]
        self.lat.set_lagrangian_steps(np.stack([e[0] for e in ent]), np.stack([e[1] for e in ent]),
                                      np.stack([e[2] for e in ent]))

    def run(self, n, staged=False):
        if not staged:
            self.stage(n)
        self.lat.step(n)
        self.t += n


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 420 and 42: multiples of every deep depth 3 ... 7 (an IB band cycle run ends with one-step
    # iterations over the whole lattice for a remainder)
    p.add_argument("--steps", type=int, default=420)
    p.add_argument("--warmup", type=int, default=42)
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="M",
                   help="BASELINE.json config: M (metric, default), K2..K5")
    p.add_argument("--nx", type=int, default=None)
    p.add_argument("--ny", type=int, default=None)
    p.add_argument("--precision", choices=["f64", "f32"], default=None)
    p.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                   help="strong (default): the configured lattice over N ranks; weak: N times the "
                        "configured width (K4 weak scaling: (nx*N) x ny, one configured lattice per rank)")
    p.add_argument("--prime-seconds", type=float, default=1.0,
                   help="untimed steps before the warmup until this much wall time has passed (the GPU "
                        "clock settles under load; reported as `prime` in the JSON line)")
    p.add_argument("--frozen", action="store_true",
                   help="IB workloads: points of iteration 250 for the whole run (round-1 workload)")
    p.add_argument("--filament-offset", type=float, default=0.0,
                   help="K5: filament m stands at (m + offset) * 128 columns (0 = on every slab edge, the BASELINE "
                        "config; 0.5 = the round-2 layout, every filament mid-slab)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU sample duration")
    p.add_argument("--no-profile-events", action="store_true", help="skip per-launch HIP events")
    p.add_argument("--rccl-self", action="store_true",
                   help="N=1 rehearsal of the multi-GPU schedule: the slab is its own RCCL neighbour")
    p.add_argument("--same-device", action="store_true",
                   help="rehearsal of the N > 1 path on one GPU: every rank uses device 0 and runs its slab as "
                        "an RCCL self ring (RCCL refuses two ranks of one communicator on one device)")
    return p.parse_args()


def cpu_baseline(nx, ny, budget_s, points=None, frozen=False):
    """The reference's own unfused sequence (equilibrium, collision, streaming, macro,
    interpolate + the literal O(N*Ns) spread gather when there are points; AoS fp64) restated in
    C (oracle/), OpenMP over the host cores, timed on a bounded number of steps of the same
    workload."""
    from oracle import oracle as O
    from cuda_iblb_11_amd import workloads as W
    node = host_cores()
    # the host cores this process may use: OMP_NUM_THREADS where the launcher sets it (the GPU
    # box grants each GPU slot its share of the node, OMP_NUM_THREADS=16 of 128 physical cores),
    # otherwise every physical core of the node
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or node["physical_cores"] or (os.cpu_count() or 1)
    threads = max(1, threads)
    kind = "port"
    try:
        O.build(native=True)
        O.load(native=True)
        native = True
    except Exception:
        O.load()
        native = False
    O.set_threads(threads)
    ns = 0 if points is None else points(0)[0].size // 2
    est = nx * ny * ns * 2e-8 / threads  # ~20 ns per delta evaluation and core
    if est > 90:
        return {"value": None, "unit": "MLUPS", "cores": threads, "kind": kind, "node": node,
                "sample": f"skipped: the reference's O(N*Ns) spread needs ~{est:.0f} s per step on {threads} cores"}
    rho, u = W.perturbed_state(nx, ny, W.SEED)
    sim = O.Simulation(nx, ny, W.TAU, W.TAU2, rho=rho, u=u, body_force=W.BODY_FORCE, point_spread=False)
    del rho, u

    def steps(t, n):  # the points of every iteration set before it (set once if frozen)
        if points is None or frozen:
            if points is not None and t == 0:
                sim.set_lagrangian(*points(250))
            sim.step(n)
            return
        for it in range(t, t + n):
            sim.set_lagrangian(*points(it))
            sim.step(1)

    t0 = time.perf_counter()
    steps(0, 1)  # warm-up + size the sample
    one = time.perf_counter() - t0
    n = int(max(1, min(50, budget_s / max(one, 1e-6))))
    t0 = time.perf_counter()
    steps(1, n)
    dt = time.perf_counter() - t0
    mlups = nx * ny * n / dt / 1e6
    return {"value": round(mlups, 3), "unit": "MLUPS", "cores": threads, "kind": kind, "node": node,
            "sample": f"{n} steps of the {nx}x{ny} f64 channel" + (f" + {ns} IB points" if ns else "") +
                      ", reference unfused AoS sequence restated in C "
                      f"(oracle/oracle.c, {'-march=native' if native else 'x86-64-v2'}, OpenMP {threads} threads), "
                      f"{dt:.1f} s"}


def host_cores():
    """Physical cores / sockets / model of the host (lscpu's counts, from /proc/cpuinfo)."""
    phys, model = set(), ""
    try:
        pid = cid = None
        for ln in open("/proc/cpuinfo"):
            k, _, v = ln.partition(":")
            k, v = k.strip(), v.strip()
            if k == "physical id":
                pid = v
            elif k == "core id":
                cid = v
            elif k == "model name" and not model:
                model = v
            elif not k and pid is not None:
                phys.add((pid, cid))
                pid = cid = None
        if pid is not None:
            phys.add((pid, cid))
    except OSError:
        pass
    return {"physical_cores": len(phys) or None, "sockets": len({p for p, _ in phys}) or None,
            "logical_cpus": os.cpu_count(), "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def pmc_valu(workload_key):
    """VALU figures of the dominant kernel per launch (profiles/pmc_valu.json, scripts/pmc_valu.py)."""
    try:
        return json.load(open(os.path.join(REPO, "profiles", "pmc_valu.json"))).get(workload_key)
    except Exception:
        return None


# vector peaks: FP32 157.3 TFLOP/s (MI355X_MICROARCH.md); FP64 vector 78.6 TFLOP/s (AMD's MI355X
# specification; half the FP32 vector rate)
VALU_PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}


_MODE_BITS = ((16, "wall split"), (64, "packed f32x2 collide"), (128, "skip regions"), (256, "preshift"),
              (512, "LDS window"), (1, "nontemporal stores"))


def deep_limiter(tm, valu, precision):
    """What binds the deep kernel that ran, from the build the library reports for its last deep launch
    (iblb_timing deep_mode / deep_vs / deep_waves_per_simd / deep_vgprs) and the SQ passes of
    profiles/pmc_valu.json (VALU issue per wave), not from a fixed string."""
    mode, vs, wps, vgprs = (int(tm.get(k, 0)) for k in ("deep_mode", "deep_vs", "deep_waves_per_simd", "deep_vgprs"))
    if wps <= 0:
        return "dependent latency and VALU issue (DESIGN.md §4)"
    feats = ", ".join(n for b, n in _MODE_BITS if mode & b) or "plain walk"
    txt = (f"VALU issue and dependent latency, not HBM: sweepk_kernel<{precision}, {vs} cell(s) per lane, MODE "
           f"{mode} = {feats}> runs {wps} wave(s) per SIMD at {vgprs} VGPRs")
    if valu and valu.get("valu_issue_share") is not None:
        s = float(valu["valu_issue_share"])
        txt += (f"; each wave issues VALU {100 * s:.0f} % of its cycles, the SIMD ~{100 * min(1.0, s * wps):.0f} % "
                f"(profiles/pmc_valu.json)")
    return txt + ". `bound` stays the contract's roofline axis (hbm); the fraction is of HBM peak (DESIGN.md §4)"


def pmc_traffic(workload_key):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except Exception:
        return None, None
    e = d.get(workload_key)
    if not e:
        return None, None
    return e.get("hbm_bytes_per_launch"), e.get("source")



def deep_label(mean):
    """K of the deep launches: one depth, or the two depths a call mixed (K-1 and K)."""
    lo, hi = int(mean), -(-mean // 1)
    return str(int(mean)) if lo == hi else f"{lo}/{int(hi)}"

def main():
    a = parse()
    # Libraries (RCCL's version banner, torch) may print to fd 1: route it to stderr and keep
    # the real stdout for the one JSON line.
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    distributed = world > 1
    if a.same_device:
        local = 0
    if distributed:
        torch.cuda.set_device(local)
        if a.same_device:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))

    import cuda_iblb_11_amd as P
    from cuda_iblb_11_amd import workloads as W

    wnx, wny, wprec, wpts, wdesc = WORKLOADS[a.workload]
    if wpts == "array":
        wdesc += (", one on every slab edge (x = 0 included)" if a.filament_offset == 0.0 else
                  ", every filament mid-slab" if a.filament_offset == 0.5 else
                  f", filament m at (m + {a.filament_offset}) * 128 columns")
    nx, ny = a.nx or wnx, a.ny or wny
    if a.scaling == "weak":
        nx *= world
    precision = a.precision or wprec
    xb, xc = P.plan_slabs(nx, world)[rank]
    # --same-device (N > 1 on one GPU): each rank runs its slab as a lattice of its own, periodic over
    # a one-rank RCCL self ring — the per-rank kernels, streams and halo exchange of the N-GPU run,
    # and this script's whole N > 1 path (process group, barriers, MAX reductions), without the
    # transfers between GPUs.  The workload's points are those of a lattice of the slab's width (K5:
    # 8 filaments per 1024 columns, one on the slab edge).
    rehearsal = distributed and a.same_device
    lnx = xc if rehearsal else nx
    points = workload_points(wpts, lnx, a.filament_offset)
    ns = 0 if points is None else points(0)[0].size // 2
    lat = P.Lattice(lnx, ny, W.TAU, W.TAU2, precision=precision, body_force=W.BODY_FORCE, device=local,
                    x_begin=0 if rehearsal else xb, x_count=xc if world > 1 and not rehearsal else 0, max_points=ns)
    rho, u = W.perturbed_state(nx, ny, W.SEED)
    lat.set_state(P.split_state(rho, 1, nx, ny, xb, xc), P.split_state(u, 2, nx, ny, xb, xc))
    del rho, u
    if rehearsal or (a.rccl_self and not distributed):
        os.environ["IBLB_RCCL_SELF"] = "1"
        lat.attach_rccl(P.rccl_unique_id(), 1, 0)
    elif distributed:
        uid = [P.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        lat.attach_rccl(uid[0], world, rank)
    drv = Driver(lat, points, a.frozen)

    # prime: the clock of an idle GPU ramps up over the first ~0.1-1 s of load; a 20-step timed
    # region (~3 ms at 4096^2) would otherwise measure the ramp (profiles/r02a_bench_*.json: 109k
    # MLUPS at 20 steps vs 125k at 500 on the same box)
    # (ranks step together: rank 0's clock decides, broadcast after every chunk)
    prime_steps, tp = 0, time.perf_counter()
    while True:
        go = time.perf_counter() - tp < a.prime_seconds
        if distributed:
            flag = torch.tensor([1.0 if go else 0.0], device="cpu" if rehearsal else "cuda")
            dist.broadcast(flag, src=0)
            go = bool(flag.item() > 0)
        if not go:
            break
        drv.run(42)  # whole deep cycles at every depth 3 ... 7
        lat.synchronize()
        prime_steps += 42
    prime_s = time.perf_counter() - tp
    # the points of the warmup and the timed steps given ahead in one schedule: nothing of the
    # timed iterations (not even the force owed at its start) is evaluated before the timer
    drv.stage(a.warmup + a.steps)
    drv.run(a.warmup, staged=True)
    lat.synchronize()
    # Launch timing for the roofline: the deep launches' own dispatch / completion signals
    # (iblb_set_profiling mode 2: no marker packets, the IB band chain's launches untimed).  At N = 1
    # they time the launches of the timed region itself, with IB too (one signal pair per K-iteration
    # cycle; round 4 bracketed every chain launch as well, +4-8 % per step, and timed IB runs in a
    # follow-up phase instead — VERDICT r4 weak #2).  At N > 1 the slab interior runs without any
    # signal (ctx_step.hip:deep_slab_step, a signal costs ~5 us per cycle there), so the same number of
    # steps (<= 100) is timed with events right afterwards.
    events_in_timed = not distributed and not a.no_profile_events
    lat.set_profiling(2 if events_in_timed else 0)
    lat.timing(reset=True)

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    drv.run(a.steps, staged=True)
    lat.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    tm = lat.timing(reset=True)
    # deep launches of the timed region and their mean depth (a call mixes depths K and K-1 so that
    # it needs no remainder launches, ctx_step.hip:deep_depth)
    deep_mean = tm["deep_iterations"] / tm["deep_launches"] if tm["deep_launches"] else float(tm["sweepk_depth"])
    if not events_in_timed and not a.no_profile_events:
        lat.set_profiling(2)
        # whole cycles only (an IB run's last n mod K iterations are one-step launches over the lattice)
        kd = int(tm["sweepk_depth"])
        drv.run(max(kd, min(a.steps, 100) // kd * kd) if kd >= 3 else min(a.steps, 100))
        lat.synchronize()
        tm = lat.timing(reset=True)
        lat.set_profiling(False)
    red_dev = "cpu" if rehearsal else "cuda"
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    launch_ms = tm["fused_ms"] / max(tm["fused_launches"], 1)
    # cells one timed launch updates (N > 1 overlapped: the interior columns of the slab)
    cells_per_launch = tm["fused_cells"] // max(tm["fused_launches"], 1)
    # dominant kernel: the two-iteration sweep where it runs (no IB owed between iterations).
    # One sweep launch reads and writes the state once (the same 144 B/cell in f64) and
    # advances its cells by two iterations.
    # (by summed launch time: with IB bands, five one-step launches over the band columns run
    # beside one deep launch over the rest of the lattice per cycle)
    sweep = tm["sweep_launches"] > 0 and tm["sweep_ms"] >= tm["fused_ms"]
    iters_per_launch = 1
    if sweep:
        launch_ms = tm["sweep_ms"] / tm["sweep_launches"]
        cells_per_launch = tm["sweep_cells"] // tm["sweep_launches"]
        iters_per_launch = 2
    # K >= 3 iterations per launch (IBLB_SWEEP_DEPTH=K): the roofline kernel wherever it runs (with IB
    # bands it advances > 97 % of the lattice updates; the trapezoids' one-step launches are reported
    # in `ib_band`)
    if tm["sweepk_launches"] > 0:
        sweep = int(tm["sweepk_depth"])
        launch_ms = tm["sweepk_ms"] / tm["sweepk_launches"]
        cells_per_launch = tm["sweepk_cells"] // tm["sweepk_launches"]
        iters_per_launch = round(deep_mean, 3)
    if a.no_profile_events:  # nothing timed per launch: name the kernel from what ran
        # (the band-cycle counter is kept without events; a deep run without IB shows as no
        # one-step launches at all, since only the boot iteration and remainders are one-step)
        depth = int(tm["sweepk_depth"])
        if tm["band_cycles"] > 0 or (ns == 0 and os.environ.get("IBLB_SWEEP", "1") != "0" and depth >= 3):
            sweep = depth
        elif ns == 0 and os.environ.get("IBLB_SWEEP", "1") != "0":
            sweep = 2
        else:
            sweep = False
        iters_per_launch = (round(deep_mean, 3) if sweep and sweep >= 3 else sweep) or 1
        launch_ms, cells_per_launch = 0.0, 0
    if distributed:
        sl = torch.tensor([launch_ms], dtype=torch.float64, device=red_dev)
        dist.all_reduce(sl, op=dist.ReduceOp.MAX)
        launch_ms = float(sl.item())

    # sanity: the state must stay finite (macro() is collective for an RCCL group)
    rho_s, _ = lat.macro()
    finite = bool(np.isfinite(rho_s).all())
    if distributed:
        fin = torch.tensor([1.0 if finite else 0.0], device=red_dev)
        dist.all_reduce(fin, op=dist.ReduceOp.MIN)
        finite = bool(fin.item() > 0)

    cells = nx * ny
    mlups = cells * a.steps / elapsed / 1e6
    bytes_per_cell = 18 * (8 if precision == "f64" else 4)
    achieved = bytes_per_cell * cells_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else None
    key = f"{precision}_{nx}x{ny}_n{world}" + (f"_ib{ns}" if ns else "") + (f"_sweep{sweep}" if sweep not in (False, True) else ("_sweep" if sweep else ""))
    traffic, traffic_src = pmc_traffic(key)
    valu = pmc_valu(key)

    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            lat.close()
            cpu = cpu_baseline(nx, ny, a.cpu_seconds, points, a.frozen)
        out = {
            "metric": METRIC,
            "value": round(mlups, 2),
            "unit": "MLUPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": precision,
            "data": "synthetic (rho = 1 + 1e-3 xi, u = 1e-3 xi, numpy seed 12345; body force 1e-6)",
            "config": {
                "workload": f"{wdesc} ({nx}x{ny}): D2Q9 channel (periodic x, bounce-back y=0, mirror y=Y-1), "
                            f"TRT+Guo, reference TAU/TAU2; "
                            + (f"{deep_label(iters_per_launch)} iterations per launch (pull-stream+collide K times, "
                               "intermediate states in registers)" if sweep else
                               "one fused pull-stream+collide launch per step")
                            + ((f"; IB: {ns} Lagrangian points, interpolate+spread every step, " +
                                ("points frozen at iteration 250 (--frozen)" if a.frozen else
                                 "points of every iteration given ahead (iblb_set_lagrangian_steps): "
                                 + ("fixed positions, u_s(it)" if wpts == "filament" else "moving positions")))
                               if ns else "")
                            + ("; IB band cycle: columns within K-1 of a forced column one iteration per launch, "
                               "the rest in the deep sweep" if ns and tm["sweepk_launches"] else ""),
                "nx": nx, "ny": ny, "global_cells": cells, "ib_points": ns,
                **({"filament_offset": a.filament_offset} if wpts == "array" else {}),
                **({"band_cycles": int(tm["band_cycles"]), "band_merged_cycles": int(tm["band_merged_cycles"]),
                    "band_par_cycles": int(tm["band_par_cycles"])}
                   if ns else {}),
                "parallelism": f"x-slab x{world}" + (" (RCCL halo)" if world > 1 and not rehearsal else "")
                               + (" (RCCL self-ring rehearsal)" if a.rccl_self and world == 1 else "")
                               + (" (same-device rehearsal: every rank a self ring over its slab on GPU 0)"
                                  if rehearsal else ""),
            },
            "ib_ms_per_step": round(tm["ib_ms"] / a.steps, 5) if ns else None,
            # IB band cycle (K iterations per cycle): lattice updates done by one-step launches over
            # the band trapezoids (incl. their ghost columns) vs the deep sweep over the gaps
            "ib_band": (None if not (ns and tm["sweepk_launches"]) else {
                "deep_lu": int(tm["sweepk_cells"] * tm["sweepk_depth"]),
                "deep_ms_per_cycle": round(tm["sweepk_ms"] / tm["sweepk_launches"], 5),
                "cycle_ms": round(elapsed / a.steps * 1e3 * tm["sweepk_depth"], 5),
                "chain": "untimed (its launches carry no events in the timed region)"}),
            # state bytes moved per second of the whole run (one read + one write per launch)
            "achieved_hbm_gbps": round(mlups * 1e6 * bytes_per_cell / iters_per_launch / 1e9, 1),
            "roofline": {
                # the roofline the fraction is taken against; what limits the deep kernels is `limiter`
                "bound": "hbm",
                "achieved": None if achieved is None else round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": None if achieved is None else round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "kernel": (f"sweepk_kernel<K={deep_label(iters_per_launch)}> (lbm_sweep_impl.h): {iters_per_launch} iterations per "
                           "launch, state read and written once"
                           + (" (slab interior; boundary sweeps on the comm stream)" if world > 1 or a.rccl_self else "")
                           if iters_per_launch > 2 else
                           "sweep2_kernel (lbm_sweep_impl.h): two iterations per launch, state read and written once"
                           if sweep else "fused_kernel (lbm_kernels.hip)")
                          + (" — not timed (--no-profile-events)" if a.no_profile_events else ""),
                "bytes_per_cell": bytes_per_cell,
                "cells_per_launch": cells_per_launch,
                "iterations_per_launch": iters_per_launch,
                # temporal blocking: the one-step algorithm needs bytes_per_cell per lattice update;
                # the rate it would have to sustain for this MLUPS, against the HBM peak
                "one_step_equivalent_gbps": round(mlups * 1e6 * bytes_per_cell / 1e9, 1),
                "one_step_equivalent_frac": round(mlups * 1e6 * bytes_per_cell / 1e9 / HBM_PEAK_GBPS, 4),
                "launch_ms": round(launch_ms, 5),
                "launch_timing": ("none (--no-profile-events)" if a.no_profile_events else
                                  "HIP events in the timed region" if events_in_timed else
                                  f"HIP events over {min(a.steps, 100)} further steps after the timed region"
                                  + (" (MAX over ranks)" if distributed else "")),
                "traffic_source": traffic_src,
                "limiter": (deep_limiter(tm, valu, precision)
                            if iters_per_launch > 2 else "HBM bandwidth (one read + one write of the state per launch)"),
            },
            # the temporally blocked kernels are bound by vector issue, not HBM: their fp64 / fp32
            # FLOP rate from the PMC FLOP count of a profiled pass over the measured launch time
            "valu": (None if valu is None or launch_ms <= 0 else {
                "achieved": round(valu["flops_per_launch"] / (launch_ms * 1e-3) / 1e12, 2),
                "peak": VALU_PEAK_TFLOPS[precision], "unit": "TFLOP/s",
                "frac": round(valu["flops_per_launch"] / (launch_ms * 1e-3) / 1e12 / VALU_PEAK_TFLOPS[precision], 4),
                "valu_issue_share": valu.get("valu_issue_share"), "source": valu.get("source")}),
            "prime": {"steps": prime_steps, "seconds": round(prime_s, 3)},
            "cpu_baseline": cpu,
            "state_finite": finite,
        }
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    lat.close()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""How far the reference's own arithmetic lets two runs of the many-point IB configuration drift
apart: the reference accumulates F_s in float (ImmersedBoundary.cu:124-125),
so a population difference of a few double ulps — what a reordered fp64 collide or the arrival
order of the spread's fp64 atomics produces — can flip an F_s component by one float ulp at a
near-tie, and the flip then spreads.  The oracle (oracle/oracle.c, the restatement) is run against
itself with its populations multiplied by (1 + mag * n), n uniform in {-2 .. 2} per population,
before every iteration; the maximum F_s difference in float ulps and the fields' relative
difference after the run are the envelope that tests/test_gpu_fused.py::test_ib_band_many_points
bounds the GPU by (2x).  Configuration = that test's: 320 x 160, 150 points in three filaments,
perturbed initial state (seed 11), body force 1e-6, 5K + 3 = 38 iterations at K = 7.
Test infrastructure (CPU, the oracle); the envelope is committed as tests/golden/ib_flip_envelope.json.
"""
import numpy as np

NX, NY, STEPS = 320, 160, 38
MAGS = (2.0 ** -52, 2.0 ** -50, 2.0 ** -48)
SEEDS = tuple(range(200, 208))


def line(xs, n, y0=3.0, dy=1.0, amp=1.5e-3):
    k = np.arange(n)
    s = np.empty(2 * n, dtype=np.float32)
    s[0::2] = xs + 0.25 * np.sin(0.3 * k)
    s[1::2] = y0 + dy * k
    us = np.zeros(2 * n, dtype=np.float32)
    us[0::2] = amp * (k / n)
    us[1::2] = -0.3 * amp * np.cos(0.2 * k)
    return s, us, (k % 7 != 3).astype(np.int32)


def points():
    return tuple(np.concatenate([p, q, r]) for p, q, r in zip(line(40.0, 30), line(60.0, 70, y0=30.0),
                                                              line(200.4, 50, y0=90.0)))


def float_ulps(a, b):
    ia = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(1 << 31) - ia, ia)
    ib = np.where(ib < 0, -(1 << 31) - ib, ib)
    return np.abs(ia - ib)


def run(O, mag=0.0, seed=0, steps=STEPS):
    """The oracle over `steps` iterations; populations perturbed by mag before every iteration."""
    from cuda_iblb_11_amd import workloads as W
    rho, u = W.perturbed_state(NX, NY, 11)
    sim = O.Simulation(NX, NY, W.TAU, W.TAU2, rho=rho, u=u, body_force=(1e-6, 0.0))
    sim.set_lagrangian(*points())
    g = np.random.default_rng(seed)
    fs = []
    for _ in range(steps):
        if mag:
            sim.f[:] = sim.f * (1 + mag * g.integers(-2, 3, sim.f.size))
        sim.step(1)
        fs.append(sim.F_s.copy())
    return sim, fs


def field_rel(x, y):
    """max over rho-1, u of max|x - y| / max|y| (rho - 1: the f64 test normalises rho by itself,
    which is ~1; rho - 1 is the stricter of the two)"""
    return max(float(np.max(np.abs((x.rho - 1) - (y.rho - 1))) / np.max(np.abs(y.rho - 1))),
               float(np.max(np.abs(x.u - y.u)) / np.max(np.abs(y.u))))


def envelope(O):
    """{mag: [(F_s ulps max, first iteration with a flip or -1, field difference), ...per seed]}"""
    ref, fref = run(O)
    out = {}
    for mag in MAGS:
        rows = []
        for seed in SEEDS:
            b, fb = run(O, mag, seed)
            ul = [int(float_ulps(x, y).max()) for x, y in zip(fref, fb)]
            first = next((i for i, v in enumerate(ul) if v > 0), -1)
            rows.append({"seed": seed, "fs_ulps": max(ul), "first_flip": first, "fields": field_rel(b, ref)})
        out[repr(mag)] = rows
    return out

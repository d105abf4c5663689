"""Pins of the CPU restatement (oracle/) — the checker every GPU parity test relies on.

The reference ships no tests and its CUDA sources cannot be built in this image (no nvcc /
CUDA runtime), so the restatement is pinned by (a) analytic known-answer tests that follow
from the reference's algorithm, (b) internal consistency between two independent forms of
the same reference kernel, (c) the reference's own nominal outputs as an envelope
(tests/golden/nominals_envelope.json).  See DESIGN.md "Oracle and parity".
"""
import json
import os

import numpy as np
import pytest

import slab_model as SM

HERE = os.path.dirname(os.path.abspath(__file__))
TAU, TAU2 = 2.806798146151282, 0.5361251085069444
W9 = np.array([4 / 9] + [1 / 9] * 4 + [1 / 36] * 4)


def test_reference_relaxation_times():
    """main.cu:314-321 with the default arguments (Re = 1, T = 1e5)."""
    from cuda_iblb_11_amd.lattice import reference_taus, RefParams
    tau, tau2 = reference_taus()
    assert abs(tau - TAU) < 1e-15 and abs(tau2 - TAU2) < 1e-15
    p = RefParams(1, 6, 48, 1.0, 1.0, 5, 1.0, 100, False, True)
    assert (p.XDIM, p.YDIM, p.T, p.ITERATIONS, p.INTERVAL) == (288, 192, 100000, 100000, 1000)
    assert abs(p.TAU - 2.806798146151282) < 1e-15


def test_streaming_push_equals_pull(oracle):
    """The literal push streaming (LatticeBoltzmann.cu:173-373) equals the independent numpy
    pull with periodic x, bounce-back bottom and same-cell mirror top."""
    rng = np.random.default_rng(0)
    for nx, ny in [(7, 5), (1, 4), (2, 2), (33, 17)]:
        f1 = rng.uniform(0, 1, 9 * nx * ny)
        f = np.zeros_like(f1)
        oracle.streaming(f1, f, nx, ny)
        assert np.array_equal(f, SM.pull_periodic(f1, nx, ny))


def test_streaming_is_a_permutation(oracle):
    """Every destination has exactly one source: streaming permutes values (mass exact)."""
    nx, ny = 9, 6
    f1 = np.arange(9 * nx * ny, dtype=np.float64)
    f = np.full_like(f1, -1)
    oracle.streaming(f1, f, nx, ny)
    assert np.array_equal(np.sort(f), f1)


def test_equilibrium_fixed_point_and_moments(oracle):
    """collision(f0, f=f0, F=0) returns f0 bit for bit; feq moments follow the reference's
    C_S = 0.57735 (rho * (1 + u^2 (1/(3 cs^2) - 1) / (2 cs^2)) for the zeroth moment)."""
    rng = np.random.default_rng(1)
    nx, ny = 10, 8
    n = nx * ny
    rho = 1 + 1e-3 * rng.uniform(-1, 1, n)
    u = 1e-2 * rng.uniform(-1, 1, 2 * n)
    f0, F = np.zeros(9 * n), np.zeros(9 * n)
    oracle.equilibrium(u, rho, f0, np.zeros(2 * n), F, nx, ny, TAU)
    assert np.all(F == 0)
    f1 = np.zeros(9 * n)
    oracle.collision(f0, f0.copy(), f1, F, TAU, TAU2, nx, ny, 0)
    assert np.array_equal(f1, f0)
    cs2 = 0.57735 ** 2
    fe = f0.reshape(n, 9)
    usq = u[:n] ** 2 + u[n:] ** 2
    assert np.allclose(fe.sum(1), rho * (1 + usq * (1 / (3 * cs2) - 1) / (2 * cs2)), rtol=0, atol=1e-15)
    assert np.allclose(fe @ SM.C_L[:, 0], rho * u[:n] / (3 * cs2), rtol=1e-10, atol=0)


def test_guo_force_moments(oracle):
    """Momentum the reference's forcing term injects: sum_i c_i F_i = (1 - 1/(2 TAU)) F / (3 cs^2)."""
    nx, ny = 4, 4
    n = nx * ny
    rng = np.random.default_rng(2)
    force = 1e-5 * rng.uniform(-1, 1, 2 * n)
    u = 1e-3 * rng.uniform(-1, 1, 2 * n)
    f0, F = np.zeros(9 * n), np.zeros(9 * n)
    oracle.equilibrium(u, np.ones(n), f0, force, F, nx, ny, TAU)
    Fm = F.reshape(n, 9)
    k = (1 - 1 / (2 * TAU)) / (3 * 0.57735 ** 2)
    assert np.allclose(Fm @ SM.C_L[:, 0], k * force[:n], rtol=1e-12, atol=0)
    assert np.allclose(Fm @ SM.C_L[:, 1], k * force[n:], rtol=1e-12, atol=0)


def test_poiseuille_kat(oracle):
    """Analytic KAT: x-uniform body force g in the reference channel.  Half-way bounce-back at
    y = -1/2 and the same-cell mirror (free slip) at y = Y - 1/2 give the half-channel profile
        u(y) = g_eff / (2 nu) * eta * (2Y - eta),   eta = y + 1/2,   nu = (TAU - 1/2)/3.
    The reference's TRT applies Guo's prefactor (1 - 1/(2 TAU)) to the odd moments too, so the
    momentum injected per step is g * (1 + 1/(2 TAU2) - 1/(2 TAU)) = 1.7545 g (g_eff)."""
    nx, ny, g = 4, 32, 1e-6
    sim = oracle.Simulation(nx, ny, TAU, TAU2, body_force=(g, 0.0))
    sim.step(20000)
    ux = sim.u[:nx * ny].reshape(ny, nx)
    assert np.all(ux == ux[:, :1])  # x-uniform
    geff = g * (1 + 0.5 / TAU2 - 0.5 / TAU)
    nu = (TAU - 0.5) / 3
    eta = np.arange(ny) + 0.5
    exact = geff / (2 * nu) * eta * (2 * ny - eta)
    err = ux[:, 0] / exact - 1
    assert np.max(np.abs(err[ny // 4:])) < 1e-3   # bulk
    assert np.max(np.abs(err)) < 2e-2             # wall cell (TRT wall offset at Lambda = 1/12)
    # no cross flow beyond the O(1e-6) compressibility the missing F_0 mass source drives
    assert np.max(np.abs(sim.u[nx * ny:])) < 1e-5 * np.max(ux)


def test_delta_kernel_moments(oracle):
    """3-point kernel (ImmersedBoundary.cu:21-81): sum_x phi(x - xs) = 1 and sum (x - xs) phi = 0
    up to the reference's truncated constants 0.33333 / 0.16667."""
    for xs in np.linspace(10.0, 11.0, 37, dtype=np.float32):
        xs = float(xs)
        nodes = range(int(np.floor(xs)) - 2, int(np.floor(xs)) + 4)
        phi0 = np.float32(0.33333 * 2)  # phi(0) of the y factor (ys = y = 0)
        phi = np.array([oracle.d_delta(xs, 0.0, x, 0) for x in nodes]) / phi0
        assert abs(phi.sum() - 1) < 5e-5
        assert abs(np.dot(np.array(nodes) - xs, phi)) < 5e-5
        assert sum(p != 0 for p in phi) <= 3
    assert oracle.d_delta(10.0, 0.0, 10, 0) == np.float32(np.float32(0.33333 * 2) * np.float32(0.33333 * 2))


def test_spread_cell_centric_equals_point_centric(oracle):
    """The literal O(N*Ns) gather (ImmersedBoundary.cu:178-231) and the 3x3 point scatter give
    bit-identical force, u and Q, including points at the x edges and epsilon = 0."""
    rng = np.random.default_rng(3)
    nx, ny = 48, 192
    n = nx * ny
    ns = 40
    s = np.empty(2 * ns, dtype=np.float32)
    s[0::2] = rng.uniform(0, nx, ns)
    s[1::2] = rng.uniform(0.5, 190, ns)
    s[0], s[2], s[4] = 0.1, nx - 0.2, np.float32(nx)
    F_s = (1e-3 * rng.uniform(-1, 1, 2 * ns)).astype(np.float32)
    eps = (rng.uniform(0, 1, ns) > 0.2).astype(np.int32)
    rho = 1 + 1e-3 * rng.uniform(-1, 1, n)
    f = rng.uniform(0.01, 0.5, 9 * n)
    outs = []
    for pc in (False, True):
        force, u, Q = np.zeros(2 * n), np.zeros(2 * n), np.zeros(1)
        oracle.spread(rho, u, f, ns, np.zeros(2 * ns, np.float32), F_s, force, s, nx, Q, eps, point_centric=pc)
        outs.append((force, u, Q))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_mass_conservation_without_force(oracle):
    """No force, u = 0 initially: walls and periodic x conserve mass; only the C_S != 1/sqrt(3)
    equilibrium mismatch can drift it, at O(u^2 * 1e-6)."""
    nx, ny = 16, 12
    rng = np.random.default_rng(4)
    rho = 1 + 1e-4 * rng.uniform(-1, 1, nx * ny)
    sim = oracle.Simulation(nx, ny, TAU, TAU2, rho=rho, u=np.zeros(2 * nx * ny))
    m0 = sim.f.sum()
    sim.step(200)
    assert abs(sim.f.sum() - m0) < 1e-12 * m0


def test_nominals_are_not_a_pin(oracle):
    """The reference's only shipped outputs (Data/Nominals: fluid snapshots at it = 1000, 50000,
    99000 and the cumulative flux of a 300x200 run, SimLog_nom.txt) come from an OLDER version of
    the code (LENGTH = 100, YDIM = 200, integer output coordinates).  Run the oracle in that
    configuration as closely as the current kinematics allow (300x200, TAU/TAU2 of SimLog_nom,
    6 cilia 50 apart, T = 1e5) and compare: the current code cannot reproduce them, so they pin
    nothing:
    * flux after iteration 0: the nominal is -2.05717e-06 (x_scale units); the current code has
      u_s = 0 at it = 0 (main.cu:200-204) on a fluid at rest, so Q is exactly 0;
    * stability: the nominal run stays at max|u| <= 4.8e-3 and rho within 1 % for 1e5 iterations;
      the current penalty IB (interpolate + spread, ImmersedBoundary.cu:94-267) with the current
      96-point cilia (main.cu:77-252) diverges within 100 iterations in the same configuration."""
    d = json.load(open(os.path.join(HERE, "golden", "nominals_envelope.json")))
    for snap in d["vector"].values():  # the committed statistics of the shipped files
        assert (snap["nx"], snap["ny"]) == (300, 200)
        assert 0.98 < snap["rho_min"] < 1 < snap["rho_max"] < 1.02 and 1e-3 < snap["u_max"] < 1e-2
    q_nominal = np.array(d["flux"]["Q"])
    assert q_nominal[0] == pytest.approx(-2.05717e-06) and np.all(np.diff(q_nominal[1:]) > 0)

    nx, ny, c_num, c_space, T = 300, 200, 6, 50.0, 100000
    speed = 0.8 * 1000 / T                      # main.cu:314 with LENGTH = 100 (SimLog_nom.txt:6)
    tau = speed * 100 / (1.0 * 0.577 ** 2) + 0.5
    tau2 = 1.0 / (12.0 * (tau - 0.5)) + 0.5
    assert (round(tau, 5), round(tau2, 5)) == (2.90291, 0.53468)  # "Relaxation times: 2.90291, 0.53468"
    x_scale = 1e6 * (1.0 / 100) * 6e-6          # main.cu:317 (l_0 = 6 um, dx = 1/LENGTH)
    sim = oracle.Simulation(nx, ny, tau, tau2)
    cil = oracle.Cilia(c_num, c_space, T, T // c_num, nx)
    umax, diverged_at = [], None
    for it in range(100):
        s, us, eps = cil.points(it)
        sim.set_lagrangian(s.copy(), us.copy(), eps.copy())
        sim.step(1)
        if it == 0:
            assert sim.flux * x_scale == 0.0 != q_nominal[0]
        m = float(np.max(np.hypot(sim.u[: nx * ny], sim.u[nx * ny:])))
        umax.append(m)
        if not np.isfinite(m) or m > 1.0:
            diverged_at = it
            break
    assert diverged_at is not None, max(umax)
    assert max(umax[:5]) < 2e-2  # the start is tame: the growth is the penalty feedback, not the kick


def test_cilia_kinematics_kats(oracle):
    """define_filament + boundary_check (main.cu:77-252): analytic pins of the beat.
    * base points (arc 0) sit at x = c_space*c_num/2 + (m - (c_num-1)/2) c_space, y = 1 exactly;
    * cilium m at iteration it has the shape of cilium 0 at it + m*p_step (metachronal lag);
    * u_s is the per-iteration displacement of the selected sample (zero at it = 0)."""
    c_num, c_space, T = 6, 48.0, 1000
    p_step = T * 1 // c_num
    cil = oracle.Cilia(c_num, c_space, T, p_step, XDIM=int(c_num * c_space))
    s, us, eps = [a.copy() for a in cil.points(0)]
    xy = s.reshape(c_num, 96, 2)
    for m in range(c_num):
        assert xy[m, 0, 1] == np.float32(1.0)
        assert xy[m, 0, 0] == np.float32(c_space * c_num / 2 + (m - (c_num - 1) / 2) * c_space)
    assert np.all(us == 0)
    prev = xy.copy()
    for it in range(1, 6):
        s, us, eps = cil.points(it)
        xy = s.reshape(c_num, 96, 2)
        d = (xy - prev).reshape(-1, 2)
        ok = np.abs(d).max(axis=1) < 1.0  # ignore points that wrapped across x = 0 / XDIM
        assert np.allclose(us.reshape(-1, 2)[ok], d[ok], atol=6e-5)  # ulps of x ~ 288 in float
        prev = xy.copy()
    # lag: cilium 1 now vs cilium 0 at it + p_step
    it = 5
    ref = oracle.Cilia(c_num, c_space, T, p_step, XDIM=int(c_num * c_space))
    for k in range(it + p_step + 1):
        r, _, _ = ref.points(k)
    a = xy[1] - [c_space, 0]
    b = r.reshape(c_num, 96, 2)[0]
    wrap = np.abs(a[:, 0] - b[:, 0]) > 100
    assert np.allclose(a[~wrap], b[~wrap], atol=1e-4)


def test_cilia_overlap_mask(oracle):
    """Densely packed cilia (c_space 12 < 2*LENGTH/c_space range) mask points that come within one
    lattice unit of a point of the preceding cilia; sparse cilia (c_space 128) never do."""
    dense = oracle.Cilia(16, 12.0, 200, 200 // 16, XDIM=16 * 12)
    masked = 0
    for it in range(0, 200, 10):
        _, _, eps = dense.points(it)
        masked = max(masked, int((eps == 0).sum()))
    assert masked > 0
    sparse = oracle.Cilia(4, 128.0, 200, 50, XDIM=512)
    for it in range(3):
        _, _, eps = sparse.points(it)
        assert np.all(eps == 1)


def _fs_line(xs, n, y0=3.0, dy=1.0, amp=1.5e-3):
    k = np.arange(n)
    s = np.empty(2 * n, dtype=np.float32)
    s[0::2] = xs + 0.25 * np.sin(0.3 * k)
    s[1::2] = y0 + dy * k
    us = np.zeros(2 * n, dtype=np.float32)
    us[0::2] = amp * (k / n)
    us[1::2] = -0.3 * amp * np.cos(0.2 * k)
    return s, us, (k % 7 != 3).astype(np.int32)


def _float_ulps(a, b):
    ia = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(1 << 31) - ia, ia)
    ib = np.where(ib < 0, -(1 << 31) - ib, ib)
    return np.abs(ia - ib)


def test_fs_float_ulp_flips(oracle):
    """Why the f64 IB parity bound with many points is 1e-8 and not 1e-10: the
    reference accumulates F_s in float (ImmersedBoundary.cu:124-125).  The restatement run against
    ITSELF, with the initial populations perturbed by one double ulp (2^-52, the size of the GPU
    collide's rounding differences), flips some F_s by a few float ulps and the fields then differ
    by ~1e-9 .. 1e-8; a perturbation (2^-50, other sign pattern) that flips none leaves them at
    ~1e-13, and an unperturbed rerun is bit-identical.  Same configuration as
    tests/test_gpu_fused.py::test_ib_band_many_points (320 x 160, 150 points, 31 iterations)."""
    from cuda_iblb_11_amd import workloads as W
    nx, ny, N = 320, 160, 320 * 160
    pts = tuple(np.concatenate([p, q, r]) for p, q, r in zip(_fs_line(40.0, 30), _fs_line(60.0, 70, y0=30.0),
                                                              _fs_line(200.4, 50, y0=90.0)))
    rho, u = W.perturbed_state(nx, ny, 11)

    def run(eps):
        f = oracle.feq(rho, u, nx, ny, W.TAU)
        f = f * (1 + eps * np.random.default_rng(3).integers(-1, 2, f.size))
        sim = oracle.Simulation(nx, ny, W.TAU, W.TAU2, rho=rho, u=u, f=f, body_force=(1e-6, 0.0))
        sim.set_lagrangian(*pts)
        fs = []
        for _ in range(31):
            sim.step(1)
            fs.append(sim.F_s.copy())
        return sim, fs

    def d(x, y):
        return max(float(np.max(np.abs((x.rho - 1) - (y.rho - 1))) / np.max(np.abs(y.rho - 1))),
                   float(np.max(np.abs(x.u - y.u)) / np.max(np.abs(y.u))))

    a, fa = run(0.0)
    a2, fa2 = run(0.0)
    assert d(a2, a) == 0.0 and all(np.array_equal(x, y) for x, y in zip(fa, fa2))
    b, fb = run(2.0 ** -52)
    flips = max(int(_float_ulps(x, y).max()) for x, y in zip(fa, fb))
    assert 1 <= flips <= 8, flips
    assert 1e-10 < d(b, a) <= 1e-8, d(b, a)
    c, fc = run(2.0 ** -50)
    assert max(int(_float_ulps(x, y).max()) for x, y in zip(fa, fc)) == 0
    assert d(c, a) <= 1e-12, d(c, a)


def test_ib_flip_envelope(oracle):
    """The envelope the GPU's many-point IB test is bounded by, pinned: the
    oracle against itself over that test's whole horizon (38 iterations = 5K + 3 at K = 7), with
    every population multiplied by 1 + mag * n (n in {-2..2}) before every iteration — the scale of
    a reordered fp64 collide (2^-52) up to a few ulps per operation chain (2^-48).  Reproduces
    tests/golden/ib_flip_envelope.json exactly (tests/golden/make_ib_flip_envelope.py); the flips are
    discrete near-ties of the float F_s sum: at 2^-52 a run either flips none (fields <= 1e-11) or the
    same component (40 ulps, fields 7.1e-9, first at iteration 12); at 2^-48 tens of ulps and fields
    up to 2e-8.  The GPU test asserts <= 2x the envelope's maxima."""
    import json
    import ib_flips
    fix = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ib_flip_envelope.json")))
    env = ib_flips.envelope(oracle)
    for mag, rows in env.items():
        for r, g in zip(rows, fix["runs"][mag]):
            assert r["fs_ulps"] == g["fs_ulps"] and r["first_flip"] == g["first_flip"], (mag, r, g)
            assert abs(r["fields"] - g["fields"]) <= 1e-3 * g["fields"], (mag, r, g)
    tiny = env[repr(2.0 ** -52)]
    assert {r["fs_ulps"] for r in tiny} == {0, 40}
    assert all((r["fields"] <= 1e-11) if r["fs_ulps"] == 0 else (6e-9 < r["fields"] < 8e-9) for r in tiny)
    big = env[repr(2.0 ** -48)]
    assert 20 <= max(r["fs_ulps"] for r in big) <= 100 and 1e-8 <= max(r["fields"] for r in big) <= 3e-8
    assert fix["max_fs_ulps"] == max(r["fs_ulps"] for rows in env.values() for r in rows)


def test_f32_model_tracks_oracle(oracle):
    """tests/f32_model.py (the float32 floor the GPU f32 parity is judged against) is the oracle's
    iteration: 11 iterations from a perturbed 64 x 48 channel agree to float32 rounding."""
    from cuda_iblb_11_amd import workloads as W
    from f32_model import F32Channel
    nx, ny = 64, 48
    rho, u = W.perturbed_state(nx, ny, 7)
    sim = oracle.Simulation(nx, ny, W.TAU, W.TAU2, rho=rho, u=u, body_force=W.BODY_FORCE)
    m = F32Channel(nx, ny, W.TAU, W.TAU2, rho, u, W.BODY_FORCE)
    sim.step(11)
    m.step(11)
    r, v = m.macro()
    n = nx * ny
    rel = lambda a, b: float(np.max(np.abs(a - b)) / np.max(np.abs(b)))
    assert rel(r - 1, sim.rho - 1) < 5e-6
    assert rel(v[:n], sim.u[:n]) < 5e-6 and rel(v[n:], sim.u[n:]) < 5e-6


def test_f32_gpu_order_over_1000_iterations(oracle):
    """tests/f32_gpu_model.py (the kernels' f32 arithmetic, op for op, on the CPU) against the oracle
    on the K1 horizon (128^2, 1000 iterations).  The round-3 order ("r03": rho * constant and
    rho (c.u) with the float32-rounded rho) lands where the GPU's round-3 f32 path was measured
    (rho - 1 1.8e-4, u_x 1.2e-6, u_y 8.4e-5, profiles/r03z/parity_f32.json): the cause of the gap to
    the 1e-4 bound.  The kernels' current order (odd part from the momentum, rho-scaled constants
    as c + (rho - 1) c) holds every field within 1e-4."""
    from cuda_iblb_11_amd import workloads as W
    from f32_gpu_model import F32GpuChannel
    nx = ny = 128
    rho, u = W.perturbed_state(nx, ny, 31)
    oracle.set_threads(min(8, os.cpu_count() or 1))
    sim = oracle.Simulation(nx, ny, W.TAU, W.TAU2, rho=rho, u=u, body_force=W.BODY_FORCE)
    sim.step(1000)
    n = nx * ny
    err = {}
    for v in ("r03", "gpu"):
        m = F32GpuChannel(nx, ny, W.TAU, W.TAU2, rho, u, W.BODY_FORCE, variant=v)
        m.step(1000)
        r, uu = m.macro()
        err[v] = {"rho-1": float(np.max(np.abs(r - sim.rho)) / np.max(np.abs(sim.rho - 1))),
                  "ux": float(np.max(np.abs(uu[:n] - sim.u[:n])) / np.max(np.abs(sim.u[:n]))),
                  "uy": float(np.max(np.abs(uu[n:] - sim.u[n:])) / np.max(np.abs(sim.u[n:])))}
    assert 1.5e-4 <= err["r03"]["rho-1"] <= 2.1e-4 and 5e-5 <= err["r03"]["uy"] <= 1.2e-4, err
    assert max(err["gpu"].values()) <= 1e-4, err

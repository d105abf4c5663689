"""Kernel-level parity of the reference-shaped HIP kernels (include/iblb.h part 1) against the
CPU restatement of the same reference kernel (oracle/oracle.c), on identical seeded inputs.

The LBM kernels and interpolate are compared BIT FOR BIT (same expression order, contraction
off on both sides).  spread scatters with fp64 atomics, so a cell reached by several points
sums in arrival order: compared to 1e-15 relative (exact when points are >= 3 cells apart).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

X, Y = 72, 40  # N = 2880, not a multiple of 128: exercises the tail guard


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _h(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _state(rng, X, Y):
    n = X * Y
    rho = 1.0 + 1e-3 * rng.uniform(-1, 1, n)
    u = 1e-3 * rng.uniform(-1, 1, 2 * n)
    force = 1e-5 * rng.uniform(-1, 1, 2 * n)
    w = np.array([4 / 9] + [1 / 9] * 4 + [1 / 36] * 4)
    f = np.tile(w, n) * (1 + 1e-3 * rng.uniform(-1, 1, 9 * n))
    return rho, u, force, f


def test_equilibrium_collision_bitexact(gpu, oracle):
    from cuda_iblb_11_amd import kernels as K
    rng = np.random.default_rng(1)
    rho, u, force, f = _state(rng, X, Y)
    tau, tau2 = 2.806798146151282, 0.5361251085069444
    n = X * Y
    f0o, Fo, f1o = np.zeros(9 * n), np.zeros(9 * n), np.zeros(9 * n)
    oracle.equilibrium(u, rho, f0o, force, Fo, X, Y, tau)
    oracle.collision(f0o, f, f1o, Fo, tau, tau2, X, Y, 0)
    import torch
    du, dr, dforce, df = _t(u), _t(rho), _t(force), _t(f)
    df0 = torch.zeros(9 * n, dtype=torch.float64, device="cuda")
    dF = torch.zeros_like(df0)
    df1 = torch.zeros_like(df0)
    K.equilibrium(du, dr, df0, dforce, dF, X, Y, tau)
    K.collision(df0, df, df1, dF, tau, tau2, X, Y, 0)
    assert np.array_equal(_h(df0), f0o)
    assert np.array_equal(_h(dF), Fo)
    assert np.array_equal(_h(df1), f1o)


@pytest.mark.parametrize("shape", [(72, 40), (5, 3), (1, 7), (130, 2)])
def test_streaming_macro_bitexact(gpu, oracle, shape):
    from cuda_iblb_11_amd import kernels as K
    Xs, Ys = shape
    rng = np.random.default_rng(2)
    n = Xs * Ys
    f1 = rng.uniform(0.01, 0.5, 9 * n)
    fo, uo, ro = np.zeros(9 * n), np.zeros(2 * n), np.zeros(n)
    oracle.streaming(f1, fo, Xs, Ys)
    oracle.macro(fo, uo, ro, Xs, Ys)
    import torch
    df = torch.zeros(9 * n, dtype=torch.float64, device="cuda")
    du = torch.zeros(2 * n, dtype=torch.float64, device="cuda")
    dr = torch.zeros(n, dtype=torch.float64, device="cuda")
    K.streaming(_t(f1), df, Xs, Ys)
    K.macro(df, du, dr, Xs, Ys)
    assert np.array_equal(_h(df), fo)
    assert np.array_equal(_h(du), uo)
    assert np.array_equal(_h(dr), ro)


def test_delta_bitexact(gpu, oracle):
    from cuda_iblb_11_amd import kernels as K
    rng = np.random.default_rng(3)
    m = 20000
    xs = rng.uniform(0, 300, m).astype(np.float32)
    ys = rng.uniform(0, 190, m).astype(np.float32)
    x = (np.rint(xs) + rng.integers(-2, 3, m)).astype(np.int32)
    y = (np.rint(ys) + rng.integers(-2, 3, m)).astype(np.int32)
    # exact half-integer and support-edge cases
    xs[:8] = np.float32([0.5, 1.5, 2.0, 2.5, 100.25, 3.0, 0.0, 287.5])
    x[:8] = np.int32([0, 0, 3, 1, 101, 1, 0, 289])
    import torch
    out = torch.zeros(m, dtype=torch.float32, device="cuda")
    K.d_delta(_t(xs), _t(ys), _t(x), _t(y), out)
    ref = np.array([oracle.d_delta(float(a), float(b), int(c), int(d)) for a, b, c, d in zip(xs, ys, x, y)],
                   dtype=np.float32)
    assert np.array_equal(_h(out), ref)


def _points(rng, ns, X, spacing):
    s = np.empty(2 * ns, dtype=np.float32)
    s[0::2] = (rng.uniform(-0.4, 0.4, ns) + np.arange(ns) * spacing) % X
    s[1::2] = rng.uniform(1.0, 180.0, ns)
    s[0] = 0.3   # x0 = 0: node x = -1 reads the previous row (reference flat index)
    s[2] = X - 0.2  # node x = X clipped in spread
    u_s = (1e-3 * rng.uniform(-1, 1, 2 * ns)).astype(np.float32)
    eps = np.ones(ns, dtype=np.int32)
    eps[5] = 0
    return s, u_s, eps


@pytest.mark.parametrize("spacing", [4.0, 0.7])
def test_interpolate_spread(gpu, oracle, spacing):
    from cuda_iblb_11_amd import kernels as K
    Xs, Ys = 96, 192
    rng = np.random.default_rng(4)
    n = Xs * Ys
    ns = 20
    rho = 1.0 + 1e-3 * rng.uniform(-1, 1, n)
    u = 1e-3 * rng.uniform(-1, 1, 2 * n)
    f = rng.uniform(0.01, 0.5, 9 * n)
    s, u_s, eps = _points(rng, ns, Xs, spacing)
    Fso = np.zeros(2 * ns, dtype=np.float32)
    oracle.interpolate(rho, u, ns, u_s, Fso, s, Xs, Ys)
    forceo, uo, Qo = np.zeros(2 * n), u.copy(), np.zeros(1)
    oracle.spread(rho, uo, f, ns, u_s, Fso, forceo, s, Xs, Qo, eps)  # literal O(N*Ns) form
    import torch
    dFs = torch.zeros(2 * ns, dtype=torch.float32, device="cuda")
    K.interpolate(_t(rho), _t(u), ns, _t(u_s), dFs, _t(s), Xs, Ys)
    assert np.array_equal(_h(dFs), Fso)
    du = _t(u.copy())
    dforce = torch.zeros(2 * n, dtype=torch.float64, device="cuda")
    dQ = torch.zeros(1, dtype=torch.float64, device="cuda")
    K.spread(_t(rho), du, _t(f), ns, _t(u_s), dFs, dforce, _t(s), Xs, dQ, _t(eps))
    fg, ug, Qg = _h(dforce), _h(du), _h(dQ)
    if spacing >= 4.0:
        assert np.array_equal(fg, forceo)
    assert np.max(np.abs(fg - forceo)) <= 1e-15 * np.max(np.abs(forceo))
    assert np.max(np.abs(ug - uo)) <= 1e-15 * np.max(np.abs(uo))
    assert abs(Qg[0] - Qo[0]) <= 1e-13 * abs(Qo[0])


@pytest.mark.parametrize("c_num,c_space,T", [(6, 48.0, 1000), (12, 24.0, 300), (64, 128.0, 5000)])
def test_cilia_kernels_bitexact(gpu, oracle, c_num, c_space, T):
    """iblb_define_filament / iblb_boundary_check (main.cu:77, 176) against the restatement,
    several consecutive iterations (lasts carries the previous positions)."""
    import torch
    from cuda_iblb_11_amd import kernels as K
    XDIM = int(c_num * c_space)
    p_step = T * 1 // c_num
    cil = oracle.Cilia(c_num, c_space, T, p_step, XDIM)
    nk = 9600 * c_num
    samples = torch.zeros(5 * nk, dtype=torch.float32, device="cuda")
    lasts = torch.zeros(2 * nk, dtype=torch.float32, device="cuda")
    bp = torch.zeros(5 * 96 * c_num, dtype=torch.float32, device="cuda")
    s = torch.zeros(2 * 96 * c_num, dtype=torch.float32, device="cuda")
    us = torch.zeros_like(s)
    eps = torch.zeros(96 * c_num, dtype=torch.int32, device="cuda")
    # small beats run past it + m*p_step == T (the reference's phase = T special case)
    iters = range(4) if c_num > 12 else range(p_step + 2)
    for it in iters:
        so, uso, eo = cil.points(it)
        K.define_filament(T, it, c_space, p_step, c_num, samples, lasts, bp)
        K.boundary_check(c_space, c_num, XDIM, it, bp, s, us, eps)
        assert np.array_equal(_h(samples), cil.samples)
        assert np.array_equal(_h(bp), cil.b_points)
        assert np.array_equal(_h(s), so) and np.array_equal(_h(us), uso) and np.array_equal(_h(eps), eo)

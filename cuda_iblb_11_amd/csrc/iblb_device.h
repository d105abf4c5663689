// iblb_device.h — device-side building blocks of the MI355X IB-LBM hot path (gfx950).
//
// Lattice: D2Q9 with the reference's velocity order (LatticeBoltzmann.cu:15-27):
//   i : 0      1      2      3       4       5      6       7        8
//   c : (0,0)  (1,0)  (0,1)  (-1,0)  (0,-1)  (1,1)  (-1,1)  (-1,-1)  (1,-1)
//   w : 4/9    1/9 x4                        1/36 x4
//
// Slab layout in HBM (one context = one x-slab [x_begin, x_begin+ncol)):
//   g[xc*col + i*plane + y]  — the nine planes of a column adjacent (plane = ny rounded up to
//   whole waves), y fastest, columns contiguous.  A slab of a group keeps `gc` ghost columns
//   on each side inside the same buffer (xc in [-gc, 0) and [ncol, ncol+gc)): its halo is
//   one contiguous block of whole columns per side, sent and received by RCCL in place.
//
// State held between steps: post-collision populations f1^{t-1} ("g").  Streaming is a
// PULL applied when g is read:
//   f^t(x,y,k) = g(x-cx_k, y-cy_k, k)                  interior, x periodic
//   f^t(x,0,k)    = g(x,0,bb(k))    k in {2,5,6}, bb = {4,7,8}   bounce-back
//   f^t(x,Y-1,k)  = g(x,Y-1,sl(k))  k in {4,8,7}, sl = {2,5,6}   same-cell mirror
// which is the reference's push streaming (LatticeBoltzmann.cu:173-373) read backwards.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace iblb {

constexpr int Q9 = 9;
__host__ __device__ constexpr int cx(int i) {
    return i == 1 || i == 5 || i == 8 ? 1 : (i == 3 || i == 6 || i == 7 ? -1 : 0);
}
__host__ __device__ constexpr int cy(int i) {
    return i == 2 || i == 5 || i == 6 ? 1 : (i == 4 || i == 7 || i == 8 ? -1 : 0);
}
__host__ __device__ constexpr double wgt(int i) {
    return i == 0 ? 4. / 9 : (i < 5 ? 1. / 9 : 1. / 36);
}
// planes a slab receives from its LEFT neighbour (cx = +1) and from its RIGHT (cx = -1)
__host__ __device__ constexpr int left_plane(int p) { return p == 0 ? 1 : (p == 1 ? 5 : 8); }
__host__ __device__ constexpr int right_plane(int p) { return p == 0 ? 3 : (p == 1 ? 6 : 7); }
__host__ __device__ constexpr int halo_slot(int k) {  // slot of plane k inside its halo triple
    return (k == 1 || k == 3) ? 0 : ((k == 5 || k == 6) ? 1 : 2);
}

struct Layout {
    int ny;      // lattice height Y
    int ncol;    // columns in this slab
    long col;    // column stride of the populations (elements)
    long plane;  // plane stride of the populations (elements)
    long rows;   // ny rounded up to whole waves: the column stride of the dense force and the
                 // boot fields (plane stride fplane)
};

// Pointers to the three halo planes of column -1 (left, planes 1,5,8) and column
// ncol (right, planes 3,6,7).  Lone slab: they point into g itself (periodic wrap); slab of a
// group: into its ghost columns -1 and ncol.
template <typename T>
struct Halo {
    const T* left[3];
    const T* right[3];
};

// Relaxation and forcing constants shared by every collide.
struct Coef {
    double omega_p, omega_m;   // 1/TAU, 1/TAU2      (LatticeBoltzmann.cu:72-73)
    double kguo;               // 1 - 1/(2 TAU)      (LatticeBoltzmann.cu:56)
    double inv_cs2, inv_cs4;   // 1/C_S^2, 1/C_S^4 with C_S = 0.57735 (LatticeBoltzmann.cu:11)
    double inv_2cs2, inv_2cs4; // 1/(2 C_S^2), 1/(2 C_S^4)
    double gx, gy;             // uniform body force (extension, 0 in the reference)
};

// Scalar pull of f^t(xc, y, k) from g (used by every non-hot kernel).
template <typename T>
__device__ __forceinline__ T pull(const T* __restrict__ g, const Layout& L, const Halo<T>& H,
                                  int xc, int y, int k) {
    if (y == 0 && cy(k) == 1) {
        const int kk = k == 2 ? 4 : (k == 5 ? 7 : 8);
        return g[kk * L.plane + xc * L.col];
    }
    if (y == L.ny - 1 && cy(k) == -1) {
        const int kk = k == 4 ? 2 : (k == 8 ? 5 : 6);
        return g[kk * L.plane + xc * L.col + y];
    }
    const int sx = xc - cx(k), sy = y - cy(k);
    if (sx < 0) return H.left[halo_slot(k)][sy];
    if (sx >= L.ncol) return H.right[halo_slot(k)][sy];
    return g[k * L.plane + (long)sx * L.col + sy];
}

// Pull of f^t(xl, y, k) from a buffer whose columns xl-1 .. xl+1 are all present: the slab's own
// columns or its ghost columns (a slab of a group holds `gc` ghost columns on each side, filled
// from the neighbours; a lone slab fills them with periodic copies when a band cycle needs them).
template <typename T>
__device__ __forceinline__ T pull_direct(const T* __restrict__ g, const Layout& L, int xl, int y, int k) {
    if (y == 0 && cy(k) == 1) return g[(k == 2 ? 4 : (k == 5 ? 7 : 8)) * L.plane + (long)xl * L.col];
    if (y == L.ny - 1 && cy(k) == -1) return g[(k == 4 ? 2 : (k == 8 ? 5 : 6)) * L.plane + (long)xl * L.col + y];
    return g[k * L.plane + (long)(xl - cx(k)) * L.col + (y - cy(k))];
}

// Storage conversion: double planes hold f, float planes hold the deviation f - w_i.
template <typename T>
struct Store;
template <>
struct Store<double> {
    static constexpr bool dev = false;
    __device__ __forceinline__ static double to_f(double v, int) { return v; }
    __device__ __forceinline__ static double from_f(double v, int) { return v; }
};
template <>
struct Store<float> {
    static constexpr bool dev = true;
    __device__ __forceinline__ static double to_f(float v, int i) { return (double)v + wgt(i); }
    __device__ __forceinline__ static float from_f(double v, int i) { return (float)(v - wgt(i)); }
};

// Macroscopic moments of one cell in the reference's summation order
// (LatticeBoltzmann.cu:396-405): rho = f0+...+f8, m = sum c f.  For deviation storage
// `rho` returns sum h (= rho - 1); the caller adds 1.
template <typename R>
__device__ __forceinline__ void moments(const R f[9], R& rho, R& mx, R& my) {
#pragma clang fp contract(on)
    rho = f[0] + f[1] + f[2] + f[3] + f[4] + f[5] + f[6] + f[7] + f[8];
    mx = ((((f[1] - f[3]) + f[5]) - f[6]) - f[7]) + f[8];
    my = ((((f[2] - f[4]) + f[5]) + f[6]) - f[7]) - f[8];
}

// TRT collision with the reference's Guo forcing (LatticeBoltzmann.cu:30-62, 64-171)
// written on the sum s = f_i + f_ibar and difference d = f_i - f_ibar of each pair
// (i, ibar) = (1,3) (2,4) (5,7) (6,8):
//   feq+ = rho w (1 + (c.u)^2/(2cs^4) - u^2/(2cs^2)),   feq- = rho w (c.u)/cs^2
//   F+   = k w (-(u.F)/cs^2 + (c.u)(c.F)/cs^4),          F-   = k w (c.F)/cs^2
//   f1_i    = f_i    - w+ (s/2 - feq+) - w- (d/2 - feq-) + F+ + F-
//   f1_ibar = f_ibar - w+ (s/2 - feq+) + w- (d/2 - feq-) + F+ - F-
//   f1_0    = f_0 - w+ (f_0 - feq_0)                      (no F_0, as in the reference)
// With E = w+ feq+ + F+ and O = w- feq- + F-:
//   f1_i = (1-w+)/2 s + (1-w-)/2 d + (E + O),   f1_ibar = (1-w+)/2 s - (1-w-)/2 d + (E - O)
// Algebraically identical to the reference; rounding differs at the 1e-16 level.  Every product
// of constants is folded once on the host (KBase: relaxation / weights; KForce: the force), so
// a pair costs ~11 operations and the per-cell moments come from the pair sums and
// differences; the multi-iteration kernels are bound by fp64 issue and register space, and the
// folded constants are kernel arguments (scalar registers) instead of per-wave recomputations.
// DEV: f holds deviations h = f - w (float storage); sum = rho - 1.
__device__ __forceinline__ double fmaR(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fmaR(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// pair p = 0..3: members a(p) (c = (1,0), (0,1), (1,1), (-1,1)) and b(p) = opposite
__host__ __device__ constexpr int pair_a(int p) { return p == 0 ? 1 : (p == 1 ? 2 : (p == 2 ? 5 : 6)); }
__host__ __device__ constexpr int pair_b(int p) { return p == 0 ? 3 : (p == 1 ? 4 : (p == 2 ? 7 : 8)); }

// Constants of the collision in the compute type R (weight class cl: 0 = axis 1/9, 1 = diagonal 1/36)
template <typename R>
struct KBase {
    R omp, opw0;           // 1 - w+,  w+ 4/9
    R opw[2], oqa[2];      // w+ w,    w+ w / (2 cs^4)
    R omwi2[2];            // w- w / cs^2
    R kw[2], kwi4[2], kwi2[2];  // k w, k w / cs^4, k w / cs^2   (k = 1 - 1/(2 TAU))
    R a1, ics2;            // 1/(2 cs^2), 1/cs^2
    R hs, hd, nhd;         // (1-w+)/2, (1-w-)/2, -(1-w-)/2
    R nck[2];              // -k w / cs^2 (the forcing's even part per weight class: u.F times it)
};
// Force-dependent constants (uniform for a body force; per cell with an IB force)
template <typename R>
struct KForce {
    R Fx, Fy, hFx, hFy;    // F, F/2
    R hE[4], gO[4];        // per pair: k w (c.F) / cs^4,  k w (c.F) / cs^2
};

template <typename R>
__host__ __device__ inline KBase<R> make_kbase(const Coef& c) {
#pragma clang fp contract(off)
    KBase<R> b;
    const R op = (R)c.omega_p, om = (R)c.omega_m, kk = (R)c.kguo;
    const R ics2 = (R)c.inv_cs2, ics4 = (R)c.inv_cs4, a2 = (R)c.inv_2cs4;
    b.omp = (R)1 - op;
    b.opw0 = op * (R)(4. / 9);
    for (int cl = 0; cl < 2; ++cl) {
        const R w = cl == 0 ? (R)(1. / 9) : (R)(1. / 36);
        b.opw[cl] = op * w;
        b.oqa[cl] = b.opw[cl] * a2;
        b.omwi2[cl] = om * w * ics2;
        b.kw[cl] = kk * w;
        b.kwi4[cl] = b.kw[cl] * ics4;
        b.kwi2[cl] = b.kw[cl] * ics2;
        b.nck[cl] = -(ics2 * b.kw[cl]);
    }
    b.a1 = (R)c.inv_2cs2;
    b.ics2 = ics2;
    b.hs = (R)0.5 * b.omp;
    b.hd = (R)0.5 * ((R)1 - om);
    b.nhd = -b.hd;
    return b;
}

// The same arithmetic on the host (uniform body force) and on the device (per-cell force), so a
// cell without IB force collides bit-identically in every kernel
template <typename R>
__host__ __device__ inline KForce<R> make_kforce(const KBase<R>& b, R Fx, R Fy) {
#pragma clang fp contract(off)
    KForce<R> k;
    k.Fx = Fx;
    k.Fy = Fy;
    k.hFx = (R)0.5 * Fx;
    k.hFy = (R)0.5 * Fy;
    const R cF[4] = {Fx, Fy, Fx + Fy, Fy - Fx};
    for (int p = 0; p < 4; ++p) {
        const int cl = p < 2 ? 0 : 1;
        k.hE[p] = cF[p] * b.kwi4[cl];
        k.gO[p] = cF[p] * b.kwi2[cl];
    }
    return k;
}

// JM (the f32 path): the odd equilibrium part from the momentum j = rho u = m + F/2 itself,
// w- feq- = (w- w / cs^2) c.j, and the rho-scaled constants as c + (rho - 1) c: the density rounded
// to float32 (rho = 1 + (rho - 1) keeps ~7 digits of a deviation ~1e-5) then enters only through
// 1/rho.  Measured on the K1 1000-iteration f32 run in the CPU emulation of this arithmetic
// (tests/f32_gpu_model.py): rho - 1 1.8e-4 -> 7.9e-5, u_y 8.9e-5 -> 3.6e-5.
template <typename R, bool DEV, bool JM = false>
__device__ __forceinline__ void collide_sd(R f[9], const R s[4], const R d[4], R rho, R sum, R ux, R uy,
                                           const KBase<R>& b, const KForce<R>& k, R jx = 0, R jy = 0) {
#pragma clang fp contract(on)  // fuse within a statement only: the same FMAs in every kernel
    const R usq = ux * ux + uy * uy;
    const R uF = ux * k.Fx + uy * k.Fy;
    const R base = -usq * b.a1;            // even equilibrium part common to all i
    // rho (1 + base), the even equilibrium factor (deviation form: minus the rest density 1)
    const R rb = DEV ? fmaR(rho, base, sum) : rho * ((R)1 + base);
    // rest population: f0 - w+ (f0 - feq0) = (1 - w+) f0 + w+ feq0
    f[0] = fmaR(b.omp, f[0], rb * b.opw0);
    // per weight class: E = P + Qa cu^2 + cu hE_p,  O = Rm cu + gO_p, with
    // P = w+ w rho (1 + base) - k w (u.F) / cs^2
    R P[2], Qa[2], Rm[2];
#pragma unroll
    for (int cl = 0; cl < 2; ++cl) {
        P[cl] = fmaR(rb, b.opw[cl], uF * b.nck[cl]);
        if (JM) {
            Qa[cl] = fmaR(sum, b.oqa[cl], b.oqa[cl]);
            Rm[cl] = b.omwi2[cl];
        } else {
            Qa[cl] = rho * b.oqa[cl];
            Rm[cl] = rho * b.omwi2[cl];
        }
    }
    // per pair: the even part A = hs s + E and the odd part B = hd d + O of the post-collision
    // pair, f_a = A + B, f_b = A - B (7-8 fp64 operations per pair; the kernels are issue-bound
    // on fp64, profiles/r02ai)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int a = pair_a(p), bb = pair_b(p);
        const int cl = p < 2 ? 0 : 1;
        const R cu = p == 0 ? ux : (p == 1 ? uy : (p == 2 ? ux + uy : uy - ux));  // c_a . u
        const R E = fmaR(cu, fmaR(Qa[cl], cu, k.hE[p]), P[cl]);
        const R cj = JM ? (p == 0 ? jx : (p == 1 ? jy : (p == 2 ? jx + jy : jy - jx))) : cu;  // c_a . j
        const R O = fmaR(Rm[cl], cj, k.gO[p]);
        const R A = fmaR(s[p], b.hs, E);
        const R B = fmaR(d[p], b.hd, O);
        f[a] = A + B;
        f[bb] = A - B;
    }
}

// The collision given rho and u explicitly (boot step)
template <typename R, bool DEV>
__device__ __forceinline__ void collide(R f[9], R rho, R drho, R ux, R uy, const KBase<R>& b, const KForce<R>& k) {
#pragma clang fp contract(on)
    R s[4], d[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        s[p] = f[pair_a(p)] + f[pair_b(p)];
        d[p] = f[pair_a(p)] - f[pair_b(p)];
    }
    collide_sd<R, DEV>(f, s, d, rho, drho, ux, uy, b, k);
}

// 1/x: v_rcp (about single precision) refined by two Newton steps (within an ulp of the
// correctly rounded quotient; ~5 fp64 operations instead of the ~12 of an IEEE division)
__device__ __forceinline__ double recip(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
    return __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
}
__device__ __forceinline__ float recip(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(r, __builtin_fmaf(-x, r, 1.f), r);
}

// The f32 (deviation storage) collide with explicit operations only (no contraction left to the
// compiler), on one cell (V = float) or on the two cells of a lane at once (V = f32x2: every
// operation one packed VALU instruction, v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32, constants
// broadcast from scalar registers).  The same operations in the same order per element, so both
// round every cell identically: the deep sweep's packed walk stays bit-identical to the one-step
// kernels.  rho-free odd part and rho-scaled constants as collide_sd's JM.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float vfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ f32x2 vfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ float vrcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ f32x2 vrcp(f32x2 x) { return f32x2{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)}; }

template <typename V>
__device__ __forceinline__ V relax_dev(V f[9], const KBase<float>& b, const KForce<float>& k) {
#pragma clang fp contract(off)
    V s[4], d[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        s[p] = f[pair_a(p)] + f[pair_b(p)];
        d[p] = f[pair_a(p)] - f[pair_b(p)];
    }
    const V sum = f[0] + ((s[0] + s[1]) + (s[2] + s[3]));
    const V mx = d[0] + (d[2] - d[3]);
    const V my = d[1] + (d[2] + d[3]);
    const V rho = (V)1.f + sum;
    V inv = vrcp(rho);  // + one Newton step (recip(float))
    inv = vfma(inv, vfma(-rho, inv, (V)1.f), inv);
    const V jx = mx + (V)k.hFx, jy = my + (V)k.hFy;
    const V ux = jx * inv, uy = jy * inv;
    const V usq = vfma(uy, uy, ux * ux);
    const V uF = vfma(uy, (V)k.Fy, ux * (V)k.Fx);
    const V base = -usq * (V)b.a1;
    const V rb = vfma(rho, base, sum);
    f[0] = vfma((V)b.omp, f[0], rb * (V)b.opw0);
    V P[2], Qa[2];
#pragma unroll
    for (int cl = 0; cl < 2; ++cl) {
        P[cl] = vfma(rb, (V)b.opw[cl], uF * (V)b.nck[cl]);
        Qa[cl] = vfma(sum, (V)b.oqa[cl], (V)b.oqa[cl]);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int cl = p < 2 ? 0 : 1;
        const V cu = p == 0 ? ux : (p == 1 ? uy : (p == 2 ? ux + uy : uy - ux));
        const V cj = p == 0 ? jx : (p == 1 ? jy : (p == 2 ? jx + jy : jy - jx));
        const V E = vfma(cu, vfma(Qa[cl], cu, (V)k.hE[p]), P[cl]);
        const V O = vfma((V)b.omwi2[cl], cj, (V)k.gO[p]);
        const V A = vfma(s[p], (V)b.hs, E);
        const V B = vfma(d[p], (V)b.hd, O);
        f[pair_a(p)] = A + B;
        f[pair_b(p)] = A - B;
    }
    return ux;
}

// One cell of a collide-stream step: f = the pulled populations f^t (deviations if DEV), k = the
// constants of the cell's force (body force + IB force).  rho and u^t = (sum c f + F/2)/rho
// (ImmersedBoundary.cu:249-255) from f, then collide in place; returns u_x (flux sample).
// Contraction is per statement (fp contract(on)), not left to the backend, so the one-step and
// the multi-iteration kernels round every cell identically whatever code surrounds them.  The
// moments come from the pair sums / differences the collision needs anyway:
// rho = f0 + s13 + s24 + s57 + s68, m_x = d13 + d57 - d68, m_y = d24 + d57 + d68.
template <typename R, bool DEV>
__device__ __forceinline__ R relax_cell(R f[9], const KBase<R>& b, const KForce<R>& k) {
#pragma clang fp contract(on)
    if constexpr (DEV) return relax_dev<R>(f, b, k);
    R s[4], d[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        s[p] = f[pair_a(p)] + f[pair_b(p)];
        d[p] = f[pair_a(p)] - f[pair_b(p)];
    }
    const R sum = f[0] + ((s[0] + s[1]) + (s[2] + s[3]));
    const R mx = d[0] + (d[2] - d[3]);
    const R my = d[1] + (d[2] + d[3]);
    const R rho = DEV ? (R)1 + sum : sum;
    const R inv = recip(rho);
    const R jx = mx + k.hFx, jy = my + k.hFy;
    const R ux = jx * inv;
    const R uy = jy * inv;
    collide_sd<R, DEV, DEV>(f, s, d, rho, sum, ux, uy, b, k, jx, jy);
    return ux;
}

// Collide constants of both compute types, folded once on the host (kernel arguments)
struct KConst {
    KBase<double> bd;
    KBase<float> bf;
    KForce<double> fd;  // the uniform body force
    KForce<float> ff;
};
inline KConst make_kconst(const Coef& c) {
    KConst k;
    k.bd = make_kbase<double>(c);
    k.bf = make_kbase<float>(c);
    k.fd = make_kforce<double>(k.bd, c.gx, c.gy);
    k.ff = make_kforce<float>(k.bf, (float)c.gx, (float)c.gy);
    return k;
}
template <typename R>
__host__ __device__ inline const KBase<R>& kbase(const KConst& k);
template <>
__host__ __device__ inline const KBase<double>& kbase<double>(const KConst& k) { return k.bd; }
template <>
__host__ __device__ inline const KBase<float>& kbase<float>(const KConst& k) { return k.bf; }
template <typename R>
__host__ __device__ inline const KForce<R>& kbody(const KConst& k);
template <>
__host__ __device__ inline const KForce<double>& kbody<double>(const KConst& k) { return k.fd; }
template <>
__host__ __device__ inline const KForce<float>& kbody<float>(const KConst& k) { return k.ff; }

// ImmersedBoundary.cu:21-81, with the reference's float/double rounding points.
// Compiled with contraction off so it matches the C restatement bit for bit.
__device__ __forceinline__ float d_delta(float xs, float ys, int x, int y) {
#pragma clang fp contract(off)
    float dx = fabsf((float)x - xs);
    float dy = fabsf((float)y - ys);
    double a = 0., b = 0., d = 0.;
    int c = 0;
    if (dx <= 1.5f) {
        if (dx <= 0.5f) { a = 0.33333; b = 1.; c = 1; d = dx; }
        else { a = 0.16667; b = 5. - 3. * (double)dx; c = -1; d = (double)(1.f - dx); }
    }
    const float deltax = (float)(a * (b + (double)c * sqrt(-3. * d * d + 1.)));
    a = 0.; b = 0.; c = 0; d = 0.;
    if (dy <= 1.5f) {
        if (dy <= 0.5f) { a = 0.33333; b = 1.; c = 1; d = dy; }
        else { a = 0.16667; b = 5. - 3. * (double)dy; c = -1; d = (double)(1.f - dy); }
    }
    const float deltay = (float)(a * (b + (double)c * sqrt(-3. * d * d + 1.)));
    return deltax * deltay;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace iblb

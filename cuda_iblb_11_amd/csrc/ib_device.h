// ib_device.h — per-point immersed-boundary bodies shared by the IB kernels (ib_kernels.hip) and
// the fused band-chain kernel (lbm_kernels.hip).
//
// Reference: ImmersedBoundary.cu:94-133 (interpolate), :138-267 (spread).  The 3-point delta is
// zero unless |x-xs| < 1.5 and |y-ys| < 1.5, so a point only touches the 3x3 nodes around
// (nearbyint(xs), nearbyint(ys)): one 16-lane group per point, one node per lane (lanes 9-15
// idle), F_s folded across the group in the reference's node order and float rounding, then each
// lane spreads its node into a dense force buffer with fp64 atomics (+ a per-(column, chunk) flag
// the collide-stream kernels read).
#pragma once

#include "iblb_kernels.h"

namespace iblb {

constexpr int LANES_PER_POINT = 16;

__device__ __forceinline__ int node_x0(float xs) { return (int)nearbyint((double)xs); }

// node (x, y) of a point's 3x3 spread, clipped to the lattice (no periodic image, as the
// reference's cell-centric gather) and to this slab's columns
__device__ __forceinline__ void spread_node(const Layout& L, int nx, int x_begin, int x, int y, float xs, float ys,
                                            float Fx, float Fy, int e, double* __restrict__ fd, long fplane,
                                            uint8_t* __restrict__ flags, int nch, int rows_per_chunk) {
#pragma clang fp contract(off)
    if (e == 0 || x < 0 || x >= nx || y < 0 || y >= L.ny) return;
    const int xc = x - x_begin;
    if (xc < 0 || xc >= L.ncol) return;
    const float del = d_delta(xs, ys, x, y);
    if (del == 0.f) return;
    const long o = (long)xc * L.rows + y;
    atomicAdd(fd + o, (double)(Fx * del) * 1. * (double)e);
    atomicAdd(fd + fplane + o, (double)(Fy * del) * 1. * (double)e);
    flags[(long)xc * nch + y / rows_per_chunk] = 1;
}

// F_s of the group's point from the per-lane node terms, in node order 0..8
__device__ __forceinline__ void fold_terms(double tx, double ty, bool valid, float& Fx, float& Fy) {
#pragma clang fp contract(off)
    Fx = 0.f;
    Fy = 0.f;
#pragma unroll
    for (int m = 0; m < 9; ++m) {
        const double ax = __shfl(tx, m, LANES_PER_POINT);
        const double ay = __shfl(ty, m, LANES_PER_POINT);
        if (__shfl((int)valid, m, LANES_PER_POINT)) {
            Fx = (float)((double)Fx + ax);
            Fy = (float)((double)Fy + ay);
        }
    }
}

// Node n's interpolation term from its nine pulled populations (ImmersedBoundary.cu:117-128 via
// macro, LatticeBoltzmann.cu:396-405)
__device__ __forceinline__ void node_term(const double f[9], float xs, float ys, int x, int y, double usx, double usy,
                                          double& tx, double& ty) {
#pragma clang fp contract(off)
    double r, mx, my;
    moments<double>(f, r, mx, my);
    const double del = d_delta(xs, ys, x, y);
    tx = 2. * (1. * 1. * del) * r * (usx - mx / r);
    ty = 2. * (1. * 1. * del) * r * (usy - my / r);
}

// Lone slab: point k (pt = k < ns, uniform over the 16-lane group), node n = lane in group:
// nodes -> F_s -> spread.  Every lane of the group must call it (shuffles).
template <typename T>
__device__ __forceinline__ void ib_point_group(const T* __restrict__ g, const Layout& L, const Halo<T>& H, int nx,
                                               bool pt, int k, int n, const float* __restrict__ s,
                                               const float* __restrict__ u_s, const int* __restrict__ eps,
                                               float* __restrict__ F_s, double* __restrict__ fd, long fplane,
                                               uint8_t* __restrict__ flags, int nch, int rows_per_chunk) {
#pragma clang fp contract(off)
    float xs = 0.f, ys = 0.f;
    int x = 0, y = 0;
    double tx = 0., ty = 0.;
    bool valid = false;
    if (pt && n < 9) {
        xs = s[2 * k + 0];
        ys = s[2 * k + 1];
        x = node_x0(xs) + cx(n);
        y = node_x0(ys) + cy(n);
        const long j = (long)y * nx + x;  // flat index without wrap (ImmersedBoundary.cu:119-122)
        if (j >= 0 && j < (long)nx * L.ny) {
            const int xj = (int)(j % nx), yj = (int)(j / nx);
            double f[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) f[q] = Store<T>::to_f(pull<T>(g, L, H, xj, yj, q), q);
            node_term(f, xs, ys, x, y, u_s[2 * k + 0], u_s[2 * k + 1], tx, ty);
            valid = true;
        }
    }
    float Fx, Fy;
    fold_terms(tx, ty, valid, Fx, Fy);
    if (!pt || n >= 9) return;
    if (n == 0) {
        F_s[2 * k + 0] = Fx;
        F_s[2 * k + 1] = Fy;
    }
    spread_node(L, nx, 0, x, y, xs, ys, Fx, Fy, eps ? eps[k] : 1, fd, fplane, flags, nch, rows_per_chunk);
}

// Slab of a group: every slab evaluates, by itself, each point that spreads into it — the point's
// nine nodes lie within 2 columns of the slab and are pulled through the IB halo (IbHalo) — and
// spreads into its own columns.  A point straddling two slabs is evaluated by both with the same
// data in the same order, so the force is bit-identical to a single slab; F_s is reported by the
// slab holding column min(x0, XDIM-1) (zeros elsewhere: the reader sums).  Needs the reference's
// invariant 0 <= nearbyint(xs) <= XDIM (boundary_check, main.cu:202-205).
// part: 0 every point, 1 the inner points (x_begin+2 <= x0 <= x_begin+ncol-3: nodes and their
// pulls inside the slab, no halo; they spread into columns >= 1 and <= ncol-2 only), 2 the others
// (need the IB halo; they spread into columns <= 2 and >= ncol-3 only).
template <typename T>
__device__ __forceinline__ void ib_slab_group(const T* __restrict__ g, const Layout& L, const IbHalo<T>& X, int nx,
                                              int x_begin, bool pt, int k, int n, const float* __restrict__ s,
                                              const float* __restrict__ u_s, const int* __restrict__ eps,
                                              float* __restrict__ F_s, double* __restrict__ fd, long fplane,
                                              uint8_t* __restrict__ flags, int nch, int rows_per_chunk, int part) {
#pragma clang fp contract(off)
    float xs = 0.f, ys = 0.f;
    int x0 = 0, x = 0, y = 0;
    bool mine = false, fs_here = true;  // fs_here: this call writes the point's F_s entry
    if (pt) {
        xs = s[2 * k + 0];
        ys = s[2 * k + 1];
        x0 = node_x0(xs);
        for (int dx = -1; dx <= 1; ++dx) {  // group-uniform: does the point spread into this slab?
            const int xx = x0 + dx;
            mine |= xx >= 0 && xx < nx && xx >= x_begin && xx < x_begin + L.ncol;
        }
        const bool inner = x0 >= x_begin + 2 && x0 <= x_begin + L.ncol - 3;
        if (part == 1) fs_here = mine = mine && inner;
        if (part == 2) {
            fs_here = !(mine && inner);  // the edge launch also zeroes the points of other slabs
            mine = mine && !inner;
        }
    }
    double tx = 0., ty = 0.;
    bool valid = false;
    if (mine && n < 9) {
        x = x0 + cx(n);
        y = node_x0(ys) + cy(n);
        const long j = (long)y * nx + x;
        if (j >= 0 && j < (long)nx * L.ny) {
            const int xj = (int)(j % nx), yj = (int)(j / nx);
            int xl = xj - x_begin;  // slab-local node column, periodic
            if (xl < -2) xl += nx;
            else if (xl > L.ncol + 1) xl -= nx;
            if (xl >= -2 && xl <= L.ncol + 1) {
                double f[9];
#pragma unroll
                for (int q = 0; q < 9; ++q) f[q] = Store<T>::to_f(pull_ib<T>(g, L, X, xl, yj, q), q);
                node_term(f, xs, ys, x, y, u_s[2 * k + 0], u_s[2 * k + 1], tx, ty);
                valid = true;
            }
        }
    }
    float Fx, Fy;
    fold_terms(tx, ty, valid, Fx, Fy);
    if (!pt || n >= 9) return;
    if (n == 0 && fs_here) {
        const int xo = x0 < nx - 1 ? x0 : nx - 1;
        const bool owner = xo >= x_begin && xo < x_begin + L.ncol;
        F_s[2 * k + 0] = owner ? Fx : 0.f;
        F_s[2 * k + 1] = owner ? Fy : 0.f;
    }
    if (mine) spread_node(L, nx, x_begin, x, y, xs, ys, Fx, Fy, eps ? eps[k] : 1, fd, fplane, flags, nch, rows_per_chunk);
}

}  // namespace iblb

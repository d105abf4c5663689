// ib_device.h — per-point immersed-boundary bodies of the IB kernels (ib_kernels.hip).
//
// Reference: ImmersedBoundary.cu:94-133 (interpolate), :138-267 (spread).  The 3-point delta is
// zero unless |x-xs| < 1.5 and |y-ys| < 1.5, so a point only touches the 3x3 nodes around
// (nearbyint(xs), nearbyint(ys)): one nine-lane group per point, one node per lane (seven groups per
// wave; the merged band launches' groups are 32 lanes, ib_next_group), F_s folded across the group
// in the reference's node order and float rounding, then each
// lane spreads its node into a dense force buffer with fp64 atomics (+ a per-(column, chunk) flag
// the collide-stream kernels read).
#pragma once

#include "lbm_vec.h"

namespace iblb {

constexpr int LANES_PER_POINT = 16;
constexpr int GHOST_PPW = 7;  // ib_point_kernel / ib_ghost_kernel: points per wave (nine lanes each)

__device__ __forceinline__ int node_x0(float xs) { return (int)nearbyint((double)xs); }

// node (x, y) of a point's 3x3 spread, clipped to the lattice (no periodic image, as the
// reference's cell-centric gather) and to the local columns [xlo, xhi) (default: the slab's own;
// x_begin: the global column of local column 0 in the caller's image)
__device__ __forceinline__ void spread_node(const Layout& L, int nx, int x_begin, int x, int y, float xs, float ys,
                                            float Fx, float Fy, int e, double* __restrict__ fd, long fplane,
                                            uint8_t* __restrict__ flags, int nch, int rows_per_chunk, int xlo = 0,
                                            int xhi = -1) {
#pragma clang fp contract(off)
    if (e == 0 || x < 0 || x >= nx || y < 0 || y >= L.ny) return;
    const int xc = x - x_begin;
    if (xc < xlo || xc >= (xhi < 0 ? L.ncol : xhi)) return;
    const float del = d_delta(xs, ys, x, y);
    if (del == 0.f) return;
    const long o = (long)xc * L.rows + y;
    atomicAdd(fd + o, (double)(Fx * del) * 1. * (double)e);
    atomicAdd(fd + fplane + o, (double)(Fy * del) * 1. * (double)e);
    flags[(long)xc * nch + y / rows_per_chunk] = 1;
}

// F_s of the group's point from the per-lane node terms, in node order 0..8 (groups of W lanes)
template <int W = LANES_PER_POINT>
__device__ __forceinline__ void fold_terms(double tx, double ty, bool valid, float& Fx, float& Fy) {
#pragma clang fp contract(off)
    Fx = 0.f;
    Fy = 0.f;
#pragma unroll
    for (int m = 0; m < 9; ++m) {
        const double ax = __shfl(tx, m, W);
        const double ay = __shfl(ty, m, W);
        if (__shfl((int)valid, m, W)) {
            Fx = (float)((double)Fx + ax);
            Fy = (float)((double)Fy + ay);
        }
    }
}

// The same fold for a group of nine lanes starting at lane `base` of the wave (ib_ghost_kernel:
// seven points per wave instead of four)
__device__ __forceinline__ void fold_terms_at(double tx, double ty, bool valid, int base, float& Fx, float& Fy) {
#pragma clang fp contract(off)
    Fx = 0.f;
    Fy = 0.f;
#pragma unroll
    for (int m = 0; m < 9; ++m) {
        const double ax = __shfl(tx, base + m);
        const double ay = __shfl(ty, base + m);
        if (__shfl((int)valid, base + m)) {
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
                                               uint8_t* __restrict__ flags, int nch, int rows_per_chunk, int base) {
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
    fold_terms_at(tx, ty, valid, base, Fx, Fy);
    if (!pt || n >= 9) return;
    if (n == 0) {
        F_s[2 * k + 0] = Fx;
        F_s[2 * k + 1] = Fy;
    }
    spread_node(L, nx, 0, x, y, xs, ys, Fx, Fy, eps ? eps[k] : 1, fd, fplane, flags, nch, rows_per_chunk);
}

// A slab with ghost columns (IbGhost, iblb_kernels.h): every slab evaluates, by itself, each point
// that spreads into its columns [clo, chi) — its own columns (one-step IB) or also the ghost
// columns an IB band trapezoid advances redundantly (band cycle) — from the columns it holds.
//
// Images: a point at node column x0 (global) appears at local column x0 - x_begin + m*nx for
// m = -1, 0, 1 (the x-periodic copies a slab's ghost columns hold; a lone slab's ghosts hold its
// own edge columns).  Each image spreads into its cells like the original (global columns clipped
// to [0, XDIM): the reference's cell-centric spread has no periodic image,
// ImmersedBoundary.cu:178-231).  The reference's flat-index quirk (ImmersedBoundary.cu:119-122:
// node j = y*XDIM + x without wrap, so x = -1 reads column XDIM-1 of row y-1, x = XDIM column 0
// of row y+1) is, in image coordinates, a pull from the node's own local column at row
// j / XDIM: the local column of global XDIM-1 next to local column x0-1 = -1 - x_begin + m*nx is
// that column itself.  A point straddling two slabs is evaluated by both from the same data in the
// same order; the force differs from a single slab's only by the arrival order of the spread
// atomics.  Every lane of the 16-lane group must call it (shuffles); pt and k are uniform over it.
template <typename T>
__device__ __forceinline__ void ib_ghost_group(const T* __restrict__ g, const Layout& L, const IbGhost& G, bool pt,
                                               int k, int n, const float* __restrict__ s,
                                               const float* __restrict__ u_s, const int* __restrict__ eps,
                                               float* __restrict__ F_s, double* __restrict__ fd, long fplane,
                                               uint8_t* __restrict__ flags, int nch, int rows_per_chunk, int imgs,
                                               int base) {
#pragma clang fp contract(off)
    float xs = 0.f, ys = 0.f;
    int x0 = 0, y0 = 0;
    bool own = false, go = false;
    if (pt) {
        xs = s[2 * k + 0];
        ys = s[2 * k + 1];
        x0 = node_x0(xs);
        y0 = node_x0(ys);
        const int xo = x0 < G.nx - 1 ? x0 : G.nx - 1;
        own = xo >= G.x_begin && xo < G.x_begin + L.ncol;
        const int xl = x0 - G.x_begin;
        const bool inner = xl >= 2 && xl <= L.ncol - 3;
        go = G.part == 0 || (G.part == 1) == inner;
        if (go && !own && n == 0 && (imgs & 1)) {  // another slab reports this point's F_s
            F_s[2 * k + 0] = 0.f;
            F_s[2 * k + 1] = 0.f;
        }
    }
    const int e = pt ? (eps ? eps[k] : 1) : 0;
    for (int m = -1; m <= 1; ++m) {
        const int xl0 = x0 - G.x_begin + m * G.nx;
        // group-uniform: does this image spread into [clo, chi)?
        const bool img = go && (imgs >> (m != 0) & 1) && (G.part != 1 || m == 0) && xl0 + 1 >= G.clo && xl0 - 1 < G.chi;
        if (!img) continue;
        double tx = 0., ty = 0.;
        bool valid = false;
        const int xn = xl0 + cx(n), x = x0 + cx(n), y = y0 + cy(n);
        if (n < 9) {
            const long j = (long)y * G.nx + x;  // flat index without wrap (ImmersedBoundary.cu:119-122)
            if (j >= 0 && j < (long)G.nx * L.ny && xn - 1 >= -G.gc && xn + 1 < L.ncol + G.gc) {
                const int yj = (int)(j / G.nx);
                double f[9];
#pragma unroll
                for (int q = 0; q < 9; ++q) f[q] = Store<T>::to_f(pull_direct<T>(g, L, xn, yj, q), q);
                node_term(f, xs, ys, x, y, u_s[2 * k + 0], u_s[2 * k + 1], tx, ty);
                valid = true;
            }
        }
        float Fx, Fy;
        fold_terms_at(tx, ty, valid, base, Fx, Fy);
        if (n == 0 && m == 0 && own) {
            F_s[2 * k + 0] = Fx;
            F_s[2 * k + 1] = Fy;
        }
        // local column of global column x in this image: x - (x_begin - m * nx) = xn
        if (n < 9)
            spread_node(L, G.nx, G.x_begin - m * G.nx, x, y, xs, ys, Fx, Fy, e, fd, fplane, flags, nch, rows_per_chunk,
                        G.clo, G.chi);
    }
}

// ---- merged band chain: the next level's force from inside a level's launch ----------------
// A band level's launch computes g^{t+j+1} from g^{t+j}; the force of level j+1 needs g^{t+j+1} at
// the nodes of the points of iteration t+j, which other waves of the same launch are writing.  So
// the point's 16-lane group recomputes this level's collide over the cells its nodes pull: node
// columns xl0-1 .. xl0+1 pull columns xl0-2 .. xl0+2, node rows y0-1 .. y0+1 (y0-2 .. y0+2 with the
// flat-index quirk) pull rows y0-3 .. y0+3 — a 5 x 7 region — with the pull, force and storage
// rounding of fused_wave (bit for bit the values the level writes), into LDS; then nodes -> F_s ->
// spread into the next level's force buffer, as ib_ghost_group.
constexpr int NEXT_RW = 5, NEXT_RH = 7, NEXT_CELLS = NEXT_RW * NEXT_RH;
constexpr int NEXT_LANES = 32;  // lanes per point: one region cell per lane (5 x 5), a second for 3 lanes (5 x 7)

// this level's post-collision values of cell (xc, y), all nine planes, as fused_wave stores them:
// the loads (pulls, chunk flag, dense force: zero where no flag is set) ...
template <typename T>
struct CellIn {
    T v[9];
    double fx, fy;
    bool hf;
};
template <typename T>
__device__ __forceinline__ void level_cell_load(const FusedArgs<T>& a, int xc, int y, int rows_per_chunk, CellIn<T>& in) {
#pragma unroll
    for (int k = 0; k < 9; ++k) in.v[k] = pull_direct<T>(a.src, a.L, xc, y, k);
    in.hf = a.flags[(long)xc * a.nch + y / rows_per_chunk] != 0;
    in.fx = a.fdense[(long)xc * a.L.rows + y];
    in.fy = a.fdense[a.fplane + (long)xc * a.L.rows + y];
}
// ... and the collide
template <typename T>
__device__ __forceinline__ void level_cell_collide(const FusedArgs<T>& a, const CellIn<T>& in, T out[9]) {
    typedef typename Calc<T>::R R;
    constexpr bool DEV = Store<T>::dev;
    R f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = (R)in.v[k];
    const KBase<R>& kb = kbase<R>(a.k);
    if (in.hf) relax_cell<R, DEV>(f, kb, make_kforce<R>(kb, (R)(a.c.gx + in.fx), (R)(a.c.gy + in.fy)));
    else relax_cell<R, DEV>(f, kb, kbody<R>(a.k));
#pragma unroll
    for (int k = 0; k < 9; ++k) out[k] = (T)f[k];
}

// point k (pt: k < nns, uniform over the group of NEXT_LANES lanes), lane n of its group, region
// slot `reg` (LDS, NEXT_CELLS x 9 values); every lane of the group must call it (shuffles).  The
// region is 5 x 5 cells (rows y0-2 .. y0+2), one per lane, unless a node crosses the lattice's x
// edge (the flat-index quirk moves it a row: 5 x 7, rows y0-3 .. y0+3).
template <typename T>
__device__ __forceinline__ void ib_next_group(const FusedArgs<T>& a, bool pt, int k, int n, int rows_per_chunk,
                                              T (*reg)[9], int imgs = 3) {
#pragma clang fp contract(off)
    const IbGhost& G = a.nG;
    const Layout& L = a.L;
    float xs = 0.f, ys = 0.f;
    int x0 = 0, y0 = 0;
    if (pt) {
        xs = a.n_s[2 * k + 0];
        ys = a.n_s[2 * k + 1];
        x0 = node_x0(xs);
        y0 = node_x0(ys);
    }
    const int e = pt ? (a.n_eps ? a.n_eps[k] : 1) : 0;
    const bool quirk = x0 - 1 < 0 || x0 + 1 >= G.nx;  // group-uniform
    const int ry0 = quirk ? y0 - 3 : y0 - 2, ncell = NEXT_RW * (quirk ? NEXT_RH : NEXT_RH - 2);
    for (int m = -1; m <= 1; ++m) {
        const int xl0 = x0 - G.x_begin + m * G.nx;
        // group-uniform: does this image spread into [clo, chi)?  (imgs: bit 0 image 0, bit 1 the others)
        const bool img = pt && (imgs >> (m != 0) & 1) && xl0 + 1 >= G.clo && xl0 - 1 < G.chi;
        if (!img) continue;
        // the region: this level's values of columns xl0-2 .. xl0+2 (cells whose own pulls stay inside
        // the buffer and rows inside the lattice; the others are never read below)
        // cell n (and n+32: the three extra cells of a 5 x 7 region)
        for (int c = n; c < ncell; c += NEXT_LANES) {
            const int xc = xl0 - 2 + c % NEXT_RW, y = ry0 + c / NEXT_RW;
            if (y >= 0 && y < L.ny && xc - 1 >= -G.gc && xc + 1 < L.ncol + G.gc) {
                CellIn<T> in;
                level_cell_load<T>(a, xc, y, rows_per_chunk, in);
                level_cell_collide<T>(a, in, reg[c]);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (a.probe == 3) {  // timing probe: the region only (a use the compiler cannot drop)
            if (reg[n % NEXT_CELLS][0] == (T)12345) a.fdnext[0] = 1.;
            continue;
        }
        double tx = 0., ty = 0.;
        bool valid = false;
        const int xn = xl0 + cx(n), x = x0 + cx(n), y = y0 + cy(n);
        if (n < 9) {
            const long j = (long)y * G.nx + x;  // flat index without wrap (ImmersedBoundary.cu:119-122)
            // the node's pulls read region columns xn-1 .. xn+1, whose own pulls reach xn-2 .. xn+2
            if (j >= 0 && j < (long)G.nx * L.ny && xn - 2 >= -G.gc && xn + 2 < L.ncol + G.gc) {
                const int yj = (int)(j / G.nx);
                const int rx = xn - (xl0 - 2), ry = yj - ry0;
                double f[9];
#pragma unroll
                for (int q = 0; q < 9; ++q) {  // pull_direct on g^{t+j+1}, from the region
                    T v;
                    if (yj == 0 && cy(q) == 1) v = reg[ry * NEXT_RW + rx][q == 2 ? 4 : (q == 5 ? 7 : 8)];
                    else if (yj == L.ny - 1 && cy(q) == -1) v = reg[ry * NEXT_RW + rx][q == 4 ? 2 : (q == 8 ? 5 : 6)];
                    else v = reg[(ry - cy(q)) * NEXT_RW + rx - cx(q)][q];
                    f[q] = Store<T>::to_f(v, q);
                }
                node_term(f, xs, ys, x, y, a.n_us[2 * k + 0], a.n_us[2 * k + 1], tx, ty);
                valid = true;
            }
        }
        float Fx, Fy;
        fold_terms<NEXT_LANES>(tx, ty, valid, Fx, Fy);
        if (a.probe == 4) {  // timing probe: no spread
            if (Fx == 12345.f) a.fdnext[0] = 1.;
            continue;
        }
        if (n < 9)
            spread_node(L, G.nx, G.x_begin - m * G.nx, x, y, xs, ys, Fx, Fy, e, a.fdnext, a.fplane, a.flnext, a.nch,
                        rows_per_chunk, G.clo, G.chi);
        // the region slot is rewritten by the next image: every lane's reads above come first
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

}  // namespace iblb

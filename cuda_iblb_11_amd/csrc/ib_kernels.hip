// ib_kernels.hip — immersed-boundary interpolation and spreading on a slab (gfx950).
//
// Reference: ImmersedBoundary.cu:94-133 (interpolate), :138-267 (spread).  The
// reference spread is a cell-centric gather over ALL points (N*Ns delta evaluations per
// step).  The 3-point delta is zero unless |x-xs| < 1.5 and |y-ys| < 1.5, so only the
// 3x3 nodes around (nearbyint(xs), nearbyint(ys)) receive anything: each point scatters
// into a dense force buffer with fp64 atomics (9*Ns delta evaluations per step).  The
// per-(column, chunk) flags tell the collide-stream kernel where the dense force must be
// read (it clears values and flag).
//
// Single slab: one 16-lane group per point does nodes -> F_s -> spread (ib_point_kernel).  Slab
// groups: each slab evaluates every point that spreads into it from a 2-column-deep IB halo
// (ib_slab_kernel, iblb_device.h IbHalo) — no collective per step.
#include "iblb_kernels.h"

namespace iblb {

namespace {
__device__ __forceinline__ int node_x0(float xs) { return (int)nearbyint((double)xs); }
}  // namespace

// One point per 16-lane group, one of its nine nodes per lane (lanes 9-15 idle): node n's rho
// and u_raw pulled from g (ImmersedBoundary.cu:117-128 via macro, LatticeBoltzmann.cu:396-405)
// and its interpolation term; F_s accumulated in the reference's node order and float rounding
// (every lane of the group folds the nine terms itself); then node n's share of the spread
// (ImmersedBoundary.cu:189-198) into the dense force.  Points are independent (a point's spread
// needs only its own F_s), so a single-slab step needs one IB launch.
constexpr int LANES_PER_POINT = 16;

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

template <typename T>
__global__ __launch_bounds__(256) void ib_point_kernel(const T* __restrict__ g, Layout L, Halo<T> H, int nx, int ns,
                                                       const float* __restrict__ s, const float* __restrict__ u_s,
                                                       const int* __restrict__ eps, float* __restrict__ F_s,
                                                       double* __restrict__ fd, long fplane,
                                                       uint8_t* __restrict__ flags, int nch, int rows_per_chunk) {
#pragma clang fp contract(off)
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int k = (int)(tid / LANES_PER_POINT), n = (int)(tid % LANES_PER_POINT);
    const bool pt = k < ns;  // no early exit: the whole group takes part in the shuffles
    float xs = 0.f, ys = 0.f;
    int x = 0, y = 0;
    double tx = 0., ty = 0.;
    bool valid = false;
    if (pt && n < 9) {
        xs = s[2 * k + 0];
        ys = s[2 * k + 1];
        x = node_x0(xs) + cx(n);
        y = node_x0(ys) + cy(n);
        const long j = (long)y * nx + x;
        if (j >= 0 && j < (long)nx * L.ny) {
            const int xj = (int)(j % nx), yj = (int)(j / nx);
            double f[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) f[q] = Store<T>::to_f(pull<T>(g, L, H, xj, yj, q), q);
            double r, mx, my;
            moments<double>(f, r, mx, my);
            const double del = d_delta(xs, ys, x, y);
            const double usx = u_s[2 * k + 0], usy = u_s[2 * k + 1];
            tx = 2. * (1. * 1. * del) * r * (usx - mx / r);
            ty = 2. * (1. * 1. * del) * r * (usy - my / r);
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

template <typename T>
hipError_t launch_ib_point(const T* g, Layout L, Halo<T> H, int nx, int ns, const float* s, const float* u_s,
                           const int* eps, float* F_s, double* fdense, long fplane, uint8_t* flags, int nch,
                           int rows_per_chunk, hipStream_t st) {
    if (ns <= 0) return hipSuccess;
    const long n = (long)LANES_PER_POINT * ns;
    ib_point_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(g, L, H, nx, ns, s, u_s, eps, F_s, fdense, fplane,
                                                                     flags, nch, rows_per_chunk);
    return hipGetLastError();
}

// Slab groups: every slab evaluates, by itself, each point that spreads into it — the point's
// nine nodes lie within 2 columns of the slab and are pulled through the IB halo (IbHalo) —
// and spreads into its own columns.  A point straddling two slabs is evaluated by both with
// the same data in the same order, so the force is bit-identical to a single slab; F_s is
// reported by the slab holding column min(x0, XDIM-1) (zeros elsewhere: the reader sums).
// Needs the reference's invariant 0 <= nearbyint(xs) <= XDIM (boundary_check, main.cu:202-205).
// part: 0 every point, 1 the inner points (x_begin+2 <= x0 <= x_begin+ncol-3: nodes and their
// pulls inside the slab, no halo; they spread into columns >= 1 and <= ncol-2 only), 2 the others
// (need the IB halo; they spread into columns <= 2 and >= ncol-3 only).
template <typename T>
__global__ __launch_bounds__(256) void ib_slab_kernel(const T* __restrict__ g, Layout L, IbHalo<T> X, int nx,
                                                      int x_begin, int ns, const float* __restrict__ s,
                                                      const float* __restrict__ u_s, const int* __restrict__ eps,
                                                      float* __restrict__ F_s, double* __restrict__ fd, long fplane,
                                                      uint8_t* __restrict__ flags, int nch, int rows_per_chunk,
                                                      int part) {
#pragma clang fp contract(off)
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int k = (int)(tid / LANES_PER_POINT), n = (int)(tid % LANES_PER_POINT);
    const bool pt = k < ns;
    float xs = 0.f, ys = 0.f;
    int x0 = 0, x = 0, y = 0;
    bool mine = false, fs_here = true;  // fs_here: this launch writes the point's F_s entry
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
                double r, mx, my;
                moments<double>(f, r, mx, my);
                const double del = d_delta(xs, ys, x, y);
                const double usx = u_s[2 * k + 0], usy = u_s[2 * k + 1];
                tx = 2. * (1. * 1. * del) * r * (usx - mx / r);
                ty = 2. * (1. * 1. * del) * r * (usy - my / r);
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

template <typename T>
hipError_t launch_ib_slab(const T* g, Layout L, IbHalo<T> X, int nx, int x_begin, int ns, const float* s,
                          const float* u_s, const int* eps, float* F_s, double* fdense, long fplane, uint8_t* flags,
                          int nch, int rows_per_chunk, hipStream_t st, int part) {
    if (ns <= 0) return hipSuccess;
    const long n = (long)LANES_PER_POINT * ns;
    ib_slab_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(g, L, X, nx, x_begin, ns, s, u_s, eps, F_s, fdense,
                                                                    fplane, flags, nch, rows_per_chunk, part);
    return hipGetLastError();
}

// Slots 3..IB_HALO_SLOTS-1 of both send buffers from the state g (slots 0-2 are written by
// the collide that produced g).  One lane per row, one block row per (side, slot).
template <typename T>
__global__ void pack_ib_halo_kernel(const T* __restrict__ g, Layout L, T* __restrict__ send_left,
                                    T* __restrict__ send_right) {
    const int y = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = 3 + (int)blockIdx.y, right = (int)blockIdx.z;
    if (y >= L.ny) return;
    const int d = send_slot_depth(s), k = send_slot_plane(right != 0, s);
    const int xc = right ? L.ncol - 1 - d : d;
    T* dst = right ? send_right : send_left;
    dst[(long)s * L.rows + y] = g[k * L.plane + (long)xc * L.col + y];
}

template <typename T>
hipError_t launch_pack_ib_halo(const T* g, Layout L, T* send_left, T* send_right, hipStream_t st) {
    dim3 grid((unsigned)((L.ny + 255) / 256), IB_HALO_SLOTS - 3, 2);
    pack_ib_halo_kernel<T><<<grid, 256, 0, st>>>(g, L, send_left, send_right);
    return hipGetLastError();
}

template hipError_t launch_ib_slab<double>(const double*, Layout, IbHalo<double>, int, int, int, const float*,
                                           const float*, const int*, float*, double*, long, uint8_t*, int, int,
                                           hipStream_t, int);
template hipError_t launch_ib_slab<float>(const float*, Layout, IbHalo<float>, int, int, int, const float*,
                                          const float*, const int*, float*, double*, long, uint8_t*, int, int,
                                          hipStream_t, int);
template hipError_t launch_pack_ib_halo<double>(const double*, Layout, double*, double*, hipStream_t);
template hipError_t launch_pack_ib_halo<float>(const float*, Layout, float*, float*, hipStream_t);
template hipError_t launch_ib_point<double>(const double*, Layout, Halo<double>, int, int, const float*, const float*,
                                            const int*, float*, double*, long, uint8_t*, int, int, hipStream_t);
template hipError_t launch_ib_point<float>(const float*, Layout, Halo<float>, int, int, const float*, const float*,
                                           const int*, float*, double*, long, uint8_t*, int, int, hipStream_t);

}  // namespace iblb

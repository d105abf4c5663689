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
#include "ib_device.h"

namespace iblb {

// Single slab: one 16-lane group per point does nodes -> F_s -> spread (ib_device.h).  Points are
// independent (a point's spread needs only its own F_s), so a single-slab step needs one IB launch.
template <typename T>
__global__ __launch_bounds__(256) void ib_point_kernel(const T* __restrict__ g, Layout L, Halo<T> H, int nx, int ns,
                                                       const float* __restrict__ s, const float* __restrict__ u_s,
                                                       const int* __restrict__ eps, float* __restrict__ F_s,
                                                       double* __restrict__ fd, long fplane,
                                                       uint8_t* __restrict__ flags, int nch, int rows_per_chunk) {
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int k = (int)(tid / LANES_PER_POINT), n = (int)(tid % LANES_PER_POINT);
    // no early exit: the whole group takes part in the shuffles
    ib_point_group<T>(g, L, H, nx, k < ns, k, n, s, u_s, eps, F_s, fd, fplane, flags, nch, rows_per_chunk);
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

// Slab groups: the points spreading into this slab, nodes through the IB halo (ib_slab_group).
template <typename T>
__global__ __launch_bounds__(256) void ib_slab_kernel(const T* __restrict__ g, Layout L, IbHalo<T> X, int nx,
                                                      int x_begin, int ns, const float* __restrict__ s,
                                                      const float* __restrict__ u_s, const int* __restrict__ eps,
                                                      float* __restrict__ F_s, double* __restrict__ fd, long fplane,
                                                      uint8_t* __restrict__ flags, int nch, int rows_per_chunk,
                                                      int part) {
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int k = (int)(tid / LANES_PER_POINT), n = (int)(tid % LANES_PER_POINT);
    ib_slab_group<T>(g, L, X, nx, x_begin, k < ns, k, n, s, u_s, eps, F_s, fd, fplane, flags, nch, rows_per_chunk,
                     part);
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

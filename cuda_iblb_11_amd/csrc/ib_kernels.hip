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
// groups (and IB band trapezoids): each slab evaluates every point that spreads into the columns
// it advances from its ghost columns (ib_ghost_kernel) — no collective per step.
#include "ib_device.h"

namespace iblb {

// Single slab: one nine-lane group per point (seven per wave, lane 63 idle) does nodes -> F_s ->
// spread (ib_device.h).  Points are independent (a point's spread needs only its own F_s), so a
// single-slab step needs one IB launch.
template <typename T>
__global__ __launch_bounds__(256) void ib_point_kernel(const T* __restrict__ g, Layout L, Halo<T> H, int nx, int ns,
                                                       const float* __restrict__ s, const float* __restrict__ u_s,
                                                       const int* __restrict__ eps, float* __restrict__ F_s,
                                                       double* __restrict__ fd, long fplane,
                                                       uint8_t* __restrict__ flags, int nch, int rows_per_chunk) {
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int w = (int)(tid >> 6), lane = (int)(tid & 63);
    const int gp = lane / 9, n = lane - 9 * gp, k = w * GHOST_PPW + gp;
    // no early exit: the whole group takes part in the shuffles
    ib_point_group<T>(g, L, H, nx, gp < GHOST_PPW && k < ns, k, n, s, u_s, eps, F_s, fd, fplane, flags, nch,
                      rows_per_chunk, 9 * gp);
}

template <typename T>
hipError_t launch_ib_point(const T* g, Layout L, Halo<T> H, int nx, int ns, const float* s, const float* u_s,
                           const int* eps, float* F_s, double* fdense, long fplane, uint8_t* flags, int nch,
                           int rows_per_chunk, hipStream_t st) {
    if (ns <= 0) return hipSuccess;
    const long n = 64L * ((ns + GHOST_PPW - 1) / GHOST_PPW);
    ib_point_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(g, L, H, nx, ns, s, u_s, eps, F_s, fdense, fplane,
                                                                     flags, nch, rows_per_chunk);
    return hipGetLastError();
}

// Slabs with ghost columns: the points (and periodic images) spreading into [clo, chi), nodes
// pulled from the buffer itself (ib_ghost_group).
template <typename T>
__global__ __launch_bounds__(256) void ib_ghost_kernel(const T* __restrict__ g, Layout L, IbGhost G, int ns,
                                                       const float* __restrict__ s, const float* __restrict__ u_s,
                                                       const int* __restrict__ eps, float* __restrict__ F_s,
                                                       double* __restrict__ fd, long fplane,
                                                       uint8_t* __restrict__ flags, int nch, int rows_per_chunk) {
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (G.sig && tid == 0) __hip_atomic_store(G.sig, G.sig_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // seven points per wave, nine lanes each (one node per lane; lane 63 idle): 43 % fewer waves than
    // 16-lane groups (the IB band cycle's chained chain evaluates every point once per level)
    const int w = (int)(tid >> 6), lane = (int)(tid & 63);
    const int gp = lane / 9, n = lane - 9 * gp;
    // group gi < ns: point gi (image 0 only when it lies in [wlo, whi)); then one group per point of
    // [wlo, whi) for its images -1 and +1 (IbGhost::wlo)
    const int gi = w * GHOST_PPW + gp;
    const bool main = gi < ns;
    const int k = main ? gi : G.wlo + (gi - ns);
    const int imgs = main ? (k >= G.wlo && k < G.whi ? 1 : 3) : 2;
    ib_ghost_group<T>(g, L, G, gp < GHOST_PPW && (main || k < G.whi), k, n, s, u_s, eps, F_s, fd, fplane, flags, nch,
                      rows_per_chunk, imgs, 9 * gp);
}

template <typename T>
hipError_t launch_ib_ghost(const T* g, Layout L, IbGhost G, int ns, const float* s, const float* u_s, const int* eps,
                           float* F_s, double* fdense, long fplane, uint8_t* flags, int nch, int rows_per_chunk,
                           hipStream_t st) {
    if (ns <= 0) return hipSuccess;
    if (G.gc < 0 || G.clo < -G.gc || G.chi > L.ncol + G.gc || G.nx < L.ncol) return hipErrorInvalidValue;
    const long n = 64L * ((ns + std::max(0, G.whi - G.wlo) + GHOST_PPW - 1) / GHOST_PPW);
    ib_ghost_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(g, L, G, ns, s, u_s, eps, F_s, fdense, fplane,
                                                                     flags, nch, rows_per_chunk);
    return hipGetLastError();
}

template hipError_t launch_ib_ghost<double>(const double*, Layout, IbGhost, int, const float*, const float*, const int*,
                                            float*, double*, long, uint8_t*, int, int, hipStream_t);
template hipError_t launch_ib_ghost<float>(const float*, Layout, IbGhost, int, const float*, const float*, const int*,
                                           float*, double*, long, uint8_t*, int, int, hipStream_t);
template hipError_t launch_ib_point<double>(const double*, Layout, Halo<double>, int, int, const float*, const float*,
                                            const int*, float*, double*, long, uint8_t*, int, int, hipStream_t);
template hipError_t launch_ib_point<float>(const float*, Layout, Halo<float>, int, int, const float*, const float*,
                                           const int*, float*, double*, long, uint8_t*, int, int, hipStream_t);

}  // namespace iblb

// lbm_sweep.hip — two iterations per launch (sweep2_kernel), the dispatch of the K-iteration
// sweeps (built per depth in lbm_sweepk<K>.hip) and the halo pack kernels; the kernels' code is
// in lbm_sweep_impl.h.
#include "lbm_sweep_impl.h"

namespace iblb {

// the K-iteration kernels are built in lbm_sweepk<K>.hip
#define IBLB_SWEEPK_EXTERN(T, K, S)                                                          \
    extern template hipError_t launch_sweepk_depth<T, K, S>(const Sweep2Args<T>&, hipStream_t); \
    extern template int deep_geometry<T, K, S>(int, int, int, int*);
#define IBLB_SWEEPK_EXTERN_K(K)                                                                               \
    IBLB_SWEEPK_EXTERN(double, K, false) IBLB_SWEEPK_EXTERN(double, K, true) IBLB_SWEEPK_EXTERN(float, K, false) \
    IBLB_SWEEPK_EXTERN(float, K, true)
IBLB_SWEEPK_EXTERN_K(3)
IBLB_SWEEPK_EXTERN_K(4)
IBLB_SWEEPK_EXTERN_K(5)
IBLB_SWEEPK_EXTERN_K(6)

template <typename T, bool SLAB>
static hipError_t launch_sweepk_slab(const Sweep2Args<T>& a, int depth, hipStream_t s) {
    if (depth == 3) return launch_sweepk_depth<T, 3, SLAB>(a, s);
    if (depth == 4) return launch_sweepk_depth<T, 4, SLAB>(a, s);
    if (depth == 5) return launch_sweepk_depth<T, 5, SLAB>(a, s);
    if (depth == 6) return launch_sweepk_depth<T, 6, SLAB>(a, s);
    return hipErrorInvalidValue;
}


template <typename T>
int sweepk_geometry(int depth, int vs, int variant, bool slab, int ny, int* nch) {
    *nch = 0;
    if (vs != 1 && vs != 2) return 0;
    switch (depth) {
        case 3: return slab ? deep_geometry<T, 3, true>(vs, variant, ny, nch) : deep_geometry<T, 3, false>(vs, variant, ny, nch);
        case 4: return slab ? deep_geometry<T, 4, true>(vs, variant, ny, nch) : deep_geometry<T, 4, false>(vs, variant, ny, nch);
        case 5: return slab ? deep_geometry<T, 5, true>(vs, variant, ny, nch) : deep_geometry<T, 5, false>(vs, variant, ny, nch);
        case 6: return slab ? deep_geometry<T, 6, true>(vs, variant, ny, nch) : deep_geometry<T, 6, false>(vs, variant, ny, nch);
        default: return 0;
    }
}
template int sweepk_geometry<double>(int, int, int, bool, int, int*);
template int sweepk_geometry<float>(int, int, int, bool, int, int*);

template <typename T>
hipError_t launch_sweepk(Sweep2Args<T> a, int depth, bool slab, hipStream_t s) {
    if (a.nsweep <= 0) return hipSuccess;
    // rows are read from row0 - 1 >= -(K-1) - VS - 1 to the last wave's row0 + 64*VS: inside the
    // 512-element guards of the buffers
    if (a.W <= 0 || a.L.ncol < 1 || a.vs <= 0 || a.map == 0 || a.L.rows % a.vs != 0 || a.L.plane % a.vs != 0 ||
        a.L.col % a.vs != 0)
        return hipErrorInvalidValue;
    if (slab && (!a.recv_left || !a.recv_right)) return hipErrorInvalidValue;
    return slab ? launch_sweepk_slab<T, true>(a, depth, s) : launch_sweepk_slab<T, false>(a, depth, s);
}

// 2-step halo of g into the send buffers (slot layout in iblb_kernels.h); one thread per
// (side, slot, row)
template <typename T>
__global__ void pack_sweep_halo_kernel(const T* __restrict__ g, Layout L, T* __restrict__ sl, T* __restrict__ sr) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long per_side = 9L * L.ny + 2;
    if (idx >= 2 * per_side) return;
    const bool left = idx < per_side;
    const long i = left ? idx : idx - per_side;
    T* buf = left ? sl : sr;
    const int c0 = left ? 0 : L.ncol - 1;
    if (i >= 9L * L.ny) {  // slot 9: wall values of the edge column
        const int w = (int)(i - 9L * L.ny);
        const int k = w == 0 ? (left ? 8 : 7) : (left ? 5 : 6);
        const int y = w == 0 ? 0 : L.ny - 1;
        buf[9 * L.rows + w] = g[(long)c0 * L.col + (long)k * L.plane + y];
        return;
    }
    const int sl_ = (int)(i / L.ny), y = (int)(i - (long)sl_ * L.ny);
    const int col = sl_ < 6 ? c0 : (left ? 1 : L.ncol - 2);
    const int k = sweep_send_plane(left, sl_);
    buf[(long)sl_ * L.rows + y] = g[(long)col * L.col + (long)k * L.plane + y];
}

template <typename T>
hipError_t launch_pack_sweep_halo(const T* g, Layout L, T* send_left, T* send_right, hipStream_t st) {
    if (L.ncol < 2) return hipErrorInvalidValue;
    const long n = 2 * (9L * L.ny + 2);
    pack_sweep_halo_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(g, L, send_left, send_right);
    return hipGetLastError();
}

// deep halo of depth K of g into both send buffers (deep_slot layout); one thread per
// (side, slot, row)
template <typename T>
__global__ void pack_deep_halo_kernel(const T* __restrict__ g, Layout L, int K, T* __restrict__ sl,
                                      T* __restrict__ sr) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int ns = deep_slots(K);
    const long per_side = (long)ns * L.ny;
    if (idx >= 2 * per_side) return;
    const bool to_left = idx < per_side;
    const long i = to_left ? idx : idx - per_side;
    const int s = (int)(i / L.ny), y = (int)(i - (long)s * L.ny);
    const int d = deep_send_depth(s, K);
    const int k = deep_send_plane(!to_left, s, K);
    const int col = to_left ? d : L.ncol - 1 - d;
    (to_left ? sl : sr)[(long)s * L.rows + y] = g[(long)col * L.col + (long)k * L.plane + y];
}

template <typename T>
hipError_t launch_pack_deep_halo(const T* g, Layout L, int depth, T* send_left, T* send_right, hipStream_t st) {
    if (depth < 3 || depth > 6 || L.ncol < depth) return hipErrorInvalidValue;
    const long n = 2L * deep_slots(depth) * L.ny;
    pack_deep_halo_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(g, L, depth, send_left, send_right);
    return hipGetLastError();
}

template hipError_t launch_pack_deep_halo<double>(const double*, Layout, int, double*, double*, hipStream_t);
template hipError_t launch_pack_deep_halo<float>(const float*, Layout, int, float*, float*, hipStream_t);
template hipError_t launch_pack_sweep_halo<double>(const double*, Layout, double*, double*, hipStream_t);
template hipError_t launch_pack_sweep_halo<float>(const float*, Layout, float*, float*, hipStream_t);
template hipError_t launch_sweep2<double>(Sweep2Args<double>, bool, hipStream_t);
template hipError_t launch_sweep2<float>(Sweep2Args<float>, bool, hipStream_t);
template hipError_t launch_sweepk<double>(Sweep2Args<double>, int, bool, hipStream_t);
template hipError_t launch_sweepk<float>(Sweep2Args<float>, int, bool, hipStream_t);

}  // namespace iblb

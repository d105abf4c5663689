// lbm_sweep.hip — two iterations per launch (sweep2_kernel) and the dispatch of the K-iteration
// sweeps (built per depth in lbm_sweepk<K>.hip); the kernels' code is in lbm_sweep_impl.h.
#include "lbm_sweep_impl.h"

namespace iblb {

// the K-iteration kernels are built in lbm_sweepk<K>.hip
#define IBLB_SWEEPK_EXTERN(T, K, S)                                                          \
    extern template hipError_t launch_sweepk_depth<T, K, S>(const Sweep2Args<T>&, hipStream_t, hipEvent_t, hipEvent_t); \
    extern template int deep_geometry<T, K, S>(int, int, int, int*);
#define IBLB_SWEEPK_EXTERN_K(K)                                                                               \
    IBLB_SWEEPK_EXTERN(double, K, false) IBLB_SWEEPK_EXTERN(double, K, true) IBLB_SWEEPK_EXTERN(float, K, false) \
    IBLB_SWEEPK_EXTERN(float, K, true)
IBLB_SWEEPK_EXTERN_K(3)
IBLB_SWEEPK_EXTERN_K(4)
IBLB_SWEEPK_EXTERN_K(5)
IBLB_SWEEPK_EXTERN_K(6)
IBLB_SWEEPK_EXTERN_K(7)

template <typename T, bool SLAB>
static hipError_t launch_sweepk_slab(const Sweep2Args<T>& a, int depth, hipStream_t s, hipEvent_t stop,
                                     hipEvent_t start) {
    if (depth == 3) return launch_sweepk_depth<T, 3, SLAB>(a, s, stop, start);
    if (depth == 4) return launch_sweepk_depth<T, 4, SLAB>(a, s, stop, start);
    if (depth == 5) return launch_sweepk_depth<T, 5, SLAB>(a, s, stop, start);
    if (depth == 6) return launch_sweepk_depth<T, 6, SLAB>(a, s, stop, start);
    if (depth == 7) return launch_sweepk_depth<T, 7, SLAB>(a, s, stop, start);
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
        case 7: return slab ? deep_geometry<T, 7, true>(vs, variant, ny, nch) : deep_geometry<T, 7, false>(vs, variant, ny, nch);
        default: return 0;
    }
}
template int sweepk_geometry<double>(int, int, int, bool, int, int*);
template int sweepk_geometry<float>(int, int, int, bool, int, int*);

template <typename T>
hipError_t launch_sweepk(Sweep2Args<T> a, int depth, bool slab, hipStream_t s, hipEvent_t stop, hipEvent_t start) {
    if (a.nsweep <= 0) return hipSuccess;
    // rows are read from row0 - 1 >= -(K-1) - VS - 1 to the last wave's row0 + 64*VS: inside the
    // 512-element guards of the buffers
    if (a.W <= 0 || a.L.ncol < 1 || a.vs <= 0 || a.L.rows % a.vs != 0 || a.L.plane % a.vs != 0 ||
        a.L.col % a.vs != 0)
        return hipErrorInvalidValue;
    return slab ? launch_sweepk_slab<T, true>(a, depth, s, stop, start)
                : launch_sweepk_slab<T, false>(a, depth, s, stop, start);
}

// the comm stream's "boundary sweeps done" signal (lbm_sweep_impl.h:edge_wait): a vector store of
// one lane with agent scope; the boundary kernel's stores were released by its end-of-kernel fence
__global__ __launch_bounds__(64) void seq_signal_kernel(unsigned* p, unsigned v) {
    if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
hipError_t launch_seq_signal(unsigned* p, unsigned v, hipStream_t s) {
    seq_signal_kernel<<<1, 64, 0, s>>>(p, v);
    return hipGetLastError();
}

// IBLB_TEST_HOLD: the word lives in host-coherent memory (a host thread sets it); one system-scope
// load per ~8 us, bounded by the wall clock so that the wave always ends
__global__ __launch_bounds__(64) void test_hold_kernel(const unsigned* word, unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        const unsigned w = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (w != 0 || wall_clock64() - t0 > ticks) break;
        __builtin_amdgcn_s_sleep(127);
    }
}
hipError_t launch_test_hold(const unsigned* word, unsigned long long ticks, hipStream_t s) {
    test_hold_kernel<<<1, 64, 0, s>>>(word, ticks);
    return hipGetLastError();
}

template hipError_t launch_sweep2<double>(Sweep2Args<double>, bool, hipStream_t);
template hipError_t launch_sweep2<float>(Sweep2Args<float>, bool, hipStream_t);
template hipError_t launch_sweepk<double>(Sweep2Args<double>, int, bool, hipStream_t, hipEvent_t, hipEvent_t);
template hipError_t launch_sweepk<float>(Sweep2Args<float>, int, bool, hipStream_t, hipEvent_t, hipEvent_t);

}  // namespace iblb

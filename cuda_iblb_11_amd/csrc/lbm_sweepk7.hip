// lbm_sweepk7.hip — the K = 7 iterations-per-launch sweeps (sweepk_kernel, lbm_sweep_impl.h),
// one translation unit per depth so that the deep kernels build in parallel.
#include "lbm_sweep_impl.h"

namespace iblb {

#define IBLB_SWEEPK_INST(T, S)                                                               \
    template hipError_t launch_sweepk_depth<T, 7, S>(const Sweep2Args<T>&, hipStream_t, hipEvent_t, hipEvent_t); \
    template int deep_geometry<T, 7, S>(int, int, int, int*);
IBLB_SWEEPK_INST(double, false)
IBLB_SWEEPK_INST(double, true)
IBLB_SWEEPK_INST(float, false)
IBLB_SWEEPK_INST(float, true)

}  // namespace iblb

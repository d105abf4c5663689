// cilia_kernels.h — launchers of the cilia kinematics kernels (cilia_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace iblb {

constexpr int CILIA_SAMPLES = 9600;  // filament samples per cilium (main.cu:81)
constexpr int CILIA_POINTS = 96;     // boundary points per cilium (main.cu:83, 344)

// main.cu:77 define_filament + the b_points selection of main.cu:158-172.
// s: [5 * 9600 * c_num] samples (x, y, arc, dx, dy), lasts [2 * 9600 * c_num], b_points [5 * 96 * c_num].
hipError_t launch_define_filament(int T, int it, double c_space, int p_step, double c_num, float* s, float* lasts,
                                  float* b_points, hipStream_t st);
// main.cu:176 boundary_check: Lagrangian s [2 * 96 * c_num], u_s, epsilon [96 * c_num].
hipError_t launch_boundary_check(double c_space, int c_num, int XDIM, int it, const float* b_points, float* s,
                                 float* u_s, int* epsilon, hipStream_t st);

}  // namespace iblb

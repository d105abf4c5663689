// ref_kernels.hip — drop-in replacements for the reference kernel launches, with the
// reference's signatures and array layouts (LatticeBoltzmann.cuh:4-10,
// ImmersedBoundary.cuh:4-8) plus a trailing stream.  Expressions keep the reference's
// evaluation order and floating-point contraction is off, so each kernel reproduces the
// C restatement (oracle/oracle.c) bit for bit.  These keep the reference's unfused data
// flow (~824 B per lattice update) and exist for drop-in compatibility and
// kernel-level parity; the fused slab path (lbm_kernels.hip) is the fast one.
#include <hip/hip_runtime.h>

#include "../../include/iblb.h"
#include "iblb_device.h"

namespace iblb {
namespace ref {

__constant__ double c_l[18] = {0., 0., 1., 0., 0., 1., -1., 0., 0., -1., 1., 1., -1., 1., -1., -1., 1., -1.};
__constant__ double t_w[9] = {4. / 9, 1. / 9, 1. / 9, 1. / 9, 1. / 9, 1. / 36, 1. / 36, 1. / 36, 1. / 36};

// LatticeBoltzmann.cu:30-62
__global__ void equilibrium_k(const double* u, const double* rho, double* f0, const double* force, double* F, int XDIM,
                              int YDIM, double TAU) {
#pragma clang fp contract(off)
    const double C_S = 0.57735;
    const long size = (long)XDIM * YDIM;
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= size) return;
    double vec[2];
    for (int i = 0; i < 9; i++) {
        f0[9 * j + i] = rho[j] * t_w[i] * (1
            + (u[0 * size + j] * c_l[2 * i + 0] + u[1 * size + j] * c_l[2 * i + 1]) / (C_S * C_S)
            + (u[0 * size + j] * c_l[2 * i + 0] + u[1 * size + j] * c_l[2 * i + 1]) * (u[0 * size + j] * c_l[2 * i + 0] + u[1 * size + j] * c_l[2 * i + 1]) / (2 * C_S * C_S * C_S * C_S)
            - (u[0 * size + j] * u[0 * size + j] + u[1 * size + j] * u[1 * size + j]) / (2 * C_S * C_S));
        vec[0] = (c_l[i * 2 + 0] - u[0 * size + j]) / (C_S * C_S) + (c_l[i * 2 + 0] * u[0 * size + j] + c_l[i * 2 + 1] * u[1 * size + j]) / (C_S * C_S * C_S * C_S) * c_l[i * 2 + 0];
        vec[1] = (c_l[i * 2 + 1] - u[1 * size + j]) / (C_S * C_S) + (c_l[i * 2 + 0] * u[0 * size + j] + c_l[i * 2 + 1] * u[1 * size + j]) / (C_S * C_S * C_S * C_S) * c_l[i * 2 + 1];
        F[9 * j + i] = (1. - 1. / (2. * TAU)) * t_w[i] * (vec[0] * force[size * 0 + j] + vec[1] * force[size * 1 + j]);
    }
}

// LatticeBoltzmann.cu:64-171
__global__ void collision_k(const double* f0, const double* f, double* f1, const double* F, double TAU, double TAU2,
                            int XDIM, int YDIM) {
#pragma clang fp contract(off)
    const long size = (long)XDIM * YDIM;
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= size) return;
    const double omega_plus = 1 / TAU;
    const double omega_minus = 1 / TAU2;
    f1[9 * j + 0] = f[9 * j + 0] - omega_plus * (f[9 * j + 0] - f0[9 * j + 0]);
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const int a = p == 0 ? 1 : (p == 1 ? 2 : (p == 2 ? 5 : 6));
        const int b = p == 0 ? 3 : (p == 1 ? 4 : (p == 2 ? 7 : 8));
        double f_plus = (f[9 * j + a] + f[9 * j + b]) / 2.;
        double f_minus = (f[9 * j + a] - f[9 * j + b]) / 2.;
        double f0_plus = (f0[9 * j + a] + f0[9 * j + b]) / 2.;
        double f0_minus = (f0[9 * j + a] - f0[9 * j + b]) / 2.;
        f1[9 * j + a] = f[9 * j + a] - omega_plus * (f_plus - f0_plus) - omega_minus * (f_minus - f0_minus) + F[9 * j + a];
        f_minus *= -1.;
        f0_minus *= -1.;
        f1[9 * j + b] = f[9 * j + b] - omega_plus * (f_plus - f0_plus) - omega_minus * (f_minus - f0_minus) + F[9 * j + b];
    }
}

// LatticeBoltzmann.cu:173-373 as a pull: each destination (cell, k) reads its single
// source; identical values to the push (each destination has exactly one writer).
__global__ void streaming_k(const double* f1, double* f, int XDIM, int YDIM) {
    const long size = (long)XDIM * YDIM;
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= size) return;
    const int x = (int)(j % XDIM), y = (int)(j / XDIM);
    for (int k = 0; k < 9; ++k) {
        long js;
        int ks = k;
        if (y == 0 && cy(k) == 1) {
            js = j; ks = k == 2 ? 4 : (k == 5 ? 7 : 8);
        } else if (y == YDIM - 1 && cy(k) == -1) {
            js = j; ks = k == 4 ? 2 : (k == 8 ? 5 : 6);
        } else {
            int sx = x - cx(k);
            sx = sx < 0 ? sx + XDIM : (sx >= XDIM ? sx - XDIM : sx);
            js = (long)(y - cy(k)) * XDIM + sx;
        }
        f[9 * j + k] = f1[9 * js + ks];
    }
}

// LatticeBoltzmann.cu:375-411
__global__ void macro_k(const double* f, double* u, double* rho, int XDIM, int YDIM) {
#pragma clang fp contract(off)
    const long size = (long)XDIM * YDIM;
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= size) return;
    double r = 0, m0 = 0, m1 = 0;
    for (int i = 0; i < 9; i++) {
        r += f[9 * j + i];
        m0 += c_l[i * 2 + 0] * f[9 * j + i];
        m1 += c_l[i * 2 + 1] * f[9 * j + i];
    }
    rho[j] = r;
    u[0 * size + j] = m0 / r;
    u[1 * size + j] = m1 / r;
}

// ImmersedBoundary.cu:94-133
__global__ void interpolate_k(const double* rho, const double* u, int Ns, const float* u_s, float* F_s, const float* s,
                              int XDIM, int YDIM) {
#pragma clang fp contract(off)
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Ns) return;
    const long size = (long)XDIM * YDIM;
    float Fx = 0.f, Fy = 0.f;
    const double xs = s[k * 2 + 0];
    const double ys = s[k * 2 + 1];
    const int x0 = (int)nearbyint(xs);
    const int y0 = (int)nearbyint(ys);
    for (int i = 0; i < 9; i++) {
        const int x = (int)nearbyint(x0 + c_l[i * 2 + 0]);
        const int y = (int)nearbyint(y0 + c_l[i * 2 + 1]);
        const long j = (long)y * XDIM + x;
        if (j < 0 || j >= size) continue;
        const double del = d_delta((float)xs, (float)ys, x, y);
        Fx = (float)((double)Fx + 2. * (1. * 1. * del) * rho[j] * ((double)u_s[2 * k + 0] - u[0 * size + j]));
        Fy = (float)((double)Fy + 2. * (1. * 1. * del) * rho[j] * ((double)u_s[2 * k + 1] - u[1 * size + j]));
    }
    F_s[2 * k + 0] = Fx;
    F_s[2 * k + 1] = Fy;
}

// ImmersedBoundary.cu:138-267 in three passes: clear force, scatter the 3x3
// contributions of every point (points in index order within one lane, so a cell's sum
// follows the reference's term order when a single point reaches it; with several
// points the fp64 atomics add in arrival order, as the reference's flux atomics do),
// then the u correction and flux.
__global__ void zero_k(double* p, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0.;
}

__global__ void spread_scatter_k(int Ns, const float* F_s, double* force, const float* s, int XDIM, int YDIM,
                                 const int* epsilon) {
#pragma clang fp contract(off)
    const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= 9L * Ns) return;
    const long size = (long)XDIM * YDIM;
    const int k = (int)(id / 9), n = (int)(id - 9L * (id / 9));
    const float xs = s[2 * k + 0], ys = s[2 * k + 1];
    const int x = (int)nearbyint((double)xs) + cx(n), y = (int)nearbyint((double)ys) + cy(n);
    if (x < 0 || x >= XDIM || y < 0 || y >= YDIM) return;
    const float del = d_delta(xs, ys, x, y);
    if (del == 0.f) return;
    const long j = (long)y * XDIM + x;
    atomicAdd(force + 0 * size + j, (double)(F_s[2 * k + 0] * del) * 1. * (double)epsilon[k]);
    atomicAdd(force + 1 * size + j, (double)(F_s[2 * k + 1] * del) * 1. * (double)epsilon[k]);
}

__global__ void spread_tail_k(const double* rho, double* u, const double* f, const double* force, int XDIM, int YDIM,
                              double* Q, int flux_column, double flux_norm) {
#pragma clang fp contract(off)
    const long size = (long)XDIM * YDIM;
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= size) return;
    u[0 * size + j] = (c_l[0 * 2 + 0] * f[9 * j + 0] + c_l[1 * 2 + 0] * f[9 * j + 1] + c_l[2 * 2 + 0] * f[9 * j + 2] +
                       c_l[3 * 2 + 0] * f[9 * j + 3] + c_l[4 * 2 + 0] * f[9 * j + 4] + c_l[5 * 2 + 0] * f[9 * j + 5] +
                       c_l[6 * 2 + 0] * f[9 * j + 6] + c_l[7 * 2 + 0] * f[9 * j + 7] + c_l[8 * 2 + 0] * f[9 * j + 8] + 0.5 * force[0 * size + j]) / rho[j];
    u[1 * size + j] = (c_l[1 * 2 + 1] * f[9 * j + 1] + c_l[1 * 2 + 1] * f[9 * j + 1] + c_l[2 * 2 + 1] * f[9 * j + 2] +
                       c_l[3 * 2 + 1] * f[9 * j + 3] + c_l[4 * 2 + 1] * f[9 * j + 4] + c_l[5 * 2 + 1] * f[9 * j + 5] +
                       c_l[6 * 2 + 1] * f[9 * j + 6] + c_l[7 * 2 + 1] * f[9 * j + 7] + c_l[8 * 2 + 1] * f[9 * j + 8] + 0.5 * force[1 * size + j]) / rho[j];
    if ((int)(j % XDIM) == flux_column) {
        const double temp = u[0 * size + j] / flux_norm;
        atomicAdd(Q, temp);  // DoubleAtomicAdd (ImmersedBoundary.cu:83-92) is native on gfx950
    }
}

__global__ void delta_k(int n, const float* xs, const float* ys, const int* x, const int* y, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = d_delta(xs[i], ys[i], x[i], y[i]);
}

inline unsigned nblk(long n) { return (unsigned)((n + 127) / 128); }  // reference block size 128 (main.cu:366)

}  // namespace ref
}  // namespace iblb

using namespace iblb::ref;

static int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? IBLB_OK : IBLB_ERR_HIP;
}
static bool bad_grid(int XDIM, int YDIM) { return XDIM < 1 || YDIM < 2; }

extern "C" int iblb_equilibrium(const double* u, const double* rho, double* f0, const double* force, double* F, int XDIM,
                                int YDIM, double TAU, void* stream) {
    if (bad_grid(XDIM, YDIM) || !u || !rho || !f0 || !force || !F) return IBLB_ERR_ARG;
    const long n = (long)XDIM * YDIM;
    equilibrium_k<<<nblk(n), 128, 0, (hipStream_t)stream>>>(u, rho, f0, force, F, XDIM, YDIM, TAU);
    return launch_status();
}

extern "C" int iblb_collision(const double* f0, const double* f, double* f1, const double* F, double TAU, double TAU2,
                              int XDIM, int YDIM, int it, void* stream) {
    (void)it;
    if (bad_grid(XDIM, YDIM) || !f0 || !f || !f1 || !F) return IBLB_ERR_ARG;
    const long n = (long)XDIM * YDIM;
    collision_k<<<nblk(n), 128, 0, (hipStream_t)stream>>>(f0, f, f1, F, TAU, TAU2, XDIM, YDIM);
    return launch_status();
}

extern "C" int iblb_streaming(const double* f1, double* f, int XDIM, int YDIM, void* stream) {
    if (bad_grid(XDIM, YDIM) || !f1 || !f || f1 == f) return IBLB_ERR_ARG;
    const long n = (long)XDIM * YDIM;
    streaming_k<<<nblk(n), 128, 0, (hipStream_t)stream>>>(f1, f, XDIM, YDIM);
    return launch_status();
}

extern "C" int iblb_macro(const double* f, double* u, double* rho, int XDIM, int YDIM, void* stream) {
    if (bad_grid(XDIM, YDIM) || !f || !u || !rho) return IBLB_ERR_ARG;
    const long n = (long)XDIM * YDIM;
    macro_k<<<nblk(n), 128, 0, (hipStream_t)stream>>>(f, u, rho, XDIM, YDIM);
    return launch_status();
}

extern "C" int iblb_interpolate(const double* rho, const double* u, int Ns, const float* u_s, float* F_s,
                                const float* s, int XDIM, int YDIM, void* stream) {
    if (bad_grid(XDIM, YDIM) || Ns < 0) return IBLB_ERR_ARG;
    if (Ns == 0) return IBLB_OK;
    if (!rho || !u || !u_s || !F_s || !s) return IBLB_ERR_ARG;
    interpolate_k<<<nblk(Ns), 128, 0, (hipStream_t)stream>>>(rho, u, Ns, u_s, F_s, s, XDIM, YDIM);
    return launch_status();
}

extern "C" int iblb_spread_ex(const double* rho, double* u, const double* f, int Ns, const float* u_s,
                              const float* F_s, double* force, const float* s, int XDIM, int YDIM, double* Q,
                              const int* epsilon, int flux_column, double flux_norm, void* stream) {
    (void)u_s;
    if (bad_grid(XDIM, YDIM) || Ns < 0 || !rho || !u || !f || !force || !Q) return IBLB_ERR_ARG;
    if (Ns > 0 && (!F_s || !s || !epsilon)) return IBLB_ERR_ARG;
    if (flux_norm == 0.) return IBLB_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long n = (long)XDIM * YDIM;
    zero_k<<<nblk(2 * n), 128, 0, st>>>(force, 2 * n);
    if (Ns > 0) spread_scatter_k<<<nblk(9L * Ns), 128, 0, st>>>(Ns, F_s, force, s, XDIM, YDIM, epsilon);
    spread_tail_k<<<nblk(n), 128, 0, st>>>(rho, u, f, force, XDIM, YDIM, Q, flux_column, flux_norm);
    return launch_status();
}

extern "C" int iblb_spread(const double* rho, double* u, const double* f, int Ns, const float* u_s, const float* F_s,
                           double* force, const float* s, int XDIM, double* Q, const int* epsilon, void* stream) {
    // ImmersedBoundary.cu:146 (size = 192*XDIM) and :259-261 (column XDIM-5, /192)
    return iblb_spread_ex(rho, u, f, Ns, u_s, F_s, force, s, XDIM, 192, Q, epsilon, XDIM - 5, 192., stream);
}

extern "C" int iblb_delta(int n, const float* xs, const float* ys, const int* x, const int* y, float* out,
                          void* stream) {
    if (n < 0 || (n > 0 && (!xs || !ys || !x || !y || !out))) return IBLB_ERR_ARG;
    if (n == 0) return IBLB_OK;
    delta_k<<<nblk(n), 128, 0, (hipStream_t)stream>>>(n, xs, ys, x, y, out);
    return launch_status();
}

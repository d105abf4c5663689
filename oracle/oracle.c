/*
 * oracle.c — CPU restatement of the reference IB-LBM hot path.  TEST INFRASTRUCTURE ONLY
 * (only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it; the
 * product never does).  Build: oracle/Makefile (-O3 -fopenmp -ffp-contract=off).
 *
 * Parity status: UNPINNED against the reference binary (the reference needs nvcc and
 * the CUDA runtime; neither is in this image).  Pinned by analytic KATs and by the
 * reference's nominal outputs as an envelope; see oracle.h and DESIGN.md.
 *
 * Each function follows the cited reference lines statement by statement; the
 * comments name the rounding points that matter for bit-level agreement.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* LatticeBoltzmann.cu:11-27 (IB copy: ImmersedBoundary.cu:14-19) */
static const double C_S = 0.57735;
static const double c_l[9 * 2] = {
    0., 0.,
    1., 0., 0., 1., -1., 0., 0., -1.,
    1., 1., -1., 1., -1., -1., 1., -1.};
static const double t_w[9] = {
    4. / 9,
    1. / 9, 1. / 9, 1. / 9, 1. / 9,
    1. / 36, 1. / 36, 1. / 36, 1. / 36};

static int g_threads = 1;
void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
int oracle_get_threads(void) { return g_threads; }

/* LatticeBoltzmann.cu:30-62.  Expression trees kept verbatim (left-to-right). */
void oracle_equilibrium(const double* u, const double* rho, double* f0, const double* force,
                        double* F, int XDIM, int YDIM, double TAU)
{
    const long size = (long)XDIM * YDIM;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (long j = 0; j < size; j++) {
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
}

/* LatticeBoltzmann.cu:64-171.  TRT: pairs (1,3) (2,4) (5,7) (6,8); no force on rest pop. */
void oracle_collision(const double* f0, const double* f, double* f1, const double* F,
                      double TAU, double TAU2, int XDIM, int YDIM, int it)
{
    (void)it; /* unused in the reference too (LatticeBoltzmann.cu:64) */
    const long size = (long)XDIM * YDIM;
    const double omega_plus = 1 / TAU;
    const double omega_minus = 1 / TAU2;
    static const int pr[4][2] = {{1, 3}, {2, 4}, {5, 7}, {6, 8}};
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (long j = 0; j < size; j++) {
        f1[9 * j + 0] = f[9 * j + 0] - omega_plus * (f[9 * j + 0] - f0[9 * j + 0]);
        for (int p = 0; p < 4; p++) {
            const int a = pr[p][0], b = pr[p][1];
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
}

/* LatticeBoltzmann.cu:173-373, push streaming with the reference's flag logic:
 * periodic x ("thru"), bounce-back on y=0 ("back"), same-cell mirror on y=YDIM-1
 * ("slip"); top/bottom win over left/right at corners. */
void oracle_streaming(const double* f1, double* f, int XDIM, int YDIM)
{
    const long size = (long)XDIM * YDIM;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (long j = 0; j < size; j++) {
        const int x = (int)(j % XDIM);
        const int y = (int)((j - j % XDIM) / XDIM);
        const int up = (y == YDIM - 1), down = (y == 0), left = (x == 0), right = (x == XDIM - 1);
        for (int i = 0; i < 9; i++) {
            int back = 0, thru = 0, slip = 0, k = i;
            long jstream = j;
            if (down || up || left || right) {
                switch (i) {
                case 0: break;
                case 1: if (right) thru = 1; break;
                case 2: if (up) slip = 1; break;
                case 3: if (left) thru = 1; break;
                case 4: if (down) back = 1; break;
                case 5: if (up) slip = 1; else if (right) thru = 1; break;
                case 6: if (up) slip = 1; else if (left) thru = 1; break;
                case 7: if (down) back = 1; else if (left) thru = 1; break;
                case 8: if (down) back = 1; else if (right) thru = 1; break;
                }
            }
            if (back) {
                static const int kb[9] = {0, 3, 4, 1, 2, 7, 8, 5, 6};
                jstream = j; k = kb[i];
            } else if (slip) {
                static const int ks[9] = {0, 1, 4, 3, 2, 8, 7, 6, 5};
                jstream = j; k = ks[i];
            } else if (thru) {
                jstream = j - (long)((XDIM - 1) * c_l[i * 2 + 0]) + (long)(XDIM * c_l[i * 2 + 1]);
                k = i;
            } else {
                jstream = j + (long)c_l[i * 2 + 0] + (long)(XDIM * c_l[i * 2 + 1]);
                k = i;
            }
            f[9 * jstream + k] = f1[9 * j + i];
        }
    }
}

/* LatticeBoltzmann.cu:375-411 */
void oracle_macro(const double* f, double* u, double* rho, int XDIM, int YDIM)
{
    const long size = (long)XDIM * YDIM;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (long j = 0; j < size; j++) {
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
}

/* ImmersedBoundary.cu:21-81.  |x - xs| in float; each 1-D factor in double, rounded to
 * float; product in float.  d = 1 - dx is a float subtraction (int 1 promoted). */
float oracle_d_delta(float xs, float ys, int x, int y)
{
    float deltax, deltay, delta;
    float dx = fabsf((float)x - xs);
    float dy = fabsf((float)y - ys);
    double a = 0., b = 0., d = 0.;
    int c = 0;
    if (dx <= 1.5) {
        if (dx <= 0.5) { a = 0.33333; b = 1.; c = 1; d = dx; }
        else { a = 0.16667; b = 5. - 3. * dx; c = -1; d = (float)(1 - dx); }
    }
    deltax = (float)(a * (b + c * sqrt(-3. * d * d + 1)));
    a = 0.; b = 0.; c = 0; d = 0.;
    if (dy <= 1.5) {
        if (dy <= 0.5) { a = 0.33333; b = 1.; c = 1; d = dy; }
        else { a = 0.16667; b = 5. - 3. * dy; c = -1; d = (float)(1 - dy); }
    }
    deltay = (float)(a * (b + c * sqrt(-3. * d * d + 1)));
    delta = deltax * deltay;
    return delta;
}

/* ImmersedBoundary.cu:94-133.  Flat index without periodic wrap (x = -1 reads the
 * previous row's last cell).  A node whose flat index leaves [0, size) is undefined
 * behaviour in the reference; here it is skipped (same rule on the GPU). */
void oracle_interpolate(const double* rho, const double* u, int Ns, const float* u_s, float* F_s,
                        const float* s, int XDIM, int YDIM)
{
    const long size = (long)XDIM * YDIM;
    for (int k = 0; k < Ns; k++) {
        F_s[2 * k + 0] = 0.;
        F_s[2 * k + 1] = 0.;
        const double xs = s[k * 2 + 0];
        const double ys = s[k * 2 + 1];
        const int x0 = (int)nearbyint(xs);
        const int y0 = (int)nearbyint(ys);
        for (int i = 0; i < 9; i++) {
            const int x = (int)nearbyint(x0 + c_l[i * 2 + 0]);
            const int y = (int)nearbyint(y0 + c_l[i * 2 + 1]);
            const long j = (long)y * XDIM + x;
            if (j < 0 || j >= size) continue;
            const double del = oracle_d_delta((float)xs, (float)ys, x, y);
            F_s[2 * k + 0] += 2. * (1. * 1. * del) * rho[j] * (u_s[2 * k + 0] - u[0 * size + j]);
            F_s[2 * k + 1] += 2. * (1. * 1. * del) * rho[j] * (u_s[2 * k + 1] - u[1 * size + j]);
        }
    }
}

/* u correction + flux of ImmersedBoundary.cu:249-264 for one cell (shared by both
 * spread restatements).  The u_y sum keeps the reference's duplicated zero term. */
static inline void spread_tail(const double* rho, double* u, const double* f, const double* force,
                               long size, long j)
{
    u[0 * size + j] = (c_l[0 * 2 + 0] * f[9 * j + 0] + c_l[1 * 2 + 0] * f[9 * j + 1] + c_l[2 * 2 + 0] * f[9 * j + 2] +
                       c_l[3 * 2 + 0] * f[9 * j + 3] + c_l[4 * 2 + 0] * f[9 * j + 4] + c_l[5 * 2 + 0] * f[9 * j + 5] +
                       c_l[6 * 2 + 0] * f[9 * j + 6] + c_l[7 * 2 + 0] * f[9 * j + 7] + c_l[8 * 2 + 0] * f[9 * j + 8] + 0.5 * force[0 * size + j]) / rho[j];
    u[1 * size + j] = (c_l[1 * 2 + 1] * f[9 * j + 1] + c_l[1 * 2 + 1] * f[9 * j + 1] + c_l[2 * 2 + 1] * f[9 * j + 2] +
                       c_l[3 * 2 + 1] * f[9 * j + 3] + c_l[4 * 2 + 1] * f[9 * j + 4] + c_l[5 * 2 + 1] * f[9 * j + 5] +
                       c_l[6 * 2 + 1] * f[9 * j + 6] + c_l[7 * 2 + 1] * f[9 * j + 7] + c_l[8 * 2 + 1] * f[9 * j + 8] + 0.5 * force[1 * size + j]) / rho[j];
}

static void spread_finish(const double* rho, double* u, const double* f, double* force, int XDIM, int YDIM,
                          double* Q, int flux_column, double flux_norm)
{
    const long size = (long)XDIM * YDIM;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (long j = 0; j < size; j++) spread_tail(rho, u, f, force, size, j);
    /* ImmersedBoundary.cu:259-264: Q += u_x/192 for every cell of column XDIM-5.  The
     * reference adds with atomics in an unspecified order; here in y order. */
    if (Q && flux_column >= 0 && flux_column < XDIM)
        for (int y = 0; y < YDIM; y++) {
            const double temp = u[(long)y * XDIM + flux_column] / flux_norm;
            Q[0] += temp;
        }
}

/* ImmersedBoundary.cu:138-267, literal cell-centric gather: every cell evaluates
 * d_delta against every point (the reference's 64-point smem tiles only change the
 * loop blocking, and its padding points contribute exact zeros). */
void oracle_spread(const double* rho, double* u, const double* f, int Ns, const float* u_s,
                   const float* F_s, double* force, const float* s, int XDIM, int YDIM,
                   double* Q, const int* epsilon, int flux_column, double flux_norm)
{
    (void)u_s;
    const long size = (long)XDIM * YDIM;
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (long j = 0; j < size; j++) {
        const int x = (int)(j % XDIM);
        const int y = (int)((j - j % XDIM) / XDIM);
        double fx = 0., fy = 0.;
        for (int k = 0; k < Ns; k++) {
            const float xs = s[2 * k + 0], ys = s[2 * k + 1];
            const float del = oracle_d_delta(xs, ys, x, y);
            /* float*float product, then *1. (double) * epsilon (ImmersedBoundary.cu:196-197) */
            fx += (double)(float)(F_s[2 * k + 0] * del) * 1. * epsilon[k];
            fy += (double)(float)(F_s[2 * k + 1] * del) * 1. * epsilon[k];
        }
        force[0 * size + j] = fx;
        force[1 * size + j] = fy;
    }
    spread_finish(rho, u, f, force, XDIM, YDIM, Q, flux_column, flux_norm);
}

/* Point-centric form of the same sum.  Non-zero deltas need |x - xs| < 1.5 and
 * |y - ys| < 1.5, i.e. the 3x3 nodes around (nearbyint(xs), nearbyint(ys)); nodes
 * outside the lattice are clipped (no periodic image, as the reference's cells simply
 * do not exist there).  Points are visited in index order, so each cell accumulates its
 * terms in the reference's order and the result is bit-identical. */
void oracle_spread_points(const double* rho, double* u, const double* f, int Ns, const float* u_s,
                          const float* F_s, double* force, const float* s, int XDIM, int YDIM,
                          double* Q, const int* epsilon, int flux_column, double flux_norm)
{
    (void)u_s;
    const long size = (long)XDIM * YDIM;
    memset(force, 0, sizeof(double) * 2 * size);
    for (int k = 0; k < Ns; k++) {
        const float xs = s[2 * k + 0], ys = s[2 * k + 1];
        const int x0 = (int)nearbyint((double)xs), y0 = (int)nearbyint((double)ys);
        for (int i = 0; i < 9; i++) {
            const int x = x0 + (int)c_l[2 * i + 0], y = y0 + (int)c_l[2 * i + 1];
            if (x < 0 || x >= XDIM || y < 0 || y >= YDIM) continue;
            const float del = oracle_d_delta(xs, ys, x, y);
            if (del == 0.f) continue;
            const long j = (long)y * XDIM + x;
            force[0 * size + j] += (double)(float)(F_s[2 * k + 0] * del) * 1. * epsilon[k];
            force[1 * size + j] += (double)(float)(F_s[2 * k + 1] * del) * 1. * epsilon[k];
        }
    }
    spread_finish(rho, u, f, force, XDIM, YDIM, Q, flux_column, flux_norm);
}

/* main.cu:56-74: Fourier coefficients of the beat, "WITHOUT MUCUS" set */
static const double A_mn[7 * 2 * 3] = {
    -0.654, 0.393, -0.097, 0.079, 0.119, 0.119, 0.009,
    1.895, -0.018, 0.158, 0.010, 0.003, 0.013, 0.040,
    0.787, -1.516, 0.032, -0.302, -0.252, -0.015, 0.035,
    -0.552, -0.126, -0.341, 0.035, 0.006, -0.029, -0.068,
    0.202, 0.716, -0.118, 0.142, 0.110, -0.013, -0.043,
    0.096, 0.263, 0.186, -0.067, -0.032, -0.002, 0.015};
static const double B_mn[7 * 2 * 3] = {
    0.0, 0.284, 0.006, -0.059, 0.018, 0.053, 0.009,
    0.0, 0.192, -0.050, 0.012, -0.007, -0.014, -0.017,
    0.0, 1.045, 0.317, 0.226, 0.004, -0.082, -0.040,
    0.0, -0.499, 0.423, 0.138, 0.125, 0.075, 0.067,
    0.0, -1.017, -0.276, -0.196, -0.037, 0.025, 0.023,
    0.0, 0.339, -0.327, -0.114, -0.105, -0.057, -0.055};
static const double PI_REF = 3.14159; /* main.cu:29 */

/* pow(float, int) of the CUDA device library, restated as float multiplications (exact
 * for the exponents 1..3 used here: pow(a,1) = a, pow(a,2) = a*a, pow(a,3) = a*(a*a)). */
static float pow_fi(float a, int b) {
    float r = a;
    for (int i = 1; i < b; i++) r = r * a;
    return r;
}

/* main.cu:77-173, one filament sample (k, m) per reference thread, threads in order. */
void oracle_define_filament(int T, int it, double c_space, int p_step, double c_num, float* s, float* lasts,
                            float* b_points)
{
    const int f_length = 9600, length = 96;
    const long nthreads = (long)f_length * (long)c_num;
    for (long threadnum = 0; threadnum < nthreads; threadnum++) {
        const int k = (int)(threadnum % f_length);
        const int m = (int)((threadnum - k) / f_length);
        float a_n[2 * 7], b_n[2 * 7];
        const float arcl = (float)(1. * k / f_length);
        int phase;
        if (it + m * p_step == T) phase = T;
        else phase = (it + m * p_step) % T;
        const float offset = (float)(1. * (m - (c_num - 1) / 2.) * c_space);
        for (int n = 0; n < 7; n++) {
            for (int h = 0; h < 2; h++) {
                a_n[2 * n + h] = 0.;
                b_n[2 * n + h] = 0.;
                for (int i = 0; i < 3; i++) {
                    a_n[2 * n + h] = (float)(a_n[2 * n + h] + A_mn[n + 14 * i + 7 * h] * pow_fi(arcl, i + 1));
                    b_n[2 * n + h] = (float)(b_n[2 * n + h] + B_mn[n + 14 * i + 7 * h] * pow_fi(arcl, i + 1));
                }
            }
        }
        float* sk = s + 5 * (k + (long)m * f_length);
        sk[0] = (float)(1. * 111 * a_n[0] * 0.5 + offset);
        sk[1] = (float)(1. * 111 * a_n[1] * 0.5);
        sk[2] = 111 * arcl;
        for (int n = 1; n < 7; n++) {
            sk[0] = (float)(sk[0] + 1. * 111 * (a_n[2 * n + 0] * cos(n * 2. * PI_REF * phase / T) + b_n[2 * n + 0] * sin(n * 2. * PI_REF * phase / T)));
            sk[1] = (float)(sk[1] + 1. * 111 * (a_n[2 * n + 1] * cos(n * 2. * PI_REF * phase / T) + b_n[2 * n + 1] * sin(n * 2. * PI_REF * phase / T)));
        }
        float* lk = lasts + 2 * (k + (long)m * f_length);
        if (it > 0) {
            sk[3] = sk[0] - lk[0];
            sk[4] = sk[1] - lk[1];
        }
        lk[0] = sk[0];
        lk[1] = sk[1];
        for (int j = m * length; j < (m + 1) * length; j++) {
            const float b_length = (float)(j % length);
            if (fabsf(sk[2] - b_length) < 0.01) {
                b_points[5 * j + 0] = sk[0];
                b_points[5 * j + 1] = sk[1];
                b_points[5 * j + 2] = sk[3];
                b_points[5 * j + 3] = sk[4];
            }
        }
    }
}

/* main.cu:176-252 */
void oracle_boundary_check(double c_space, int c_num, int XDIM, int it, const float* b_points, float* s,
                           float* u_s, int* epsilon)
{
    const int length = 96;
    const int Np = length * c_num;
    for (int j = 0; j < Np; j++) {
        s[2 * j + 0] = (float)((c_space * c_num) / 2. + b_points[5 * j + 0]);
        if (s[2 * j + 0] < 0) s[2 * j + 0] = s[2 * j + 0] + XDIM;
        else if (s[2 * j + 0] > XDIM) s[2 * j + 0] = s[2 * j + 0] - XDIM;
        s[2 * j + 1] = b_points[5 * j + 1] + 1;
        if (it == 0) { u_s[2 * j + 0] = 0.; u_s[2 * j + 1] = 0.; }
        else { u_s[2 * j + 0] = b_points[5 * j + 2]; u_s[2 * j + 1] = b_points[5 * j + 3]; }
        epsilon[j] = 1;
    }
    const int r_max = (int)(2 * length / c_space);
    for (int j = 0; j < Np; j++) {
        const int m = (j - j % length) / length;
        const float x_m = s[2 * j + 0], y_m = s[2 * j + 1];
        for (int r = 1; r < r_max; r++)
            for (int l = 0; l < length; l++) {
                const int mm = (m - r < 0) ? m - r + c_num : m - r;
                const float x_l = s[2 * (l + mm * length) + 0];
                const float y_l = s[2 * (l + mm * length) + 1];
                if (fabsf(x_l - x_m) < 1 && fabsf(y_l - y_m) < 1) epsilon[j] = 0;
            }
    }
}

/* main.cu:852-909: one iteration on f_stream. */
void oracle_step(oracle_state* st, int it)
{
    const int X = st->XDIM, Y = st->YDIM;
    const long size = (long)X * Y;
    oracle_equilibrium(st->u, st->rho, st->f0, st->force, st->F, X, Y, st->TAU);
    oracle_collision(st->f0, st->f, st->f1, st->F, st->TAU, st->TAU2, X, Y, it);
    oracle_streaming(st->f1, st->f, X, Y);
    oracle_macro(st->f, st->u, st->rho, X, Y);
    const int have_bf = st->body_force[0] != 0. || st->body_force[1] != 0.;
    if (st->Ns > 0) {
        oracle_interpolate(st->rho, st->u, st->Ns, st->u_s, st->F_s, st->s, X, Y);
        if (!have_bf) {
            if (st->point_spread)
                oracle_spread_points(st->rho, st->u, st->f, st->Ns, st->u_s, st->F_s, st->force, st->s, X, Y,
                                     st->Q, st->epsilon, st->flux_column, st->flux_norm);
            else
                oracle_spread(st->rho, st->u, st->f, st->Ns, st->u_s, st->F_s, st->force, st->s, X, Y,
                              st->Q, st->epsilon, st->flux_column, st->flux_norm);
            return;
        }
        /* extension: force = spread + body force, then the u correction and flux */
        if (st->point_spread)
            oracle_spread_points(st->rho, st->u, st->f, st->Ns, st->u_s, st->F_s, st->force, st->s, X, Y,
                                 NULL, st->epsilon, -1, 1.);
        else
            oracle_spread(st->rho, st->u, st->f, st->Ns, st->u_s, st->F_s, st->force, st->s, X, Y,
                          NULL, st->epsilon, -1, 1.);
        for (long j = 0; j < size; j++) {
            st->force[j] += st->body_force[0];
            st->force[size + j] += st->body_force[1];
        }
    } else {
        /* no-IB variant: force is the uniform body force (0 in the reference) */
        for (long j = 0; j < size; j++) {
            st->force[j] = st->body_force[0];
            st->force[size + j] = st->body_force[1];
        }
    }
    spread_finish(st->rho, st->u, st->f, st->force, X, Y, st->Q, st->flux_column, st->flux_norm);
}

void oracle_run(oracle_state* st, int it0, int nsteps)
{
    for (int n = 0; n < nsteps; n++) oracle_step(st, it0 + n);
}

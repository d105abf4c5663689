/*
 * san_main.c — TEST INFRASTRUCTURE: drives every function of the CPU restatement (oracle.c) under
 * AddressSanitizer / UndefinedBehaviorSanitizer (sanitizers on the CPU path; the GPU
 * path has none on this pool).  Built by oracle/Makefile.san, run by tests/test_sanitize.py.
 * A 96 x 48 channel with IB points at the lattice's x edges (the flat-index quirk of
 * ImmersedBoundary.cu:119-122), next to the walls, and an overlap-masked one; both spread forms;
 * the cilia kinematics of two cilia (main.cu:77-252); the d_delta support edge.  Exit 0 = clean
 * (the sanitizers abort on a finding).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define NX 96
#define NY 48
#define N (NX * NY)

static double* alloc(size_t n) {
    double* p = (double*)calloc(n, sizeof(double));
    if (!p) exit(2);
    return p;
}

static int finite_all(const double* a, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (!isfinite(a[i])) return 0;
    return 1;
}

int main(void) {
    oracle_set_threads(1);
    double *f = alloc(9 * N), *f0 = alloc(9 * N), *f1 = alloc(9 * N), *F = alloc(9 * N);
    double *rho = alloc(N), *u = alloc(2 * N), *force = alloc(2 * N), *Q = alloc(1);
    for (int j = 0; j < N; ++j) {
        rho[j] = 1.0 + 1e-3 * sin(0.37 * j);
        u[j] = 1e-3 * cos(0.11 * j);
        u[N + j] = 1e-3 * sin(0.05 * j);
    }
    oracle_equilibrium(u, rho, f, force, F, NX, NY, 2.8068);  /* f = feq (main.cu:722) */
    /* points: x = 0.2 and x = XDIM - 0.3 (nodes across the x edge), y next to both walls, eps 0 */
    enum { NS = 8 };
    float s[2 * NS] = {0.2f, 10.f, NX - 0.3f, 20.f, 40.4f, 0.6f, 41.5f, NY - 1.4f, 60.f, 24.f, 61.f, 25.f, 1.5f, 1.5f, 80.2f, 33.3f};
    float us[2 * NS], Fs[2 * NS];
    int eps[NS] = {1, 1, 1, 1, 1, 0, 1, 1};
    for (int k = 0; k < 2 * NS; ++k) us[k] = 1e-3f * (float)((k % 3) - 1);
    oracle_state st;
    memset(&st, 0, sizeof st);
    st.XDIM = NX; st.YDIM = NY; st.TAU = 2.8068; st.TAU2 = 0.5361;
    st.f = f; st.f0 = f0; st.f1 = f1; st.F = F; st.rho = rho; st.u = u; st.force = force; st.Q = Q;
    st.Ns = NS; st.s = s; st.u_s = us; st.F_s = Fs; st.epsilon = eps;
    st.body_force[0] = 1e-6; st.flux_column = NX - 5; st.flux_norm = 192.0;
    for (int mode = 0; mode < 2; ++mode) {  /* the literal O(N*Ns) gather, then the point scatter */
        st.point_spread = mode;
        oracle_run(&st, 0, 6);
    }
    st.Ns = 0;  /* no-IB variant */
    oracle_run(&st, 12, 4);
    /* the delta's support edge and beyond */
    float dsum = 0.f;
    for (int dx = -3; dx <= 3; ++dx) dsum += oracle_d_delta(10.5f, 10.5f, 10 + dx, 10);
    /* cilia: four cilia 48 apart, XDIM = 192 (main.cu:77-252).  Fewer than 2 LENGTH / c_space cilia
     * make boundary_check's neighbour index m - r + c_num negative (main.cu:214-248, restated as is):
     * an out-of-bounds read the reference's own check XDIM >= 2 LENGTH (main.cu:303) excludes, and
     * the one ASan found on the first run of this harness with two cilia. */
    const int c_num = 4, T = 1000, CX = 192;
    float* samp = (float*)calloc((size_t)5 * 9600 * c_num, sizeof(float));
    float* lasts = (float*)calloc((size_t)2 * 9600 * c_num, sizeof(float));
    float* bp = (float*)calloc((size_t)5 * 96 * c_num, sizeof(float));
    float* cs = (float*)calloc((size_t)2 * 96 * c_num, sizeof(float));
    float* cu = (float*)calloc((size_t)2 * 96 * c_num, sizeof(float));
    int* ce = (int*)calloc((size_t)96 * c_num, sizeof(int));
    if (!samp || !lasts || !bp || !cs || !cu || !ce) return 2;
    for (int it = 0; it < 3; ++it) {
        oracle_define_filament(T, it, 48.0, T / c_num, (double)c_num, samp, lasts, bp);
        oracle_boundary_check(48.0, c_num, CX, it, bp, cs, cu, ce);
    }
    const int ok = finite_all(f, 9 * N) && finite_all(rho, N) && finite_all(u, 2 * N) && isfinite(*Q) && isfinite(dsum);
    printf("{\"ok\": %s, \"Q\": %.17g, \"delta_sum\": %.9g, \"cilia_x0\": %.6g}\n", ok ? "true" : "false", *Q,
           (double)dsum, (double)cs[0]);
    free(f); free(f0); free(f1); free(F); free(rho); free(u); free(force); free(Q);
    free(samp); free(lasts); free(bp); free(cs); free(cu); free(ce);
    return ok ? 0 : 1;
}

/*
 * oracle.h — CPU restatement of the reference IB-LBM hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (cuda_iblb_11_amd, libiblb.so) never links or calls it.
 *
 * Every function restates one reference kernel (file:line under /root/reference/
 * CUDA_IBLB_11) in plain C with the reference's array layouts, loop orders and
 * float/double rounding points, compiled with -ffp-contract=off.  One documented
 * generalisation: `spread` takes YDIM (the reference hard-codes size = 192*XDIM,
 * ImmersedBoundary.cu:146; identical for YDIM == 192).
 *
 * Parity status: the reference's CUDA sources need nvcc + the CUDA runtime, neither of
 * which exists in this image, so the reference cannot be built here (see DESIGN.md
 * "Oracle and parity").  This restatement is pinned by analytic known-answer tests and
 * by the reference's own nominal output files (Data/Nominals) as an envelope — NOT by
 * reference-generated vectors: parity against the reference binary is UNPINNED.
 */
#ifndef IBLB_ORACLE_H
#define IBLB_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

/* LatticeBoltzmann.cu:30-62 */
void oracle_equilibrium(const double* u, const double* rho, double* f0, const double* force,
                        double* F, int XDIM, int YDIM, double TAU);
/* LatticeBoltzmann.cu:64-171 */
void oracle_collision(const double* f0, const double* f, double* f1, const double* F,
                      double TAU, double TAU2, int XDIM, int YDIM, int it);
/* LatticeBoltzmann.cu:173-373 (push form, literal switch logic) */
void oracle_streaming(const double* f1, double* f, int XDIM, int YDIM);
/* LatticeBoltzmann.cu:375-411 */
void oracle_macro(const double* f, double* u, double* rho, int XDIM, int YDIM);
/* ImmersedBoundary.cu:21-81 */
float oracle_d_delta(float xs, float ys, int x, int y);
/* ImmersedBoundary.cu:94-133 */
void oracle_interpolate(const double* rho, const double* u, int Ns, const float* u_s, float* F_s,
                        const float* s, int XDIM, int YDIM);
/* ImmersedBoundary.cu:138-267, cell-centric O(N*Ns) gather exactly as the reference
 * (tiles of 64 points, all points evaluated for every cell). */
void oracle_spread(const double* rho, double* u, const double* f, int Ns, const float* u_s,
                   const float* F_s, double* force, const float* s, int XDIM, int YDIM,
                   double* Q, const int* epsilon, int flux_column, double flux_norm);
/* Same result as oracle_spread, point-centric: only the 3x3 nodes around each point can
 * have a non-zero delta, so each point scatters into those (in point order, so each
 * cell's sum has the reference's term order). */
void oracle_spread_points(const double* rho, double* u, const double* f, int Ns, const float* u_s,
                          const float* F_s, double* force, const float* s, int XDIM, int YDIM,
                          double* Q, const int* epsilon, int flux_column, double flux_norm);

/* Cilia kinematics (the reference's Lagrangian source, main.cu:56-252).
 * define_filament: 9600 samples per cilium of the Fourier beat shape (A_mn/B_mn "without
 * mucus", main.cu:56-74); boundary points b_points[5*96*c_num] are the samples whose arc
 * position lies within 0.01 of an integer (main.cu:158-172; where two samples qualify, the
 * later one in thread order is kept).  boundary_check: s, u_s and the overlap mask epsilon
 * (main.cu:176-252; all of s is written before the mask is evaluated). */
void oracle_define_filament(int T, int it, double c_space, int p_step, double c_num, float* s, float* lasts,
                            float* b_points);
void oracle_boundary_check(double c_space, int c_num, int XDIM, int it, const float* b_points, float* s,
                           float* u_s, int* epsilon);

/* One reference iteration main.cu:852-909 on host arrays:
 * equilibrium -> collision -> streaming -> macro -> [interpolate -> spread].
 * body_force (2 doubles, may be NULL) is added to force after spread (extension;
 * NULL or zeros reproduce the reference).  Ns == 0 runs the no-IB variant, where
 * force = body_force and u = (sum c f + force/2)/rho.  point_spread selects
 * oracle_spread_points (1) or the literal O(N*Ns) oracle_spread (0). */
typedef struct oracle_state {
    int XDIM, YDIM;
    double TAU, TAU2;
    double* f;     /* [9N] post-stream populations   */
    double* f0;    /* [9N] scratch                    */
    double* f1;    /* [9N] scratch                    */
    double* F;     /* [9N] scratch                    */
    double* rho;   /* [N]                              */
    double* u;     /* [2N]                             */
    double* force; /* [2N]                             */
    double* Q;     /* [1]                              */
    int Ns;
    const float* s; const float* u_s; float* F_s; const int* epsilon;
    double body_force[2];
    int flux_column; double flux_norm;
    int point_spread;
} oracle_state;

void oracle_step(oracle_state* st, int it);
void oracle_run(oracle_state* st, int it0, int nsteps);

/* Threads the OpenMP loops use (1 = serial). */
void oracle_set_threads(int n);
int  oracle_get_threads(void);

#ifdef __cplusplus
}
#endif
#endif

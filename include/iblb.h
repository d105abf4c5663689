/*
 * iblb.h — C ABI of the MI355X-native immersed-boundary lattice-Boltzmann hot path.
 *
 * Replaces the hot path of ptheywood/CUDA_IBLB_11 (reference @ /root/reference):
 *   LatticeBoltzmann.cuh:4-10  equilibrium / collision / streaming / macro kernels
 *   ImmersedBoundary.cuh:4-8   interpolate / spread kernels
 *   main.cu:817-934            the per-step launch sequence that drives them
 *
 * Two layers are exported:
 *
 *  (1) Reference-shaped entry points (iblb_equilibrium ... iblb_spread).  Same names,
 *      same argument lists and the same array layouts as the reference kernels
 *      (device pointers; f/f0/f1/F are AoS [9*j+i], u/force are SoA [a*size+j],
 *      Lagrangian arrays are interleaved float xy), plus a trailing HIP stream.
 *      A maintainer replaces `kernel<<<grid, block, 0, s>>>(args)` in main.cu by
 *      `iblb_kernel(args, s)`.  They keep the reference's unfused data flow and exist
 *      for drop-in compatibility and kernel-by-kernel parity, not for speed.
 *
 *  (2) The fused context API (iblb_create ... iblb_destroy).  One context owns one
 *      x-slab of the lattice on one GPU, stores the populations SoA (y fastest) and
 *      advances the exact reference time step
 *        equilibrium -> collision -> streaming -> macro -> interpolate -> spread
 *      (main.cu:852-909): without IB one bandwidth-bound kernel advances up to seven
 *      iterations (temporal blocking, the deep sweep), with IB a band cycle of K iterations
 *      (the deep sweep beside a chain of small launches around the points).  Host arrays crossing this boundary use the reference layouts
 *      restricted to the slab: cell j = y * x_count + (x - x_begin).
 *
 * Conventions: every function returns IBLB_OK (0) or a negative IBLB_ERR_* code;
 * no C++ exception crosses the ABI.  The caller owns host buffers, the library owns
 * device buffers.  One host thread per context.  Context calls are synchronous on
 * return (results are in the caller's buffers).  The reference had no error
 * channel other than cudaGetLastError() at the call sites (main.cu:724-728,
 * 854-887, 902-922); here the code is returned and iblb_last_error() explains it.
 */
#ifndef IBLB_H
#define IBLB_H

#ifdef __cplusplus
extern "C" {
#endif

#define IBLB_OK               0
#define IBLB_ERR_ARG         -1   /* invalid argument / shape                      */
#define IBLB_ERR_HIP         -2   /* HIP runtime error (message in last_error)     */
#define IBLB_ERR_STATE       -3   /* call not valid in the current context state   */
#define IBLB_ERR_COMM        -4   /* RCCL / transport error                        */
#define IBLB_ERR_NOMEM       -5   /* device or host allocation failed              */
#define IBLB_ERR_UNSUPPORTED -6   /* feature not built / not available             */
#define IBLB_ERR_NODEVICE    -7   /* no HIP device visible                         */

#define IBLB_PREC_F64 0          /* populations stored and collided in double      */
#define IBLB_PREC_F32 1          /* populations stored as float deviations f - w_i */

#define IBLB_UNIQUE_ID_BYTES 128 /* size of the RCCL unique id blob               */

/* ABI version of this header: bumped whenever a struct crossing the ABI changes layout (iblb_config,
 * iblb_timing, iblb_cilia).  5: iblb_timing's band_cycles ... deep_iterations (round 4), the
 * size-checked iblb_get_timing_ex (round 5).  6: iblb_timing's dev_wait_launches and deep_mode ... deep_vgprs, and
 * iblb_set_wait_timeout (round 6).  Compare with iblb_abi_version() at run time. */
#define IBLB_ABI_VERSION 6

/* ---------------------------------------------------------------------------------
 * (1) Reference-shaped kernels.  All pointers are DEVICE pointers.  `stream` is a
 * hipStream_t (NULL = default stream).  Launch is asynchronous, like the reference's
 * <<< >>> launches; the return value reports launch errors only.
 * ------------------------------------------------------------------------------- */

/* LatticeBoltzmann.cu:30 equilibrium(u, rho, f0, force, F, XDIM, YDIM, TAU) */
int iblb_equilibrium(const double* u, const double* rho, double* f0, const double* force,
                     double* F, int XDIM, int YDIM, double TAU, void* stream);

/* LatticeBoltzmann.cu:64 collision(f0, f, f1, F, TAU, TAU2, XDIM, YDIM, it) — `it` unused as in the reference */
int iblb_collision(const double* f0, const double* f, double* f1, const double* F,
                   double TAU, double TAU2, int XDIM, int YDIM, int it, void* stream);

/* LatticeBoltzmann.cu:173 streaming(f1, f, XDIM, YDIM) */
int iblb_streaming(const double* f1, double* f, int XDIM, int YDIM, void* stream);

/* LatticeBoltzmann.cu:375 macro(f, u, rho, XDIM, YDIM) */
int iblb_macro(const double* f, double* u, double* rho, int XDIM, int YDIM, void* stream);

/* ImmersedBoundary.cu:94 interpolate(rho, u, Ns, u_s, F_s, s, XDIM, YDIM) */
int iblb_interpolate(const double* rho, const double* u, int Ns, const float* u_s, float* F_s,
                     const float* s, int XDIM, int YDIM, void* stream);

/* ImmersedBoundary.cu:138 spread(rho, u, f, Ns, u_s, F_s, force, s, XDIM, Q, epsilon).
 * Like the reference it assumes YDIM == 192 (`size = 192 * XDIM`, ImmersedBoundary.cu:146)
 * and accumulates Q += u_x(XDIM-5, y)/192 (ImmersedBoundary.cu:259-264). */
int iblb_spread(const double* rho, double* u, const double* f, int Ns, const float* u_s,
                const float* F_s, double* force, const float* s, int XDIM, double* Q,
                const int* epsilon, void* stream);

/* spread with the grid height, flux column and flux divisor made explicit
 * (YDIM == 192, flux_column == XDIM-5, flux_norm == 192 reproduces iblb_spread). */
int iblb_spread_ex(const double* rho, double* u, const double* f, int Ns, const float* u_s,
                   const float* F_s, double* force, const float* s, int XDIM, int YDIM,
                   double* Q, const int* epsilon, int flux_column, double flux_norm,
                   void* stream);

/* ImmersedBoundary.cu:21 d_delta, evaluated on the device for n (xs, ys, x, y) tuples
 * (parity hook for the 3-point kernel). */
int iblb_delta(int n, const float* xs, const float* ys, const int* x, const int* y,
               float* out, void* stream);

/* main.cu:77 define_filament(T, it, c_space, p_step, c_num, s, lasts, b_points): cilia beat
 * shape, s = the reference's d_boundary [5*9600*c_num], lasts [2*9600*c_num], b_points
 * [5*96*c_num].  Where two samples qualify for one boundary point the later one in thread
 * order is kept (the reference leaves that race unspecified). */
int iblb_define_filament(int T, int it, double c_space, int p_step, double c_num, float* s,
                         float* lasts, float* b_points, void* stream);

/* main.cu:176 boundary_check(c_space, c_num, XDIM, it, b_points, s, u_s, epsilon): Lagrangian
 * points s [2*96*c_num], velocities u_s and overlap mask epsilon [96*c_num]. */
int iblb_boundary_check(double c_space, int c_num, int XDIM, int it, const float* b_points,
                        float* s, float* u_s, int* epsilon, void* stream);

/* ---------------------------------------------------------------------------------
 * (2) Fused context API.
 * ------------------------------------------------------------------------------- */

typedef struct iblb_ctx iblb_ctx;

typedef struct iblb_config {
    int    nx, ny;            /* global lattice XDIM x YDIM (main.cu:270-271,298)          */
    double tau, tau2;         /* TAU, TAU2 (main.cu:320-321)                               */
    int    precision;         /* IBLB_PREC_F64 (default) or IBLB_PREC_F32                  */
    double body_force[2];     /* uniform force added to force^t every step; (0,0) = ref.  */
    double flux_norm;         /* Q += u_x / flux_norm; reference literal 192 (IB.cu:261)   */
    int    flux_column;       /* global column sampled for Q; reference XDIM-5 (IB.cu:259) */
    int    device;            /* HIP device ordinal                                        */
    int    x_begin, x_count;  /* owned columns [x_begin, x_begin + x_count); x_count <= 0
                                 means the whole lattice (single slab)                     */
    int    max_points;        /* Lagrangian point capacity; 0 disables the IB kernels      */
} iblb_config;

typedef struct iblb_timing {
    long long steps;           /* reference steps completed                              */
    long long fused_launches;  /* collide-stream launches timed                          */
    double    fused_ms;        /* summed duration of the timed collide-stream launches   */
    double    ib_ms;           /* summed duration of IB phases (interp + spread)         */
    double    halo_ms;         /* summed duration of halo exchanges                      */
    double    fused_bytes;     /* algorithmic bytes per cell of the collide-stream kernel */
    long long cells;           /* cells owned by this context                            */
    long long fused_cells;     /* lattice updates done by the timed collide-stream launches */
    /* two-iteration launches (temporal blocking, lbm_sweep.hip): each reads and writes the
     * state once (fused_bytes per cell) and advances its cells by two iterations */
    long long sweep_launches;  /* timed two-iteration launches                           */
    double    sweep_ms;        /* their summed duration                                  */
    long long sweep_cells;     /* cells they covered (lattice updates = 2 x sweep_cells) */
    /* deep launches (IBLB_SWEEP_DEPTH = K >= 3): state read and written once for K (or K-1)
     * iterations */
    long long sweepk_launches;
    double    sweepk_ms;
    long long sweepk_cells;    /* cells they covered; lattice updates = sweepk_cells x the launches'
                                * depths (deep_iterations / deep_launches on average) */
    long long sweepk_depth;    /* K, the configured depth */
    /* IB band cycles run (ctx_band.hip), and how many of them ran the merged chain; counted
     * whether or not profiling events are on */
    long long band_cycles;
    long long band_merged_cycles;
    long long band_par_cycles;  /* of those, run with the last level beside the deep sweep (lone slab) */
    /* deep launches (lone slab, slab interiors, band cycles) and the iterations they advanced, counted
     * whether or not profiling events are on: a call of n iterations mixes depths K and K-1 so that
     * no two-iteration or one-step remainder is left where n allows it (ctx_step.hip:deep_depth) */
    long long deep_launches;
    long long deep_iterations;
    /* launches of an RCCL group slab whose waves waited on a device word instead of a queue wait
     * (the slab hand-off, iblb_set_wait_timeout below); counted without profiling */
    long long dev_wait_launches;
    /* the build of the last deep launch (lone slab, slab interior or band cycle's deep sweep): its
     * MODE bits (lbm_sweep_impl.h), cells per lane, resident waves per SIMD and VGPRs per lane */
    long long deep_mode, deep_vs, deep_waves_per_simd, deep_vgprs;
} iblb_timing;

/* Reference defaults: 288x192, TAU/TAU2 for Re=1, T=1e5 (main.cu:267-321). */
int iblb_config_default(iblb_config* cfg);

int  iblb_create(const iblb_config* cfg, iblb_ctx** out);
void iblb_destroy(iblb_ctx* ctx);
const char* iblb_last_error(const iblb_ctx* ctx);   /* NULL ctx: last create() error */
const char* iblb_version(void);
int  iblb_abi_version(void);                       /* IBLB_ABI_VERSION the library was built with */
int  iblb_device_count(int* n);

/* Initial state (main.cu:636-754).  rho [N], u [2N] SoA, force [2N] SoA (force^0, may be
 * NULL = 0), f [9N] AoS post-stream populations (NULL = feq(rho, u) exactly as the
 * reference's initial `equilibrium` launch, main.cu:722-754).  N = x_count * ny.
 * rho == NULL and u == NULL: rho = 1, u = 0 (the reference's initial values). */
int iblb_set_state(iblb_ctx* ctx, const double* rho, const double* u, const double* f,
                   const double* force);

/* Lagrangian points for the next immersed-boundary evaluation (main.cu:834 boundary_check
 * outputs): s [2ns] xy, u_s [2ns] xy, epsilon [ns] (NULL = all 1).  Global coordinates.
 * A slab of a group needs >= 3 columns and the reference's invariant 0 <= s_x <= XDIM
 * (boundary_check wraps s_x into it, main.cu:202-205); IBLB_ERR_ARG otherwise. */
int iblb_set_lagrangian(iblb_ctx* ctx, int ns, const float* s, const float* u_s,
                        const int* epsilon);

/* Lagrangian points of the next `nsteps` iterations, given ahead (the reference computes a
 * new s, u_s, epsilon every iteration before its IB step, main.cu:822-841, 900-909): iteration
 * t0 + i (t0 = iblb_get_step at the call) uses entry i; after the last entry the points stay
 * those of entry nsteps-1.  Same result as iblb_set_lagrangian(entry i) before each of those
 * iterations, but iblb_step can then advance several iterations per launch (IB band cycle)
 * where the points of one cycle force only part of the lattice.  s, u_s [nsteps][2ns] xy,
 * epsilon [nsteps][ns] (NULL = all 1).  iblb_set_lagrangian / iblb_set_cilia end the schedule. */
int iblb_set_lagrangian_steps(iblb_ctx* ctx, int nsteps, int ns, const float* s, const float* u_s,
                              const int* epsilon);

/* On-device cilia kinematics (main.cu:822-841): when set, every iblb_step iteration `it`
 * first runs define_filament + boundary_check for `it` and uses their s, u_s, epsilon as the
 * Lagrangian points of that iteration (no host round trip).  c_num <= 0 or NULL disables.
 * Needs max_points >= 96 * c_num.  Excludes iblb_set_lagrangian while active. */
typedef struct iblb_cilia {
    int    c_num;    /* cilia (main.cu:268)                                        */
    double c_space;  /* spacing of the cilium bases in lattice units (main.cu:280) */
    int    T;        /* beat period in iterations (main.cu:299)                    */
    int    p_step;   /* phase lag of neighbouring cilia, T*c_fraction/c_num (main.cu:336) */
} iblb_cilia;
int iblb_set_cilia(iblb_ctx* ctx, const iblb_cilia* cilia);
/* Current Lagrangian points (the reference's d_s, d_u_s, d_epsilon; any may be NULL). */
int iblb_get_lagrangian(iblb_ctx* ctx, float* s, float* u_s, int* epsilon);

/* Advance nsteps reference iterations (main.cu:852-909 each). */
int iblb_step(iblb_ctx* ctx, int nsteps);

/* Macroscopic fields after the last step as the reference holds them after `spread`:
 * rho [N] = sum f (macro), u [2N] SoA = (sum c f + force/2)/rho.  Either may be NULL. */
int iblb_get_macro(iblb_ctx* ctx, double* rho, double* u);
/* Post-stream populations f^t [9N] AoS (the reference's d_f after streaming). */
int iblb_get_populations(iblb_ctx* ctx, double* f);
/* force^t [2N] SoA as the reference's d_force after spread (plus body_force). */
int iblb_get_force(iblb_ctx* ctx, double* force);
/* Lagrangian force F_s [2ns] of the last interpolation.  Collective in an RCCL group; in a
 * local group each slab holds the F_s of the points whose column min(x0, XDIM-1) it owns and
 * zeros for the others (sum over the slabs). */
int iblb_get_lagrangian_force(iblb_ctx* ctx, float* F_s);
/* Cumulative flux Q (ImmersedBoundary.cu:259-264).  With a multi-slab RCCL group this
 * is the sum over all ranks; with a local group it is this slab's share. */
int iblb_get_flux(iblb_ctx* ctx, double* Q);
int iblb_get_step(iblb_ctx* ctx, long long* steps);
/* Non-finite (NaN / Inf) stored populations of the current state, counted over every cell
 * of the lattice (summed over the ranks of an RCCL group: collective).  The driver checks it
 * at every output iteration (the reference's penalty IB can diverge). */
int iblb_count_nonfinite(iblb_ctx* ctx, long long* count);

/* Timing: when enabled (1) every collide-stream launch is bracketed by HIP events on the
 * stream it runs on; iblb_get_timing() returns the sums (and resets them if reset).  enabled = 2:
 * only the deep (K-iteration) launches are timed, by their own dispatch / completion signals (no
 * marker packets; the IB band cycle's chain launches run untimed), so that a timed region with IB
 * keeps its schedule. */
int iblb_set_profiling(iblb_ctx* ctx, int enabled);
int iblb_get_timing(iblb_ctx* ctx, iblb_timing* t, int reset);
/* The same, writing at most `bytes` bytes of the struct (pass sizeof(iblb_timing) of the header the
 * caller was built with: an older, shorter iblb_timing gets its own fields only).  iblb_get_timing
 * writes sizeof(iblb_timing) of THIS header. */
int iblb_get_timing_ex(iblb_ctx* ctx, iblb_timing* t, unsigned long bytes, int reset);
/* The stream the context launches on (hipStream_t), for callers that add work. */
int iblb_get_stream(iblb_ctx* ctx, void** stream);
/* Block until all work of the context is done. */
int iblb_synchronize(iblb_ctx* ctx);

/* ---- x-slab decomposition -------------------------------------------------------
 * Slabs are ordered along x (periodic).  Every population buffer of a slab holds ghost
 * columns on both sides (3K per side, K = IBLB_SWEEP_DEPTH); a halo exchange of depth d
 * sends the d whole edge columns of the current state to each neighbour and receives the
 * neighbours' into the ghost columns, in place (no packing): d = 1 for a one-step
 * iteration, 3 when an owed IB force is evaluated from the ghosts, K per K-iteration deep
 * cycle, 3K per IB band cycle whose trapezoids cross a slab edge.
 *
 * Local group: n contexts of ONE process (any devices with peer access) linked
 * left-to-right; iblb_group_step() advances them together.  Synchronous transport,
 * meant for testing the decomposition on one GPU.
 *
 * RCCL group: one context per process; rank 0 creates the id, it is broadcast by the
 * caller (e.g. torch.distributed), every rank attaches; iblb_step() then exchanges
 * halos with ncclSend/ncclRecv on a second stream, overlapped with the collide of the
 * interior columns (IBLB_OVERLAP=0 in the environment selects the sequential schedule).
 * With an RCCL group iblb_step, iblb_set_lagrangian and every reader are collective. */
int iblb_link_local(iblb_ctx** ctxs, int n);
int iblb_group_step(iblb_ctx** ctxs, int n, int nsteps);
int iblb_rccl_unique_id(char id[IBLB_UNIQUE_ID_BYTES]);
int iblb_attach_rccl(iblb_ctx* ctx, const char id[IBLB_UNIQUE_ID_BYTES], int nranks, int rank);
/* Bound of the RCCL group's device-side waits, in seconds of wall-clock time (default 600, or
 * IBLB_WAIT_TIMEOUT_S from the environment at iblb_create).  Inside a run of deep cycles a slab's
 * kernels wait for the boundary work of the previous cycle on a device word rather than in the
 * hardware queue; that work follows the cycle's halo exchange, i.e. the neighbour ranks.  A rank
 * whose host reaches its next iblb_step late (writing output, a checkpoint, the caller's own work)
 * delays those waits like RCCL's own kernels and changes no result; only a wait longer than this
 * bound fails: the iblb_step / iblb_synchronize that sees it returns IBLB_ERR_COMM and the state
 * must be set again.  Set it at least as long as the longest pause any rank takes between calls. */
int iblb_set_wait_timeout(iblb_ctx* ctx, double seconds);

/* Whole-lattice rho [nx*ny] and u [2*nx*ny] (reference layout, j = y*XDIM + x) on rank `root`
 * of an RCCL group: the output gather the reference's single-GPU BigData writer needs
 * (main.cu:938-971) when the lattice is split over GPUs.  Collective; the other ranks may
 * pass NULL.  A single slab returns iblb_get_macro. */
int iblb_gather_macro(iblb_ctx* ctx, int root, double* rho, double* u);

/* ---- checkpoint / restart (absent in the reference; its jobs run 1e5+ steps, cilia6.sh) --
 * iblb_save_checkpoint writes this context's slab: the stored populations in their storage
 * precision, step count, cumulative flux Q, Lagrangian points and cilia kinematics state
 * (written to path.tmp, then renamed).  iblb_load_checkpoint restores it into a context
 * created with the same lattice, slab, precision, tau/tau2 and body force (and enough
 * max_points); stepping on from there is bit-identical to the uninterrupted run up to the
 * summation order of the IB spread.  Each rank of a group saves / loads its own file;
 * restore before iblb_link_local, before or after iblb_attach_rccl. */
int iblb_save_checkpoint(iblb_ctx* ctx, const char* path);
int iblb_load_checkpoint(iblb_ctx* ctx, const char* path);

#ifdef __cplusplus
}
#endif
#endif /* IBLB_H */

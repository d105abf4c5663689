// iblb_kernels.h — host-callable launchers of the slab kernels (used by iblb_ctx.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "iblb_device.h"

namespace iblb {

// Cells per lane of the collide-stream kernel: 16 bytes per lane per plane.
template <typename T>
constexpr int vec_of() { return 16 / (int)sizeof(T); }

// A slab's view of the points for IB with ghost columns (launch_ib_ghost below)
struct IbGhost {
    int nx, x_begin;
    int gc;        // ghost columns holding valid data (node pulls outside are skipped)
    int clo, chi;  // local columns that receive force
    int part;
    // the launch's first lane stores sig_val to *sig (agent scope) when the kernel starts: the kernels
    // before it in its stream are complete (the IB band cycle's exchange, ctx_band.hip)
    unsigned* sig = nullptr;
    unsigned sig_val = 0;
    // points [wlo, whi): their images -1 / +1 in groups of their own after the ns point groups (as
    // FusedArgs::wlo)
    int wlo = 0, whi = 0;
};

template <typename T>
struct FusedArgs {
    const T* src;
    T* dst;
    Layout L;
    Halo<T> H;          // column -1 / ncol planes (periodic images or ghost columns)
    int col_begin;      // first local column handled by this launch
    int col_step;       // distance between the columns of this launch (1 = contiguous range)
    int ncols;          // columns handled by this launch
    const int* cols;    // column table (device): column k of the launch is cols[col_begin + k]
                        // (nullptr: col_begin + k * col_step); IB bands of the K-iteration cycle
    int nch;            // 64*V-row chunks per column
    uint8_t* flags;     // per (column, chunk): dense IB force present (nullptr: no IB); the
                        // wave that consumes a chunk's force clears its values and its flag
                        // (columns -gc .. ncol+gc-1 addressable: the pointer is at column 0)
    double* fdense;     // dense IB force, x plane then y plane (column stride rows; column 0)
    long fplane;
    int flux_col;       // local column sampled for Q (>= 0), or -1 (none: never column -1, a ghost column)
    double flux_norm;
    double* Q;
    Coef c;
    KConst k;           // collide constants folded on the host (iblb_device.h)
    int variant;        // kernel variant (MODE bits of lbm_kernels.hip), 0 = default
    // IB band patches (band cycle, rows restricted): with row_tab set, cols holds 5 ints per entry
    // from col_begin on, {column, first chunk, end chunk, first row, end row}, and launch entry e
    // covers chunks [first, end) of its column (nchl waves per entry, the extra ones exit).  Q is
    // sampled on rows [first row, end row) only; store_rows: the populations too (other rows of
    // the column belong to the deep sweep).
    int row_tab = 0;
    int nchl = 0;
    int store_rows = 0;
    // Merged band chain (ctx_band.hip): the force of this level is read, not consumed (fkeep: the
    // IB waves below read it too); the waves of the entries clear the force buffer fdclr / flclr
    // of the level before (consumed by the previous launch) at their (column, chunk); clr_waves
    // more waves clear it at columns clr_lo .. clr_lo+clr_w-1 and clr_hi .. clr_hi+clr_w-1 (nch
    // chunks each); nns > 0: after those,
    // 16 lanes per point (nns points of the next level's iteration) evaluate the next level's force
    // from this launch's source (ib_next_group, ib_device.h) into fdnext / flnext.
    int fkeep = 0;
    double* fdclr = nullptr;
    uint8_t* flclr = nullptr;
    int clr_waves = 0, clr_lo = 0, clr_hi = 0, clr_w = 0;
    int nns = 0;
    IbGhost nG{};
    const float* n_s = nullptr;
    const float* n_us = nullptr;
    const int* n_eps = nullptr;
    double* fdnext = nullptr;
    uint8_t* flnext = nullptr;
    // points [wlo, whi): their periodic images (m = -1, +1) are evaluated by groups of their own after
    // the nns point groups, whose groups then take image m = 0 only (a point at the lattice's x edge
    // has two images in a slab touching that edge, which one group would walk one after the other)
    int wlo = 0, whi = 0;
    // vhalf (band cycle, f32): the launch's entry waves take 64 * V/2 rows (row_tab chunks in those
    // units); the IB flags stay per 64 * V rows, read at chunk / 2 and not cleared by these waves (two
    // waves share one: a flag left set over zeroed force takes the forced collide with force 0, bit
    // for bit the unforced one; a merged level's fdclr values are still cleared, their flag kept)
    int vhalf = 0;
    int probe = 0;  // timing probe IBLB_PROBE_LEVEL (WRONG results): 1 point groups skipped, 2 entry waves skipped,
                    // 3 point groups end after their region, 4 before their spread (5 / 6, the spread
                    // with plain stores / without chunk flags: round 5, profiles/r05/probe, removed)
};

// Two iterations per launch (lbm_sweep.hip): g^t -> g^{t+2}, no IB force owed in between.
// IB band cycle with its last level beside the deep sweep (and a group slab's boundary sweeps): a patch output region the
// last level stores and the deep sweep must not: local columns [x0, x1] (inclusive) x rows [y0, y1)
// (even bounds, so that a lane's two cells are both in or both out)
struct SkipBox {
    int x0, x1, y0, y1;
};
constexpr int MAX_SKIP = 96;

template <typename T>
struct Sweep2Args {
    const T* src;        // g^t
    T* dst;              // g^{t+K} (the other buffer)
    Layout L;
    int col_begin;       // sweep s covers output columns [col_begin + s*col_step, + W) ∩ [.., col_end)
    int col_step;
    int col_end;
    int nsweep;
    int W;               // output columns per sweep (wave)
    int vs;              // cells per lane; rows, col and plane multiples of vs
    int nch;             // set by launch_sweep2
    int variant;         // deep sweeps: bit 0 nontemporal stores, bit 1 the f32 wall split
    int nsweep_w = 0;    // wall split (set by the launcher): sweeps of each wall chunk,
    int wall_ch0 = 0;    // inner chunks between the wall chunks,
    int wall_top = 0;    // and the first row of the top wall chunk
    int cus;             // deep sweeps, balanced widths: CUs the launch's stream may use (0 = all)
    int flux_col;        // local column sampled for Q (every iteration), or -1
    int fskip0, fskip1;  // rows [fskip0, fskip1) of the flux column are not sampled (an IB band
                         // patch covers them: its trapezoid's last level adds their flux)
    double flux_norm;
    double* Q;
    Coef c;
    KConst k;            // collide constants folded on the host (iblb_device.h)
    // Device-side ordering of a slab's interior and boundary sweeps (ghost-column builds only,
    // ctx_step.hip:deep_slab_step).  An edge wave is one whose output columns reach below wait_lo or
    // above wait_hi (wait_lo = INT_MAX: every wave).  wait_seq: edge waves first wait until
    // *wait_seq - wait_val >= 0, bounded by wait_ticks of the device's constant wall clock
    // (wall_clock64; the context's wait timeout, 600 s by default: a neighbour rank that is late
    // by less never fails the wait); past it they set *wait_err and go on, and the host reports the
    // call as failed.  done_cnt: edge waves add 1 when their stores are released (agent scope), and
    // the host learns their number from *edge_waves (set by the launcher).  nullptr: no wait / no signal.
    const unsigned* wait_seq = nullptr;
    unsigned wait_val = 0;
    int wait_lo = 0, wait_hi = 0;
    unsigned* wait_err = nullptr;
    unsigned long long wait_ticks = 0;
    unsigned* done_cnt = nullptr;
    int* edge_waves = nullptr;  // host pointer, written by launch_sweepk (not read on the device)
    int* kinfo = nullptr;       // host pointer: {MODE, VS, resident waves per SIMD, VGPRs} of the build launched
    int edge_trim = 0;          // balanced sweeps: the first and last sweep this many columns narrower
    int nskip = 0;       // > 0: the patch output regions below are left to the band's last level,
    SkipBox skip[MAX_SKIP];  // sorted by x0, disjoint in columns (a lone slab's deep sweep, a group slab's interior and boundary sweeps)
};

// ghost: false = lone slab (columns outside [0, ncol) are the periodic images; also the interior
// columns of a group slab, which read none); true = columns outside [0, ncol) are the ghost
// columns of the buffer itself (a group slab's boundary sweeps after the halo exchange)
template <typename T>
hipError_t launch_sweep2(Sweep2Args<T> a, bool ghost, hipStream_t s);
// K = depth (3 .. 6) iterations per launch: g^t -> g^{t+K}; ghost as above (a
// boundary sweep of output columns [0, K) reads columns -K .. 2K-1).  col_step 0: balanced widths.
// start / stop: recorded by the kernel's dispatch / completion signals (no marker packets)
template <typename T>
hipError_t launch_sweepk(Sweep2Args<T> a, int depth, bool ghost, hipStream_t s, hipEvent_t stop = nullptr,
                         hipEvent_t start = nullptr);
// *p = v after the stream's previous work (one lane, an agent-scope store: the release of the
// previous kernel's stores is its end-of-kernel fence)
hipError_t launch_seq_signal(unsigned* p, unsigned v, hipStream_t s);
// Test hold (IBLB_TEST_HOLD, ctx_step.hip:exchange): one wave that polls the host-coherent *word
// until it is non-zero or `ticks` of the device wall clock have passed, so that the work queued
// behind it on `s` starts late, as behind a neighbour rank that reaches its exchange late.
hipError_t launch_test_hold(const unsigned* word, unsigned long long ticks, hipStream_t s);
// Resident waves per CU of a deep-sweep configuration; *nch = its row chunks for ny rows.
template <typename T>
int sweepk_geometry(int depth, int vs, int variant, bool ghost, int ny, int* nch);

// Launch geometry of the collide-stream kernel: one wave per (column, 64*V-row chunk).
inline int chunks_per_column(int ny, int V) { return (ny + 64 * V - 1) / (64 * V); }

template <typename T>
hipError_t launch_fused(const FusedArgs<T>& a, hipStream_t s, hipEvent_t stop = nullptr);  // stop: recorded at the end

// Step 0 of a fresh state: collide f^0 with explicit rho^0, u^0, force^0 (no pull).
template <typename T>
hipError_t launch_boot(const T* src, T* dst, Layout L, const double* rho0, const double* u0,
                       const double* force0, long fplane, Coef c, KConst k, hipStream_t s);

// Macroscopic output in the reference layout (slab-local j = y*ncol + xc):
// rho = sum f, u = (sum c f + force/2)/rho with force = g + dense IB force.
template <typename T>
hipError_t launch_macro_out(const T* g, Layout L, Halo<T> H, const double* fdense, long fplane,
                            double gx, double gy, double* rho, double* u, hipStream_t s);

// Post-stream populations f^t in the reference AoS layout [9*j+i] (raw: no pull).
template <typename T>
hipError_t launch_pop_out(const T* g, Layout L, Halo<T> H, double* f, int raw, hipStream_t s);

// q(u^t) of the current state for the flux column (added to *out).
template <typename T>
hipError_t launch_flux(const T* g, Layout L, Halo<T> H, const double* fdense, long fplane,
                       double gx, double gy, int xc, double flux_norm, double* out, hipStream_t s);

// Non-finite stored populations of the slab's own cells (rows < ny, all nine planes), added to
// *count (one double: an exact integer up to 2^53).
template <typename T>
hipError_t launch_count_nonfinite(const T* g, Layout L, double* count, hipStream_t s);

// Reference AoS populations [9*j+i] -> slab planes (deviation form for float).
template <typename T>
hipError_t launch_pop_in(const double* f, T* g, Layout L, hipStream_t s);

// Reference SoA field [comp*N + j] (j = y*ncol + xc) <-> slab layout [comp*fplane + xc*col + y].
hipError_t launch_field_in(const double* ref, double* lay, Layout L, int ncomp, long fplane, hipStream_t s);
hipError_t launch_field_out(const double* lay, double* ref, Layout L, int ncomp, long fplane, double add0,
                            double add1, hipStream_t s);

// Immersed boundary (global coordinates; the slab owns columns [x_begin, x_begin+ncol)).
// Single slab: nodes + interpolation + spread of every point in one launch.
template <typename T>
hipError_t launch_ib_point(const T* g, Layout L, Halo<T> H, int nx, int ns, const float* s, const float* u_s,
                           const int* eps, float* F_s, double* fdense, long fplane, uint8_t* flags, int nch,
                           int rows_per_chunk, hipStream_t st);
// A slab with ghost columns (a slab of a group after a halo exchange of depth >= gc, or a lone
// slab whose ghosts hold periodic copies): every point whose 3x3 spread reaches local columns
// [clo, chi) — each periodic image of it, x0 - x_begin + m * nx for m = -1, 0, 1 — pulls its nodes
// from the buffer (columns -gc .. ncol+gc-1) and spreads into the cells of [clo, chi) (global
// columns clipped to [0, XDIM) as the reference's cell-centric spread).  F_s: the slab holding
// column min(x0, XDIM-1) writes the point's F_s, the others zero (readers sum).  part: 0 every
// point, 1 the inner points (2 <= x0 - x_begin <= ncol-3: nodes and pulls inside the slab, no
// ghost needed), 2 the others.
// (IbGhost: declared with FusedArgs above)
template <typename T>
hipError_t launch_ib_ghost(const T* g, Layout L, IbGhost G, int ns, const float* s, const float* u_s, const int* eps,
                           float* F_s, double* fdense, long fplane, uint8_t* flags, int nch, int rows_per_chunk,
                           hipStream_t st);

}  // namespace iblb

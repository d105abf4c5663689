// iblb_kernels.h — host-callable launchers of the slab kernels (used by iblb_ctx.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "iblb_device.h"

namespace iblb {

// Cells per lane of the collide-stream kernel: 16 bytes per lane per plane.
template <typename T>
constexpr int vec_of() { return 16 / (int)sizeof(T); }

template <typename T>
struct FusedArgs {
    const T* src;
    T* dst;
    Layout L;
    Halo<T> H;
    T* send_left[3];    // planes {3,6,7} of column 0 (nullptr = not sent)
    T* send_right[3];   // planes {1,5,8} of column ncol-1
    int col_begin;      // first local column handled by this launch
    int col_step;       // distance between the columns of this launch (1 = contiguous range)
    int ncols;          // columns handled by this launch
    const int* cols;    // column table (device): column k of the launch is cols[col_begin + k]
                        // (nullptr: col_begin + k * col_step); IB bands of the K-iteration cycle
    int nch;            // 64*V-row chunks per column
    uint8_t* flags;     // per (column, chunk): dense IB force present (nullptr: no IB); the
                        // wave that consumes a chunk's force clears its values and its flag
    double* fdense;     // dense IB force, x plane then y plane (same col stride)
    long fplane;
    int flux_col;       // local column sampled for Q, or -1
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
};

// The band chain of one IB band cycle in ONE launch (lbm_kernels.hip band_kernel): workgroup q
// runs patch q's whole trapezoid, level j = 0 .. K-1: the IB of the level's points whose node
// column x0 lies in the patch (force^{t+j} from level j-1, or from g^t at j = 0 when owed), a
// workgroup barrier, the one-step collide of the level's entries (fused_wave), a barrier.  The
// patches' columns are disjoint and apart, so workgroups never share a cell, a force value or a
// flag.  Bit-identical to the launch-per-level chain (same bodies, same data; spread atomics in
// another order).
constexpr int BAND_MAX_K = 6;
constexpr int BAND_PT = 2 + 3 * BAND_MAX_K;  // ints per patch in the patch table
template <typename T>
struct BandArgs {
    FusedArgs<T> f;                  // the collide arguments common to every level (cols = the
                                     // entry table, row_tab = 1); src / dst / H / entries per level
    const T* src[BAND_MAX_K];        // level j reads src[j] (g^t, then the scratch levels) ...
    T* dst[BAND_MAX_K];              // ... and writes dst[j] (the last level: g^{t+K}, patch rows)
    Halo<T> H0;                      // periodic images of g^t (the only level that can reach x = 0)
    // patch q: pt[q*BAND_PT + 0..1] = the x0 range [lo, hi] (local) of its points, then per level
    // j: {first entry, entries, chunks per entry} at pt[q*BAND_PT + 2 + 3j]
    const int* pt;
    int npatch;
    int K;
    int ib0;                         // level 0 evaluates force^t from g^t (owed)
    const float* ps[BAND_MAX_K];     // the points of level j (iteration t+j-1; j = 0: the current)
    const float* pus[BAND_MAX_K];
    const int* pe[BAND_MAX_K];
    int ns;
    int nx;
    int x_begin;
    int slab;                        // a slab of a group: IB by ib_slab_group (no halo is reached)
    IbHalo<T> X;
    float* F_s;
    int rows_per_chunk;              // of the IB flags (64 * V)
};
template <typename T>
hipError_t launch_band(const BandArgs<T>& a, hipStream_t s);

// Two iterations per launch (lbm_sweep.hip): g^t -> g^{t+2}, no IB force owed in between.
// 2-step halo of a slab (SWEEP_HALO_SLOTS slots of L.rows elements per side):
//   from the left  neighbour: 0-2 col -1 {1,5,8}, 3-5 col -1 {0,2,4}, 6-8 col -2 {1,5,8},
//                             9: [0] col -1 plane 7 at y = 0, [1] col -1 plane 6 at y = Y-1
//   from the right neighbour: 0-2 col ncol {3,6,7}, 3-5 col ncol {0,2,4}, 6-8 col ncol+1 {3,6,7},
//                             9: [0] col ncol plane 8 at y = 0, [1] col ncol plane 5 at y = Y-1
// (slot 9: the same-cell wall values of the halo column's own collide).  Slots 0-2 are the
// one-step halo, so a one-step launch can follow a two-step exchange.
constexpr int SWEEP_HALO_SLOTS = 10;
// slot of plane k of the d-th column beyond the slab edge (d = 0, 1) in the left / right 2-step
// halo (-1: not carried)
__host__ __device__ constexpr int sweep_slot(bool left, int d, int k) {
    return (left ? cx(k) == 1 : cx(k) == -1) ? (d == 0 ? halo_slot(k) : 6 + halo_slot(k))
                                             : (d == 0 && cx(k) == 0 ? 3 + (k == 0 ? 0 : (k == 2 ? 1 : 2)) : -1);
}
// plane carried in slot s (< 9) of the halo sent to the left (my columns 0, 1) / right neighbour
__host__ __device__ constexpr int sweep_send_plane(bool to_left, int s) {
    return (s >= 3 && s < 6) ? 2 * (s - 3) : (to_left ? right_plane(s % 3) : left_plane(s % 3));
}

template <typename T>
struct Sweep2Args {
    const T* src;        // g^t
    T* dst;              // g^{t+2} (the other buffer)
    Layout L;
    const T* recv_left;  // slab of a group: 2-step halos received from the neighbours
    const T* recv_right; // (lone slab: columns -2, -1, ncol, ncol+1 are the periodic images)
    T* send_left;        // slab of a group: 2-step halos for the neighbours, written by the waves
    T* send_right;       //   of columns 0, 1 / ncol-2, ncol-1
    int col_begin;       // sweep s covers output columns [col_begin + s*col_step, + W) ∩ [.., col_end)
    int col_step;
    int col_end;
    int nsweep;
    int W;               // output columns per sweep (wave)
    int vs;              // cells per lane; rows, col and plane multiples of vs
    int nch;             // set by launch_sweep2
    int variant;         // MODE bits (nontemporal loads / stores, no prefetch)
    int map;             // 1: linear, chunk fastest; 0: 4 sweeps per workgroup, XCD-contiguous;
                         // 2: linear order in XCD-contiguous ranges (default)
    int alt;             // odd sweeps walk right to left (neighbours read their shared edges together)
    int cus;             // deep sweeps, balanced widths: CUs the launch's stream may use (0 = all)
    int xcds;            // deep sweeps, map 2: XCDs the workgroups are dealt over (0 = 8)
    const int* sweep_tab;  // deep sweeps: sweep s covers [sweep_tab[2s], sweep_tab[2s+1]) (device;
                           // nullptr: col_begin / col_step / W); the force-free gaps between IB bands
    int tab_rows;          // sweep_tab entries of 4 ints: + chunk range [tab[4s+2], tab[4s+3]) of the
                           // sweep (the columns of an IB band outside its patch rows)
    int flux_col;        // local column sampled for Q (both iterations), or -1
    double flux_norm;
    double* Q;
    Coef c;
    KConst k;            // collide constants folded on the host (iblb_device.h)
};

// slab: true = the group kernel (halo columns from recv_*, send buffers written); false = lone
// slab (periodic images) or interior columns of a group slab (no halo, no sends)
template <typename T>
hipError_t launch_sweep2(Sweep2Args<T> a, bool slab, hipStream_t s);
// K = depth (3 .. 6) iterations per launch: g^t -> g^{t+K}; map 1 or 2.  slab = false: lone
// slab (periodic columns) or interior columns of a group slab; slab = true: columns beyond the
// edges from the deep halo (deep_slot) in recv_left / recv_right, and (send_left != nullptr) the
// output columns [0, K) / [ncol-K, ncol) also written into the deep halo of the send buffers
// (what launch_pack_deep_halo makes of them).  col_step 0: balanced widths.
template <typename T>
hipError_t launch_sweepk(Sweep2Args<T> a, int depth, bool slab, hipStream_t s);
// Resident waves per CU of a deep-sweep configuration; *nch = its row chunks for ny rows.
template <typename T>
int sweepk_geometry(int depth, int vs, int variant, bool slab, int ny, int* nch);
// The deep halo of depth K of state g into both send buffers.
template <typename T>
hipError_t launch_pack_deep_halo(const T* g, Layout L, int depth, T* send_left, T* send_right, hipStream_t st);
// The 2-step halo of state g into both send buffers (after a one-step launch or an IB exchange).
template <typename T>
hipError_t launch_pack_sweep_halo(const T* g, Layout L, T* send_left, T* send_right, hipStream_t st);

// Launch geometry of the collide-stream kernel: one wave per (column, 64*V-row chunk).
inline int chunks_per_column(int ny, int V) { return (ny + 64 * V - 1) / (64 * V); }

template <typename T>
hipError_t launch_fused(const FusedArgs<T>& a, hipStream_t s);

// Step 0 of a fresh state: collide f^0 with explicit rho^0, u^0, force^0 (no pull).
template <typename T>
hipError_t launch_boot(const T* src, T* dst, Layout L, const double* rho0, const double* u0,
                       const double* force0, long fplane, T* const send_left[3], T* const send_right[3],
                       Coef c, KConst k, hipStream_t s);

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
// Slab groups: the points spreading into this slab, nodes pulled through the IB halo.  part: 0
// all, 1 inner points only (no halo needed), 2 the points near the slab edges.
template <typename T>
hipError_t launch_ib_slab(const T* g, Layout L, IbHalo<T> X, int nx, int x_begin, int ns, const float* s,
                          const float* u_s, const int* eps, float* F_s, double* fdense, long fplane, uint8_t* flags,
                          int nch, int rows_per_chunk, hipStream_t st, int part = 0);
// IB halo slots 3.. of both send buffers from the state g.
template <typename T>
hipError_t launch_pack_ib_halo(const T* g, Layout L, T* send_left, T* send_right, hipStream_t st);

}  // namespace iblb

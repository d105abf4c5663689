// lbm_sweep_impl.h — the temporally blocked kernels (templates), shared by lbm_sweep.hip (two
// iterations per launch, dispatch, halo packing) and lbm_sweepk{3,4,5,6}.hip (the K-iteration
// kernels of one depth each: separate translation units build in parallel).
//
// Two reference iterations per launch (temporal blocking along x).
//
// The one-step collide-stream kernel (lbm_kernels.hip) already moves the algorithmic minimum of
// one iteration, 144 B/LU in f64, at ~96 % of the measured HBM copy rate.  Below that floor the
// only lever is to touch the state less often: this kernel reads g^t once and writes g^{t+2}
// once, keeping the intermediate post-collision state g^{t+1} in registers.
//
// One wave = one (sweep, chunk): a chunk of 64*VS rows (lane l owns rows y0 .. y0+VS-1) and a
// sweep of W output columns [xa, xb).  The wave walks x = xa-1 .. xb:
//   step 1  g1[x]   = collide(pull(g0)) for its rows, plus ONE extra cell per lane: lane 0 the row
//                     below the chunk (cs-1), lane 63 the row above (cs+64*VS).  Those are the
//                     only g1 values of other chunks that step 2 pulls (c_y = +-1 planes).
//   step 2  g2[x-1] = collide(pull(g1)) from the register window g1[x-2] (planes 1,5,8),
//                     g1[x-1] (0,2,4 and the wall cells), g1[x] (3,6,7); +-1-row pulls are DPP
//                     lane shifts whose end lanes take the extra cells.
// Per cell and iteration the arithmetic is the one of fused_kernel (same relax_cell, same
// storage rounding), so the result is bit-identical to two one-step launches.  Cost: the g1
// columns xa-1 and xb are recomputed by the neighbouring sweeps and each lane collides VS+1
// cells in step 1 (the extra cell is live in 2 lanes of 64).
//
// Algorithmic HBM bytes per launch: one read + one write of the state = 144 B per cell (f64) for
// TWO lattice updates, plus the (W+2)/W re-read of the sweep edges.
//
// Lone slab: columns -2, -1, ncol, ncol+1 are the periodic images.  Slab of a group (SLAB): they
// are the ghost columns of the buffer itself, filled by the halo exchange (whole columns, in place).
#pragma once

#include <hip/hip_ext.h>

#include <climits>

#include "lbm_vec.h"

namespace iblb {

// sweep only (MODE bits 1, 2 as in lbm_vec.h): no software prefetch of the next column (two-step
// sweeps); the deep sweep's wall split (sweepk_kernel)
#ifndef IBLB_WALK_UL
#define IBLB_WALK_UL 1  // the LDS-window walks load the next column unconditionally (0: round 6's A/B base)
#endif
enum { MODE_NO_PREFETCH = 8, MODE_SPLIT = 16, MODE_PACK = 64, MODE_SKIP = 128, MODE_PRESHIFT = 256, MODE_LDSWIN = 512,
       MODE_WT_STORE = 1024 };

namespace {

// pointer to plane k of column x (x in [-2, ncol+1]); x is wave-uniform.  SLAB: ghost columns
// in the buffer; else the periodic image.
template <typename T, bool SLAB>
__device__ __forceinline__ const T* sweep_col(const Sweep2Args<T>& a, int x, int k) {
    const Layout& L = a.L;
    if (SLAB || (x >= 0 && x < L.ncol)) return a.src + (long)x * L.col + (long)k * L.plane;
    const int xw = x < 0 ? x + L.ncol : x - L.ncol;
    return a.src + (long)xw * L.col + (long)k * L.plane;
}

// g0(x, y, k) for the wall cells (y = 0 or Y-1) of column x
template <typename T, bool SLAB>
__device__ __forceinline__ T wall_val(const Sweep2Args<T>& a, int x, int k, int y) {
    return sweep_col<T, SLAB>(a, x, k)[y];
}

// a sampled flux row: inside the lattice and outside the rows an IB band patch accounts for
template <typename T>
__device__ __forceinline__ bool flux_row(const Sweep2Args<T>& a, int y) {
    return y < a.L.ny && (y < a.fskip0 || y >= a.fskip1);
}

// rows y0 .. y0+VS-1 of plane pointer p shifted by one row: DIR = +1 -> rows y-1, DIR = -1 ->
// rows y+1, built from the aligned values v of this lane's rows; the end lane takes *edge (no
// edge: the end lane keeps whatever the shift left, it is a ghost row whose value is not used)
template <typename T, int VS, int DIR>
__device__ __forceinline__ void shift_rows(const T v[VS], const T* edge, int lane, T r[VS]) {
    if (DIR > 0) {
        T prev = lane_shift<+1>(v[VS - 1]);
        if (edge && lane == 0) prev = *edge;
        r[0] = prev;
#pragma unroll
        for (int e = 1; e < VS; ++e) r[e] = v[e - 1];
    } else {
        T next = lane_shift<-1>(v[0]);
        if (edge && lane == 63) next = *edge;
#pragma unroll
        for (int e = 0; e < VS - 1; ++e) r[e] = v[e + 1];
        r[VS - 1] = next;
    }
}

// Row-vector access at a wave-uniform base + this lane's 32-bit byte offset: the compiler keeps
// the base in SGPRs (global_load/store saddr form) and every access shares one offset VGPR.
// readfirstlane makes the base an opaque SGPR value, so the compiler cannot re-associate the
// lane offset into a per-lane 64-bit address (2 VGPRs per access).
template <typename P>
__device__ __forceinline__ P* sgpr_ptr(P* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (P*)(((uint64_t)hi << 32) | lo);
}
#define IBLB_GLOBAL __attribute__((address_space(1)))

template <typename T, int VS, int MODE>
__device__ __forceinline__ void ld_rows(const T* base, unsigned off, T v[VS]) {
    typedef typename VT<T, VS>::type vec;
    const IBLB_GLOBAL vec* p = (const IBLB_GLOBAL vec*)((const IBLB_GLOBAL char*)sgpr_ptr(base) + off);
    const vec x = (MODE & MODE_NT_LOAD) ? __builtin_nontemporal_load(p) : *p;
#pragma unroll
    for (int e = 0; e < VS; ++e) v[e] = x[e];
}

template <typename T, int VS, int MODE>
__device__ __forceinline__ void st_rows(T* base, unsigned off, const T v[VS]) {
    typedef typename VT<T, VS>::type vec;
    vec x;
#pragma unroll
    for (int e = 0; e < VS; ++e) x[e] = v[e];
    IBLB_GLOBAL vec* p = (IBLB_GLOBAL vec*)((IBLB_GLOBAL char*)sgpr_ptr(base) + off);
    if (MODE & MODE_NT_STORE) __builtin_nontemporal_store(x, p);
    else *p = x;
}

// Raw g0 rows of one column step: the 9 source planes at this lane's rows, plus the same-cell
// values the walls need from planes whose pull column is not x (7, 8 at y = 0; 5, 6 at y = Y-1)
template <typename T, int VS>
struct Raw {
    T v[9][VS];
    T e[9];  // wave-edge rows: row0-1 of the c_y = +1 planes, row0+64*VS of the c_y = -1 planes
    T w[6];  // g0(x, 0, 7), g0(x, 0, 8), g0(x, Y-1, 5), g0(x, Y-1, 6) (wall lanes only); MODE_PRESHIFT:
             // g0(x, 0, 4), g0(x, Y-1, 2)
};

// rows of the wave start at row0 = cs - VS (uniform); lane byte offset off
template <typename T, int VS, int MODE, bool SLAB>
__device__ __forceinline__ void load_raw(const Sweep2Args<T>& a, int x, int row0, unsigned off, bool bot, bool top,
                                         Raw<T, VS>& r) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const T* p = sweep_col<T, SLAB>(a, x - cx(k), k) + row0;
        ld_rows<T, VS, MODE>(p, off, r.v[k]);
        // the ghost lanes' own pulls reach one row beyond the wave (uniform address)
        if (cy(k) == 1) r.e[k] = p[-1];
        if (cy(k) == -1) r.e[k] = p[64 * VS];
    }
    r.w[0] = r.w[1] = r.w[2] = r.w[3] = (T)0;
    if (bot) {
        r.w[0] = wall_val<T, SLAB>(a, x, 7, 0);
        r.w[1] = wall_val<T, SLAB>(a, x, 8, 0);
    }
    if (top) {
        r.w[2] = wall_val<T, SLAB>(a, x, 5, a.L.ny - 1);
        r.w[3] = wall_val<T, SLAB>(a, x, 6, a.L.ny - 1);
    }
}

// pull of the 9 populations of this lane's rows from one column triple of a post-collision
// state held as aligned row vectors (pk[k]: plane k of column x - c_x(k)): planes with c_y = 0 as
// they are, c_y = +1 from the row below (DPP shift up), c_y = -1 from the row above, the end
// lanes taking edge[k] (the row beyond the wave; nullptr: garbage, see below); the walls
// from the same cell of the middle column (planes 2, 4 of this lane's rows, 7 and 8 of row 0,
// 5 and 6 of this lane's rows for the top row).  The end lanes' out-of-wave neighbours are garbage: those lanes are the
// sweep's ghost rows.
template <typename T, int VS>
__device__ __forceinline__ void pull_window(const T (*pk[9])[VS], const T* edge, const T (&m2)[VS], const T (&m4)[VS],
                                            T m7, T m8, const T (&m5)[VS], const T (&m6)[VS], int lane, int r0,
                                            int et, T s[9][VS], bool walls = true) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        if (cy(k) == 0) {
#pragma unroll
            for (int e = 0; e < VS; ++e) s[k][e] = (*pk[k])[e];
        } else if (cy(k) == 1) {
            shift_rows<T, VS, +1>(*pk[k], edge ? edge + k : nullptr, lane, s[k]);
        } else {
            shift_rows<T, VS, -1>(*pk[k], edge ? edge + k : nullptr, lane, s[k]);
        }
    }
    if (!walls) return;  // wave-uniform: the wave holds neither wall row
    if (r0 == 0) {  // bounce-back on y = 0 (LatticeBoltzmann.cu:328-340)
        s[2][0] = m4[0];
        s[5][0] = m7;
        s[6][0] = m8;
    }
    if (et >= 0 && et < VS) {  // same-cell mirror on y = Y-1 (LatticeBoltzmann.cu:341-353)
#pragma unroll
        for (int e = 0; e < VS; ++e)
            if (e == et) { s[4][e] = m2[e]; s[8][e] = m5[e]; s[7][e] = m6[e]; }
    }
}

}  // namespace

// The walk of one wave over the output columns [xa, xb): step 1 makes g1 of columns xa-1 .. xb
// in walking order, step 2 makes g2 of the middle column of the last three.  REV walks from xb
// down to xa-1 (the window mirrored: A = g1[x+2], C = g1[x]); alternate sweeps walking towards
// each other read their shared edge columns at the same time, so one fetch serves both.
// Returns this lane's flux partial.
template <typename T, int VS, int MODE, bool SLAB, bool REV>
__device__ __forceinline__ double sweep_walk(const Sweep2Args<T>& a, int xa, int xb, int row0, unsigned off,
                                             int lane, int r0, int et, bool owner, bool bot, bool top) {
    typedef typename Calc<T>::R R;
    constexpr bool DEV = Store<T>::dev;
    const Layout L = a.L;
    // first, last and next column of the walk
    const int x0 = REV ? xb : xa - 1, x1 = REV ? xa - 1 : xb, dx = REV ? -1 : 1;

    // g1 window: A = g1[x-2dx] (planes with c_x = dx used), B = g1[x-dx], C = g1[x]
    T A[9][VS], B[9][VS];
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int e = 0; e < VS; ++e) { A[k][e] = 0; B[k][e] = 0; }
    double q = 0.;

    // software prefetch of the next column (MODE_NO_PREFETCH: load at use, fewer VGPRs)
    constexpr bool PF = !(MODE & MODE_NO_PREFETCH);
    Raw<T, VS> nxt;
    if (PF) load_raw<T, VS, MODE, SLAB>(a, x0, row0, off, bot, top, nxt);
    for (int i = 0, x = x0; i <= xb - xa + 1; ++i, x += dx) {
        Raw<T, VS> cur;
        if (PF) {
            cur = nxt;
            load_raw<T, VS, MODE, SLAB>(a, x == x1 ? x : x + dx, row0, off, bot, top, nxt);
        } else {
            load_raw<T, VS, MODE, SLAB>(a, x, row0, off, bot, top, cur);
        }

        // ---- step 1: g1[x] ----
        T C[9][VS];
        {
            const T(*pk[9])[VS];
#pragma unroll
            for (int k = 0; k < 9; ++k) pk[k] = &cur.v[k];
            T s[9][VS];
            T t5[VS], t6[VS];
#pragma unroll
            for (int e = 0; e < VS; ++e) { t5[e] = cur.w[2]; t6[e] = cur.w[3]; }
            pull_window<T, VS>(pk, cur.e, cur.v[2], cur.v[4], cur.w[0], cur.w[1], t5, t6, lane, r0, et, s);
            const bool flux1 = x == a.flux_col && x >= xa && x < xb;
#pragma unroll
            for (int e = 0; e < VS; ++e) {
                R f[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) f[k] = (R)s[k][e];
                const R ux = relax_cell<R, DEV>(f, kbase<R>(a.k), kbody<R>(a.k));
                if (flux1 && owner && flux_row(a, r0 + e)) q += (double)ux / a.flux_norm;
#pragma unroll
                for (int k = 0; k < 9; ++k) C[k][e] = (T)f[k];
            }
        }

        // ---- step 2: g2[x-dx] from the window ----
        if (i >= 2) {
            const int xo = x - dx;
            const T(*pk[9])[VS];
            // plane k of g2[xo] pulls from g1[xo - c_x(k)]: c_x = dx -> A, c_x = -dx -> C
#pragma unroll
            for (int k = 0; k < 9; ++k) pk[k] = cx(k) == dx ? &A[k] : (cx(k) == -dx ? &C[k] : &B[k]);
            T s[9][VS];
            pull_window<T, VS>(pk, nullptr, B[2], B[4], B[7][0], B[8][0], B[5], B[6], lane, r0, et, s);
            const bool flux2 = xo == a.flux_col;
#pragma unroll
            for (int e = 0; e < VS; ++e) {
                R f[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) f[k] = (R)s[k][e];
                const R ux = relax_cell<R, DEV>(f, kbase<R>(a.k), kbody<R>(a.k));
                if (flux2 && owner && flux_row(a, r0 + e)) q += (double)ux / a.flux_norm;
#pragma unroll
                for (int k = 0; k < 9; ++k) s[k][e] = (T)f[k];
            }
            if (owner) {
                T* dst = a.dst + (long)xo * L.col + row0;
#pragma unroll
                for (int k = 0; k < 9; ++k) st_rows<T, VS, MODE>(dst + (long)k * L.plane, off, s[k]);
            }
        }

        // ---- rotate the window ----
#pragma unroll
        for (int k = 0; k < 9; ++k)
#pragma unroll
            for (int e = 0; e < VS; ++e) { A[k][e] = B[k][e]; B[k][e] = C[k][e]; }
    }
    return q;
}

// wave -> (sweep, chunk), chunk fastest, with that linear order dealt to the eight XCDs in
// contiguous ranges (blocks b and b+8 share an XCD: the dispatcher deals workgroups round-robin over
// all eight whatever the stream's CU mask, profiles/r02n_xcc_probe.txt), so the edge columns of
// neighbouring sweeps are re-read from the L2 that just fetched them.  Odd sweeps walk right to
// left: neighbours read their shared edge columns at about the same time.
__device__ __forceinline__ void linear_item(int nch, int wv, int& sw, int& ch) {
    int b = (int)blockIdx.x;
    const int q = (int)gridDim.x / 8;
    if (b < 8 * q) b = (b % 8) * q + b / 8;
    const int gw = b * 4 + wv;
    sw = gw / nch;
    ch = gw - sw * nch;
}

// One wave = (sweep, chunk).  Lane l holds rows r0 = cs - VS + l*VS .. r0+VS-1: lanes 1..62 own
// the chunk's 62*VS output rows [cs, cs + 62*VS), lanes 0 and 63 are ghost rows (the g1 values
// of the rows just outside the chunk that step 2 pulls).  Ghost rows and rows >= ny compute
// garbage that no owned row reads.
template <typename T, int VS, int MODE, bool SLAB>
__global__ __launch_bounds__(256) void sweep2_kernel(Sweep2Args<T> a) {
    typedef typename Calc<T>::R R;
    static_assert(sizeof(R) == sizeof(T), "the window keeps g1 in the storage type");
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int sw, ch;
    linear_item(a.nch, wv, sw, ch);
    if (sw >= a.nsweep || ch >= a.nch) return;
    const int xa = a.col_begin + sw * a.col_step;
    const int xb = min(xa + a.W, a.col_end);
    const int cs = ch * (62 * VS);
    const int row0 = cs - VS;  // first row of the wave (lane 0)
    const int r0 = row0 + lane * VS;
    const unsigned off = (unsigned)(lane * VS * (int)sizeof(T));
    const int et = a.L.ny - 1 - r0;  // element of the top row, if in [0, VS)
    const bool owner = lane >= 1 && lane <= 62 && r0 < a.L.ny;
    const bool bot = r0 == 0;
    const bool top = et >= 0 && et < VS;
    const double q = (sw & 1)
                         ? sweep_walk<T, VS, MODE, SLAB, true>(a, xa, xb, row0, off, lane, r0, et, owner, bot, top)
                         : sweep_walk<T, VS, MODE, SLAB, false>(a, xa, xb, row0, off, lane, r0, et, owner, bot, top);
    if (a.flux_col >= xa && a.flux_col < xb) {
        const double qs = wave_sum(q);
        if (lane == 0) atomicAdd(a.Q, qs);
    }
}

template <typename T, int VS, int MODE>
static hipError_t launch_sweep_mode(const Sweep2Args<T>& a, bool slab, unsigned blocks, hipStream_t s) {
    if (slab) sweep2_kernel<T, VS, MODE, true><<<blocks, 256, 0, s>>>(a);
    else sweep2_kernel<T, VS, MODE, false><<<blocks, 256, 0, s>>>(a);
    return hipGetLastError();
}

// (variant: nontemporal stores, software prefetch of the next column — the measured best of the
// round-1 variants, profiles/r01p_tune_*.log; the others are no longer built)
template <typename T, int VS>
static hipError_t launch_sweep_vs(const Sweep2Args<T>& a, bool slab, unsigned blocks, hipStream_t s) {
    return launch_sweep_mode<T, VS, MODE_NT_STORE>(a, slab, blocks, s);
}

template <typename T>
hipError_t launch_sweep2(Sweep2Args<T> a, bool slab, hipStream_t s) {
    if (a.nsweep <= 0) return hipSuccess;
    // rows are read up to VS+1 below 0 and up to nch*62*VS + VS (< rows + 62*VS + VS + 1): inside
    // the 512-element guards of the buffers (iblb_ctx.hip)
    if (a.W <= 0 || a.L.ncol < 2 || a.vs <= 0 || a.L.rows % a.vs != 0 || a.L.plane % a.vs != 0 || a.L.col % a.vs != 0)
        return hipErrorInvalidValue;
    a.nch = (a.L.ny + 62 * a.vs - 1) / (62 * a.vs);
    const unsigned blocks = (unsigned)(((long)a.nsweep * a.nch + 3) / 4);
    constexpr int V = vec_of<T>();
    if (a.vs == V) return launch_sweep_vs<T, V>(a, slab, blocks, s);
    if (a.vs == V / 2) return launch_sweep_vs<T, V / 2>(a, slab, blocks, s);
    return hipErrorInvalidValue;
}

// ---- K iterations per launch (lone slab, K = 3 .. 6) ------------------------------------------
// sweepk_kernel: g^t -> g^{t+K}, the walk keeping K-1 register windows (g^{t+1} .. g^{t+K-1}).
// Same wave geometry, order and walking directions as sweep2_kernel.  Valid rows shrink by one
// per level at the wave's edges (the +-1-row pulls of the end lanes take garbage from level 2
// on), so each edge carries G ghost lanes with G * VS >= K - 1 rows.  Each level's cell
// arithmetic is fused_kernel's (relax_cell): bit-identical to K one-step launches.
//
// Software-pipelined walk over the level-1 columns xa-(K-1) .. xb+(K-2) (dx = +1, or -1 from
// the right end): iteration i makes level 1 of column x from the rows loaded in the previous
// iteration, issues the loads of column x + dx, then makes level l = 2 .. K of column
// x - (l-1)*dx from level l-1's window.  The loads fly while K-1 levels of arithmetic run, and
// every level (level 1 included) keeps only its two previous columns between iterations.
// Wall rows (y = 0, Y-1) are patched only by the waves that hold them (a wave-uniform branch).
//
// Algorithmic HBM bytes per launch: one read + one write of the state (144 B per cell in f64)
// for K lattice updates, plus the edge re-reads of neighbouring sweeps (served by L2 under the
// XCD-contiguous alternating order).

// plane k of column x of a lone slab, x periodic (x may lie up to K columns outside)
template <typename T>
__device__ __forceinline__ const T* col_periodic(const Sweep2Args<T>& a, int x, int k) {
    const int n = a.L.ncol;
    int xw = x % n;
    if (xw < 0) xw += n;
    return a.src + (long)xw * a.L.col + (long)k * a.L.plane;
}

// plane k of column x for the deep walk: a lone slab wraps periodically; a slab of a group
// (SLAB) reads the ghost columns of its buffer (K of them per side after the halo exchange)
template <typename T, bool SLAB, int K>
__device__ __forceinline__ const T* col_deep(const Sweep2Args<T>& a, int x, int k) {
    if (!SLAB) return col_periodic<T>(a, x, k);
    return a.src + (long)x * a.L.col + (long)k * a.L.plane;
}

// ---- buffer-resource addressing of the lone-slab walk ----------------------------------------
// A column's nine planes are loaded through one buffer resource (V#, 4 SGPRs) whose base is the
// column (minus the buffer guard, so that every offset is non-negative): the plane offsets are
// loop-invariant SGPRs (soffset) and the lane's row offset a loop-invariant VGPR (voffset).  Per
// walk step that leaves one periodic wrap and one 64-bit multiply per column instead of the
// 64-bit plane-address arithmetic of every load (which, with one wave per SIMD, cost an issue
// slot each: ~150 scalar instructions per step).
constexpr int BUF_GUARD = 512;  // elements in front of every population buffer (iblb_ctx.hip GUARD)

template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t col_rsrc(const T* col) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(col - BUF_GUARD), (short)0, 0x7fffffff, 0x00020000);
}
// column x of a lone slab, x periodic (|x| within one period of the slab, as in the walk)
template <typename T>
__device__ __forceinline__ const T* col_wrap(const Sweep2Args<T>& a, int x) {
    const int n = a.L.ncol;
    int xw = x < 0 ? x + n : (x >= n ? x - n : x);
    if ((unsigned)xw >= (unsigned)n) {  // a slab narrower than the walk's reach
        xw = x % n;
        if (xw < 0) xw += n;
    }
    return a.src + (long)xw * a.L.col;
}
// column x of the walk: periodic (lone slab) or a ghost column of the buffer (SLAB)
template <typename T, bool SLAB>
__device__ __forceinline__ const T* col_at(const Sweep2Args<T>& a, int x) {
    return SLAB ? a.src + (long)x * a.L.col : col_wrap(a, x);
}
// The walk's column pointers kept from step to step (UL walks, round 6): the next column to load (pn,
// its periodic index xn in a lone slab) and the output column (pd) advance by one column stride
// instead of a periodic wrap and a 64-bit multiply per step (~30 scalar instructions, an issue slot
// each at one wave per SIMD)
template <typename T>
struct ColPtrs {
    const T* pn;
    int xn;
    T* pd;
};
template <typename T, bool SLAB, int DX>
__device__ __forceinline__ void col_step(const Sweep2Args<T>& a, const T*& p, int& xw) {
    p += DX * (long)a.L.col;
    if (!SLAB) {
        xw += DX;
        if (DX > 0 && xw == a.L.ncol) {
            xw = 0;
            p = a.src;
        }
        if (DX < 0 && xw < 0) {
            xw = a.L.ncol - 1;
            p = a.src + (long)(a.L.ncol - 1) * a.L.col;
        }
    }
}
template <typename T, int VS, int MODE>
__device__ __forceinline__ void ld_rows_buf(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, T v[VS]) {
    typedef typename VT<T, VS>::type vec;
    constexpr int aux = (MODE & MODE_NT_LOAD) ? 2 : 0;
    constexpr int B = VS * (int)sizeof(T);
    vec x;
    if constexpr (B == 16) x = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, aux));
    else if constexpr (B == 8) x = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, aux));
    else x = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, aux));
#pragma unroll
    for (int e = 0; e < VS; ++e) v[e] = x[e];
}
template <typename T>
__device__ __forceinline__ T ld_one_buf(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    if constexpr (sizeof(T) == 8) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
    else return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
template <typename T, int VS, int MODE>
__device__ __forceinline__ void st_rows_buf(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, const T v[VS]) {
    typedef typename VT<T, VS>::type vec;
    vec x;
#pragma unroll
    for (int e = 0; e < VS; ++e) x[e] = v[e];
    // MODE_WT_STORE (a slab interior's edge waves): sc1, write-through — the handed-off columns leave
    // the XCD's L2 with the store, so the wave's signal needs no L2-wide release (Guideline 16 R1)
    constexpr int aux = (MODE & MODE_WT_STORE) ? 16 : (MODE & MODE_NT_STORE) ? 2 : 0;
    constexpr int B = VS * (int)sizeof(T);
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    if constexpr (B == 16) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), r, voff, soff, aux);
    else if constexpr (B == 8) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, x), r, voff, soff, aux);
    else __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), r, voff, soff, aux);
}
// the loop-invariant offsets of one wave (bytes): the lane's rows, the two wave-edge rows
struct BufOfs {
    unsigned lane, lo, hi;  // voffset of the lane's rows, of row row0-1, of row row0+64*VS
    unsigned plane;         // bytes between planes
};

// rc: the buffer resources of columns x-1, x, x+1
template <typename T, int VS, int MODE, bool SLAB, int K>
__device__ __forceinline__ void load_raw_periodic(const Sweep2Args<T>& a, int x, int row0, unsigned off, bool bot,
                                                  bool top, Raw<T, VS>& r, const BufOfs& bo,
                                                  const __amdgpu_buffer_rsrc_t (&rc)[3]) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const __amdgpu_buffer_rsrc_t rk = rc[1 - cx(k)];
        const unsigned so = (unsigned)k * bo.plane;
        if (MODE & MODE_PRESHIFT) {
            // the lane's rows of the pull itself: rows r0 - c_y .. (one row off the lane's alignment; no
            // wave-edge value and no lane shift at level 1)
            ld_rows_buf<T, VS, MODE>(rk, bo.lane, so - cy(k) * (int)sizeof(T), r.v[k]);
        } else {
            ld_rows_buf<T, VS, MODE>(rk, bo.lane, so, r.v[k]);
            if (cy(k) == 1) r.e[k] = ld_one_buf<T>(rk, bo.lo, so);
            if (cy(k) == -1) r.e[k] = ld_one_buf<T>(rk, bo.hi, so);
        }
    }
    r.w[0] = r.w[1] = r.w[2] = r.w[3] = r.w[4] = r.w[5] = (T)0;
    if (bot) {
        r.w[0] = col_deep<T, SLAB, K>(a, x, 7)[0];
        r.w[1] = col_deep<T, SLAB, K>(a, x, 8)[0];
        if (MODE & MODE_PRESHIFT) r.w[4] = col_deep<T, SLAB, K>(a, x, 4)[0];
    }
    if (top) {
        r.w[2] = col_deep<T, SLAB, K>(a, x, 5)[a.L.ny - 1];
        r.w[3] = col_deep<T, SLAB, K>(a, x, 6)[a.L.ny - 1];
        if (MODE & MODE_PRESHIFT) r.w[5] = col_deep<T, SLAB, K>(a, x, 2)[a.L.ny - 1];
    }
}

// f32, two cells per lane: both cells' collides as one packed f32x2 computation (relax_dev)
template <typename T, int VS, int MODE>
constexpr bool packed_pair() { return sizeof(T) == 4 && VS == 2 && (MODE & MODE_PACK); }
template <typename T, int VS>
__device__ __forceinline__ void relax_pair(const T (&s)[9][VS], const Sweep2Args<T>& a, bool flux, int fown, double& q,
                                           T (&out)[9][VS]) {
    f32x2 f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = f32x2{(float)s[k][0], (float)s[k][1]};
    const f32x2 ux = relax_dev<f32x2>(f, kbase<float>(a.k), kbody<float>(a.k));
    if (flux) {  // wave-uniform branch; the lane condition as a select (no exec-mask branch)
        const double t0 = (double)ux.x / a.flux_norm, t1 = (double)ux.y / a.flux_norm;
        q += (fown & 1) ? t0 : 0.;
        q += (fown & 2) ? t1 : 0.;
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        out[k][0] = (T)f[k].x;
        out[k][1] = (T)f[k].y;
    }
}

// one column of level l+1 from a window of level l (A = older, B = middle, C = newer column in
// walking direction DX): the output is B's column; flux: add u_x of the owned rows to q
// ASH: A's populations that wait in the LDS window arrive already at their pull's rows
// (lds_pop_read); the others are pulled as usual (LDS window only: no wall rows in those waves)
template <typename T, int VS, int DX, int MODE = 0, bool ASH = false>
__device__ __forceinline__ void level_from_window(const T (&A)[9][VS], const T (&B)[9][VS], const T (&C)[9][VS],
                                                  const Sweep2Args<T>& a, int lane, int r0, int et, bool walls,
                                                  bool flux, int fown, double& q, T (&out)[9][VS]) {
    typedef typename Calc<T>::R R;
    constexpr bool DEV = Store<T>::dev;
    const T(*pk[9])[VS];
#pragma unroll
    for (int k = 0; k < 9; ++k) pk[k] = cx(k) == DX ? &A[k] : (cx(k) == -DX ? &C[k] : &B[k]);
    T s[9][VS];
    pull_window<T, VS>(pk, nullptr, B[2], B[4], B[7][0], B[8][0], B[5], B[6], lane, r0, et, s, walls);
    if constexpr (ASH) {
#pragma unroll
        for (int k = 0; k < 9; ++k)
            if (cx(k) == DX && cy(k) != 0)  // (the diagonal movers: in LDS in both precisions)
#pragma unroll
                for (int e = 0; e < VS; ++e) s[k][e] = A[k][e];
    }
    if constexpr (packed_pair<T, VS, MODE>()) {
        relax_pair<T, VS>(s, a, flux, fown, q, out);
        return;
    }
#pragma unroll
    for (int e = 0; e < VS; ++e) {
        R f[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) f[k] = (R)s[k][e];
        const R ux = relax_cell<R, DEV>(f, kbase<R>(a.k), kbody<R>(a.k));
        if (flux) {  // wave-uniform branch; the lane condition as a select (no exec-mask branch)
            const double t = (double)ux / a.flux_norm;
            q += ((fown >> e) & 1) ? t : 0.;
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) out[k][e] = (T)f[k];
    }
}

// level 1 of one column from its loaded g^t rows
template <typename T, int VS, int MODE = 0>
__device__ __forceinline__ void level_from_raw(const Raw<T, VS>& cur, const Sweep2Args<T>& a, int lane, int r0, int et,
                                               bool walls, bool flux, int fown, double& q, T (&out)[9][VS]) {
    typedef typename Calc<T>::R R;
    constexpr bool DEV = Store<T>::dev;
    const T(*pk[9])[VS];
#pragma unroll
    for (int k = 0; k < 9; ++k) pk[k] = &cur.v[k];
    T s[9][VS];
    T t5[VS], t6[VS];
#pragma unroll
    for (int e = 0; e < VS; ++e) { t5[e] = cur.w[2]; t6[e] = cur.w[3]; }
    if (MODE & MODE_PRESHIFT) {  // loaded at the pull's rows; the walls' same-cell values are uniform loads
        T m2[VS], m4[VS];
#pragma unroll
        for (int e = 0; e < VS; ++e) { m2[e] = cur.w[5]; m4[e] = cur.w[4]; }
#pragma unroll
        for (int k = 0; k < 9; ++k)
#pragma unroll
            for (int e = 0; e < VS; ++e) s[k][e] = cur.v[k][e];
        if (walls) {
            if (r0 == 0) {  // bounce-back on y = 0 (LatticeBoltzmann.cu:328-340)
                s[2][0] = m4[0];
                s[5][0] = cur.w[0];
                s[6][0] = cur.w[1];
            }
            if (et >= 0 && et < VS) {  // same-cell mirror on y = Y-1 (LatticeBoltzmann.cu:341-353)
#pragma unroll
                for (int e = 0; e < VS; ++e)
                    if (e == et) { s[4][e] = m2[e]; s[8][e] = t5[e]; s[7][e] = t6[e]; }
            }
        }
    } else {
        pull_window<T, VS>(pk, cur.e, cur.v[2], cur.v[4], cur.w[0], cur.w[1], t5, t6, lane, r0, et, s, walls);
    }
    if constexpr (packed_pair<T, VS, MODE>()) {
        relax_pair<T, VS>(s, a, flux, fown, q, out);
        return;
    }
#pragma unroll
    for (int e = 0; e < VS; ++e) {
        R f[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) f[k] = (R)s[k][e];
        const R ux = relax_cell<R, DEV>(f, kbase<R>(a.k), kbody<R>(a.k));
        if (flux) {  // wave-uniform branch; the lane condition as a select (no exec-mask branch)
            const double t = (double)ux / a.flux_norm;
            q += ((fown >> e) & 1) ? t : 0.;
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) out[k][e] = (T)f[k];
    }
}

template <typename T, int VS>
__device__ __forceinline__ void copy_col(T (&d)[9][VS], const T (&s)[9][VS]) {
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int e = 0; e < VS; ++e) d[k][e] = s[k][e];
}

// MODE_SKIP: the patch output regions (left to the band cycle's last level) a walk meets.  The walk's
// output columns are monotonic, so the wave keeps the region it is at or before: its index sp, its
// columns in scalar registers and whether this lane's rows r0 .. r0+VS-1 lie in its rows; it moves
// on (reading the next region from the kernel arguments) only when the walk passes the region.
struct SkipState {
    int sp, x0, x1;
    bool rows;
};
template <typename T, int VS, bool REV>
__device__ __forceinline__ void skip_load(const Sweep2Args<T>& a, int r0, SkipState& st) {
    if (st.sp >= 0 && st.sp < a.nskip) {
        const SkipBox b = a.skip[st.sp];
        st.x0 = b.x0;
        st.x1 = b.x1;
        st.rows = r0 >= b.y0 && r0 + VS <= b.y1;
    } else {  // no region left on this side: a column range no output column reaches
        st.x0 = INT_MAX;
        st.x1 = INT_MIN;
        st.rows = false;
    }
}
template <typename T, int VS, bool REV>
__device__ __forceinline__ bool skip_rows(const Sweep2Args<T>& a, int c, int r0, SkipState& st) {
    if (!REV) {
        while (st.sp < a.nskip && c > st.x1) {
            ++st.sp;
            skip_load<T, VS, REV>(a, r0, st);
        }
    } else {
        while (st.sp >= 0 && c < st.x0) {
            --st.sp;
            skip_load<T, VS, REV>(a, r0, st);
        }
    }
    return c >= st.x0 && c <= st.x1 && st.rows;
}

// Iteration i of the walk (column x = x0 + i*dx): level 1 of x from the rows loaded in the
// previous iteration, then the loads of column x + dx (they fly during the remaining levels),
// then level l = 2 .. K of column x - (l-1)*dx from level l-1's window: WA / WB = its columns
// made two and one iterations ago, and N = the one made in this iteration.  Level l starts at
// iteration 2(l-1), when its window holds three valid columns; its columns in [xa, xb) (stored at
// level K, counted in the flux) all come later.  (Running every level from iteration 0 instead,
// on not-yet-valid windows, lets the compiler hoist the collide constants out of the walk and
// needs more registers than the wave has: measured 40 % slower, profiles/r02c_*.)
// LDS window (MODE_LDSWIN, f64 inner chunks of the wall split, two cells per lane): the three
// populations of a level's column that move along the walk (c_x = DX) are needed two iterations after
// they are made; they wait in LDS (two slots by iteration parity, 16 B per lane and population, 144 KB
// per workgroup at K = 7) instead of VGPRs, so the register window keeps only the three c_x = 0
// populations of the middle column: 256 VGPRs + 4 AGPRs instead of 256 + 142 at K = 7, no AGPR moves
// in the walk (profiles/r04/ldswin).
template <typename T, int VS, int MODE, bool WL>
constexpr bool lds_window() { return (MODE & MODE_LDSWIN) && VS == 2 && !WL; }
// the moving populations kept in LDS: f64 all three; f32 (three waves per SIMD, round 5) the two
// diagonal ones, so that twelve waves' windows fit a CU's LDS (147 of 160 KB) — the third stays in
// registers (a two-column rotation, like the register window)
template <typename T>
constexpr bool lds_pop(int k) { return sizeof(T) == 8 || cy(k) != 0; }
template <typename T>
constexpr int lds_npop() { return sizeof(T) == 8 ? 3 : 2; }
template <typename T, int K, int VS>
constexpr int lds_window_wave() { return 2 * (K - 1) * lds_npop<T>() * 64 * VS; }  // elements per wave
// A moving population read back from its LDS slot (q: this lane's vector) at the rows its pull takes
// (round 6): c_y = +1 reads rows r0-1 .. r0+VS-2, c_y = -1 rows r0+1 .. r0+VS — the neighbour lane's
// element through the address instead of a DPP row shift after the read (the end lanes read their
// neighbour block's element or the padding: ghost rows).  c_y = 0: the lane's own vector.
template <typename T, int VS>
__device__ __forceinline__ typename VT<T, VS>::type lds_pop_read(const typename VT<T, VS>::type* q, int cyk) {
    typedef typename VT<T, VS>::type vec;
    if (cyk == 0) return *q;
    const T* e0 = (const T*)q - cyk;
    vec v;
#pragma unroll
    for (int e = 0; e < VS; ++e) v[e] = e0[e];
    return v;
}

// UL (the LDS-window walks, round 6): the next column's loads are unconditional, the last step loading
// columns it already read (x - DX .. x + DX: inside the walk's reach): the loaded column then needs no
// select against the old one at the loop's back edge (18 v_mov_b64 per f64 step)
template <typename T, int VS, int MODE, int K, bool SLAB, bool REV, bool LW, bool UL = false>
__device__ __forceinline__ void sweepk_iter(const Sweep2Args<T>& a, int i, int nl1, int x0, int xa, int xb, int row0,
                                            unsigned off, int lane, int r0, int et, bool owner, bool bot, bool top,
                                            bool walls, T (&WA)[K - 1][9][VS], T (&WB)[K - 1][9][VS],
                                            Raw<T, VS>& cur, double& q, const BufOfs& bo,
                                            __amdgpu_buffer_rsrc_t (&rc)[3], bool fin, int fi, int fown, SkipState& sp,
                                            T* lw, ColPtrs<T>& cp) {
    constexpr int DX = REV ? -1 : 1;
    const int x = x0 + i * DX;
    if constexpr (UL) cp.pd += DX * (long)a.L.col;  // output column x - (K-1) DX
    T N[9][VS];
    typedef typename VT<T, VS>::type vec;
    // LDS window, f64: level l+1's moving populations are read from LDS before level l is computed (and
    // level 2's before level 1), so that the read's latency hides behind a level's arithmetic instead of
    // stalling the one wave of the SIMD at the start of every level (+12 VGPRs).  The slot read is
    // written only after its own level's compute, so reading it one level early is the same value.
    constexpr bool PREF = LW && sizeof(T) == 8;
    vec pre[lds_npop<T>()];
    auto lds_slot = [&](int l) { return (vec*)(lw + ((i & 1) * (K - 1) + (l - 2)) * lds_npop<T>() * 64 * VS); };
    // (the moving populations in LDS, in slot order, and their c_y)
    auto lds_cy = [](int p) {
        int q = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k)
            if (cx(k) == DX && lds_pop<T>(k)) {
                if (q == p) return cy(k);
                ++q;
            }
        return 0;
    };
    if constexpr (PREF) {
#pragma unroll
        for (int p = 0; p < lds_npop<T>(); ++p) pre[p] = lds_pop_read<T, VS>(lds_slot(2) + p * 64, lds_cy(p));
    }
    // fin: the flux column is one of the sweep's outputs; level l reaches it at step fi + l - 1
    level_from_raw<T, VS, MODE>(cur, a, lane, r0, et, walls, fin && i == fi, fown, q, N);
    if (UL || i + 1 < nl1) {
        // the resources of the next column triple: one new column
        const int xl = UL && i + 1 >= nl1 ? x - DX : x;
        __amdgpu_buffer_rsrc_t rn;
        if constexpr (UL) {  // column xl + 2 DX: the last step keeps the previous one (x + DX)
            if (i + 1 < nl1) col_step<T, SLAB, DX>(a, cp.pn, cp.xn);
            rn = col_rsrc(cp.pn);
        } else {
            rn = col_rsrc(col_at<T, SLAB>(a, xl + 2 * DX));
        }
        if (DX > 0) {
            rc[0] = rc[1];
            rc[1] = rc[2];
            rc[2] = rn;
        } else {
            rc[2] = rc[1];
            rc[1] = rc[0];
            rc[0] = rn;
        }
        load_raw_periodic<T, VS, MODE, SLAB, K>(a, xl + DX, row0, off, bot, top, cur, bo, rc);
    }
#pragma unroll
    for (int l = 2; l <= K; ++l) {
        const int c = x - (l - 1) * DX;
        const bool flux = fin && i == fi + l - 1;
        T out[9][VS];
        const bool made = i >= 2 * (l - 1);
        vec* ls = nullptr;
        if constexpr (LW) {  // slot of parity i: the column made two iterations ago, then this one's
            ls = lds_slot(l);
            int p = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k)
                if (cx(k) == DX && lds_pop<T>(k)) {
                    const vec v = PREF ? pre[p] : lds_pop_read<T, VS>(ls + p * 64, cy(k));
#pragma unroll
                    for (int e = 0; e < VS; ++e) WA[l - 2][k][e] = v[e];
                    ++p;
                }
            if constexpr (PREF)
                if (l < K) {
#pragma unroll
                    for (int p2 = 0; p2 < lds_npop<T>(); ++p2) pre[p2] = lds_pop_read<T, VS>(lds_slot(l + 1) + p2 * 64, lds_cy(p2));
                }
        }
        if (made) level_from_window<T, VS, DX, MODE, LW>(WA[l - 2], WB[l - 2], N, a, lane, r0, et, walls, flux, fown, q, out);
        // level K's columns of the made steps are exactly the sweep's outputs [xa, xb)
        bool keep = owner;
        if constexpr ((MODE & MODE_SKIP) != 0)
            if (made && l == K) keep = owner && !skip_rows<T, VS, REV>(a, c, r0, sp);
        if (made && l == K && keep) {
            const __amdgpu_buffer_rsrc_t rd = col_rsrc<T>(UL ? cp.pd : a.dst + (long)c * a.L.col);
#pragma unroll
            for (int k = 0; k < 9; ++k) st_rows_buf<T, VS, MODE>(rd, bo.lane, (unsigned)k * bo.plane, out[k]);
        }
        if constexpr (LW) {
            int p = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k)
                if (cx(k) == DX) {
                    if (lds_pop<T>(k)) {
                        vec v;
#pragma unroll
                        for (int e = 0; e < VS; ++e) v[e] = N[k][e];
                        ls[p * 64] = v;
                        ++p;
                    } else {  // (f32) the register rotation of this population
#pragma unroll
                        for (int e = 0; e < VS; ++e) {
                            WA[l - 2][k][e] = WB[l - 2][k][e];
                            WB[l - 2][k][e] = N[k][e];
                        }
                    }
                }
#pragma unroll
            for (int k = 0; k < 9; ++k)
                if (cx(k) == 0)
#pragma unroll
                    for (int e = 0; e < VS; ++e) WB[l - 2][k][e] = N[k][e];
        } else {
            copy_col<T, VS>(WA[l - 2], WB[l - 2]);
            copy_col<T, VS>(WB[l - 2], N);
        }
        // N becomes level l's column for level l+1, made or not: out is left unset when level l is not
        // made, and level l+1 is then not made either (made(l+1) implies made(l) two iterations back and
        // now), so whatever N holds there is never used.  Unconditional, the copy is a renaming (the
        // compiler folds the unset branch away); under `made` it cost 18 v_mov_b64 per level, 108 of
        // the f64 inner walk step's 144 (round 6).  f64 with the LDS window or one cell
        // per lane (the wall walks); without the window at two cells per lane (the f64 band cycle's deep
        // sweep) the renamed windows take 160 instead of 142 AGPRs, which
        // leaves the band chain's kernels no registers beside the deep sweep's waves (K3 cycle 0.219 ->
        // 0.277 ms); f32: the renamed windows need more registers than three waves per SIMD leave.
        if (l < K && ((sizeof(T) == 8 && (LW || VS == 1)) || made)) copy_col<T, VS>(N, out);
    }
}

// The walk over the level-1 columns.  (Unrolling it by two or three so that the window columns
// are renamed instead of copied measured 10-20 % slower: more live registers, profiles/r02d_*.)
// WL: the wave holds a wall row (compile-time, so that the waves of the other chunks carry no
// wall code and keep no wall planes of the windows live)
// NOFLUX: the sweep holds no flux column (the waves of all sweeps but one): the walk is built without
// the per-level flux test and its branch (round 6: the test's spilled SGPRs cost a v_readlane and a
// compare per level and cell of every wave)
template <typename T, int VS, int MODE, int K, bool SLAB, bool REV, bool WL, bool NOFLUX = false>
__device__ __forceinline__ double sweepk_walk(const Sweep2Args<T>& a, int xa, int xb, int row0, unsigned off,
                                              int lane, int r0, int et, bool owner, bool bot_, bool top_, T* lw) {
    const bool walls = WL, bot = WL && bot_, top = WL && top_;
    const int x0 = REV ? xb + K - 2 : xa - (K - 1);
    const int nl1 = xb - xa + 2 * (K - 1);  // level-1 columns xa-(K-1) .. xb+(K-2)
    T WA[K - 1][9][VS], WB[K - 1][9][VS];
#pragma unroll
    for (int l = 0; l < K - 1; ++l)
#pragma unroll
        for (int k = 0; k < 9; ++k)
#pragma unroll
            for (int e = 0; e < VS; ++e) WA[l][k][e] = WB[l][k][e] = (T)0;
    double q = 0.;
    BufOfs bo;
    bo.lane = (unsigned)((row0 + BUF_GUARD) * (int)sizeof(T)) + off;
    bo.lo = (unsigned)((row0 - 1 + BUF_GUARD) * (int)sizeof(T));
    bo.hi = (unsigned)((row0 + 64 * VS + BUF_GUARD) * (int)sizeof(T));
    bo.plane = (unsigned)(a.L.plane * (long)sizeof(T));
    Raw<T, VS> cur;
    __amdgpu_buffer_rsrc_t rc[3];
    rc[0] = col_rsrc(col_at<T, SLAB>(a, x0 - 1));
    rc[1] = col_rsrc(col_at<T, SLAB>(a, x0));
    rc[2] = col_rsrc(col_at<T, SLAB>(a, x0 + 1));
    constexpr int DX = REV ? -1 : 1;
    ColPtrs<T> cp;
    cp.pn = col_at<T, SLAB>(a, x0 + DX);
    {
        const int n = a.L.ncol;
        int xw = (x0 + DX) % n;
        cp.xn = xw < 0 ? xw + n : xw;
    }
    cp.pd = a.dst + (long)(x0 - K * DX) * a.L.col;  // (advanced before its first use: column x0 - (K-1) DX)
    load_raw_periodic<T, VS, MODE, SLAB, K>(a, x0, row0, off, bot, top, cur, bo, rc);
    const bool fin = !NOFLUX && a.flux_col >= 0 && a.flux_col >= xa && a.flux_col < xb;
    const int fi = REV ? xb + K - 2 - a.flux_col : a.flux_col - xa + K - 1;  // step of level 1 at the flux column
    // bit e: row r0 + e is owned and its flux sampled; one VGPR computed once (testing the IB
    // band's skipped flux rows inside the walk's flux branch changed the compiled loop: +2 % per
    // launch, profiles/r03ab)
    int fown = 0;
#pragma unroll
    for (int e = 0; e < VS; ++e) fown |= (owner && flux_row(a, r0 + e)) ? 1 << e : 0;
    // (a main loop without the per-level `made` checks, after 2(K-1) window-filling iterations,
    // lets the compiler hoist the collide constants into registers: VGPR spills, 512 VGPRs)
    SkipState sp{0, INT_MAX, INT_MIN, false};  // MODE_SKIP: the first region not left of the sweep (REV: right)
    if constexpr ((MODE & MODE_SKIP) != 0) {
        if (!REV)
            while (sp.sp < a.nskip && a.skip[sp.sp].x1 < xa) ++sp.sp;
        else
            for (sp.sp = a.nskip - 1; sp.sp >= 0 && a.skip[sp.sp].x0 >= xb; --sp.sp) {
            }
        skip_load<T, VS, REV>(a, r0, sp);
    }
    // (round 6 also tried two steps per trip with WA and WB swapping roles, the window's rotation a
    // renaming: the compiler kept the windows in AGPRs, 1399 instructions per f64 step against 1392)
    constexpr bool LW = lds_window<T, VS, MODE, WL>();
    for (int i = 0; i < nl1; ++i)
        sweepk_iter<T, VS, MODE, K, SLAB, REV, LW, LW && IBLB_WALK_UL>(a, i, nl1, x0, xa, xb, row0, off, lane, r0, et, owner,
                                                                    bot, top, walls, WA, WB, cur, q, bo, rc, fin, fi, fown,
                                                                    sp, lw, cp);
    return q;
}

template <int K, int VS>
constexpr int ghost_lanes() { return (K - 1 + VS - 1) / VS; }

// Wall split (MODE_SPLIT; balanced sweeps, or fixed ones such as a slab's boundary sweeps, round 4).
// The rows split into a bottom wall chunk [0, OWN1),
// the inner rows [OWN1, a.wall_top) in chunks of OWN*VS and a top wall chunk [a.wall_top, ny), where
// OWN1 = 64 - 2(K-1) rows is one wave of one cell per lane.  The inner chunks are walked by the
// kernel's VS-cell walk without wall code (a.nsweep sweeps each); the two wall chunks by a one-cell
// walk with the wall rules (a.nsweep_w sweeps each), listed after them.  The kernel is built for
// WPE waves per SIMD (f32: 3 instead of 2): the one-cell wall walk needs fewer registers than the
// inner walk, so neither spills (the VS-cell wall walk spilled 15 dwords and ran ~1.4x slower per
// column, profiles/r03sp).
__device__ __forceinline__ void split_item(const int nin, const int nsw_in, int wv, int& sw, int& ch, bool& wall) {
    int b = (int)blockIdx.x;
    const int q = (int)gridDim.x / 8;
    if (b < 8 * q) b = (b % 8) * q + b / 8;
    const int gw = b * 4 + wv;
    const int ni = nsw_in * nin;
    wall = gw >= ni;
    if (!wall) {
        sw = gw / nin;
        ch = gw - sw * nin;
    } else {
        const int g2 = gw - ni;
        sw = g2 >> 1;
        ch = g2 & 1;  // 0: bottom, 1: top
    }
}

// A slab interior's edge wave waits for the comm stream's boundary sweeps of the previous cycle
// (Sweep2Args::wait_seq) instead of the whole launch waiting behind a cross-queue barrier packet
// (~9 us per cycle, profiles/r04/bsplit).  The protocol of MI355X_MICROARCH.md (inter-workgroup
// visibility): the producer's stores are released by its kernel's end-of-kernel fence, then a
// signal kernel stores the sequence number (agent scope); here one relaxed agent-scope poll per
// ~0.2 us (s_sleep), then an agent-scope acquire (this CU's L1) drained by vmcnt(0) before the
// wave's first load.  Each waiting wave acquires for itself, so no workgroup barrier is needed.
// The producer sits behind the cycle's RCCL exchange, i.e. behind the neighbour ranks' hosts: a rank
// that reaches its next iblb_step late (a file write, a checkpoint, the caller's own work) keeps these
// waves spinning for as long, as it keeps RCCL's own kernels spinning.  So the bound is wall-clock
// time, not a poll count: `ticks` of the constant device clock (the context's wait timeout, 600 s by
// default), only so that a signal that never comes (a failed comm stream or peer) cannot
// leave the grid spinning for ever; past it the wave flags *err and goes on, and the call fails.
__device__ __forceinline__ void edge_wait(const unsigned* seq, unsigned val, unsigned* err, unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        const unsigned s = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if ((int)(s - val) >= 0) break;
        if (wall_clock64() - t0 > ticks) {
            if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The edge wave's stores released, then counted (MI355X_MICROARCH.md, Valid forms: every storing
// wave's vmcnt(0), the agent-scope release, the asm wait the compiler may otherwise drop after it,
// then the agent-scope atomic add; each edge wave signals for itself).
// wt: every store of the wave was write-through (sc1): drained by vmcnt(0), no release needed (R1).
// (The L2-wide release of plain stores, one per edge wave, cost the 512-column interior 7 us per launch,
// profiles/r05/hs.)
__device__ __forceinline__ void edge_done(unsigned* cnt, bool wt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!wt) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Balanced sweep s of nsw over [cb, ce): floor/ceil((ce - cb) / nsw) columns; trim > 0 makes the first
// and last sweeps `trim` columns narrower (a slab interior's edge waves, which also wait and signal)
__host__ __device__ inline void balanced_range(int cb, int ce, int trim, int s, int nsw, int& xa, int& xb) {
    const long n = (long)(ce - cb) + 2L * trim;
    xa = cb - trim + (int)(s * n / nsw);
    xb = cb - trim + (int)((s + 1) * n / nsw);
    xa = xa < cb ? cb : xa;
    xb = xb > ce ? ce : xb;
    xb = xb < xa ? xa : xb;  // (the launcher keeps trim below every sweep's share: never empty there)
}

// G ghost lanes at each wave edge (G * VS >= K - 1 rows)
template <typename T, int VS, int MODE, int K, bool SLAB, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void sweepk_kernel(Sweep2Args<T> a) {
    constexpr int G = ghost_lanes<K, VS>();
    constexpr int OWN = 64 - 2 * G;  // owned lanes per wave
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    T* lw = nullptr;
    if constexpr (lds_window<T, VS, MODE, false>()) {
        // (16 B of padding at each end: the shifted reads of lds_pop_read reach one element beyond a
        // block at the wave's end lanes, whose rows are ghost rows)
        constexpr int PAD = 16 / (int)sizeof(T);
        __shared__ __attribute__((aligned(16))) T lwin[4 * lds_window_wave<T, K, VS>() + 2 * PAD];
        lw = lwin + PAD + wv * lds_window_wave<T, K, VS>() + lane * VS;
    }
    int sw, ch, nsw = a.nsweep;
    bool wall = false;
    if (MODE & MODE_SPLIT) {
        split_item(a.wall_ch0, a.nsweep, wv, sw, ch, wall);
        if (wall) nsw = a.nsweep_w;
        if (sw >= nsw) return;
    } else {
        linear_item(a.nch, wv, sw, ch);
        if (sw >= nsw || ch >= a.nch) return;
    }
    int xa, xb;
    if (a.col_step > 0) {
        xa = a.col_begin + sw * a.col_step;
        xb = min(xa + a.W, a.col_end);
    } else {  // balanced: nsw sweeps of floor/ceil((col_end - col_begin) / nsw) columns
        balanced_range(a.col_begin, a.col_end, a.edge_trim, sw, nsw, xa, xb);
    }
    const bool edge = SLAB && (xa < a.wait_lo || xb > a.wait_hi);
    // an edge wave that signals its stores: write-through in the wall-split walks (the slab builds)
    const bool wt = (MODE & MODE_SPLIT) && edge && a.done_cnt;
    if constexpr (SLAB)
        if (a.wait_seq && edge) edge_wait(a.wait_seq, a.wait_val, a.wait_err, a.wait_ticks);
    const bool rev = sw & 1;
    double q;
    if ((MODE & MODE_SPLIT) && wall) {  // a wall chunk: one cell per lane, the wall walk
        constexpr int G1 = ghost_lanes<K, 1>(), OWN1 = 64 - 2 * G1;
        const int cs = ch == 0 ? 0 : a.wall_top;
        const int row0 = cs - G1;
        const int r0 = row0 + lane;
        const unsigned off = (unsigned)(lane * (int)sizeof(T));
        const int et = a.L.ny - 1 - r0;
        const bool owner = lane >= G1 && lane < 64 - G1 && r0 < a.L.ny && (ch == 1 || r0 < OWN1);
        if constexpr (SLAB) {
            if (wt) {
                constexpr int MW = MODE | MODE_WT_STORE;
                q = rev ? sweepk_walk<T, 1, MW, K, SLAB, true, true>(a, xa, xb, row0, off, lane, r0, et, owner, r0 == 0, et == 0, lw)
                        : sweepk_walk<T, 1, MW, K, SLAB, false, true>(a, xa, xb, row0, off, lane, r0, et, owner, r0 == 0, et == 0, lw);
                goto walked;
            }
        }
        // f64: the wall waves are nearly as long as the inner ones, so the flux-free walk here too (f32: the
        // flux-free one-cell walks measured slower on the K5-width slab, profiles/r06/rings2)
        if (sizeof(T) == 4 || (a.flux_col >= 0 && a.flux_col >= xa && a.flux_col < xb))
            q = rev ? sweepk_walk<T, 1, MODE, K, SLAB, true, true>(a, xa, xb, row0, off, lane, r0, et, owner, r0 == 0, et == 0, lw)
                    : sweepk_walk<T, 1, MODE, K, SLAB, false, true>(a, xa, xb, row0, off, lane, r0, et, owner, r0 == 0, et == 0, lw);
        else
            q = rev ? sweepk_walk<T, 1, MODE, K, SLAB, true, true, true>(a, xa, xb, row0, off, lane, r0, et, owner, r0 == 0,
                                                                       et == 0, lw)
                    : sweepk_walk<T, 1, MODE, K, SLAB, false, true, true>(a, xa, xb, row0, off, lane, r0, et, owner, r0 == 0,
                                                                        et == 0, lw);
    } else if (MODE & MODE_SPLIT) {  // an inner chunk: no wall row within reach of its own rows
        constexpr int OWN1 = 64 - 2 * ghost_lanes<K, 1>();
        const int cs = OWN1 + ch * (OWN * VS);
        const int row0 = cs - G * VS;
        const int r0 = row0 + lane * VS;
        const unsigned off = (unsigned)(lane * VS * (int)sizeof(T));
        const int et = a.L.ny - 1 - r0;
        const bool owner = lane >= G && lane < 64 - G && r0 < a.wall_top;
        if constexpr (SLAB) {
            if (wt) {
                constexpr int MW = MODE | MODE_WT_STORE;
                q = rev ? sweepk_walk<T, VS, MW, K, SLAB, true, false>(a, xa, xb, row0, off, lane, r0, et, owner, false, false, lw)
                        : sweepk_walk<T, VS, MW, K, SLAB, false, false>(a, xa, xb, row0, off, lane, r0, et, owner, false, false, lw);
                goto walked;
            }
        }
        if (sizeof(T) == 4 || (a.flux_col >= 0 && a.flux_col >= xa && a.flux_col < xb))  // (f32: spills 20 B)
            q = rev ? sweepk_walk<T, VS, MODE, K, SLAB, true, false>(a, xa, xb, row0, off, lane, r0, et, owner, false, false, lw)
                    : sweepk_walk<T, VS, MODE, K, SLAB, false, false>(a, xa, xb, row0, off, lane, r0, et, owner, false, false, lw);
        else
            q = rev ? sweepk_walk<T, VS, MODE, K, SLAB, true, false, true>(a, xa, xb, row0, off, lane, r0, et, owner, false, false, lw)
                    : sweepk_walk<T, VS, MODE, K, SLAB, false, false, true>(a, xa, xb, row0, off, lane, r0, et, owner, false, false, lw);
    } else {
        const int cs = ch * (OWN * VS);
        const int row0 = cs - G * VS;
        const int r0 = row0 + lane * VS;
        const unsigned off = (unsigned)(lane * VS * (int)sizeof(T));
        const int et = a.L.ny - 1 - r0;
        const bool owner = lane >= G && lane < 64 - G && r0 < a.L.ny;
        const bool bot = r0 == 0;
        const bool top = et >= 0 && et < VS;
        // wave-uniform: does the wave hold a wall row (y = 0 or Y-1, ghost lanes included)?
        const bool walls = row0 <= 0 || row0 + 64 * VS >= a.L.ny;
        q = walls ? (rev ? sweepk_walk<T, VS, MODE, K, SLAB, true, true>(a, xa, xb, row0, off, lane, r0, et, owner, bot, top, lw)
                         : sweepk_walk<T, VS, MODE, K, SLAB, false, true>(a, xa, xb, row0, off, lane, r0, et, owner, bot, top, lw))
                  : (rev ? sweepk_walk<T, VS, MODE, K, SLAB, true, false>(a, xa, xb, row0, off, lane, r0, et, owner, bot, top, lw)
                         : sweepk_walk<T, VS, MODE, K, SLAB, false, false>(a, xa, xb, row0, off, lane, r0, et, owner, bot, top, lw));
    }
walked:
    if (a.flux_col >= 0 && a.flux_col >= xa && a.flux_col < xb) {
        const double qs = wave_sum(q);
        if (lane == 0) atomicAdd(a.Q, qs);
    }
    if constexpr (SLAB)
        if (a.done_cnt && edge) edge_done(a.done_cnt, wt);
}

// Waves of one instantiation resident per CU (256-thread workgroups), and on `cus` CUs (0: all).
template <typename T, int VS, int MODE, int K, bool SLAB, int WPE>
static long waves_per_cu() {
    static long cached = 0;
    if (cached) return cached;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sweepk_kernel<T, VS, MODE, K, SLAB, WPE>, 256, 0) !=
            hipSuccess ||
        nb <= 0)
        return 0;
    cached = (long)nb * 4;
    return cached;
}
template <typename T, int VS, int MODE, int K, bool SLAB, int WPE>
static long resident_waves(int cus) {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        return 0;
    return waves_per_cu<T, VS, MODE, K, SLAB, WPE>() * (cus > 0 ? std::min(cus, ncu) : ncu);
}

// wall split: sweeps of a wall chunk per sweep of an inner chunk, in quarters.  With one-cell wall
// walks (no spills) the launch time is the inner waves' whatever the ratio: M f32 0.319-0.322 ms per
// launch for 0.5 ... 1.5 (profiles/r03s1); the first split (two-cell wall walks with spills) needed 2
// (0.305-0.320 ms, profiles/r03sp, r03r2).
constexpr int WALL_SWEEPS_X4 = 4;

template <typename T, int VS, int MODE, int K, bool SLAB, int WPE>
static hipError_t launch_sweepk_mode(Sweep2Args<T> b, hipStream_t s, hipEvent_t stop, hipEvent_t start) {
    long waves;
    if (b.col_step <= 0) {
        // balanced sweeps: the wave count a whole number of device-wide rounds (the waves of one
        // launch all do the same work, so a partial last round idles the chip), sweeps close to
        // the requested W columns
        const long n = b.col_end - b.col_begin;
        const long slots = resident_waves<T, VS, MODE, K, SLAB, WPE>(b.cus);
        long ns = (n + b.W - 1) / b.W;
        if (MODE & MODE_SPLIT) {
            // wall split: nin inner chunks with ns sweeps, the two wall chunks with ns * r sweeps each
            const long nin = b.wall_ch0, r4 = VS == 1 ? 6 : WALL_SWEEPS_X4;  // VS 1: wall walks ~1.4x the inner
            if (slots > 0) {
                const long rounds = std::max(1L, (ns * (4 * nin + 2 * r4) / 4 + slots / 2) / slots);
                ns = std::max(1L, 4 * rounds * slots / (4 * nin + 2 * r4));
            }
            b.nsweep = (int)std::min(ns, n);
            b.nsweep_w = (int)std::min((ns * r4 + 3) / 4, n);
            waves = (long)b.nsweep * nin + 2L * b.nsweep_w;
        } else {
            if (slots > 0) {
                const long rounds = std::max(1L, (ns * b.nch + slots / 2) / slots);
                ns = std::max(1L, rounds * slots / b.nch);
            }
            b.nsweep = (int)std::min(ns, n);
            waves = (long)b.nsweep * b.nch;
        }
    } else if (MODE & MODE_SPLIT) {  // fixed sweeps (a slab's boundary sweeps): the wall chunks too
        b.nsweep_w = b.nsweep;
        waves = (long)b.nsweep * b.wall_ch0 + 2L * b.nsweep_w;
    } else {
        waves = (long)b.nsweep * b.nch;
    }
    if (b.col_step <= 0 && b.edge_trim > 0) {
        // the first and last sweeps keep at least one column: trim < every sweep's share
        const long n = b.col_end - b.col_begin;
        const long nsw = std::max((long)b.nsweep, (MODE & MODE_SPLIT) ? (long)b.nsweep_w : 0L);
        b.edge_trim = (int)std::min((long)b.edge_trim, std::max(0L, n / std::max(1L, nsw) - 1));
    }
    if (b.edge_waves) {  // the waves that will add to done_cnt (sweepk_kernel's `edge`)
        auto edges = [&](int nsw) {
            int e = 0;
            for (int sw = 0; sw < nsw; ++sw) {
                int xa, xb;
                if (b.col_step > 0) {
                    xa = b.col_begin + sw * b.col_step;
                    xb = std::min(xa + b.W, b.col_end);
                } else {
                    balanced_range(b.col_begin, b.col_end, b.edge_trim, sw, nsw, xa, xb);
                }
                e += (xa < b.wait_lo || xb > b.wait_hi) ? 1 : 0;
            }
            return e;
        };
        *b.edge_waves = (MODE & MODE_SPLIT) ? edges(b.nsweep) * b.wall_ch0 + 2 * edges(b.nsweep_w)
                                            : edges(b.nsweep) * b.nch;
    }
    if (b.kinfo) {  // which build ran (iblb_timing: the bench line's limiter names it)
        static int vgprs = -1;
        if (vgprs < 0) {
            hipFuncAttributes fa{};
            vgprs = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&sweepk_kernel<T, VS, MODE, K, SLAB, WPE>)) ==
                            hipSuccess
                        ? fa.numRegs
                        : 0;
        }
        b.kinfo[0] = MODE;
        b.kinfo[1] = VS;
        b.kinfo[2] = (int)(waves_per_cu<T, VS, MODE, K, SLAB, WPE>() / 4);
        b.kinfo[3] = vgprs;
    }
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    if (stop || start)  // the events ride on the kernel's own signals: no marker packets around it
        hipExtLaunchKernelGGL(sweepk_kernel<T, VS, MODE, K, SLAB, WPE>, dim3(blocks), dim3(256), 0, s, start, stop, 0, b);
    else
        sweepk_kernel<T, VS, MODE, K, SLAB, WPE><<<blocks, 256, 0, s>>>(b);
    return hipGetLastError();
}

// the wall split (variant bit 1): two cells per lane in the inner chunks; f32 at three waves per
// SIMD, f64 at one
template <typename T, int VS>
constexpr bool wall_split_built() { return VS == 2 || VS == 1; }

template <typename T, int VS, int K, bool SLAB>
static hipError_t launch_sweepk_vs(const Sweep2Args<T>& a, hipStream_t s, hipEvent_t stop, hipEvent_t start) {
    constexpr int G = ghost_lanes<K, VS>();
    const int rows_per_wave = (64 - 2 * G) * VS;  // owned rows
    Sweep2Args<T> b = a;
    b.nch = (a.L.ny + rows_per_wave - 1) / rows_per_wave;
    if constexpr (wall_split_built<T, VS>()) {
        // rows: [0, OWN1) bottom wall chunk, inner chunks of rows_per_wave, top wall chunk from an even
        // row (two-cell lanes of the inner chunks never straddle it) holding the last OWN1 or fewer rows
        constexpr int OWN1 = 64 - 2 * ghost_lanes<K, 1>();
        const int top = (a.L.ny - OWN1 + 1) & ~1;
        // f32, one cell per lane (a group slab's band cycle): the split with the skip regions too
        constexpr bool SPLIT_SKIP = sizeof(T) == 4 && VS == 1 && !SLAB;
        if ((a.variant & 2) && (VS == 2 || (a.variant & 64)) && (a.nskip == 0 || SPLIT_SKIP) && top > OWN1) {
            b.wall_top = top;
            b.wall_ch0 = (top - OWN1 + rows_per_wave - 1) / rows_per_wave;
            if constexpr (SPLIT_SKIP) {
                constexpr int WPE = 3;  // (four waves: 6 dwords of scratch spills)
                if (a.nskip > 0) {
                    if (a.variant & 32)
                        return launch_sweepk_mode<T, VS, 1 | MODE_SPLIT | MODE_PRESHIFT | MODE_SKIP, K, SLAB, WPE>(b, s, stop,
                                                                                                         start);
                    return launch_sweepk_mode<T, VS, 1 | MODE_SPLIT | MODE_SKIP, K, SLAB, WPE>(b, s, stop, start);
                }
            }
            // bit 3: the inner chunks packed, two waves per SIMD (the packed inner walk needs 191 VGPRs;
            // forced to three waves it spills 21 dwords: 0.417 vs 0.323 ms per M f32 launch, profiles/r04/pack)
            constexpr int WPE = sizeof(T) == 4 ? (VS == 2 ? 3 : 4) : (VS == 2 ? 1 : 2);
            if constexpr (sizeof(T) == 4 && VS == 2)
                if (a.variant & 8) {
                    // bit 7 (round 5): two of the three moving populations in LDS, three waves per SIMD
                    if constexpr (!SLAB)
                        if (a.variant & 128)
                            return launch_sweepk_mode<T, VS, 1 | MODE_SPLIT | MODE_PACK | MODE_LDSWIN, K, SLAB, 3>(b, s, stop,
                                                                                                         start);
                    return launch_sweepk_mode<T, VS, 1 | MODE_SPLIT | MODE_PACK, K, SLAB, 2>(b, s, stop, start);
                }
            // bit 7 (f64, two cells per lane, with bit 5): the LDS window of the inner chunks
            if constexpr (sizeof(T) == 8 && VS == 2)
                if ((a.variant & 160) == 160)
                    return launch_sweepk_mode<T, VS, 1 | MODE_SPLIT | MODE_PRESHIFT | MODE_LDSWIN, K, SLAB, WPE>(b, s, stop,
                                                                                                           start);
            if (a.variant & 32)
                return launch_sweepk_mode<T, VS, 1 | MODE_SPLIT | MODE_PRESHIFT, K, SLAB, WPE>(b, s, stop, start);
            if (a.variant & 1) return launch_sweepk_mode<T, VS, 1 | MODE_SPLIT, K, SLAB, WPE>(b, s, stop, start);
            return launch_sweepk_mode<T, VS, MODE_SPLIT, K, SLAB, WPE>(b, s, stop, start);
        }
    }
    // the IB band cycle's deep and boundary sweeps beside its last level: patch output rows left out
    if (a.nskip > 0) return launch_sweepk_mode<T, VS, 1 | MODE_SKIP, K, SLAB, 1>(b, s, stop, start);
    // variants: bit 0 = nontemporal stores (default), 0 = plain; bit 3 (f32, two cells per lane): the
    // packed collide (both cells in one f32x2 computation, relax_dev)
    if constexpr (sizeof(T) == 4 && VS == 2)
        if (a.variant & 8) return launch_sweepk_mode<T, VS, 1 | MODE_PACK, K, SLAB, 1>(b, s, stop, start);
    // bit 5 without bit 1: level 1 loads each plane at its pull's rows (no wave-edge loads, no lane
    // shift) in every chunk.  Slower than the plain walk (M f64 0.559 vs 0.521 ms per launch,
    // profiles/r04/split64): the wall waves, which set the launch time here, wait on the wall rows'
    // uniform loads.  With bit 1 (the split) the inner chunks take it and the wall waves have slack.
    if ((a.variant & 34) == 32) return launch_sweepk_mode<T, VS, 1 | MODE_PRESHIFT, K, SLAB, 1>(b, s, stop, start);
    if (a.variant & 1) return launch_sweepk_mode<T, VS, 1, K, SLAB, 1>(b, s, stop, start);
    return launch_sweepk_mode<T, VS, 0, K, SLAB, 1>(b, s, stop, start);
}

// cells per lane: 2 or 1 (4 in f32 measured slower: one wave per SIMD, profiles/r01d4_*)
template <typename T, int K, bool SLAB>
hipError_t launch_sweepk_depth(const Sweep2Args<T>& a, hipStream_t s, hipEvent_t stop, hipEvent_t start) {
    if (a.vs == 2) return launch_sweepk_vs<T, 2, K, SLAB>(a, s, stop, start);
    if (a.vs == 1) return launch_sweepk_vs<T, 1, K, SLAB>(a, s, stop, start);
    return hipErrorInvalidValue;
}


// resident waves per CU and waves per launch column-chunk geometry of one configuration (the
// context sizes the CUs it reserves for the boundary sweeps with it)
template <typename T, int K, bool SLAB>
int deep_geometry(int vs, int variant, int ny, int* nch) {
    if (vs == 2) {
        *nch = (ny + (64 - 2 * ghost_lanes<K, 2>()) * 2 - 1) / ((64 - 2 * ghost_lanes<K, 2>()) * 2);
        return (int)((variant & 1) ? waves_per_cu<T, 2, 1, K, SLAB, 1>() : waves_per_cu<T, 2, 0, K, SLAB, 1>());
    }
    *nch = (ny + (64 - 2 * ghost_lanes<K, 1>()) - 1) / (64 - 2 * ghost_lanes<K, 1>());
    return (int)((variant & 1) ? waves_per_cu<T, 1, 1, K, SLAB, 1>() : waves_per_cu<T, 1, 0, K, SLAB, 1>());
}

}  // namespace iblb

// lbm_kernels.hip — fused pull-stream + TRT/Guo collide for gfx950, and the slab
// support kernels (boot step, macro/population/flux readers, layout conversion).
//
// Hot kernel: fused_kernel.  Per lattice update it reads the 9 populations once and
// writes them once: 144 B/LU in double, 72 B/LU in float (algorithmic minimum).
// Reference data flow it replaces: equilibrium -> collision -> streaming -> macro ->
// spread's u correction (LatticeBoltzmann.cu:30-411, ImmersedBoundary.cu:249-264),
// ~824 B/LU there.
#include <hip/hip_ext.h>

#include "lbm_vec.h"
#include "ib_device.h"

namespace iblb {

// merged band chain: clear the force buffer the previous launch consumed at (column xc, chunk ch)
// (the lane's rows y0 .. y0+V-1; clear_flag false: half-height waves, two of them per flag, leave it set)
template <int V>
__device__ __forceinline__ void band_clear(double* fd, uint8_t* fl, long fplane, int rows, int nch, int xc, int ch,
                                           int y0, int lane, bool clear_flag = true) {
    const long fi = (long)xc * nch + ch;
    if (fl[fi]) {
        double* p = fd + (long)xc * rows + y0;
#pragma unroll
        for (int e = 0; e < V; ++e) { p[e] = 0.; p[fplane + e] = 0.; }
        if (lane == 0 && clear_flag) fl[fi] = 0;
    }
}

// One wave = one (column, chunk of 64*V rows); lane l owns rows y0 .. y0+V-1.
// Column-uniform decisions (halo source, flux column, IB flag) are scalar branches.  Walls are
// per-lane fixes of the first / last row.  Columns outside [0, ncol) (IB band trapezoids over a
// slab's ghost columns) are addressed directly.
template <typename T, int V, bool IB, int MODE>
__device__ __forceinline__ void fused_wave(const FusedArgs<T>& a, const int gw, const int lane) {
    typedef typename VT<T, V>::type vec;
    typedef typename Calc<T>::R R;
    constexpr bool DEV = Store<T>::dev;
    int xc, ch, ya = 0, yb = a.L.rows;  // rows sampled for Q (and stored, store_rows)
    if (a.row_tab) {  // an IB patch entry: chunks [e[1], e[2]) of column e[0]
        if (gw >= a.ncols * a.nchl) return;
        const int* e = a.cols + a.col_begin + 5 * (gw / a.nchl);
        ch = __builtin_amdgcn_readfirstlane(e[1]) + gw % a.nchl;
        if (ch >= __builtin_amdgcn_readfirstlane(e[2])) return;
        xc = __builtin_amdgcn_readfirstlane(e[0]);
        ya = __builtin_amdgcn_readfirstlane(e[3]);
        yb = __builtin_amdgcn_readfirstlane(e[4]);
    } else {
        if (gw >= a.ncols * a.nch) return;
        xc = a.cols ? __builtin_amdgcn_readfirstlane(a.cols[a.col_begin + gw / a.nch])
                    : a.col_begin + (gw / a.nch) * a.col_step;
        ch = gw - (gw / a.nch) * a.nch;
    }
    const Layout L = a.L;
    const int cs = ch * (64 * V);
    const int y0 = cs + lane * V;
    const long cb = (long)xc * L.col;
    const T* __restrict__ src = a.src;

    const T* p0 = src + cb;
    const T* p2 = src + 2 * L.plane + cb;
    const T* p4 = src + 4 * L.plane + cb;
    const T *p1, *p5, *p8, *p3, *p6, *p7;
    if (xc == 0) {
        p1 = a.H.left[0]; p5 = a.H.left[1]; p8 = a.H.left[2];
    } else {
        p1 = src + 1 * L.plane + cb - L.col; p5 = src + 5 * L.plane + cb - L.col; p8 = src + 8 * L.plane + cb - L.col;
    }
    if (xc == L.ncol - 1) {
        p3 = a.H.right[0]; p6 = a.H.right[1]; p7 = a.H.right[2];
    } else {
        p3 = src + 3 * L.plane + cb + L.col; p6 = src + 6 * L.plane + cb + L.col; p7 = src + 7 * L.plane + cb + L.col;
    }

    // pull: c_y = 0 planes aligned, c_y = +1 planes from row y-1, c_y = -1 planes from row y+1
    vec v0 = ld_plane<T, V, MODE>(p0 + y0);
    vec v1 = ld_plane<T, V, MODE>(p1 + y0);
    vec v3 = ld_plane<T, V, MODE>(p3 + y0);
    vec v2 = ld_shifted<T, V, MODE, +1>(p2, y0, cs, lane);
    vec v5 = ld_shifted<T, V, MODE, +1>(p5, y0, cs, lane);
    vec v6 = ld_shifted<T, V, MODE, +1>(p6, y0, cs, lane);
    vec v4 = ld_shifted<T, V, MODE, -1>(p4, y0, cs, lane);
    vec v7 = ld_shifted<T, V, MODE, -1>(p7, y0, cs, lane);
    vec v8 = ld_shifted<T, V, MODE, -1>(p8, y0, cs, lane);
    if (y0 == 0) {  // bounce-back on y = 0 (LatticeBoltzmann.cu:328-340)
        v2[0] = src[(4 * L.plane + cb)];
        v5[0] = src[(7 * L.plane + cb)];
        v6[0] = src[(8 * L.plane + cb)];
    }
    const int et = L.ny - 1 - y0;
    if (et >= 0 && et < V) {  // same-cell mirror on y = Y-1 (LatticeBoltzmann.cu:341-353)
        const long top = cb + L.ny - 1;
        const T t2 = src[(2 * L.plane + top)], t5 = src[(5 * L.plane + top)],
                t6 = src[(6 * L.plane + top)];
#pragma unroll
        for (int e = 0; e < V; ++e)
            if (e == et) { v4[e] = t2; v8[e] = t5; v7[e] = t6; }
    }

    // dense IB force for this (column, chunk), consumed and cleared (vhalf: the flag of the 64*2V-row
    // chunk this half-height wave lies in, left set: the other half-height wave may not have read it)
    const long fi = (long)xc * a.nch + (a.vhalf ? ch >> 1 : ch);
    bool has_f = false;
    if (IB) has_f = a.flags[fi] != 0;
    double fxv[V], fyv[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { fxv[e] = 0.; fyv[e] = 0.; }
    if (IB && has_f) {
        double* fx = a.fdense + (long)xc * L.rows + y0;
        double* fy = a.fdense + a.fplane + (long)xc * L.rows + y0;
#pragma unroll
        for (int e = 0; e < V; ++e) { fxv[e] = fx[e]; fyv[e] = fy[e]; }
        if (!a.fkeep) {
#pragma unroll
            for (int e = 0; e < V; ++e) { fx[e] = 0.; fy[e] = 0.; }
            if (lane == 0 && !a.vhalf) a.flags[fi] = 0;  // only this wave reads this flag
        }
    }
    if (IB && a.flclr) band_clear<V>(a.fdclr, a.flclr, a.fplane, L.rows, a.nch, xc, a.vhalf ? ch >> 1 : ch, y0, lane, !a.vhalf);

    const bool do_flux = a.flux_col >= 0 && xc == a.flux_col;  // (-1: none; ghost column -1 is a real column)
    double q = 0.;
#pragma unroll
    for (int e = 0; e < V; ++e) {
        R f[9] = {(R)v0[e], (R)v1[e], (R)v2[e], (R)v3[e], (R)v4[e], (R)v5[e], (R)v6[e], (R)v7[e], (R)v8[e]};
        const KBase<R>& kb = kbase<R>(a.k);
        // body force only: the host-folded constants; with an IB force: the same fold per cell
        const R ux = (IB && has_f) ? relax_cell<R, DEV>(f, kb, make_kforce<R>(kb, (R)(a.c.gx + fxv[e]), (R)(a.c.gy + fyv[e])))
                                   : relax_cell<R, DEV>(f, kb, kbody<R>(a.k));
        if (do_flux && y0 + e < L.ny && y0 + e >= ya && y0 + e < yb) q += (double)ux / a.flux_norm;
        v0[e] = (T)f[0]; v1[e] = (T)f[1]; v2[e] = (T)f[2]; v3[e] = (T)f[3]; v4[e] = (T)f[4];
        v5[e] = (T)f[5]; v6[e] = (T)f[6]; v7[e] = (T)f[7]; v8[e] = (T)f[8];
    }
    T* dst = a.dst + cb + y0;
    if (!a.store_rows || (y0 >= ya && y0 + V <= yb)) {
        st_plane<T, V, MODE>(dst, v0);
        st_plane<T, V, MODE>(dst + 1 * L.plane, v1);
        st_plane<T, V, MODE>(dst + 2 * L.plane, v2);
        st_plane<T, V, MODE>(dst + 3 * L.plane, v3);
        st_plane<T, V, MODE>(dst + 4 * L.plane, v4);
        st_plane<T, V, MODE>(dst + 5 * L.plane, v5);
        st_plane<T, V, MODE>(dst + 6 * L.plane, v6);
        st_plane<T, V, MODE>(dst + 7 * L.plane, v7);
        st_plane<T, V, MODE>(dst + 8 * L.plane, v8);
    } else if (y0 + V > ya && y0 < yb) {  // a lane across the patch's first or last row
#pragma unroll
        for (int e = 0; e < V; ++e)
            if (y0 + e >= ya && y0 + e < yb) {
                dst[e] = v0[e]; dst[e + 1 * L.plane] = v1[e]; dst[e + 2 * L.plane] = v2[e];
                dst[e + 3 * L.plane] = v3[e]; dst[e + 4 * L.plane] = v4[e]; dst[e + 5 * L.plane] = v5[e];
                dst[e + 6 * L.plane] = v6[e]; dst[e + 7 * L.plane] = v7[e]; dst[e + 8 * L.plane] = v8[e];
            }
    }
    if (do_flux) {
        q = wave_sum(q);
        if (lane == 0) atomicAdd(a.Q, q);
    }
}

template <typename T, int V, bool IB, int MODE>
__global__ __launch_bounds__(256) void fused_kernel(FusedArgs<T> a) {
    fused_wave<T, V, IB, MODE>(a, __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)),
                               threadIdx.x & 63);
}

// A level of the merged band chain (FusedArgs: fkeep, fdclr, clr_waves, nns): the 32-lane point
// groups of the next level's IB (ib_next_group) first — the launch's longest waves, dispatched before
// the others — then the waves of the table entries (fused_wave), then clr_waves clear-only waves.  The
// roles are wave-uniform; the point groups synchronise only within their wave (LDS region per group).
// (VW: cells per lane of the entry waves, V/2 with FusedArgs::vhalf; the IB flags stay per 64*V rows)
template <typename T, int V, int MODE, int VW = V>
__global__ __launch_bounds__(256) void band_level_kernel(FusedArgs<T> a) {
    __shared__ T reg[256 / NEXT_LANES][NEXT_CELLS][9];
    const int lane = threadIdx.x & 63;
    const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int ngroups = a.nns > 0 ? a.nns + max(0, a.whi - a.wlo) : 0;
    const int pw = (ngroups * NEXT_LANES + 63) / 64;
    if (gw < pw) {
        if (a.probe == 1) return;
        const long t = (long)gw * 64 + lane;
        const int gi = (int)(t / NEXT_LANES), n = (int)(t % NEXT_LANES);
        // group gi < nns: point gi (image 0 only when it lies in [wlo, whi)); then one group per point
        // of [wlo, whi) for its images -1 and +1 (FusedArgs::wlo)
        const bool main = gi < a.nns;
        const int k = main ? gi : a.wlo + (gi - a.nns);
        const int imgs = main ? (k >= a.wlo && k < a.whi ? 1 : 3) : 2;  // bit 0: m = 0, bit 1: m = +-1
        ib_next_group<T>(a, main || k < a.whi, k, n, 64 * V, reg[threadIdx.x / NEXT_LANES], imgs);
        return;
    }
    const int w = gw - pw, ew = a.ncols * a.nchl;
    if (w < ew) {
        if (a.probe != 2) fused_wave<T, VW, true, MODE>(a, w, lane);
        return;
    }
    if (w < ew + a.clr_waves) {
        const int c = w - ew, per = a.clr_w * a.nch;
        const int r = c < per ? c : c - per;
        const int xc = (c < per ? a.clr_lo : a.clr_hi) + r / a.nch, ch = r % a.nch;
        band_clear<V>(a.fdclr, a.flclr, a.fplane, a.L.rows, a.nch, xc, ch, ch * 64 * V + lane * V, lane);
    }
}

template <typename T, int MODE>
hipError_t launch_band_level_mode(const FusedArgs<T>& a, unsigned blocks, hipStream_t s, hipEvent_t stop) {
    constexpr int V = vec_of<T>();
    if constexpr (sizeof(T) == 4)
        if (a.vhalf) {
            if (stop)
                hipExtLaunchKernelGGL(band_level_kernel<T, V, MODE, V / 2>, dim3(blocks), dim3(256), 0, s, nullptr, stop, 0,
                                      a);
            else
                band_level_kernel<T, V, MODE, V / 2><<<blocks, 256, 0, s>>>(a);
            return hipGetLastError();
        }
    if (stop)
        hipExtLaunchKernelGGL(band_level_kernel<T, V, MODE>, dim3(blocks), dim3(256), 0, s, nullptr, stop, 0, a);
    else
        band_level_kernel<T, V, MODE><<<blocks, 256, 0, s>>>(a);
    return hipGetLastError();
}

template <typename T, int MODE>
hipError_t launch_fused_mode(const FusedArgs<T>& a, unsigned blocks, hipStream_t s, hipEvent_t stop) {
    constexpr int V = vec_of<T>();
    if (a.row_tab && (a.nns > 0 || a.clr_waves > 0)) return launch_band_level_mode<T, MODE>(a, blocks, s, stop);
    if constexpr (sizeof(T) == 4)
        if (a.vhalf) {  // band levels in half-height waves (f32: two cells per lane, 128-row chunks)
            if (!a.row_tab) return hipErrorInvalidValue;
            if (stop)
                hipExtLaunchKernelGGL(fused_kernel<T, V / 2, true, MODE>, dim3(blocks), dim3(256), 0, s, nullptr, stop, 0, a);
            else
                fused_kernel<T, V / 2, true, MODE><<<blocks, 256, 0, s>>>(a);
            return hipGetLastError();
        }
    if (stop) {  // the event rides on the kernel's own completion signal: no marker packet after it
        if (a.flags)
            hipExtLaunchKernelGGL(fused_kernel<T, V, true, MODE>, dim3(blocks), dim3(256), 0, s, nullptr, stop, 0, a);
        else
            hipExtLaunchKernelGGL(fused_kernel<T, V, false, MODE>, dim3(blocks), dim3(256), 0, s, nullptr, stop, 0, a);
    } else if (a.flags) {
        fused_kernel<T, V, true, MODE><<<blocks, 256, 0, s>>>(a);
    } else {
        fused_kernel<T, V, false, MODE><<<blocks, 256, 0, s>>>(a);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_fused(const FusedArgs<T>& a, hipStream_t s, hipEvent_t stop) {
    long waves = (long)a.ncols * (a.row_tab ? a.nchl : a.nch);
    if (a.row_tab && a.nns > 0) waves += ((long)(a.nns + std::max(0, a.whi - a.wlo)) * NEXT_LANES + 63) / 64;
    if (a.row_tab) waves += a.clr_waves;
    if (waves <= 0) return hipSuccess;
    if (a.row_tab && (a.nns > 0 || a.clr_waves > 0) && !a.flags) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    switch (a.variant) {
        case 1: return launch_fused_mode<T, 1>(a, blocks, s, stop);
        case 2: return launch_fused_mode<T, 2>(a, blocks, s, stop);
        case 3: return launch_fused_mode<T, 3>(a, blocks, s, stop);
        case 4: return launch_fused_mode<T, 4>(a, blocks, s, stop);
        case 5: return launch_fused_mode<T, 5>(a, blocks, s, stop);
        case 6: return launch_fused_mode<T, 6>(a, blocks, s, stop);
        case 7: return launch_fused_mode<T, 7>(a, blocks, s, stop);
        default: return launch_fused_mode<T, 0>(a, blocks, s, stop);
    }
}

// ---- boot step: collide f^0 with given rho^0, u^0, force^0 (main.cu:720-754, it = 0) --
template <typename T>
__global__ __launch_bounds__(256) void boot_kernel(const T* __restrict__ src, T* __restrict__ dst, Layout L,
                                                   const double* __restrict__ rho0, const double* __restrict__ u0,
                                                   const double* __restrict__ force0, long fplane, Coef c,
                                                   KConst kc) {
    typedef typename Calc<T>::R R;
    constexpr bool DEV = Store<T>::dev;
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)L.ncol * L.ny) return;
    const int xc = (int)(idx / L.ny), y = (int)(idx - (long)xc * L.ny);
    const long o = (long)xc * L.col + y, of = (long)xc * L.rows + y;
    R f[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) f[i] = (R)src[i * L.plane + o];
    const double rho = rho0[of];
    const R ux = (R)u0[of], uy = (R)u0[fplane + of];
    const R Fx = (R)(c.gx + (force0 ? force0[of] : 0.)), Fy = (R)(c.gy + (force0 ? force0[fplane + of] : 0.));
    const KBase<R>& kb = kbase<R>(kc);
    collide<R, DEV>(f, (R)rho, (R)(rho - 1.0), ux, uy, kb, make_kforce<R>(kb, Fx, Fy));
#pragma unroll
    for (int i = 0; i < 9; ++i) dst[i * L.plane + o] = (T)f[i];
}

template <typename T>
hipError_t launch_boot(const T* src, T* dst, Layout L, const double* rho0, const double* u0, const double* force0,
                       long fplane, Coef c, KConst k, hipStream_t s) {
    const long n = (long)L.ncol * L.ny;
    boot_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(src, dst, L, rho0, u0, force0, fplane, c, k);
    return hipGetLastError();
}

// ---- readers ------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void pull_cell(const T* g, const Layout& L, const Halo<T>& H, int xc, int y, double f[9]) {
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = Store<T>::to_f(pull<T>(g, L, H, xc, y, k), k);
}

// rho = sum f in the reference order (LatticeBoltzmann.cu:396-399); u corrected as in
// ImmersedBoundary.cu:249-255.  Contraction off: matches the C restatement bit for bit
// given the same populations.
template <typename T>
__global__ void macro_out_kernel(const T* __restrict__ g, Layout L, Halo<T> H, const double* __restrict__ fdense,
                                 long fplane, double gx, double gy, double* __restrict__ rho_out,
                                 double* __restrict__ u_out) {
#pragma clang fp contract(off)
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long N = (long)L.ncol * L.ny;
    if (idx >= N) return;
    const int y = (int)(idx / L.ncol), xc = (int)(idx - (long)y * L.ncol);  // reference order j = y*ncol + xc
    double f[9];
    pull_cell<T>(g, L, H, xc, y, f);
    double r, mx, my;
    moments<double>(f, r, mx, my);
    const long o = (long)xc * L.rows + y;
    const double Fx = (fdense ? fdense[o] : 0.) + gx;
    const double Fy = (fdense ? fdense[fplane + o] : 0.) + gy;
    if (rho_out) rho_out[idx] = r;
    if (u_out) {
        u_out[idx] = (mx + 0.5 * Fx) / r;
        u_out[N + idx] = (my + 0.5 * Fy) / r;
    }
}

template <typename T>
hipError_t launch_macro_out(const T* g, Layout L, Halo<T> H, const double* fdense, long fplane, double gx, double gy,
                            double* rho, double* u, hipStream_t s) {
    const long n = (long)L.ncol * L.ny;
    macro_out_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(g, L, H, fdense, fplane, gx, gy, rho, u);
    return hipGetLastError();
}

// raw != 0: g holds unstreamed f^0 (boot phase), read each cell in place.
template <typename T>
__global__ void pop_out_kernel(const T* __restrict__ g, Layout L, Halo<T> H, double* __restrict__ f_out, int raw) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)L.ncol * L.ny) return;
    const int y = (int)(idx / L.ncol), xc = (int)(idx - (long)y * L.ncol);
    double f[9];
    if (raw) {
#pragma unroll
        for (int k = 0; k < 9; ++k) f[k] = Store<T>::to_f(g[k * L.plane + (long)xc * L.col + y], k);
    } else {
        pull_cell<T>(g, L, H, xc, y, f);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) f_out[9 * idx + k] = f[k];
}

template <typename T>
hipError_t launch_pop_out(const T* g, Layout L, Halo<T> H, double* f, int raw, hipStream_t s) {
    const long n = (long)L.ncol * L.ny;
    pop_out_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(g, L, H, f, raw);
    return hipGetLastError();
}

template <typename T>
__global__ void flux_kernel(const T* __restrict__ g, Layout L, Halo<T> H, const double* __restrict__ fdense,
                            long fplane, double gx, double gy, int xc, double flux_norm, double* out) {
#pragma clang fp contract(off)
    double q = 0.;
    for (int y = threadIdx.x; y < L.ny; y += blockDim.x) {
        double f[9];
        pull_cell<T>(g, L, H, xc, y, f);
        double r, mx, my;
        moments<double>(f, r, mx, my);
        const long o = (long)xc * L.rows + y;
        const double Fx = (fdense ? fdense[o] : 0.) + gx;
        q += ((mx + 0.5 * Fx) / r) / flux_norm;
    }
    q = wave_sum(q);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, q);
}

template <typename T>
hipError_t launch_flux(const T* g, Layout L, Halo<T> H, const double* fdense, long fplane, double gx, double gy, int xc,
                       double flux_norm, double* out, hipStream_t s) {
    flux_kernel<T><<<1, 256, 0, s>>>(g, L, H, fdense, fplane, gx, gy, xc, flux_norm, out);
    return hipGetLastError();
}

// one block per (column, plane): the rows of one plane of one column are contiguous
template <typename T>
__global__ void count_nonfinite_kernel(const T* __restrict__ g, Layout L, double* count) {
    const int xc = (int)blockIdx.x, k = (int)blockIdx.y;
    const T* p = g + (long)xc * L.col + (long)k * L.plane;
    int bad = 0;
    for (int y = threadIdx.x; y < L.ny; y += blockDim.x) bad += !isfinite(p[y]);
    const double n = wave_sum((double)bad);
    if ((threadIdx.x & 63) == 0 && n > 0.) atomicAdd(count, n);
}

template <typename T>
hipError_t launch_count_nonfinite(const T* g, Layout L, double* count, hipStream_t s) {
    if (L.ncol <= 0) return hipSuccess;
    count_nonfinite_kernel<T><<<dim3((unsigned)L.ncol, 9), 256, 0, s>>>(g, L, count);
    return hipGetLastError();
}

// ---- layout conversion ------------------------------------------------------------------
template <typename T>
__global__ void pop_in_kernel(const double* __restrict__ f, T* __restrict__ g, Layout L) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)L.ncol * L.ny) return;
    const int y = (int)(idx / L.ncol), xc = (int)(idx - (long)y * L.ncol);
#pragma unroll
    for (int k = 0; k < 9; ++k) g[k * L.plane + (long)xc * L.col + y] = Store<T>::from_f(f[9 * idx + k], k);
}

template <typename T>
hipError_t launch_pop_in(const double* f, T* g, Layout L, hipStream_t s) {
    const long n = (long)L.ncol * L.ny;
    pop_in_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(f, g, L);
    return hipGetLastError();
}

__global__ void field_in_kernel(const double* __restrict__ ref, double* __restrict__ lay, Layout L, int ncomp, long fplane) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long N = (long)L.ncol * L.ny;
    if (idx >= N) return;
    const int y = (int)(idx / L.ncol), xc = (int)(idx - (long)y * L.ncol);
    for (int a = 0; a < ncomp; ++a) lay[a * fplane + (long)xc * L.rows + y] = ref[a * N + idx];
}

__global__ void field_out_kernel(const double* __restrict__ lay, double* __restrict__ ref, Layout L, int ncomp,
                                 long fplane, double add0, double add1) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long N = (long)L.ncol * L.ny;
    if (idx >= N) return;
    const int y = (int)(idx / L.ncol), xc = (int)(idx - (long)y * L.ncol);
    for (int a = 0; a < ncomp; ++a)
        ref[a * N + idx] = (lay ? lay[a * fplane + (long)xc * L.rows + y] : 0.) + (a == 0 ? add0 : add1);
}

hipError_t launch_field_in(const double* ref, double* lay, Layout L, int ncomp, long fplane, hipStream_t s) {
    const long n = (long)L.ncol * L.ny;
    field_in_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(ref, lay, L, ncomp, fplane);
    return hipGetLastError();
}

hipError_t launch_field_out(const double* lay, double* ref, Layout L, int ncomp, long fplane, double add0, double add1,
                            hipStream_t s) {
    const long n = (long)L.ncol * L.ny;
    field_out_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(lay, ref, L, ncomp, fplane, add0, add1);
    return hipGetLastError();
}

#define IBLB_INST(T)                                                                                            \
    template hipError_t launch_fused<T>(const FusedArgs<T>&, hipStream_t, hipEvent_t);                                \
    template hipError_t launch_boot<T>(const T*, T*, Layout, const double*, const double*, const double*, long,  \
                                       Coef, KConst, hipStream_t);                                                  \
    template hipError_t launch_macro_out<T>(const T*, Layout, Halo<T>, const double*, long, double, double,      \
                                            double*, double*, hipStream_t);                                     \
    template hipError_t launch_pop_out<T>(const T*, Layout, Halo<T>, double*, int, hipStream_t);                     \
    template hipError_t launch_flux<T>(const T*, Layout, Halo<T>, const double*, long, double, double, int,      \
                                       double, double*, hipStream_t);                                           \
    template hipError_t launch_pop_in<T>(const double*, T*, Layout, hipStream_t);                                \
    template hipError_t launch_count_nonfinite<T>(const T*, Layout, double*, hipStream_t);

IBLB_INST(double)
IBLB_INST(float)

}  // namespace iblb

// lbm_vec.h — register-level helpers shared by the collide-stream kernels (lbm_kernels.hip,
// lbm_sweep.hip): 16-byte plane loads/stores, nontemporal variants, DPP lane shifts.
#pragma once

#include "iblb_kernels.h"

namespace iblb {

template <typename T, int V>
struct VT {
    typedef T type __attribute__((ext_vector_type(V)));
};

// 16-byte load at a 16-byte aligned address.
template <typename T, int V>
__device__ __forceinline__ typename VT<T, V>::type lda(const T* p) {
    return *reinterpret_cast<const typename VT<T, V>::type*>(p);
}
// 16-byte load at an element-aligned (misaligned by one element) address.
template <typename T, int V>
__device__ __forceinline__ typename VT<T, V>::type ldu(const T* p) {
    typename VT<T, V>::type r;
    __builtin_memcpy(&r, p, sizeof(r));
    return r;
}
template <typename T, int V>
__device__ __forceinline__ void sta(T* p, typename VT<T, V>::type v) {
    *reinterpret_cast<typename VT<T, V>::type*>(p) = v;
}

// Compute type: double storage collides in double, float storage in float
// (deviation form keeps rho ~ 1 out of the float mantissa).
template <typename T>
struct Calc { typedef double R; };
template <>
struct Calc<float> { typedef float R; };

// Kernel variants (MODE bits), selected per context for A/B measurement:
//   MODE_NT_STORE  populations written with nontemporal stores
//   MODE_NT_LOAD   populations read with nontemporal loads (each element is read once)
//   MODE_SHIFT     all planes loaded 16-B aligned; the +-1-row shift of the c_y != 0 planes
//                  is done in registers (DPP wave_shr / wave_shl by one lane) with one scalar
//                  load per wave for the element across the chunk edge, instead of
//                  misaligned 16-B loads
enum { MODE_NT_STORE = 1, MODE_NT_LOAD = 2, MODE_SHIFT = 4 };

template <typename T, int V, int MODE>
__device__ __forceinline__ typename VT<T, V>::type ld_plane(const T* p) {
    typedef typename VT<T, V>::type vec;
    if (MODE & MODE_NT_LOAD) return __builtin_nontemporal_load(reinterpret_cast<const vec*>(p));
    return lda<T, V>(p);
}
template <typename T, int V, int MODE>
__device__ __forceinline__ void st_plane(T* p, typename VT<T, V>::type v) {
    typedef typename VT<T, V>::type vec;
    if (MODE & MODE_NT_STORE) __builtin_nontemporal_store(v, reinterpret_cast<vec*>(p));
    else sta<T, V>(p, v);
}

// Move a 32/64-bit value one lane up (dir = +1: lane l receives lane l-1) or down
// (dir = -1: lane l receives lane l+1) across the whole wave with DPP.
// bound_ctrl: the lane without a source (lane 0 / lane 63) reads 0, so no register has to be
// initialised with an "old" value first (one v_mov_b32 less per shifted dword)
template <int DIR>
__device__ __forceinline__ int dpp_shift(int v) {
    return __builtin_amdgcn_mov_dpp(v, DIR > 0 ? 0x138 : 0x130, 0xf, 0xf, true);
}
template <int DIR>
__device__ __forceinline__ double lane_shift(double v) {
    const int lo = dpp_shift<DIR>(__double2loint(v));
    const int hi = dpp_shift<DIR>(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
template <int DIR>
__device__ __forceinline__ float lane_shift(float v) {
    return __int_as_float(dpp_shift<DIR>(__float_as_int(v)));
}

// Rows y0-1 .. y0+V-2 (DIR = +1, planes with c_y = +1) or y0+1 .. y0+V (DIR = -1) of plane
// pointer p (column base), for a wave covering rows [cs, cs + 64V).
template <typename T, int V, int MODE, int DIR>
__device__ __forceinline__ typename VT<T, V>::type ld_shifted(const T* p, int y0, int cs, int lane) {
    typedef typename VT<T, V>::type vec;
    if (!(MODE & MODE_SHIFT)) return ldu<T, V>(p + y0 - DIR);
    const vec a = ld_plane<T, V, MODE>(p + y0);
    vec r;
    if (DIR > 0) {
        // element 0 = last element of the previous lane; lane 0: row cs-1 (scalar load)
        T prev = lane_shift<+1>(a[V - 1]);
        const T edge = p[cs - 1];
        if (lane == 0) prev = edge;
        r[0] = prev;
#pragma unroll
        for (int e = 1; e < V; ++e) r[e] = a[e - 1];
    } else {
        T next = lane_shift<-1>(a[0]);
        const T edge = p[cs + 64 * V];
        if (lane == 63) next = edge;
#pragma unroll
        for (int e = 0; e < V - 1; ++e) r[e] = a[e + 1];
        r[V - 1] = next;
    }
    return r;
}

}  // namespace iblb

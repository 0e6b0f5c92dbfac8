// device.hpp -- CDNA4 (gfx950) device helpers shared by the SpMV kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace spmv {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// Streamed matrix data (col/val) is read exactly once per SpMV: load it with
// the non-temporal hint so it does not displace x from L2 / Infinity Cache.
__device__ __forceinline__ i32x4 ld_stream4(const int32_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const i32x4 *>(p));
}
__device__ __forceinline__ f64x2 ld_stream2(const double *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(p));
}
__device__ __forceinline__ i32x2 ld_stream2(const int32_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const i32x2 *>(p));
}
__device__ __forceinline__ double ld_stream(const double *p) {
    return __builtin_nontemporal_load(p);
}
__device__ __forceinline__ int32_t ld_stream(const int32_t *p) {
    return __builtin_nontemporal_load(p);
}

// x gathers: plain cached loads (x is the re-used operand).
__device__ __forceinline__ double ld_x(const double *x, int32_t c) { return x[c]; }

// y = a*b + c as a rounded multiply followed by a rounded add.  Keeps the
// per-row arithmetic identical to the reference's `tmp += val*x`
// (src/opt_crs.cpp:62-66) as compiled without contraction, so sequential-order
// kernels (ELL, DIA, 1-lane CSR) are bit-exact against oracle/.
__device__ __forceinline__ double madd(double a, double b, double c) {
    return __dadd_rn(c, __dmul_rn(a, b));
}

// Sum over aligned groups of G lanes (G power of two <= 64); every lane of a
// group ends with the group total.  Butterfly order is fixed -> deterministic.
template <int G>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = __dadd_rn(v, __shfl_xor(v, o, 64));
    return v;
}

// 64-bit DPP move (two 32-bit v_mov_dpp).  Lanes the control does not feed
// (or rows outside ROWMASK) read 0.
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWMASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWMASK, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// group_sum<G> with the offsets below 16 taken by DPP instead of ds_bpermute,
// bit-identical to group_sum<G> (same pairs, same order; IEEE addition is
// commutative, so v + v[i ^ o] is the same sum in both lanes of a pair):
// offset 8 is the row rotation by 8 (lane i reads (i + 8) mod 16 = i ^ 8);
// offset 4 the row rotation by 4, which reads a lane holding v[i ^ 4] once
// the offset-8 step has made every row 8-periodic (G >= 16; for G = 8 it
// stays a ds_bpermute); offsets 2 and 1 are the quad permutations
// [2,3,0,1] and [1,0,3,2], exactly i ^ 2 and i ^ 1.
template <int G>
__device__ __forceinline__ double group_sum_dpp(double v) {
#pragma unroll
    for (int o = G / 2; o >= 16; o >>= 1) v = __dadd_rn(v, __shfl_xor(v, o, 64));
    if constexpr (G >= 16) {
        v = __dadd_rn(v, dpp_f64<0x128>(v));  // row_ror:8
        v = __dadd_rn(v, dpp_f64<0x124>(v));  // row_ror:4
    } else if constexpr (G == 8) {
        v = __dadd_rn(v, __shfl_xor(v, 4, 64));
    }
    if constexpr (G >= 4) v = __dadd_rn(v, dpp_f64<0x4E>(v));  // quad_perm [2,3,0,1]
    if constexpr (G >= 2) v = __dadd_rn(v, dpp_f64<0xB1>(v));  // quad_perm [1,0,3,2]
    return v;
}

// Inclusive prefix sum of an int across the 64-lane wave (Hillis-Steele).
__device__ __forceinline__ int wave_inclusive_sum(int v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// Segmented inclusive scan across the wave: a lane with `start` begins a new
// segment.  Returns the running sum of the lane's segment up to and including
// the lane.  Combination order is a fixed tree (deterministic).
__device__ __forceinline__ double wave_seg_scan(double v, bool start, int lane) {
    int f = start ? 1 : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        double tv = __shfl_up(v, o, 64);
        int tf = __shfl_up(f, o, 64);
        if (lane >= o) {
            if (!f) v = __dadd_rn(tv, v);
            f |= tf;
        }
    }
    return v;
}

}  // namespace spmv

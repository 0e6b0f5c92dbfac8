// k_ell.hip -- sliced ELL SpMV for gfx950: the opt_ell hot loop
// (src/opt_ell.cpp:75-89, y[r] += x[col] * val over the row's slots)
// re-laid out for wave64.
//
// One wave = one slice of 64 consecutive rows, one lane = one row.  Slots are
// interleaved by 4 (see EllDev): at step q a lane issues one 16-byte load of
// 4 column indices and two 16-byte loads of 4 values (slots 0-1 from the
// quad's first KiB of values, 2-3 from its second) -- every wave instruction
// reads 1 KiB contiguous -- then 4 x gathers.  The slice width is
// wave-uniform, so the loop has no divergence.  Each row is summed
// sequentially in slot order with a rounded multiply + rounded add, i.e. the
// same arithmetic as opt_crs/opt_ell (bit-exact against oracle/).  Padding
// slots carry val = 0 and repeat a real column of the row.  With PERM the
// slices hold rows sorted by length (JDS, src/opt_jds.cpp:29-71, 91-103) and
// y is written through the permutation.
//
// O32 (x below 4 GB, a slice below 2 GB): the wave's slice base is
// wave-uniform (SGPR) and every load addresses it, or x, plus a 32-bit byte
// offset (the global_load saddr form), instead of 64-bit per-lane addresses.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

template <bool O32>
__device__ __forceinline__ const char *ell_at(const void *base, int64_t byte_off) {
    if constexpr (O32) return (const char *)base + (uint32_t)byte_off;
    else return (const char *)base + byte_off;
}

template <int UNROLL, bool ADD, bool PERM, bool O32 = false>
__global__ __launch_bounds__(256) void ell_slice_kernel(int64_t m, int64_t n_slices,
                                                        const int32_t *__restrict__ perm,
                                                        const int64_t *__restrict__ slice_off,
                                                        const int32_t *__restrict__ col,
                                                        const double *__restrict__ val,
                                                        const double *__restrict__ x,
                                                        double *__restrict__ y) {
    const int64_t slice = (int64_t)blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (slice >= n_slices) return;
    const int64_t srow = slice * 64 + lane;
    // JDS: the matrix row, loaded before the slots so its latency hides
    // behind them instead of trailing the wave
    const int64_t row = PERM ? (srow < m ? (int64_t)perm[srow] : 0) : srow;
    const int64_t base = slice_off[slice];
    const int64_t quads = (slice_off[slice + 1] - base) >> 8;  // (width/4)
    const int32_t *cs = col + base;  // wave-uniform slice bases
    const double *vs = val + base;
    auto ldc = [&](int64_t q) { return ld_stream4((const int32_t *)ell_at<O32>(cs, (q * 256 + lane * 4) * 4)); };
    auto ldv = [&](int64_t q, int h) {
        return ld_stream2((const double *)ell_at<O32>(vs, (q * 256 + h * 128 + lane * 2) * 8));
    };
    auto ldx = [&](int c) -> double {
        if constexpr (O32) return *(const double *)((const char *)x + (uint32_t)c * 8u);
        else return ld_x(x, c);
    };
    double acc = 0.0;
    int64_t q = 0;
    for (; q + UNROLL <= quads; q += UNROLL) {
        i32x4 c[UNROLL];
        f64x2 a[UNROLL], b[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            c[u] = ldc(q + u);
            a[u] = ldv(q + u, 0);
            b[u] = ldv(q + u, 1);
        }
        double g[UNROLL][4];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            g[u][0] = ldx(c[u].x);
            g[u][1] = ldx(c[u].y);
            g[u][2] = ldx(c[u].z);
            g[u][3] = ldx(c[u].w);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            acc = madd(a[u].x, g[u][0], acc);
            acc = madd(a[u].y, g[u][1], acc);
            acc = madd(b[u].x, g[u][2], acc);
            acc = madd(b[u].y, g[u][3], acc);
        }
    }
    for (; q < quads; ++q) {
        const i32x4 c = ldc(q);
        const f64x2 a = ldv(q, 0);
        const f64x2 b = ldv(q, 1);
        const double g0 = ldx(c.x), g1 = ldx(c.y), g2 = ldx(c.z), g3 = ldx(c.w);
        acc = madd(a.x, g0, acc);
        acc = madd(a.y, g1, acc);
        acc = madd(b.x, g2, acc);
        acc = madd(b.y, g3, acc);
    }
    if (srow < m) {
        if (ADD) y[row] = __dadd_rn(y[row], acc);
        else __builtin_nontemporal_store(acc, y + row);  // not re-read: streamed out
    }
}

template <int U, bool O32>
static void launch_ell_uo(const spmv_plan_s *p, const double *x, double *y, size_t lds) {
    const EllDev &e = p->ell;
    const int64_t blocks = (e.n_slices + 3) / 4;
    if (e.perm)
        hipLaunchKernelGGL((ell_slice_kernel<U, false, true, O32>), dim3((unsigned)blocks), dim3(256), lds,
                           p->stream, p->m, e.n_slices, e.perm, e.slice_off, e.col, e.val, x, y);
    else
        hipLaunchKernelGGL((ell_slice_kernel<U, false, false, O32>), dim3((unsigned)blocks), dim3(256), lds,
                           p->stream, p->m, e.n_slices, e.perm, e.slice_off, e.col, e.val, x, y);
}

template <int U>
static void launch_ell_u(const spmv_plan_s *p, const double *x, double *y, size_t lds) {
    // 32-bit offsets: x below 4 GB and a slice's values below 2 GB
    bool o32 = p->n < ((int64_t)1 << 29) && (int64_t)p->ell.max_width * 64 * 8 < ((int64_t)1 << 31);
    if (const char *v = probe_env("SPMV_LAUNCH_ELL_O32")) o32 = o32 && std::atoi(v) != 0;
    if (o32) launch_ell_uo<U, true>(p, x, y, lds);
    else launch_ell_uo<U, false>(p, x, y, lds);
}

constexpr int kEllLdsKb = 64;  // LDS per workgroup of a large ELL launch: 2 workgroups per CU

int launch_ell(const spmv_plan_s *p, const double *x, double *y) {
    const EllDev &e = p->ell;
    if (e.n_slices == 0) return SPMV_SUCCESS;
    // Above 256 MB of slots the launch requests 64 KB of LDS: two workgroups
    // (8 waves, ~48 KB of slots in flight) per CU instead of the 8 the
    // registers allow -- fewer concurrent streams, as DIA's cap (config 4,
    // same plans: 2.421-2.425 -> 2.382-2.387 ms over three plans,
    // profiles/round4/probe/c4_ell_window_variants.jsonl).
    // The product runs 2 quads (4 slots each) per lane per iteration; the
    // probe build adds launch-time unroll 1 / 4 and LDS-request variants.
    size_t lds = (size_t)e.slots * sizeof(double) >= kStreamVmmMinBytes ? kEllLdsKb * 1024 : 0;
#ifdef SPMV_PROBES
    int unroll = e.unroll;
    if (const char *v = probe_env("SPMV_LAUNCH_ELL_UNROLL")) unroll = std::atoi(v);
    if (const char *v = probe_env("SPMV_LAUNCH_ELL_LDS_KB")) lds = (size_t)std::atoi(v) * 1024;
    switch (unroll) {
        case 1: launch_ell_u<1>(p, x, y, lds); break;
        case 4: launch_ell_u<4>(p, x, y, lds); break;
        default: launch_ell_u<2>(p, x, y, lds);
    }
#else
    launch_ell_u<2>(p, x, y, lds);
#endif
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

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
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

template <int UNROLL, bool ADD, bool PERM>
__global__ __launch_bounds__(256) void ell_slice_kernel(int64_t m, int64_t n_slices,
                                                        const int32_t *__restrict__ perm,
                                                        const int64_t *__restrict__ slice_off,
                                                        const int32_t *__restrict__ col,
                                                        const double *__restrict__ val,
                                                        const double *__restrict__ x,
                                                        double *__restrict__ y) {
    const int64_t slice = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (slice >= n_slices) return;
    const int64_t base = slice_off[slice];
    const int64_t quads = (slice_off[slice + 1] - base) >> 8;  // (width/4)
    const int32_t *cp = col + base + lane * 4;
    const double *vp = val + base + lane * 2;
    double acc = 0.0;
    int64_t q = 0;
    for (; q + UNROLL <= quads; q += UNROLL) {
        i32x4 c[UNROLL];
        f64x2 a[UNROLL], b[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            c[u] = ld_stream4(cp + (q + u) * 256);
            a[u] = ld_stream2(vp + (q + u) * 256);
            b[u] = ld_stream2(vp + (q + u) * 256 + 128);
        }
        double g[UNROLL][4];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            g[u][0] = ld_x(x, c[u].x);
            g[u][1] = ld_x(x, c[u].y);
            g[u][2] = ld_x(x, c[u].z);
            g[u][3] = ld_x(x, c[u].w);
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
        const i32x4 c = ld_stream4(cp + q * 256);
        const f64x2 a = ld_stream2(vp + q * 256);
        const f64x2 b = ld_stream2(vp + q * 256 + 128);
        const double g0 = ld_x(x, c.x), g1 = ld_x(x, c.y), g2 = ld_x(x, c.z), g3 = ld_x(x, c.w);
        acc = madd(a.x, g0, acc);
        acc = madd(a.y, g1, acc);
        acc = madd(b.x, g2, acc);
        acc = madd(b.y, g3, acc);
    }
    const int64_t srow = slice * 64 + lane;
    if (srow < m) {
        const int64_t row = PERM ? (int64_t)perm[srow] : srow;  // JDS: back to matrix order
        if (ADD) y[row] = __dadd_rn(y[row], acc);
        else y[row] = acc;
    }
}

template <int U>
static void launch_ell_u(const spmv_plan_s *p, const double *x, double *y, size_t lds) {
    const EllDev &e = p->ell;
    const int64_t blocks = (e.n_slices + 3) / 4;
    if (e.perm)
        hipLaunchKernelGGL((ell_slice_kernel<U, false, true>), dim3((unsigned)blocks), dim3(256), lds, p->stream,
                           p->m, e.n_slices, e.perm, e.slice_off, e.col, e.val, x, y);
    else
        hipLaunchKernelGGL((ell_slice_kernel<U, false, false>), dim3((unsigned)blocks), dim3(256), lds,
                           p->stream, p->m, e.n_slices, e.perm, e.slice_off, e.col, e.val, x, y);
}

int launch_ell(const spmv_plan_s *p, const double *x, double *y) {
    const EllDev &e = p->ell;
    if (e.n_slices == 0) return SPMV_SUCCESS;
    // probe build: launch-time unroll / LDS request (workgroups per CU)
    int unroll = e.unroll;
    size_t lds = 0;
    if (const char *v = probe_env("SPMV_LAUNCH_ELL_UNROLL")) unroll = std::atoi(v);
    if (const char *v = probe_env("SPMV_LAUNCH_ELL_LDS_KB")) lds = (size_t)std::atoi(v) * 1024;
    switch (unroll) {  // quads (4 slots each) per lane per iteration
        case 1: launch_ell_u<1>(p, x, y, lds); break;
        case 4: launch_ell_u<4>(p, x, y, lds); break;
        default: launch_ell_u<2>(p, x, y, lds);
    }
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

// k_dia.hip -- DIA SpMV for gfx950: replaces the serial opt_dia loop
// (src/opt_dia.cpp:65-97, y[col+off-ioff] += diag*x[col], plus a leaked
// tmp[m+n-1] per call at :80).
//
// Row-indexed diagonals: val[d*mp + r] = A[r, r + off[d]].  One lane = two
// rows; the diagonal loop is wave-uniform and the offsets are loaded as scalars.
// Each value load is coalesced (consecutive rows), each x load is coalesced
// and re-used across the diagonals through L1/L2, so HBM sees ~8 B per stored
// slot + x + y.  Diagonals are summed in ascending offset order, i.e.
// ascending column order with rounded multiply + add: bit-identical to the
// sequential opt_crs row sum.  Out-of-range slots hold 0 and read a clamped,
// in-bounds x entry.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

// Two rows per lane: one 16-byte load of val[d*mp + r .. r+1] per diagonal
// (mp = m rounded up to even), so a wave instruction streams 1 KiB.
template <int UNROLL>
__global__ __launch_bounds__(256) void dia_kernel(int64_t m, int64_t mp, int64_t n, int n_diags,
                                                  const int32_t *__restrict__ off,
                                                  const double *__restrict__ val,
                                                  const double *__restrict__ x,
                                                  double *__restrict__ y) {
    const int64_t r = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (r >= m) return;
    double acc0 = 0.0, acc1 = 0.0;
    auto xat = [&](int64_t c) { return x[c < 0 ? 0 : (c >= n ? n - 1 : c)]; };
    int d = 0;
    for (; d + UNROLL <= n_diags; d += UNROLL) {
        f64x2 v[UNROLL];
        double g0[UNROLL], g1[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = ld_stream2(val + (int64_t)(d + u) * mp + r);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t c = r + off[d + u];
            g0[u] = xat(c);
            g1[u] = xat(c + 1);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            acc0 = madd(v[u].x, g0[u], acc0);
            acc1 = madd(v[u].y, g1[u], acc1);
        }
    }
    for (; d < n_diags; ++d) {
        const f64x2 v = ld_stream2(val + (int64_t)d * mp + r);
        const int64_t c = r + off[d];
        acc0 = madd(v.x, xat(c), acc0);
        acc1 = madd(v.y, xat(c + 1), acc1);
    }
    y[r] = acc0;
    if (r + 1 < m) y[r + 1] = acc1;
}

int launch_dia(const spmv_plan_s *p, const double *x, double *y) {
    const DiaDev &d = p->dia;
    if (p->m == 0) return SPMV_SUCCESS;
    const int64_t pairs = (p->m + 1) / 2;
    const int64_t blocks = (pairs + 255) / 256;
    hipLaunchKernelGGL((dia_kernel<8>), dim3((unsigned)blocks), dim3(256), 0, p->stream, p->m, d.mp,
                       p->n, d.n_diags, d.off, d.val, x, y);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

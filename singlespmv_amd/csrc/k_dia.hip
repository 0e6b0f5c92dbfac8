// k_dia.hip -- DIA SpMV for gfx950: replaces the serial opt_dia loop
// (src/opt_dia.cpp:65-97, y[col+off-ioff] += diag*x[col], plus a leaked
// tmp[m+n-1] per call at :80).
//
// Row-indexed diagonals: val[d*m + r] = A[r, r + off[d]].  One lane = one
// row; the diagonal loop is wave-uniform and the offsets are loaded as scalars.
// Each value load is coalesced (consecutive rows), each x load is coalesced
// and re-used across the diagonals through L1/L2, so HBM sees ~8 B per stored
// slot + x + y.  Diagonals are summed in ascending offset order, i.e.
// ascending column order with rounded multiply + add: bit-identical to the
// sequential opt_crs row sum.  Out-of-range slots hold 0 and read a clamped,
// in-bounds x entry.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

template <int UNROLL>
__global__ __launch_bounds__(256) void dia_kernel(int64_t m, int64_t n, int n_diags,
                                                  const int32_t *__restrict__ off,
                                                  const double *__restrict__ val,
                                                  const double *__restrict__ x,
                                                  double *__restrict__ y) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    double acc = 0.0;
    int d = 0;
    for (; d + UNROLL <= n_diags; d += UNROLL) {
        double v[UNROLL], g[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = ld_stream(val + (int64_t)(d + u) * m + r);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            int64_t c = r + off[d + u];
            c = c < 0 ? 0 : (c >= n ? n - 1 : c);
            g[u] = x[c];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc = madd(v[u], g[u], acc);
    }
    for (; d < n_diags; ++d) {
        const double v = ld_stream(val + (int64_t)d * m + r);
        int64_t c = r + off[d];
        c = c < 0 ? 0 : (c >= n ? n - 1 : c);
        acc = madd(v, x[c], acc);
    }
    y[r] = acc;
}

int launch_dia(const spmv_plan_s *p, const double *x, double *y) {
    const DiaDev &d = p->dia;
    if (p->m == 0) return SPMV_SUCCESS;
    const int64_t blocks = (p->m + 255) / 256;
    hipLaunchKernelGGL((dia_kernel<8>), dim3((unsigned)blocks), dim3(256), 0, p->stream, p->m, p->n,
                       d.n_diags, d.off, d.val, x, y);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

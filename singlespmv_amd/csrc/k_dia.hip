// k_dia.hip -- DIA SpMV for gfx950: replaces the serial opt_dia loop
// (src/opt_dia.cpp:65-97, y[col+off-ioff] += diag*x[col], plus a leaked
// tmp[m+n-1] per call at :80).
//
// Row-indexed diagonals, blocked: the 512 rows of workgroup b hold every
// diagonal contiguously, val[(b*n_diags + d)*512 + r%512] = A[r, r + off[d]],
// so a workgroup streams ONE contiguous n_diags*4 KB block (the first layout,
// diagonal-major val[d*mp + r], read 64 streams 160 MB apart at config 4:
// 1.81 ms vs the blocked layout's, profiles/round1/probe/dia_blocked_ab.jsonl).
// One lane = two rows; the diagonal loop is wave-uniform and the offsets are
// loaded as scalars, so HBM sees ~8 B per stored slot + x + y.  Diagonals are summed in ascending offset order, i.e.
// ascending column order with rounded multiply + add: bit-identical to the
// sequential opt_crs row sum.  Out-of-range slots hold 0 and read a clamped,
// in-bounds x entry.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

// Two rows per lane: one 16-byte load of the lane's two rows per diagonal, so
// a wave instruction streams 1 KiB.
//
// LDSX: the workgroup's 512 rows need x over ONE contiguous column window
// [r0 + off_min, r0 + 511 + off_max + 1]; it is staged once into LDS with
// coalesced loads and every diagonal reads its pair x[c], x[c+1] from there,
// so the only HBM stream left is val (and x once).  Without LDSX (diagonal
// span too wide for the window) x is read from global memory per diagonal.
template <int UNROLL, bool LDSX, int YMODE = 0>
__global__ __launch_bounds__(256) void dia_kernel(int64_t m, int64_t mp, int64_t n, int n_diags,
                                                  const int32_t *__restrict__ off, int32_t off_min, int32_t win,
                                                  const double *__restrict__ val,
                                                  const double *__restrict__ x,
                                                  double *__restrict__ y, int32_t group) {
    extern __shared__ double xs[];
    const int64_t r0 = 2 * (int64_t)blockIdx.x * blockDim.x;
    const int64_t r = r0 + 2 * threadIdx.x;
    // group > 0 (DiaDev::group): blocks interleaved per group of `group`
    // consecutive blocks, diagonal by diagonal (the block's diagonal d at
    // stride gt*512); else one contiguous n_diags*4 KB block
    int64_t vbase = (int64_t)blockIdx.x * n_diags * kDiaBlockRows, dstride = kDiaBlockRows;
    if (group > 0) {
        const int64_t t = blockIdx.x / group, g = blockIdx.x - t * group;
        const int64_t rest = mp / kDiaBlockRows - t * group;
        vbase = (t * group * n_diags + g) * kDiaBlockRows;
        dstride = (rest < group ? rest : group) * kDiaBlockRows;
    }
    const double *vb = val + vbase + 2 * threadIdx.x;
    auto xat = [&](int64_t c) { return x[c < 0 ? 0 : (c >= n ? n - 1 : c)]; };
    if (LDSX) {
        // out-of-range columns only meet zero-filled slots: any finite x works
        const int64_t c0 = r0 + off_min;
        for (int i = threadIdx.x; i < win; i += blockDim.x) xs[i] = xat(c0 + i);
        __syncthreads();
    }
    if (r >= m) return;
    double acc0 = 0.0, acc1 = 0.0;
    const int lbase = 2 * threadIdx.x - off_min;  // LDS index of column r + 0
    int d = 0;
    for (; d + UNROLL <= n_diags; d += UNROLL) {
        f64x2 v[UNROLL];
        double g0[UNROLL], g1[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = ld_stream2(vb + (int64_t)(d + u) * dstride);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (LDSX) {
                const int li = lbase + off[d + u];
                g0[u] = xs[li];
                g1[u] = xs[li + 1];
            } else {
                const int64_t c = r + off[d + u];
                g0[u] = xat(c);
                g1[u] = xat(c + 1);
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            acc0 = madd(v[u].x, g0[u], acc0);
            acc1 = madd(v[u].y, g1[u], acc1);
        }
    }
    for (; d < n_diags; ++d) {
        const f64x2 v = ld_stream2(vb + (int64_t)d * dstride);
        double a, b;
        if (LDSX) {
            const int li = lbase + off[d];
            a = xs[li];
            b = xs[li + 1];
        } else {
            const int64_t c = r + off[d];
            a = xat(c);
            b = xat(c + 1);
        }
        acc0 = madd(v.x, a, acc0);
        acc1 = madd(v.y, b, acc1);
    }
    // y is written once and not re-read: the row pair as one 16-byte
    // nontemporal store where y is 16-byte aligned (r is even)
    if (r + 1 < m && (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
        f64x2 yv;
        yv.x = acc0;
        yv.y = acc1;
        // YMODE 1 (probe A/B): ordinary 16-byte stores (y lines stay in L2)
        if constexpr (YMODE == 1) *reinterpret_cast<f64x2 *>(y + r) = yv;
        else __builtin_nontemporal_store(yv, reinterpret_cast<f64x2 *>(y + r));
    } else {
        y[r] = acc0;
        if (r + 1 < m) y[r + 1] = acc1;
    }
}

// LDS x window of a 512-row workgroup: 512 rows + diagonal span + 1
constexpr int kDiaMaxWin = 8192;  // doubles (64 KB)
// LDS requested per workgroup (KB), at least the window: > 80 KB = one per CU
constexpr int kDiaLdsKb = 96;

int launch_dia(const spmv_plan_s *p, const double *x, double *y) {
    const DiaDev &d = p->dia;
    if (p->m == 0) return SPMV_SUCCESS;
    if (d.n_diags == 0) {  // no stored diagonal: y = 0
        SPMV_HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * (size_t)p->m, p->stream));
        return SPMV_SUCCESS;
    }
    const int64_t pairs = (p->m + 1) / 2;
    const int64_t blocks = (pairs + 255) / 256;
    const int32_t off_min = d.off_host.front(), off_max = d.off_host.back();
    const int64_t win = 512 + (int64_t)off_max - off_min + 1;
    // The LDS request caps the workgroups per CU (kDiaLdsKb: one, 4 waves,
    // 32 KB of values in flight; the x window alone would allow 8): fewer
    // value streams keep the HBM channels out of the oversubscribed mode some
    // placements fall into.  Config 4, launch variants on the same plans:
    // 1.476-1.527 ms at 1 per CU, 1.500-1.594 at 2, 1.537-1.641 at 8
    // (profiles/round3/probe/dia_occupancy_paired_c4.jsonl,
    // dia_unroll_occupancy_c4.jsonl; profiles/round3/README.md)
    // Below the size at which DIA values take VMM handles (kDiaVmmMinBytes,
    // 256 MB) the launch keeps the x window's own occupancy: 64 diagonals,
    // same plans, 200 K rows (100 MB) 0.0166 ms uncapped vs 0.0188 capped;
    // 2 M rows (1 GB) 0.163 vs 0.159; 6 M rows (3 GB) 0.486 vs 0.466
    // (profiles/round4/probe/dia_cap_{200k,2m,6m}.jsonl)
    const bool big = (size_t)d.n_diags * (size_t)d.mp * sizeof(double) >= kDiaVmmMinBytes;
    int kb = d.lds_kb >= 0 ? d.lds_kb : (big ? kDiaLdsKb : 0);
    if (const char *e = probe_env("SPMV_LAUNCH_DIA_LDS_KB")) kb = std::atoi(e);
    const int dbg = launch_dbg(d.dbg);
    const size_t lds = std::max(sizeof(double) * (size_t)win, (size_t)kb * 1024);
#ifdef SPMV_PROBES
    if (win <= kDiaMaxWin && (dbg & 12)) {  // probe A/B: 4 (dbg 4) / 16 (dbg 8) diagonals in flight per lane
        if (dbg & 4)
            hipLaunchKernelGGL((dia_kernel<4, true>), dim3((unsigned)blocks), dim3(256), lds, p->stream, p->m, d.mp,
                               p->n, d.n_diags, d.off, off_min, (int32_t)win, d.val, x, y, d.group);
        else
            hipLaunchKernelGGL((dia_kernel<16, true>), dim3((unsigned)blocks), dim3(256), lds, p->stream, p->m, d.mp,
                               p->n, d.n_diags, d.off, off_min, (int32_t)win, d.val, x, y, d.group);
        SPMV_HIP_TRY(hipGetLastError());
        return SPMV_SUCCESS;
    }
    if (win <= kDiaMaxWin && (dbg & 2)) {  // probe A/B: ordinary y stores
        hipLaunchKernelGGL((dia_kernel<8, true, 1>), dim3((unsigned)blocks), dim3(256), lds,
                           p->stream, p->m, d.mp, p->n, d.n_diags, d.off, off_min, (int32_t)win, d.val, x, y, d.group);
        SPMV_HIP_TRY(hipGetLastError());
        return SPMV_SUCCESS;
    }
#endif
    if (win <= kDiaMaxWin && !(dbg & 1))
        hipLaunchKernelGGL((dia_kernel<8, true>), dim3((unsigned)blocks), dim3(256), lds,
                           p->stream, p->m, d.mp, p->n, d.n_diags, d.off, off_min, (int32_t)win, d.val, x, y, d.group);
    else
        hipLaunchKernelGGL((dia_kernel<8, false>), dim3((unsigned)blocks), dim3(256), 0, p->stream, p->m, d.mp,
                           p->n, d.n_diags, d.off, off_min, 0, d.val, x, y, d.group);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

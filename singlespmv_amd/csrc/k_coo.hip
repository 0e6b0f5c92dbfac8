// k_coo.hip -- COO SpMV for gfx950: the opt_coo plugin (src/opt_coo.cpp:34-46:
// zero y, then `#pragma omp atomic` y[r] += val*x[c] per entry).
//
// Entries are row-sorted (plans are built from CSR) and padded to whole
// 128-entry units (CooDev).  One wave takes U units per step; in a unit lane l
// owns entries 2l and 2l+1, so every row / col / val load instruction reads
// 512 B / 512 B / 1 KiB of whole lines, and the U units' loads are issued
// together.  Per unit: the lane adds its two products when they share a row,
// a fixed-tree segmented scan over equal-row runs carries rows from lane to
// lane, and the last lane of every run issues ONE f64 atomic add
// (global_atomic_add_f64) -- a lane whose two entries straddle a row boundary
// closes the first row itself.  A row inside one unit is therefore exact and
// deterministic; a row split across units gets several atomic adds whose
// order (hence rounding) may vary, as in the reference's OpenMP atomics.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

// one unit: rows r0 <= r1 (or -1 padding), products p0, p1 of entries 2l, 2l+1
__device__ __forceinline__ void coo_unit(int32_t r0, int32_t r1, double p0, double p1, int lane,
                                         double *__restrict__ y) {
    const bool joined = r0 == r1;
    int32_t pr1 = __shfl_up(r1, 1, 64);  // the previous lane's last row
    if (lane == 0) pr1 = -2;
    const double v = joined ? __dadd_rn(p0, p1) : p1;
    const bool start = !joined || pr1 != r0;
    const double S = wave_seg_scan(v, start, lane);
    double C = __shfl_up(S, 1, 64);  // the open run arriving from the left
    if (pr1 != r0) C = 0.0;
    int32_t nr0 = __shfl_down(r0, 1, 64);
    if (lane == 63) nr0 = -2;
    if (!joined && r0 >= 0) atomicAdd(&y[r0], __dadd_rn(C, p0));
    if (nr0 != r1 && r1 >= 0) atomicAdd(&y[r1], S);
}

template <int U>
__global__ __launch_bounds__(256) void coo_pair_kernel(int64_t n_units, const int32_t *__restrict__ row,
                                                       const int32_t *__restrict__ col,
                                                       const double *__restrict__ val,
                                                       const double *__restrict__ x, double *__restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t u0 = wave * U; u0 < n_units; u0 += nwaves * U) {
        i32x2 r[U], c[U];
        f64x2 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u0 + u < n_units) {  // wave-uniform
                const int64_t off = (u0 + u) * kCooUnit + lane * 2;
                r[u] = ld_stream2(row + off);
                c[u] = ld_stream2(col + off);
                a[u] = ld_stream2(val + off);
            } else {
                r[u] = i32x2{-1, -1};
                c[u] = i32x2{0, 0};
                a[u] = f64x2{0.0, 0.0};
            }
        }
        double g0[U], g1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            g0[u] = ld_x(x, c[u].x);
            g1[u] = ld_x(x, c[u].y);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            coo_unit(r[u].x, r[u].y, __dmul_rn(a[u].x, g0[u]), __dmul_rn(a[u].y, g1[u]), lane, y);
    }
}

template <int U>
static void launch_coo_u(const spmv_plan_s *p, double *y, const double *x, int64_t max_blocks) {
    const CooDev &c = p->coo;
    const int64_t waves = (c.n_units + U - 1) / U;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, max_blocks));
    hipLaunchKernelGGL((coo_pair_kernel<U>), dim3((unsigned)blocks), dim3(256), 0, p->stream, c.n_units, c.row,
                       c.col, c.val, x, y);
}

int launch_coo(const spmv_plan_s *p, const double *x, double *y) {
    if (p->m) SPMV_HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * (size_t)p->m, p->stream));
    phase_mark(p);  // zero_y | segment
    if (p->coo.n_units == 0) return SPMV_SUCCESS;
    int64_t max_blocks = INT32_MAX;  // one step per wave: short waves interleave best
#ifdef SPMV_PROBES
    // probe build: units per step, grid cap (workgroups of 4 waves)
    int u = 4;
    if (const char *v = probe_env("SPMV_LAUNCH_COO_U")) u = std::atoi(v);
    if (const char *v = probe_env("SPMV_LAUNCH_COO_BLOCKS")) max_blocks = std::atoll(v);
    switch (u) {
        case 1: launch_coo_u<1>(p, y, x, max_blocks); break;
        case 2: launch_coo_u<2>(p, y, x, max_blocks); break;
        case 8: launch_coo_u<8>(p, y, x, max_blocks); break;
        default: launch_coo_u<4>(p, y, x, max_blocks);
    }
#else
    launch_coo_u<4>(p, y, x, max_blocks);
#endif
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

// k_coo.hip -- COO SpMV for gfx950: the opt_coo plugin (src/opt_coo.cpp:34-46:
// zero y, then `#pragma omp atomic` y[r] += val*x[c] per entry).
//
// Entries are row-sorted (plans are built from CSR).  One wave takes 64
// consecutive entries per step (coalesced 4 B + 4 B + 8 B loads), forms the
// products, runs a fixed-tree segmented scan over equal-row runs and lets the
// last lane of every run issue ONE f64 atomic add (global_atomic_add_f64) --
// 1 atomic per row per wave instead of one per entry.  A row inside one
// wave-step is therefore exact and deterministic; a row split across steps
// gets several atomic adds whose order (hence rounding) may vary, as in the
// reference's OpenMP atomics.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

__global__ __launch_bounds__(256) void coo_segment_kernel(int64_t nnz, const int32_t *__restrict__ row,
                                                          const int32_t *__restrict__ col,
                                                          const double *__restrict__ val,
                                                          const double *__restrict__ x,
                                                          double *__restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t base = wave * 64; base < nnz; base += nwaves * 64) {
        const int64_t j = base + lane;
        const bool ok = j < nnz;
        const int32_t r = ok ? ld_stream(row + j) : -1;
        const double v = ok ? __dmul_rn(ld_stream(val + j), ld_x(x, ld_stream(col + j))) : 0.0;
        const int32_t rprev = __shfl_up(r, 1, 64);
        const bool start = lane == 0 || rprev != r;
        const double s = wave_seg_scan(v, start, lane);
        const int32_t rnext = __shfl_down(r, 1, 64);
        const bool last = lane == 63 || rnext != r;
        if (ok && last) atomicAdd(&y[r], s);
    }
}

int launch_coo(const spmv_plan_s *p, const double *x, double *y) {
    if (p->m) SPMV_HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * (size_t)p->m, p->stream));
    phase_mark(p);  // zero_y | segment
    if (p->nnz == 0) return SPMV_SUCCESS;
    const int64_t waves = (p->nnz + 63) / 64;
    const int64_t blocks = std::min<int64_t>((waves + 3) / 4, 256 * 64);
    hipLaunchKernelGGL(coo_segment_kernel, dim3((unsigned)blocks), dim3(256), 0, p->stream, p->nnz, p->coo.row,
                       p->coo.col, p->coo.val, x, y);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

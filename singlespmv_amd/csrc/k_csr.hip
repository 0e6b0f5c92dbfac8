// k_csr.hip -- CSR SpMV for gfx950: the opt_crs hot loop
// (src/opt_crs.cpp:57-69, `y[i] = sum_j val[j] * x[idx[j]]`) re-designed for
// wave64.
//
// csr_vec4<L, RP>: a group of L lanes (L | 64) owns one row.  The group walks
// the row from its 16-byte-aligned start a = ptr[i] & ~3 in chunks of 4*L
// entries; each lane issues ONE 16-byte load of 4 column indices and TWO
// 16-byte loads of 4 values (non-temporal: streamed once), so a wave
// instruction covers 1 KiB contiguous when rows are contiguous.  Entries
// outside [ptr[i], ptr[i+1]) are masked (no gather).  Each lane sums its
// entries in order, then the group reduces with a fixed butterfly; lane 0
// writes y[i] (β = 0, idempotent).
//
// Algorithmic bytes per row: 12*nnz_i + rp bytes + 8 (y) and the
// x gathers (8*n total, counted once).
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

// LIST: the rows come from a length bin (rows[]), not 0..m-1 (adaptive CSR)
template <int L, typename RP, bool LIST>
__global__ __launch_bounds__(256) void csr_vec4_kernel(int64_t m, const int32_t *__restrict__ rows,
                                                       const RP *__restrict__ rp,
                                                       const int32_t *__restrict__ col,
                                                       const double *__restrict__ val,
                                                       const double *__restrict__ x,
                                                       double *__restrict__ y) {
    const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t g = gtid / L;
    const int lane = threadIdx.x & (L - 1);
    if (g >= m) return;  // whole groups exit together (L | 256)
    const int64_t row = LIST ? (int64_t)rows[g] : g;
    const int64_t s = rp[row];
    const int64_t e = rp[row + 1];
    double acc = 0.0;
    for (int64_t j = (s & ~(int64_t)3) + 4 * lane; j < e; j += 4 * L) {
        const i32x4 c = ld_stream4(col + j);
        const f64x2 v01 = ld_stream2(val + j);
        const f64x2 v23 = ld_stream2(val + j + 2);
        // masked gathers: only entries of this row
        const double x0 = (j + 0 >= s && j + 0 < e) ? ld_x(x, c.x) : 0.0;
        const double x1 = (j + 1 >= s && j + 1 < e) ? ld_x(x, c.y) : 0.0;
        const double x2 = (j + 2 >= s && j + 2 < e) ? ld_x(x, c.z) : 0.0;
        const double x3 = (j + 3 >= s && j + 3 < e) ? ld_x(x, c.w) : 0.0;
        if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, x0, acc);
        if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, x1, acc);
        if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, x2, acc);
        if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, x3, acc);
    }
    acc = group_sum<L>(acc);
    if (lane == 0) y[row] = acc;
}

// One 256-thread workgroup per row (the longest-row bin of adaptive CSR):
// four waves stride the row in 1 KiB chunks, each reduces with the fixed
// butterfly, and the four wave sums are added in wave order (deterministic).
template <typename RP>
__global__ __launch_bounds__(256) void csr_block_kernel(const int32_t *__restrict__ rows, const RP *__restrict__ rp,
                                                        const int32_t *__restrict__ col,
                                                        const double *__restrict__ val,
                                                        const double *__restrict__ x, double *__restrict__ y) {
    __shared__ double part[4];
    const int64_t row = rows[blockIdx.x];
    const int64_t s = rp[row];
    const int64_t e = rp[row + 1];
    double acc = 0.0;
    for (int64_t j = (s & ~(int64_t)3) + 4 * threadIdx.x; j < e; j += 4 * 256) {
        const i32x4 c = ld_stream4(col + j);
        const f64x2 v01 = ld_stream2(val + j);
        const f64x2 v23 = ld_stream2(val + j + 2);
        if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, ld_x(x, c.x), acc);
        if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, ld_x(x, c.y), acc);
        if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, ld_x(x, c.z), acc);
        if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, ld_x(x, c.w), acc);
    }
    acc = group_sum<64>(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) y[row] = __dadd_rn(__dadd_rn(part[0], part[1]), __dadd_rn(part[2], part[3]));
}

// Adaptive CSR in ONE launch: workgroup ranges map to the length bins
// (blk_off), so all bins run concurrently instead of back to back; the bin
// test is workgroup-uniform (no divergence).  Bin b has L = kCsrBinLanes[b]
// lanes per row; the last bin is one workgroup per row.
struct CsrBinTable {
    int64_t blk_off[kCsrBins + 1];  // first workgroup of each bin, in launch order
    int64_t row_off[kCsrBins + 1];  // first row (in bin_rows) of each bin
};
// launch order: the longest rows first (their workgroups run longest), so
// the short-row bins fill in behind them instead of forming the tail
constexpr int kCsrLaunchOrder[kCsrBins] = {7, 6, 5, 4, 3, 2, 1, 0};

// ADD: y[yrow[row]] += sum (the HYB/JDS overflow, one writer per row);
// otherwise y[row] = sum
template <int L, typename RP, bool ADD>
__device__ __forceinline__ void csr_rows_body(int64_t wg, int64_t nrows, const int32_t *__restrict__ rows,
                                              const RP *__restrict__ rp, const int32_t *__restrict__ col,
                                              const double *__restrict__ val, const double *__restrict__ x,
                                              double *__restrict__ y, const int32_t *__restrict__ yrow) {
    const int64_t g = (wg * 256 + threadIdx.x) / L;
    const int lane = threadIdx.x & (L - 1);
    if (g >= nrows) return;
    const int64_t row = rows[g];
    const int64_t s = rp[row];
    const int64_t e = rp[row + 1];
    double acc = 0.0;
    for (int64_t j = (s & ~(int64_t)3) + 4 * lane; j < e; j += 4 * L) {
        const i32x4 c = ld_stream4(col + j);
        const f64x2 v01 = ld_stream2(val + j);
        const f64x2 v23 = ld_stream2(val + j + 2);
        const double x0 = (j + 0 >= s && j + 0 < e) ? ld_x(x, c.x) : 0.0;
        const double x1 = (j + 1 >= s && j + 1 < e) ? ld_x(x, c.y) : 0.0;
        const double x2 = (j + 2 >= s && j + 2 < e) ? ld_x(x, c.z) : 0.0;
        const double x3 = (j + 3 >= s && j + 3 < e) ? ld_x(x, c.w) : 0.0;
        if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, x0, acc);
        if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, x1, acc);
        if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, x2, acc);
        if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, x3, acc);
    }
    acc = group_sum<L>(acc);
    if (lane == 0) {
        if (ADD) {
            const int64_t yi = yrow[row];
            y[yi] = __dadd_rn(y[yi], acc);
        } else {
            y[row] = acc;
        }
    }
}

template <typename RP, bool ADD>
__global__ __launch_bounds__(256) void csr_adaptive_kernel(CsrBinTable t, const int32_t *__restrict__ rows,
                                                           const RP *__restrict__ rp,
                                                           const int32_t *__restrict__ col,
                                                           const double *__restrict__ val,
                                                           const double *__restrict__ x, double *__restrict__ y,
                                                           const int32_t *__restrict__ yrow) {
    __shared__ double part[4];
    const int64_t blk = blockIdx.x;
    int k = 0;
    while (k < kCsrBins - 1 && blk >= t.blk_off[k + 1]) ++k;  // uniform
    const int b = kCsrLaunchOrder[k];
    const int64_t wg = blk - t.blk_off[k];
    const int32_t *br = rows + t.row_off[b];
    const int64_t n = t.row_off[b + 1] - t.row_off[b];
    switch (b) {
        case 0: csr_rows_body<1, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 1: csr_rows_body<2, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 2: csr_rows_body<4, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 3: csr_rows_body<8, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 4: csr_rows_body<16, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 5: csr_rows_body<32, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 6: csr_rows_body<64, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        default: {
            // one workgroup per row: four wave sums added in wave order
            const int64_t row = br[wg];
            const int64_t s = rp[row];
            const int64_t e = rp[row + 1];
            double acc = 0.0;
            for (int64_t j = (s & ~(int64_t)3) + 4 * threadIdx.x; j < e; j += 4 * 256) {
                const i32x4 c = ld_stream4(col + j);
                const f64x2 v01 = ld_stream2(val + j);
                const f64x2 v23 = ld_stream2(val + j + 2);
                if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, ld_x(x, c.x), acc);
                if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, ld_x(x, c.y), acc);
                if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, ld_x(x, c.z), acc);
                if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, ld_x(x, c.w), acc);
            }
            acc = group_sum<64>(acc);
            if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
            __syncthreads();
            if (threadIdx.x == 0) {
                const double sum = __dadd_rn(__dadd_rn(part[0], part[1]), __dadd_rn(part[2], part[3]));
                if (ADD) {
                    const int64_t yi = yrow[row];
                    y[yi] = __dadd_rn(y[yi], sum);
                } else {
                    y[row] = sum;
                }
            }
        }
    }
}

// one launch of the adaptive kernel over length bins (bin_off: host offsets)
template <typename RP, bool ADD>
static int launch_adaptive(const spmv_plan_s *p, const int64_t *bin_off, const int32_t *bin_rows, const RP *rp,
                           const int32_t *col, const double *val, const double *x, double *y,
                           const int32_t *yrow) {
    CsrBinTable t;
    t.blk_off[0] = 0;
    for (int b = 0; b <= kCsrBins; ++b) t.row_off[b] = bin_off[b];
    for (int k = 0; k < kCsrBins; ++k) {
        const int b = kCsrLaunchOrder[k];
        const int64_t n = bin_off[b + 1] - bin_off[b];
        const int L = kCsrBinLanes[b];
        t.blk_off[k + 1] = t.blk_off[k] + (L >= 256 ? n : (n * L + 255) / 256);
    }
    if (t.blk_off[kCsrBins] == 0) return SPMV_SUCCESS;
    hipLaunchKernelGGL((csr_adaptive_kernel<RP, ADD>), dim3((unsigned)t.blk_off[kCsrBins]), dim3(256), 0, p->stream,
                       t, bin_rows, rp, col, val, x, y, yrow);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

template <int L, typename RP>
static int launch_csr_t(const spmv_plan_s *p, int64_t nrows, const int32_t *rows, const double *x, double *y) {
    const int64_t threads = nrows * L;
    const int64_t blocks = (threads + 255) / 256;
    if (blocks == 0) return SPMV_SUCCESS;
    if (rows)
        hipLaunchKernelGGL((csr_vec4_kernel<L, RP, true>), dim3((unsigned)blocks), dim3(256), 0, p->stream, nrows,
                           rows, (const RP *)p->csr.row_ptr, p->csr.col, p->csr.val, x, y);
    else
        hipLaunchKernelGGL((csr_vec4_kernel<L, RP, false>), dim3((unsigned)blocks), dim3(256), 0, p->stream, nrows,
                           rows, (const RP *)p->csr.row_ptr, p->csr.col, p->csr.val, x, y);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

template <typename RP>
static int launch_csr_lanes(const spmv_plan_s *p, int lanes, int64_t nrows, const int32_t *rows, const double *x,
                            double *y) {
    switch (lanes) {
        case 1: return launch_csr_t<1, RP>(p, nrows, rows, x, y);
        case 2: return launch_csr_t<2, RP>(p, nrows, rows, x, y);
        case 4: return launch_csr_t<4, RP>(p, nrows, rows, x, y);
        case 8: return launch_csr_t<8, RP>(p, nrows, rows, x, y);
        case 16: return launch_csr_t<16, RP>(p, nrows, rows, x, y);
        case 32: return launch_csr_t<32, RP>(p, nrows, rows, x, y);
        case 64: return launch_csr_t<64, RP>(p, nrows, rows, x, y);
        case 256:
            if (nrows > 0) {
                hipLaunchKernelGGL((csr_block_kernel<RP>), dim3((unsigned)nrows), dim3(256), 0, p->stream, rows,
                                   (const RP *)p->csr.row_ptr, p->csr.col, p->csr.val, x, y);
                SPMV_HIP_TRY(hipGetLastError());
            }
            return SPMV_SUCCESS;
        default: set_error("csr lanes must be a power of two in [1,64]"); return SPMV_ERROR_INVALID_VALUE;
    }
}

template <typename RP>
static int launch_csr_rp(const spmv_plan_s *p, const double *x, double *y) {
    const CsrDev &c = p->csr;
    if (!c.bin_rows) return launch_csr_lanes<RP>(p, c.lanes, p->m, nullptr, x, y);
    // adaptive: every bin in one launch (workgroup ranges per bin)
    return launch_adaptive<RP, false>(p, c.bin_off, c.bin_rows, (const RP *)c.row_ptr, c.col, c.val, x, y, nullptr);
}

int launch_csr(const spmv_plan_s *p, const double *x, double *y) {
    return p->csr.rp64 ? launch_csr_rp<int64_t>(p, x, y) : launch_csr_rp<int32_t>(p, x, y);
}

// ---- HYB overflow: CSR-vector over the overflow rows, y[row] += sum -------
template <int L>
__global__ __launch_bounds__(256) void hyb_overflow_kernel(int64_t nrows, const int32_t *__restrict__ rows,
                                                           const int64_t *__restrict__ rp,
                                                           const int32_t *__restrict__ col,
                                                           const double *__restrict__ val,
                                                           const double *__restrict__ x,
                                                           double *__restrict__ y) {
    const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = gtid / L;
    const int lane = threadIdx.x & (L - 1);
    if (r >= nrows) return;
    const int64_t s = rp[r];
    const int64_t e = rp[r + 1];
    double acc = 0.0;
    for (int64_t j = (s & ~(int64_t)3) + 4 * lane; j < e; j += 4 * L) {
        const i32x4 c = ld_stream4(col + j);
        const f64x2 v01 = ld_stream2(val + j);
        const f64x2 v23 = ld_stream2(val + j + 2);
        if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, ld_x(x, c.x), acc);
        if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, ld_x(x, c.y), acc);
        if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, ld_x(x, c.z), acc);
        if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, ld_x(x, c.w), acc);
    }
    acc = group_sum<L>(acc);
    if (lane == 0) {
        const int32_t row = rows[r];
        y[row] = __dadd_rn(y[row], acc);  // single writer per row
    }
}

int launch_hyb_overflow(const spmv_plan_s *p, const double *x, double *y) {
    const HybDev &h = p->hyb;
    if (h.n_rows == 0) return SPMV_SUCCESS;
    if (h.bin_rows)  // overflow rows binned by their overflow length
        return launch_adaptive<int64_t, true>(p, h.bin_off, h.bin_rows, h.row_ptr, h.col, h.val, x, y, h.rows);
    const int L = 64;
    const int64_t blocks = (h.n_rows * L + 255) / 256;
    hipLaunchKernelGGL((hyb_overflow_kernel<64>), dim3((unsigned)blocks), dim3(256), 0, p->stream,
                       h.n_rows, h.rows, h.row_ptr, h.col, h.val, x, y);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

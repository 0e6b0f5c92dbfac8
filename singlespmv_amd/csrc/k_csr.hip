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

#include <algorithm>
#include <climits>
#include <vector>

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

// csr_win<L, RP>: csr_vec4 with x staged through LDS (north star: "x[]
// staged through LDS").  Workgroup w owns rows [w*256/L, (w+1)*256/L) and the
// plan knows the column window [win[2w], win[2w] + win[2w+1]) they read
// (csr_plan_window).  The lane's first chunk of col/val is loaded first, the
// window is copied into LDS with coalesced loads while those are in flight,
// and after one barrier every gather is a ds_read_b64 instead of an L1/L2
// request.  A span of -1 (columns too spread) keeps the global gathers.  Each
// lane sums the same entries in the same order and the group reduces with the
// same butterfly as csr_vec4_kernel<L>: y is bit-identical to it.
template <int L, typename RP>
__global__ __launch_bounds__(256) void csr_win_kernel(int64_t m, const int32_t *__restrict__ win,
                                                      const RP *__restrict__ rp, const int32_t *__restrict__ col,
                                                      const double *__restrict__ val, const double *__restrict__ x,
                                                      double *__restrict__ y) {
    extern __shared__ double xs[];
    const int64_t g = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
    const int lane = threadIdx.x & (L - 1);
    const int32_t lo = win[2 * blockIdx.x], span = win[2 * blockIdx.x + 1];
    const bool live = g < m;  // whole groups (L | 256); the barrier needs every thread
    int64_t s = 0, e = 0;
    if (live) {
        s = rp[g];
        e = rp[g + 1];
    }
    double acc = 0.0;
    if (span < 0) {  // workgroup-uniform: global gathers
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
    } else {
        int64_t j = (s & ~(int64_t)3) + 4 * lane;
        i32x4 c = {0, 0, 0, 0};
        f64x2 v01 = {0.0, 0.0}, v23 = {0.0, 0.0};
        if (j < e) {
            c = ld_stream4(col + j);
            v01 = ld_stream2(val + j);
            v23 = ld_stream2(val + j + 2);
        }
        for (int i = threadIdx.x; i < span; i += 256) xs[i] = x[(int64_t)lo + i];
        __syncthreads();
        while (j < e) {
            // entries outside [s, e) (the aligned start, the padding) are
            // never read from the window: their columns may lie outside it
            const double x0 = (j + 0 >= s && j + 0 < e) ? xs[c.x - lo] : 0.0;
            const double x1 = (j + 1 >= s && j + 1 < e) ? xs[c.y - lo] : 0.0;
            const double x2 = (j + 2 >= s && j + 2 < e) ? xs[c.z - lo] : 0.0;
            const double x3 = (j + 3 >= s && j + 3 < e) ? xs[c.w - lo] : 0.0;
            if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, x0, acc);
            if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, x1, acc);
            if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, x2, acc);
            if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, x3, acc);
            j += 4 * L;
            if (j < e) {
                c = ld_stream4(col + j);
                v01 = ld_stream2(val + j);
                v23 = ld_stream2(val + j + 2);
            }
        }
    }
    acc = group_sum<L>(acc);
    if (live && lane == 0) y[g] = acc;
}

// Plan-time LDS x windows (csr_win_kernel, ell_slice_kernel<..., WIN>):
// workgroup w covers the entries [bounds[w*stride], bounds[min((w+1)*stride,
// nb)]) of `col` (CSR: row pointers, `stride` rows per workgroup; ELL: slice
// offsets, 4 slices per workgroup); its window is the smallest and largest
// column there, span = hi - lo + 1, or -1 beyond kCsrMaxWin.  One 256-thread
// block per workgroup.
template <typename B>
__global__ __launch_bounds__(256) void window_scan(int64_t nb, int stride, const B *__restrict__ bounds,
                                                   const int32_t *__restrict__ col, int32_t *__restrict__ win) {
    __shared__ int32_t red[2][4];
    const int64_t r0 = (int64_t)blockIdx.x * stride;
    const int64_t r1 = r0 + stride < nb ? r0 + stride : nb;
    const int64_t b = bounds[r0], e = bounds[r1];
    int32_t lo = INT32_MAX, hi = -1;
    for (int64_t j = b + threadIdx.x; j < e; j += 256) {
        const int32_t c = col[j];
        lo = c < lo ? c : lo;
        hi = c > hi ? c : hi;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = lo;
        red[1][threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            lo = red[0][w] < lo ? red[0][w] : lo;
            hi = red[1][w] > hi ? red[1][w] : hi;
        }
        if (hi < 0) {  // no entries
            win[2 * blockIdx.x] = 0;
            win[2 * blockIdx.x + 1] = 0;
        } else {
            const int64_t span = (int64_t)hi - lo + 1;
            win[2 * blockIdx.x] = lo;
            win[2 * blockIdx.x + 1] = span <= kCsrMaxWin ? (int32_t)span : -1;
        }
    }
}

int plan_x_window(spmv_plan_s *p, int64_t nb, int stride, const void *bounds, bool bounds64, const int32_t *col,
                  XWindow *out) {
    *out = XWindow{};
    if (nb <= 0) return SPMV_SUCCESS;
    const int64_t nwg = (nb + stride - 1) / stride;
    void *q = nullptr;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(int32_t) * 2 * (size_t)nwg));
    int32_t *dwin = (int32_t *)q;
    if (bounds64)
        hipLaunchKernelGGL(window_scan<int64_t>, dim3((unsigned)nwg), dim3(256), 0, p->stream, nb, stride,
                           (const int64_t *)bounds, col, dwin);
    else
        hipLaunchKernelGGL(window_scan<int32_t>, dim3((unsigned)nwg), dim3(256), 0, p->stream, nb, stride,
                           (const int32_t *)bounds, col, dwin);
    SPMV_HIP_TRY(hipGetLastError());
    std::vector<int32_t> h(2 * (size_t)nwg);
    SPMV_HIP_TRY(hipMemcpyAsync(h.data(), dwin, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost, p->stream));
    SPMV_HIP_TRY(hipStreamSynchronize(p->stream));
    int64_t wgs = 0;
    int mx = 0;
    for (int64_t w = 0; w < nwg; ++w)
        if (h[2 * w + 1] >= 0) {
            ++wgs;
            mx = std::max(mx, h[2 * w + 1]);
        }
    if (wgs == 0) {
        p->arena.free(dwin);
        return SPMV_SUCCESS;
    }
    out->win = dwin;
    out->wgs = wgs;
    out->max = std::max(mx, 1);
    return SPMV_SUCCESS;
}

// After the CSR is on the device (either build path): per-workgroup windows
// for the in-order kernel (lanes > 0); x_window = -1 turns them off.
int csr_plan_window(spmv_plan_s *p, const spmv_options_t &o) {
    CsrDev &c = p->csr;
    if (o.x_window < 0 || c.lanes <= 0 || p->m == 0) return SPMV_SUCCESS;
    SPMV_RETURN_IF(plan_x_window(p, p->m, 256 / c.lanes, c.row_ptr, c.rp64, c.col, &c.xw));
    if (c.xw.win) p->kernel_name = "csr_win_kernel<" + std::to_string(c.lanes) + ">";
    return SPMV_SUCCESS;
}

template <int L, typename RP>
static int launch_csr_win_t(const spmv_plan_s *p, const double *x, double *y) {
    const int64_t blocks = (p->m * L + 255) / 256;
    hipLaunchKernelGGL((csr_win_kernel<L, RP>), dim3((unsigned)blocks), dim3(256),
                       sizeof(double) * (size_t)p->csr.xw.max, p->stream, p->m, p->csr.xw.win,
                       (const RP *)p->csr.row_ptr, p->csr.col, p->csr.val, x, y);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

template <typename RP>
static int launch_csr_win(const spmv_plan_s *p, const double *x, double *y) {
    switch (p->csr.lanes) {
        case 1: return launch_csr_win_t<1, RP>(p, x, y);
        case 2: return launch_csr_win_t<2, RP>(p, x, y);
        case 4: return launch_csr_win_t<4, RP>(p, x, y);
        case 8: return launch_csr_win_t<8, RP>(p, x, y);
        case 16: return launch_csr_win_t<16, RP>(p, x, y);
        case 32: return launch_csr_win_t<32, RP>(p, x, y);
        case 64: return launch_csr_win_t<64, RP>(p, x, y);
        default: set_error("csr lanes must be a power of two in [1,64]"); return SPMV_ERROR_INVALID_VALUE;
    }
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
    if (c.xw.win) return launch_csr_win<RP>(p, x, y);
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

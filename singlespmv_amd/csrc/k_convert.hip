// k_convert.hip -- on-device format conversion, modelled on
// the CSR5 conversion pipeline (CSR5_cuda/detail/cuda/format_cuda.h:21-718:
// partition pointers by binary search of row_ptr, descriptor bit-flags by
// atomicOr, tile transposes) -- for a CSR that already lives in HBM, so a
// 1 G-nnz matrix never round-trips through the host.
//
//   CSR: int64 -> int32 row pointers (or a device copy), col/val copies.
//   SS : non-empty-row ordinals by a device exclusive scan, empty-row
//        compaction, row-start flags by atomicOr, first-row ordinal per tile
//        by binary search, and the 64-lane x sigma tile transpose.
// Unlike CSR5's in-place transpose (anonymouslib_cuda.h:203-204) the
// caller's arrays are never modified.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "device.hpp"
#include "internal.hpp"

namespace spmv {

int csr_x_windows_device(spmv_plan_s *p, const int64_t *d_rp);

namespace {

constexpr int kScanBlock = 1024;

// ---- exclusive scan of int64 (three-phase, recursive on block sums) ---------
__global__ __launch_bounds__(kScanBlock) void scan_block_sums(const int64_t *__restrict__ in, int64_t n,
                                                              int64_t *__restrict__ sums) {
    __shared__ int64_t s[kScanBlock];
    const int64_t i = (int64_t)blockIdx.x * kScanBlock + threadIdx.x;
    s[threadIdx.x] = i < n ? in[i] : 0;
    __syncthreads();
    for (int o = kScanBlock / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(kScanBlock) void scan_block_apply(const int64_t *__restrict__ in, int64_t n,
                                                               const int64_t *__restrict__ offs,
                                                               int64_t *__restrict__ out) {
    __shared__ int64_t s[kScanBlock];
    const int64_t i = (int64_t)blockIdx.x * kScanBlock + threadIdx.x;
    const int64_t v = i < n ? in[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kScanBlock; o <<= 1) {  // Hillis-Steele inclusive
        const int64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    if (i < n) out[i] = offs[blockIdx.x] + s[threadIdx.x] - v;  // exclusive
}

int exclusive_scan(spmv_plan_s *p, const int64_t *in, int64_t *out, int64_t n, hipStream_t st,
                   std::vector<void *> &tmp) {
    if (n == 0) return SPMV_SUCCESS;
    const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
    int64_t *sums, *offs;
    SPMV_RETURN_IF(scratch_malloc(&sums, sizeof(int64_t) * nb, "sums"));
    tmp.push_back(sums);
    SPMV_RETURN_IF(scratch_malloc(&offs, sizeof(int64_t) * nb, "offs"));
    tmp.push_back(offs);
    hipLaunchKernelGGL(scan_block_sums, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, sums);
    if (nb > 1) SPMV_RETURN_IF(exclusive_scan(p, sums, offs, nb, st, tmp));
    else SPMV_HIP_TRY(hipMemsetAsync(offs, 0, sizeof(int64_t), st));
    hipLaunchKernelGGL(scan_block_apply, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, offs, out);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

// ---- CSR ------------------------------------------------------------------
__global__ void rp_to_i32(const int64_t *__restrict__ rp, int64_t n, int32_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int32_t)rp[i];
}

// ---- SS -------------------------------------------------------------------
__global__ void nonempty_flags(const int64_t *__restrict__ rp, int64_t m, int64_t *__restrict__ f) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < m; r += (int64_t)gridDim.x * blockDim.x)
        f[r] = rp[r + 1] > rp[r] ? 1 : 0;
}

// nzord = exclusive scan of the flags: scatter ordinal -> row, empty -> list
__global__ void compact_rows(const int64_t *__restrict__ rp, const int64_t *__restrict__ nzord, int64_t m,
                             int32_t *__restrict__ nzrow, int32_t *__restrict__ empty) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < m; r += (int64_t)gridDim.x * blockDim.x) {
        if (rp[r + 1] > rp[r]) nzrow[nzord[r]] = (int32_t)r;
        else empty[r - nzord[r]] = (int32_t)r;
    }
}

// the bit of every row start (and of the padding's dummy segment) via atomicOr
__global__ void start_flags(const int64_t *__restrict__ rp, int64_t m, int64_t nnz, int sigma,
                            uint32_t *__restrict__ flags) {
    const int64_t T = 64 * (int64_t)sigma;
    const int W = ss_flag_words(sigma);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= m; r += (int64_t)gridDim.x * blockDim.x) {
        int64_t pos;
        if (r < m) {
            if (rp[r + 1] <= rp[r]) continue;
            pos = rp[r];
        } else {
            if (nnz % T == 0) continue;
            pos = nnz;
        }
        const int64_t t = pos / T, li = pos % T, k = li % sigma;
        atomicOr(&flags[(t * W + k / 32) * 64 + li / sigma], 1u << (k % 32));
    }
}

// first-row ordinal of every tile: binary search of row_ptr (CSR5's
// generate_partition_pointer_s1_kernel, format_cuda.h:21-42)
__global__ void tile_ordinals(const int64_t *__restrict__ rp, int64_t m, const int64_t *__restrict__ nzord,
                              int64_t n_nonempty, int sigma, int64_t n_tiles, int32_t *__restrict__ tord) {
    const int64_t T = 64 * (int64_t)sigma;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tiles; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t target = t * T;
        int64_t lo = 0, hi = m;  // first r with rp[r] >= target
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (rp[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        tord[t] = (int32_t)(lo < m ? nzord[lo] : n_nonempty);
    }
}

// tile transpose: col position t*T + (k/4)*256 + lane*4 + k%4, val position
// t*T + (k/4)*256 + (k%4/2)*128 + lane*2 + k%2 <- nnz t*T + lane*sigma + k
__global__ void tile_transpose(const int32_t *__restrict__ col, const double *__restrict__ val, int64_t nnz,
                               int sigma, int64_t total, int32_t *__restrict__ tcol, double *__restrict__ tval) {
    const int64_t T = 64 * (int64_t)sigma;
    for (int64_t pos = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pos < total;
         pos += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = pos / T, w = pos % T;
        const int64_t q = w >> 8, lane = (w >> 2) & 63, k = q * 4 + (w & 3);
        const int64_t i = t * T + lane * sigma + k;
        tcol[pos] = i < nnz ? col[i] : 0;
        const int64_t r = w & 255, vlane = (r & 127) >> 1, vk = q * 4 + (r >> 7) * 2 + (r & 1);
        const int64_t vi = t * T + vlane * sigma + vk;
        tval[pos] = vi < nnz ? val[vi] : 0.0;
    }
}

// x window of every tile (ss_tile_windows, formats.cpp): one wave per tile
// reduces the column range of its 64 x sigma positions (padding: column 0)
__global__ __launch_bounds__(256) void tile_windows(const int32_t *__restrict__ col, int64_t nnz, int sigma,
                                                    int64_t n_tiles, int32_t *__restrict__ win) {
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= n_tiles) return;
    const int64_t T = 64 * (int64_t)sigma;
    int lo = INT32_MAX, hi = -1;
    for (int64_t i = t * T + lane; i < (t + 1) * T; i += 64) {
        const int c = i < nnz ? col[i] : 0;
        lo = c < lo ? c : lo;
        hi = c > hi ? c : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o, 64));
        hi = max(hi, __shfl_xor(hi, o, 64));
    }
    if (lane == 0) {
        const bool fits = hi - lo < kSsWinCols;
        win[2 * t] = fits ? lo : 0;
        win[2 * t + 1] = fits ? hi - lo + 1 : 0;
    }
}

// CSR values of a row-group plan in halves (CsrDev::val_halves)
__global__ void csr_val_halves_kernel(const double *__restrict__ val, int64_t nnz, int64_t total,
                                      double *__restrict__ out) {
    for (int64_t pos = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pos < total;
         pos += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = csr_val_halves_entry(pos);
        out[pos] = e < nnz ? val[e] : 0.0;
    }
}

// input checks of validate_csr (capi.cpp) on device data: bad[0] counts
// decreasing row pointers, bad[1] columns outside [0, n)
__global__ void check_csr(const int64_t *__restrict__ rp, int64_t m, const int32_t *__restrict__ col, int64_t nnz,
                          int64_t n, unsigned long long *__restrict__ bad) {
    unsigned long long b0 = 0, b1 = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) b0 += rp[i + 1] < rp[i];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride)
        b1 += (col[i] < 0) | ((int64_t)col[i] >= n);
    if (b0) atomicAdd(&bad[0], b0);
    if (b1) atomicAdd(&bad[1], b1);
}

__global__ void rp32_to_64(const int32_t *__restrict__ rp, int64_t n, int64_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = rp[i];
}

__global__ void scale_kernel(double *__restrict__ y, int64_t n, double alpha) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = __dmul_rn(alpha, y[i]);
}

inline unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65536)); }

}  // namespace

int exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, hipStream_t st, std::vector<void *> &tmp) {
    return exclusive_scan(nullptr, in, out, n, st, tmp);
}

int widen_row_ptr_device(const int32_t *d_rp32, int64_t m, int64_t **d_rp64) {
    *d_rp64 = nullptr;
    SPMV_RETURN_IF(scratch_malloc(d_rp64, 8 * (size_t)(m + 1), "d_rp64"));
    hipLaunchKernelGGL(rp32_to_64, dim3(grid_for(m + 1)), dim3(256), 0, 0, d_rp32, m + 1, *d_rp64);
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(*d_rp64);
        *d_rp64 = nullptr;
        set_error(std::string("row_ptr widening: ") + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    return SPMV_SUCCESS;
}

int launch_scale(const spmv_plan_s *p, double *y, double alpha) {
    if (p->m == 0 || alpha == 1.0) return SPMV_SUCCESS;
    hipLaunchKernelGGL(scale_kernel, dim3(grid_for(p->m)), dim3(256), 0, p->stream, y, p->m, alpha);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

int validate_csr_device(const int64_t *d_rp, int64_t m, const int32_t *d_col, int64_t nnz, int64_t n) {
    int64_t ends[2] = {0, 0};
    SPMV_HIP_TRY(hipMemcpy(&ends[0], d_rp, 8, hipMemcpyDeviceToHost));
    SPMV_HIP_TRY(hipMemcpy(&ends[1], d_rp + m, 8, hipMemcpyDeviceToHost));
    SPMV_CHECK_ARG(ends[0] == 0, "row_ptr[0] != 0");
    SPMV_CHECK_ARG(ends[1] == nnz, "row_ptr[m] != nnz");
    unsigned long long *bad, hbad[2] = {0, 0};
    SPMV_RETURN_IF(scratch_malloc(&bad, sizeof(hbad), "bad"));
    (void)hipMemset(bad, 0, sizeof(hbad));
    hipLaunchKernelGGL(check_csr, dim3(grid_for(std::max(m, nnz))), dim3(256), 0, 0, d_rp, m, d_col, nnz, n, bad);
    hipError_t e = hipMemcpy(hbad, bad, sizeof(hbad), hipMemcpyDeviceToHost);
    (void)hipFree(bad);
    if (e != hipSuccess) {
        set_error(std::string("device CSR validation: ") + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    SPMV_CHECK_ARG(hbad[0] == 0, "row_ptr is not non-decreasing");
    SPMV_CHECK_ARG(hbad[1] == 0, "column index outside [0, n)");
    return SPMV_SUCCESS;
}

// Device-input plan builders.  d_rp/d_col/d_val are device pointers on the
// plan's device; they are only read.
int build_csr_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                     const spmv_options_t &o, double mean_row) {
    CsrDev &c = p->csr;
    const hipStream_t st = p->stream;
    c.rp64 = p->nnz >= (int64_t)INT32_MAX - 64 || o.csr_row_ptr64 != 0 || probe_env("SPMV_CSR_FORCE_RP64");
    void *q;
    SPMV_RETURN_IF(p->arena.alloc(&q, (c.rp64 ? 8 : 4) * (size_t)(p->m + 1)));
    c.row_ptr = q;
    if (c.rp64) SPMV_HIP_TRY(hipMemcpyAsync(q, d_rp, 8 * (size_t)(p->m + 1), hipMemcpyDeviceToDevice, st));
    else hipLaunchKernelGGL(rp_to_i32, dim3(grid_for(p->m + 1)), dim3(256), 0, st, d_rp, p->m + 1, (int32_t *)q);
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(int32_t) * (size_t)(p->nnz + kPad)));
    c.col = (int32_t *)q;
    if (p->nnz) SPMV_HIP_TRY(hipMemcpyAsync(c.col, d_col, 4 * (size_t)p->nnz, hipMemcpyDeviceToDevice, st));
    SPMV_HIP_TRY(hipMemsetAsync(c.col + p->nnz, 0, 4 * kPad, st));
    SPMV_HIP_TRY(hipStreamSynchronize(st));
    (void)mean_row;
    // lanes per row / length bins from the row pointers (m+1 values to the host)
    std::vector<int64_t> hrp((size_t)p->m + 1);
    SPMV_HIP_TRY(hipMemcpy(hrp.data(), d_rp, 8 * (size_t)(p->m + 1), hipMemcpyDeviceToHost));
    SPMV_RETURN_IF(csr_plan_lanes(p, hrp.data(), p->m, o));
    c.val_halves = csr_val_halves_wanted(c);
    const int64_t vtotal = c.val_halves ? (p->nnz + 255) / 256 * 256 : p->nnz;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(double) * (size_t)(vtotal + kPad)));
    c.val = (double *)q;
    if (c.val_halves) {
        hipLaunchKernelGGL(csr_val_halves_kernel, dim3(grid_for(vtotal)), dim3(256), 0, st, d_val, p->nnz, vtotal,
                           c.val);
    } else if (p->nnz) {
        SPMV_HIP_TRY(hipMemcpyAsync(c.val, d_val, 8 * (size_t)p->nnz, hipMemcpyDeviceToDevice, st));
    }
    SPMV_HIP_TRY(hipMemsetAsync(c.val + vtotal, 0, 8 * kPad, st));
    SPMV_HIP_TRY(hipGetLastError());
    SPMV_HIP_TRY(hipStreamSynchronize(st));
    if (c.lanes > 0) SPMV_RETURN_IF(csr_x_windows_device(p, d_rp));
    csr_finish_info(p);
    return SPMV_SUCCESS;
}

// csr_x_windows on the device (formats.cpp): the column range [lo, hi] of
// each kCsrWinGroup-row granule's entries (hi = -1: none), one workgroup each
__global__ __launch_bounds__(256) void csr_window_kernel(const int64_t *__restrict__ rp, int64_t m,
                                                         const int32_t *__restrict__ col, int32_t *__restrict__ lo,
                                                         int32_t *__restrict__ hi) {
    __shared__ int32_t smin[256], smax[256];
    const int64_t b = blockIdx.x;
    const int64_t e0 = rp[b * kCsrWinGroup];
    const int64_t r1 = (b + 1) * kCsrWinGroup < m ? (b + 1) * kCsrWinGroup : m;
    const int64_t e1 = rp[r1];
    int32_t mn = INT32_MAX, mx = -1;
    for (int64_t j = e0 + threadIdx.x; j < e1; j += 256) {
        const int32_t c = col[j];
        mn = c < mn ? c : mn;
        mx = c > mx ? c : mx;
    }
    smin[threadIdx.x] = mn;
    smax[threadIdx.x] = mx;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            smin[threadIdx.x] = min(smin[threadIdx.x], smin[threadIdx.x + o]);
            smax[threadIdx.x] = max(smax[threadIdx.x], smax[threadIdx.x + o]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        lo[b] = smax[0] < 0 ? 0 : smin[0];
        hi[b] = smax[0];
    }
}

int csr_x_windows_device(spmv_plan_s *p, const int64_t *d_rp) {
    const int64_t ng = (p->m + kCsrWinGroup - 1) / kCsrWinGroup;
    if (ng == 0) return SPMV_SUCCESS;
    int32_t *d = nullptr;
    SPMV_RETURN_IF(scratch_malloc(&d, 2 * sizeof(int32_t) * (size_t)ng, "d"));
    hipLaunchKernelGGL(csr_window_kernel, dim3((unsigned)ng), dim3(256), 0, p->stream, d_rp, p->m, p->csr.col, d,
                       d + ng);
    std::vector<int32_t> lo((size_t)ng), hi((size_t)ng);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(lo.data(), d, sizeof(int32_t) * (size_t)ng, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hi.data(), d + ng, sizeof(int32_t) * (size_t)ng, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    SPMV_HIP_TRY(e);
    return csr_windows_finish(p, lo, hi);
}

int build_ss_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                    const spmv_options_t &o, double mean_row) {
    SsDev &s = p->ss;
    const hipStream_t st = p->stream;
    s.sigma = o.ss_sigma > 0 ? o.ss_sigma : auto_ss_sigma(mean_row);
    if (!ss_sigma_ok(s.sigma)) {
        set_error("ss_sigma must be one of 4,8,12,16,20,24,32,48,64");
        return SPMV_ERROR_INVALID_VALUE;
    }
    ss_probe_options(s);
    const int W = ss_flag_words(s.sigma);
    const int64_t m = p->m, nnz = p->nnz, T = 64 * (int64_t)s.sigma;
    s.n_tiles = (nnz + T - 1) / T;
    // scratch freed on every exit path (after the stream drains)
    struct Scratch {
        hipStream_t st;
        std::vector<void *> v;
        ~Scratch() {
            (void)hipStreamSynchronize(st);
            for (void *t : v) (void)hipFree(t);
        }
    } scratch{st, {}};
    std::vector<void *> &tmp = scratch.v;
    // non-empty ordinals
    int64_t *flg = nullptr, *nzord = nullptr;
    SPMV_RETURN_IF(scratch_malloc(&flg, 8 * (size_t)std::max<int64_t>(m + 1, 1), "flg"));
    tmp.push_back(flg);
    SPMV_RETURN_IF(scratch_malloc(&nzord, 8 * (size_t)std::max<int64_t>(m + 1, 1), "nzord"));
    tmp.push_back(nzord);
    hipLaunchKernelGGL(nonempty_flags, dim3(grid_for(m)), dim3(256), 0, st, d_rp, m, flg);
    SPMV_HIP_TRY(hipMemsetAsync(flg + m, 0, 8, st));
    SPMV_RETURN_IF(exclusive_scan(p, flg, nzord, m + 1, st, tmp));
    SPMV_HIP_TRY(hipMemcpyAsync(&s.n_nonempty, nzord + m, 8, hipMemcpyDeviceToHost, st));
    SPMV_HIP_TRY(hipStreamSynchronize(st));
    s.n_empty = m - s.n_nonempty;
    void *q;
    if (s.n_empty > 0) {
        SPMV_RETURN_IF(p->arena.alloc(&q, 4 * (size_t)std::max<int64_t>(s.n_nonempty, 1)));
        s.nzrow = (int32_t *)q;
        SPMV_RETURN_IF(p->arena.alloc(&q, 4 * (size_t)s.n_empty));
        s.empty_rows = (int32_t *)q;
        hipLaunchKernelGGL(compact_rows, dim3(grid_for(m)), dim3(256), 0, st, d_rp, nzord, m, s.nzrow, s.empty_rows);
    }
    const int64_t total = s.n_tiles * T;
    SPMV_RETURN_IF(p->arena.alloc(&q, 4 * (size_t)std::max<int64_t>(s.n_tiles * 64 * W, 1)));
    s.flags = (uint32_t *)q;
    SPMV_HIP_TRY(hipMemsetAsync(s.flags, 0, 4 * (size_t)std::max<int64_t>(s.n_tiles * 64 * W, 1), st));
    hipLaunchKernelGGL(start_flags, dim3(grid_for(m + 1)), dim3(256), 0, st, d_rp, m, nnz, s.sigma, s.flags);
    SPMV_RETURN_IF(p->arena.alloc(&q, 4 * (size_t)std::max<int64_t>(s.n_tiles, 1)));
    s.tile_ord = (int32_t *)q;
    hipLaunchKernelGGL(tile_ordinals, dim3(grid_for(s.n_tiles)), dim3(256), 0, st, d_rp, m,
                       nzord, s.n_nonempty, s.sigma, s.n_tiles, s.tile_ord);
    SPMV_RETURN_IF(p->arena.alloc(&q, 4 * (size_t)std::max<int64_t>(total, 1)));
    s.col = (int32_t *)q;
    SPMV_RETURN_IF(p->arena.alloc(&q, 8 * (size_t)std::max<int64_t>(total, 1)));
    s.val = (double *)q;
    hipLaunchKernelGGL(tile_transpose, dim3(grid_for(total)), dim3(256), 0, st, d_col, d_val, nnz, s.sigma, total,
                       s.col, s.val);
    SPMV_RETURN_IF(p->arena.alloc(&q, 8 * (size_t)std::max<int64_t>(s.n_tiles, 1)));
    s.win = (int32_t *)q;
    if (s.n_tiles > 0)
        hipLaunchKernelGGL(tile_windows, dim3((unsigned)((s.n_tiles + 3) / 4)), dim3(256), 0, st, d_col, nnz, s.sigma,
                           s.n_tiles, s.win);
    SPMV_RETURN_IF(p->arena.alloc(&q, 16 * (size_t)std::max<int64_t>(s.n_tiles, 1)));
    s.ht = (double *)q;
    SPMV_RETURN_IF(p->arena.alloc(&q, 4 * (size_t)std::max<int64_t>(s.n_tiles, 1)));
    s.tail_ord = (int32_t *)q;
    SPMV_RETURN_IF(ss_plan_tail_ord(p));
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        set_error(std::string("device SS conversion: ") + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    ss_finish_info(p);
    return SPMV_SUCCESS;
}

}  // namespace spmv

// k_devbuild.hip -- DIA, sliced ELL, HYB, JDS and COO plans from a CSR that
// already lives in HBM (the CSR5 conversion pipeline's role,
// CSR5_cuda/detail/cuda/format_cuda.h:21-718), and the diagonal census AUTO
// needs to pick DIA.  Only the row pointers visit the host (slice widths, the
// JDS order, the HYB width and overflow rows are functions of the row lengths
// alone, computed by the same host code as the host builders); columns and
// values move HBM -> HBM.  Every layout is byte-identical to the host
// builder's (formats.cpp), checked by spmv_plan_digest in the GPU tests.
//
//   DIA : occupied diagonals by a mark + wave-compacted census (the host's
//         occ[] sweep, src/opt_dia.cpp:29-45), then one thread per row fills
//         its slots of the 512-row blocks (src/opt_dia.cpp:47-56 re-laid out):
//         duplicates are added in entry order, as the host build does.
//   ELL : one wave per 64-row slice, one lane per row, 16-byte column and
//         value stores in the interleaved slot order (src/opt_ell.cpp:28-52).
//   HYB / JDS : the ELL fill over the capped (and, JDS, length-sorted) rows,
//         plus a wave per overflow row copying its entries past K.
//   COO : row ids per entry, columns / values copied, 128-entry unit padding.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "device.hpp"
#include "internal.hpp"

namespace spmv {

namespace {

inline unsigned grid_for(int64_t n, int per = 256) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, 65536));
}

// ---- DIA census -------------------------------------------------------------
// occ[col - row + m - 1] = 1 for every entry (benign byte races: all write 1)
__global__ __launch_bounds__(256) void dia_mark_kernel(const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                       int64_t m, uint8_t *__restrict__ occ) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < m; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = rp[r + 1];
        for (int64_t j = rp[r]; j < e; ++j) occ[col[j] - r + m - 1] = 1;
    }
}

// the occupied diagonals, compacted: one atomic per wave (ballot + popcount)
__global__ __launch_bounds__(256) void dia_census_kernel(const uint8_t *__restrict__ occ, int64_t N, int64_t m,
                                                         int32_t cap, unsigned long long *__restrict__ cnt,
                                                         int32_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // every lane of a wave runs the same trip count (the ballot is wave-wide)
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); base < N; base += stride) {
        const int64_t d = base + lane;
        const bool on = d < N && occ[d];
        const unsigned long long mask = __ballot(on);
        if (!mask) continue;
        unsigned long long first = 0;
        if (lane == 0) first = atomicAdd(cnt, (unsigned long long)__popcll(mask));
        first = __shfl(first, 0, 64);
        if (on) {
            const unsigned long long below = mask & ((1ull << lane) - 1ull);
            const unsigned long long at = first + (unsigned long long)__popcll(below);
            if (at < (unsigned long long)cap) out[at] = (int32_t)(d - (m - 1));
        }
    }
}

// ---- DIA fill -----------------------------------------------------------------
// One thread per row: its entries in CSR order, each to the slot of its
// diagonal in the row's 512-row block (the layout of build_dia, formats.cpp).
// A slot receives 0.0 + v on its first visit and slot + v on a later one
// (duplicates), exactly the host build's `val[at] += v` from a zero-filled
// buffer; a column above every earlier column of the row cannot have been
// visited, so it is a plain store.  Diagonal lookup: an int16 table in LDS
// indexed by (col - row - off_min) when the offsets span <= kDiaLut, else a
// binary search of the ascending offsets.
constexpr int kDiaLut = 16384;

template <bool LUT>
__global__ __launch_bounds__(256) void dia_fill_kernel(const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                       const double *__restrict__ val, int64_t m,
                                                       const int32_t *__restrict__ off, int nd, int32_t off_min,
                                                       int32_t span, int64_t group, int64_t nblk,
                                                       double *__restrict__ out) {
    __shared__ int16_t lut[LUT ? kDiaLut : 1];
    if constexpr (LUT) {
        for (int i = threadIdx.x; i < span; i += blockDim.x) lut[i] = -1;
        __syncthreads();
        for (int d = threadIdx.x; d < nd; d += blockDim.x) lut[off[d] - off_min] = (int16_t)d;
        __syncthreads();
    }
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < m; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = r / kDiaBlockRows, rl = r % kDiaBlockRows;
        int64_t bbase = b * nd * kDiaBlockRows, dstride = kDiaBlockRows;
        if (group > 0) {  // interleaved groups (k_dia.hip, probe build)
            const int64_t t = b / group, g = b - t * group, gt = group < nblk - t * group ? group : nblk - t * group;
            bbase = (t * group * nd + g) * kDiaBlockRows;
            dstride = gt * kDiaBlockRows;
        }
        const int64_t e = rp[r + 1];
        int32_t cmax = -1;
        for (int64_t j = rp[r]; j < e; ++j) {
            const int32_t c = col[j];
            const double v = val[j];
            const int32_t o = (int32_t)((int64_t)c - r);
            int di;
            if constexpr (LUT) {
                di = lut[o - off_min];
            } else {
                int lo = 0, hi = nd - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (off[mid] < o) lo = mid + 1;
                    else hi = mid;
                }
                di = lo;
            }
            double *slot = out + bbase + (int64_t)di * dstride + rl;
            if (c > cmax) {
                *slot = __dadd_rn(0.0, v);
                cmax = c;
            } else {
                *slot = __dadd_rn(*slot, v);
            }
        }
    }
}

// ---- sliced ELL fill ------------------------------------------------------------
// One wave per slice, lane li = slice row li (matrix row order[s*64 + li]
// for JDS); each quad of slots leaves as one 16-byte column store and two
// 16-byte value stores (slots 0-1, 2-3 of the quad's two 1-KiB value halves).
// Padding: the row's last real column (0 for an empty row), value 0.
__global__ __launch_bounds__(256) void ell_fill_kernel(const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                       const double *__restrict__ val, int64_t m,
                                                       const int32_t *__restrict__ order,
                                                       const int64_t *__restrict__ slice_off, int64_t n_slices,
                                                       int32_t *__restrict__ ecol, double *__restrict__ eval) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int li = threadIdx.x & 63;
    if (s >= n_slices) return;
    const int64_t base = slice_off[s];
    const int64_t w = (slice_off[s + 1] - base) / 64;
    const int64_t sr = s * 64 + li;
    int64_t rs = 0, len = 0;
    if (sr < m) {
        const int64_t row = order ? (int64_t)order[sr] : sr;
        rs = rp[row];
        len = rp[row + 1] - rs;
        len = len < w ? len : w;  // w <= cap: cap is a multiple of 4 (or INT32_MAX)
    }
    int32_t last = 0;
    for (int64_t q = 0; q < w / 4; ++q) {
        i32x4 c;
        double v[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int64_t k = 4 * q + kk;
            int32_t ck = last;
            double vk = 0.0;
            if (k < len) {
                ck = col[rs + k];
                vk = val[rs + k];
                last = ck;
            }
            c[kk] = ck;
            v[kk] = vk;
        }
        *reinterpret_cast<i32x4 *>(ecol + base + q * 256 + li * 4) = c;
        f64x2 a, b;
        a.x = v[0];
        a.y = v[1];
        b.x = v[2];
        b.y = v[3];
        *reinterpret_cast<f64x2 *>(eval + base + q * 256 + li * 2) = a;
        *reinterpret_cast<f64x2 *>(eval + base + q * 256 + 128 + li * 2) = b;
    }
}

// ---- HYB / JDS overflow: a wave per overflow row copies entries K.. ----------
__global__ __launch_bounds__(256) void overflow_copy_kernel(const int64_t *__restrict__ rp,
                                                            const int32_t *__restrict__ col,
                                                            const double *__restrict__ val, int64_t K,
                                                            const int32_t *__restrict__ rows,
                                                            const int64_t *__restrict__ orp, int64_t n_rows,
                                                            int32_t *__restrict__ ocol, double *__restrict__ oval) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n_rows) return;
    const int64_t src = rp[rows[i]] + K, dst = orp[i], cnt = orp[i + 1] - dst;
    for (int64_t t = lane; t < cnt; t += 64) {
        ocol[dst + t] = col[src + t];
        oval[dst + t] = val[src + t];
    }
}

// column order of the rows: bad[0] counts entries below their predecessor
// (disorder), bad[1] entries equal to it (duplicates)
__global__ __launch_bounds__(256) void rows_order_kernel(const int64_t *__restrict__ rp,
                                                         const int32_t *__restrict__ col, int64_t m,
                                                         unsigned long long *__restrict__ bad) {
    unsigned long long d = 0, q = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < m; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = rp[r + 1];
        for (int64_t j = rp[r] + 1; j < e; ++j) {
            d += col[j] < col[j - 1];
            q += col[j] == col[j - 1];
        }
    }
    if (d) atomicAdd(bad, d);
    if (q) atomicAdd(bad + 1, q);
}

// ---- COO row ids -------------------------------------------------------------------
__global__ __launch_bounds__(256) void coo_rows_kernel(const int64_t *__restrict__ rp, int64_t m,
                                                       int32_t *__restrict__ row) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < m; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = rp[r + 1];
        for (int64_t j = rp[r]; j < e; ++j) row[j] = (int32_t)r;
    }
}

// scratch freed on every exit path (after the stream drains)
struct Scratch {
    hipStream_t st;
    std::vector<void *> v;
    ~Scratch() {
        (void)hipStreamSynchronize(st);
        for (void *t : v) (void)hipFree(t);
    }
};

template <typename T>
int plan_alloc(spmv_plan_s *p, T **dst, int64_t count) {
    void *q = nullptr;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(T) * (size_t)std::max<int64_t>(count, 1)));
    *dst = (T *)q;
    return SPMV_SUCCESS;
}

// host array -> a new plan allocation (count elements; pad zeroed elements after)
template <typename T>
int plan_upload(spmv_plan_s *p, T **dst, const T *src, int64_t count, int64_t pad = 0) {
    SPMV_RETURN_IF(plan_alloc(p, dst, count + pad));
    if (count > 0) SPMV_HIP_TRY(hipMemcpyAsync(*dst, src, sizeof(T) * (size_t)count, hipMemcpyHostToDevice, p->stream));
    if (pad > 0) SPMV_HIP_TRY(hipMemsetAsync(*dst + count, 0, sizeof(T) * (size_t)pad, p->stream));
    return SPMV_SUCCESS;
}

int sync_or_error(spmv_plan_s *p, const char *what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    if (e != hipSuccess) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        (void)hipGetLastError();
        return SPMV_ERROR_HIP;
    }
    return SPMV_SUCCESS;
}

// the ELL part (cap, order: JDS) of a plan from a device CSR
int ell_fill_device(spmv_plan_s *p, const DevCsr &A, int cap, const int32_t *h_order, const int32_t *d_order) {
    EllDev &e = p->ell;
    if (const char *u = probe_env("SPMV_ELL_UNROLL")) e.unroll = std::atoi(u);
    e.n_slices = (A.m + 63) / 64;
    std::vector<int64_t> off;
    const int maxw = ell_slice_offsets(A.h_rp, A.m, cap, h_order, off);
    const int64_t total = off[(size_t)e.n_slices];
    SPMV_RETURN_IF(plan_upload(p, &e.slice_off, off.data(), e.n_slices + 1));
    SPMV_RETURN_IF(plan_alloc(p, &e.col, total));
    SPMV_RETURN_IF(plan_alloc(p, &e.val, total));
    if (e.n_slices > 0 && total > 0)
        hipLaunchKernelGGL(ell_fill_kernel, dim3((unsigned)((e.n_slices + 3) / 4)), dim3(256), 0, p->stream, A.d_rp,
                           A.d_col, A.d_val, A.m, d_order, e.slice_off, e.n_slices, e.col, e.val);
    SPMV_RETURN_IF(sync_or_error(p, "device ELL fill"));
    ell_finish_info(p, maxw, total);
    return SPMV_SUCCESS;
}

// the overflow CSR (entries K.. of the rows longer than K) from a device CSR
int overflow_device(spmv_plan_s *p, const DevCsr &A, int K) {
    HybDev &h = p->hyb;
    std::vector<int32_t> rows;
    std::vector<int64_t> orp;
    overflow_layout(A.h_rp, A.m, K, rows, orp);
    SPMV_RETURN_IF(overflow_upload_index(p, rows, orp));
    SPMV_RETURN_IF(plan_alloc(p, &h.col, h.nnz + kPad));
    SPMV_RETURN_IF(plan_alloc(p, &h.val, h.nnz + kPad));
    SPMV_HIP_TRY(hipMemsetAsync(h.col + h.nnz, 0, sizeof(int32_t) * kPad, p->stream));
    SPMV_HIP_TRY(hipMemsetAsync(h.val + h.nnz, 0, sizeof(double) * kPad, p->stream));
    if (h.n_rows > 0)
        hipLaunchKernelGGL(overflow_copy_kernel, dim3((unsigned)((h.n_rows + 3) / 4)), dim3(256), 0, p->stream, A.d_rp,
                           A.d_col, A.d_val, (int64_t)K, h.rows, h.row_ptr, h.n_rows, h.col, h.val);
    return sync_or_error(p, "device overflow copy");
}

}  // namespace

// Occupied diagonals of a device CSR, ascending (dia_offsets of formats.cpp):
// kDiaRefused when there are more than max_diags or the zero fill exceeds
// max_fill, SPMV_SUCCESS when DIA fits, else an error status.
int dia_offsets_device(spmv_plan_s *p, const DevCsr &A, int max_diags, double max_fill, std::vector<int32_t> &offs) {
    offs.clear();
    const int64_t N = A.m + A.n - 1;
    if (N <= 0) return SPMV_SUCCESS;
    const hipStream_t st = p->stream;
    Scratch scratch{st, {}};
    uint8_t *occ = nullptr;
    SPMV_RETURN_IF(scratch_malloc(&occ, (size_t)N, "occ"));
    scratch.v.push_back(occ);
    unsigned long long *cnt = nullptr;
    SPMV_RETURN_IF(scratch_malloc(&cnt, sizeof(unsigned long long), "cnt"));
    scratch.v.push_back(cnt);
    int32_t *out = nullptr;
    SPMV_RETURN_IF(scratch_malloc(&out, sizeof(int32_t) * (size_t)(max_diags + 1), "out"));
    scratch.v.push_back(out);
    SPMV_HIP_TRY(hipMemsetAsync(occ, 0, (size_t)N, st));
    SPMV_HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st));
    if (A.m > 0 && A.nnz > 0)
        hipLaunchKernelGGL(dia_mark_kernel, dim3(grid_for(A.m)), dim3(256), 0, st, A.d_rp, A.d_col, A.m, occ);
    hipLaunchKernelGGL(dia_census_kernel, dim3(grid_for(N, 1024)), dim3(256), 0, st, occ, N, A.m, max_diags + 1, cnt,
                       out);
    unsigned long long n_occ = 0;
    SPMV_HIP_TRY(hipGetLastError());
    SPMV_HIP_TRY(hipMemcpyAsync(&n_occ, cnt, sizeof(n_occ), hipMemcpyDeviceToHost, st));
    SPMV_HIP_TRY(hipStreamSynchronize(st));
    if (n_occ > (unsigned long long)max_diags) return kDiaRefused;
    offs.resize((size_t)n_occ);
    if (n_occ) SPMV_HIP_TRY(hipMemcpy(offs.data(), out, sizeof(int32_t) * (size_t)n_occ, hipMemcpyDeviceToHost));
    std::sort(offs.begin(), offs.end());
    if ((double)offs.size() * (double)A.m > max_fill * (double)std::max<int64_t>(A.nnz, 1)) return kDiaRefused;
    return SPMV_SUCCESS;
}

int rows_order_device(spmv_plan_s *p, const DevCsr &A, int *order) {
    *order = kRowsStrict;
    if (A.m == 0 || A.nnz == 0) return SPMV_SUCCESS;
    Scratch scratch{p->stream, {}};
    unsigned long long *bad = nullptr, hb[2] = {0, 0};
    SPMV_RETURN_IF(scratch_malloc(&bad, sizeof(hb), "bad"));
    scratch.v.push_back(bad);
    SPMV_HIP_TRY(hipMemsetAsync(bad, 0, sizeof(hb), p->stream));
    hipLaunchKernelGGL(rows_order_kernel, dim3(grid_for(A.m)), dim3(256), 0, p->stream, A.d_rp, A.d_col, A.m, bad);
    SPMV_HIP_TRY(hipGetLastError());
    SPMV_HIP_TRY(hipMemcpyAsync(hb, bad, sizeof(hb), hipMemcpyDeviceToHost, p->stream));
    SPMV_HIP_TRY(hipStreamSynchronize(p->stream));
    *order = hb[0] ? kRowsUnsorted : hb[1] ? kRowsSorted : kRowsStrict;
    return SPMV_SUCCESS;
}

int build_dia_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o) {
    DiaDev &d = p->dia;
    const int maxd = o.dia_max_diags > 0 ? o.dia_max_diags : 1024;
    const double fill = o.dia_max_fill > 0 ? o.dia_max_fill : 3.0;
    std::vector<int32_t> offs;
    const int st = dia_offsets_device(p, A, maxd, fill, offs);
    if (st == kDiaRefused) {
        set_error("DIA: matrix has too many diagonals or too much zero fill for the DIA format");
        return SPMV_ERROR_NOT_SUPPORTED;
    }
    SPMV_RETURN_IF(st);
    d.n_diags = (int)offs.size();
    d.off_host = offs;
    d.mp = (A.m + kDiaBlockRows - 1) / kDiaBlockRows * kDiaBlockRows;
    const int64_t slots = (int64_t)d.n_diags * d.mp;
    if (const char *e = probe_env("SPMV_DIA_GROUP")) d.group = std::max(0, std::atoi(e));
    if (const char *e = probe_env("SPMV_DIA_DEBUG")) d.dbg = std::atoi(e);
    if (const char *e = probe_env("SPMV_DIA_LDS_KB")) d.lds_kb = std::atoi(e);
    SPMV_RETURN_IF(plan_upload(p, &d.off, offs.data(), d.n_diags));
    // the value buffer as build_dia places it: AUTO puts >= 256 MB straight
    // into 2-MB VMM handles at a 1-GB-aligned VA
    const size_t vbytes = (size_t)std::max<int64_t>(slots, 1) * sizeof(double);
    spmv_options_t oo = o;
    SPMV_RETURN_IF(placement_mode_check(oo.placement));
    if (oo.placement == SPMV_PLACEMENT_AUTO)
        oo.placement = vbytes >= kDiaVmmMinBytes ? SPMV_PLACEMENT_VMM : SPMV_PLACEMENT_PLAIN;
    const bool vmm_now = oo.placement == SPMV_PLACEMENT_VMM && !probe_env("SPMV_PLACEMENT_MODE");
    if (vmm_now) {
        void *q = nullptr;
        SPMV_RETURN_IF(p->arena.alloc_vmm(&q, vbytes, kVmmChunk, p->device, kVmmAlign));
        d.val = (double *)q;
        d.placement = SPMV_PLACEMENT_VMM;
    } else {
        SPMV_RETURN_IF(plan_alloc(p, &d.val, std::max<int64_t>(slots, 1)));
    }
    SPMV_HIP_TRY(hipMemsetAsync(d.val, 0, vbytes, p->stream));
    if (slots > 0 && A.nnz > 0) {
        const int32_t off_min = offs.front(), span = offs.back() - offs.front() + 1;
        const int64_t nblk = d.mp / kDiaBlockRows;
        if (span <= kDiaLut)
            hipLaunchKernelGGL(dia_fill_kernel<true>, dim3(grid_for(A.m)), dim3(256), 0, p->stream, A.d_rp, A.d_col,
                               A.d_val, A.m, d.off, d.n_diags, off_min, span, (int64_t)d.group, nblk, d.val);
        else
            hipLaunchKernelGGL(dia_fill_kernel<false>, dim3(grid_for(A.m)), dim3(256), 0, p->stream, A.d_rp, A.d_col,
                               A.d_val, A.m, d.off, d.n_diags, off_min, span, (int64_t)d.group, nblk, d.val);
    }
    SPMV_RETURN_IF(sync_or_error(p, "device DIA fill"));
    if (!vmm_now) SPMV_RETURN_IF(dia_placement(p, A.m, A.n, vbytes, oo));
    dia_finish_info(p);
    return SPMV_SUCCESS;
}

int build_ell_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &) {
    return ell_fill_device(p, A, INT32_MAX, nullptr, nullptr);
}

int build_hyb_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o) {
    const int K = hyb_width(A.h_rp, A.m, o);
    SPMV_RETURN_IF(ell_fill_device(p, A, K, nullptr, nullptr));
    const int64_t ell_slots = p->stored_slots;
    SPMV_RETURN_IF(overflow_device(p, A, K));
    hyb_finish_info(p, K, ell_slots);
    return SPMV_SUCCESS;
}

int build_jds_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o) {
    std::vector<int32_t> order;
    int K = 0;
    const bool identity = jds_layout(A.h_rp, A.m, A.nnz, o, order, &K);
    if (!identity) SPMV_RETURN_IF(plan_upload(p, &p->ell.perm, order.data(), A.m));
    SPMV_RETURN_IF(ell_fill_device(p, A, K, identity ? nullptr : order.data(), p->ell.perm));
    const int64_t ell_slots = p->stored_slots;
    SPMV_RETURN_IF(overflow_device(p, A, K));
    jds_finish_info(p, identity, ell_slots);
    return SPMV_SUCCESS;
}

int build_coo_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &) {
    CooDev &c = p->coo;
    c.n_units = (A.nnz + kCooUnit - 1) / kCooUnit;
    const int64_t total = c.n_units * kCooUnit;
    SPMV_RETURN_IF(plan_alloc(p, &c.row, total));
    SPMV_RETURN_IF(plan_alloc(p, &c.col, total));
    SPMV_RETURN_IF(plan_alloc(p, &c.val, total));
    const int64_t pad = total - A.nnz;
    if (pad > 0) {
        SPMV_HIP_TRY(hipMemsetAsync(c.row + A.nnz, 0xFF, sizeof(int32_t) * (size_t)pad, p->stream));  // row -1
        SPMV_HIP_TRY(hipMemsetAsync(c.col + A.nnz, 0, sizeof(int32_t) * (size_t)pad, p->stream));
        SPMV_HIP_TRY(hipMemsetAsync(c.val + A.nnz, 0, sizeof(double) * (size_t)pad, p->stream));
    }
    if (A.nnz > 0) {
        SPMV_HIP_TRY(hipMemcpyAsync(c.col, A.d_col, sizeof(int32_t) * (size_t)A.nnz, hipMemcpyDeviceToDevice, p->stream));
        SPMV_HIP_TRY(hipMemcpyAsync(c.val, A.d_val, sizeof(double) * (size_t)A.nnz, hipMemcpyDeviceToDevice, p->stream));
        hipLaunchKernelGGL(coo_rows_kernel, dim3(grid_for(A.m)), dim3(256), 0, p->stream, A.d_rp, A.m, c.row);
    }
    SPMV_RETURN_IF(sync_or_error(p, "device COO build"));
    coo_finish_info(p);
    return SPMV_SUCCESS;
}


// ---- layout digest (spmv_plan_digest) ------------------------------------------
namespace {

struct ArrayRef {
    const char *name;
    const void *ptr;
    int64_t bytes;
};

// the device arrays of a plan with their logical sizes (what the builders
// write; allocation rounding and per-execute scratch excluded)
int plan_arrays(const spmv_plan_s *p, std::vector<ArrayRef> &a) {
    a.clear();
    auto add = [&](const char *name, const void *ptr, int64_t bytes) {
        if (ptr && bytes > 0) a.push_back(ArrayRef{name, ptr, bytes});
    };
    switch (p->format) {
        case SPMV_FORMAT_CSR: {
            const CsrDev &c = p->csr;
            add("row_ptr", c.row_ptr, (c.rp64 ? 8 : 4) * (p->m + 1));
            add("col", c.col, 4 * (p->nnz + kPad));
            add("val", c.val, 8 * ((c.val_halves ? (p->nnz + 255) / 256 * 256 : p->nnz) + kPad));
            add("bin_rows", c.bin_rows, 4 * p->m);
            add("win0", c.win0, 4 * ((p->m + kCsrWinGroup - 1) / kCsrWinGroup));
            return SPMV_SUCCESS;
        }
        case SPMV_FORMAT_SS: {
            const SsDev &s = p->ss;
            const int64_t total = s.n_tiles * 64 * s.sigma;
            add("col", s.col, 4 * total);
            add("val", s.val, 8 * total);
            add("flags", s.flags, 4 * 64 * ss_flag_words(s.sigma) * s.n_tiles);
            add("win", s.win, 8 * s.n_tiles);
            add("tile_ord", s.tile_ord, 4 * s.n_tiles);
            add("nzrow", s.nzrow, 4 * s.n_nonempty);
            add("empty_rows", s.empty_rows, 4 * s.n_empty);
            return SPMV_SUCCESS;
        }
        case SPMV_FORMAT_ELL:
        case SPMV_FORMAT_HYB:
        case SPMV_FORMAT_JDS: {
            const EllDev &e = p->ell;
            add("slice_off", e.slice_off, 8 * (e.n_slices + 1));
            add("ell_col", e.col, 4 * e.slots);
            add("ell_val", e.val, 8 * e.slots);
            add("perm", e.perm, 4 * p->m);
            if (p->format != SPMV_FORMAT_ELL) {
                const HybDev &h = p->hyb;
                add("ovf_rows", h.rows, 4 * h.n_rows);
                add("ovf_row_ptr", h.row_ptr, 8 * (h.n_rows + 1));
                add("ovf_bin_rows", h.bin_rows, 4 * h.n_rows);
                add("ovf_col", h.col, 4 * (h.nnz + kPad));
                add("ovf_val", h.val, 8 * (h.nnz + kPad));
            }
            return SPMV_SUCCESS;
        }
        case SPMV_FORMAT_DIA:
            add("off", p->dia.off, 4 * (int64_t)p->dia.n_diags);
            add("val", p->dia.val, 8 * (int64_t)p->dia.n_diags * p->dia.mp);
            return SPMV_SUCCESS;
        case SPMV_FORMAT_COO: {
            const int64_t total = p->coo.n_units * kCooUnit;
            add("row", p->coo.row, 4 * total);
            add("col", p->coo.col, 4 * total);
            add("val", p->coo.val, 8 * total);
            return SPMV_SUCCESS;
        }
        case SPMV_FORMAT_CSS: {
            const CssDev &c = p->css;
            const int64_t nb = (int64_t)c.P * c.nwg, total = p->stored_slots;
            add("woff", c.woff, 8 * (c.n_lists + 1));
            add("wlen", c.wlen, 4 * c.n_lists);
            add("bstart", c.bstart, 8 * (nb + 1));
            add("rmap", c.rmap, 4 * c.n_rmap);
            add("moff", c.moff, 8 * (nb + 1));
            add("merge", c.merge, 12 * c.split_rows);
            add("col", c.col, 4 * total);
            add("slot", c.row, (2 * total) & ~(int64_t)3);  // whole words (total is a multiple of 256 when interleaved)
            add("val", c.val, 8 * total);
            return SPMV_SUCCESS;
        }
    }
    if (p->format == SPMV_FORMAT_BIN) {
        const BinDev &B = p->bin;
        const int64_t E1 = B.mul_entries + kBinMulSlack, S = B.n_strips, NR = B.n_blocks * B.n_bins;
        add("bin_row0", B.bin_row0, 4 * (B.n_bins + 1));
        add("run_off", B.run_off, 8 * (NR + 1));
        add("srun_off", B.srun_off, 8 * (NR + 1));
        add("val1", B.val1, 8 * E1);
        add("cs1", B.cs1, (2 * E1) & ~(int64_t)3);
        add("slot2", B.slot2, (2 * B.slot_entries) & ~(int64_t)3);
        add("dst1", B.dst1, 4 * (E1 >> B.pad_log));
        add("mtab", B.mtab, 4 * (B.slot_entries / 8));
        add("lstart", B.lstart, 8 * S);
        add("lshift", B.lshift, 8 * S);
        add("lcode", B.lcode, 4 * B.long_entries);
        return SPMV_SUCCESS;
    }
    set_error("spmv_plan_digest: unknown format");
    return SPMV_ERROR_NOT_SUPPORTED;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// sum over the array's 4-byte words of mix(word, position): order-free, so
// any grid gives the same digest; a 4-byte tail word is zero-extended
__global__ __launch_bounds__(256) void digest_kernel(const uint32_t *__restrict__ w, int64_t nwords,
                                                     unsigned long long *__restrict__ out) {
    uint64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (int64_t)gridDim.x * blockDim.x)
        acc += mix64(((uint64_t)w[i] << 32 | 0x9E37u) ^ mix64((uint64_t)i + 0x632BE59BD9B4E019ull));
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

}  // namespace

}  // namespace spmv

using namespace spmv;

extern "C" int spmv_plan_digest(spmv_plan_t p, uint64_t *digests, int32_t cap, int32_t *n_arrays) {
    SPMV_CHECK_ARG(p != nullptr && n_arrays != nullptr && (cap <= 0 || digests != nullptr), "bad arguments");
    std::vector<ArrayRef> a;
    SPMV_RETURN_IF(plan_arrays(p, a));
    *n_arrays = (int32_t)a.size();
    int cur = -1;
    SPMV_HIP_TRY(hipGetDevice(&cur));
    if (cur != p->device) SPMV_HIP_TRY(hipSetDevice(p->device));
    unsigned long long *d = nullptr;
    SPMV_RETURN_IF(scratch_malloc(&d, sizeof(unsigned long long) * std::max<size_t>(a.size(), 1), "d"));
    hipError_t e = hipMemset(d, 0, sizeof(unsigned long long) * std::max<size_t>(a.size(), 1));
    for (size_t k = 0; k < a.size() && e == hipSuccess; ++k) {
        // logical sizes are multiples of 4 bytes (int32 / int64 / f64 arrays)
        const int64_t nw = a[k].bytes / 4;
        hipLaunchKernelGGL(digest_kernel, dim3(grid_for(nw, 1024)), dim3(256), 0, p->stream,
                           (const uint32_t *)a[k].ptr, nw, d + k);
        e = hipGetLastError();
    }
    std::vector<unsigned long long> h(a.size());
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    if (e == hipSuccess && !a.empty()) e = hipMemcpy(h.data(), d, sizeof(unsigned long long) * a.size(), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) {
        set_error(std::string("spmv_plan_digest: ") + hipGetErrorString(e));
        (void)hipGetLastError();
        return SPMV_ERROR_HIP;
    }
    for (size_t k = 0; k < a.size() && (int32_t)k < cap; ++k) digests[k] = (uint64_t)h[k] ^ (uint64_t)a[k].bytes;
    return SPMV_SUCCESS;
}

extern "C" const char *spmv_plan_digest_name(spmv_plan_t p, int32_t k) {
    std::vector<ArrayRef> a;
    if (!p || k < 0 || plan_arrays(p, a) != SPMV_SUCCESS || k >= (int32_t)a.size()) return "";
    return a[(size_t)k].name;
}

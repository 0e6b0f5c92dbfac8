// k_bin_build.hip -- BIN fill from a CSR already in HBM (build_bin_device in
// build_bin.cpp drives it).  The OptimizeProblem counterpart is opt_ss's
// host-side segment build (src/opt_ss.cpp:52-142); here a 1 G-entry matrix
// never round-trips through the host: only the row pointers (to cut the row
// bins) and the (bin, strip) entry counts (to lay out the segments) visit it.
//
// One thread per CSR entry j throughout:
//   bin   b = last bin whose first entry <= j     (binary search, NB + 1 starts)
//   row   r = last row of b whose first entry <= j (binary search in row_ptr)
//   strip t = col[j] / C
//   k       = ordinal of j among row r's entries in strip t
//             (= j - first entry of r in strip t; rows must have
//              non-decreasing strips, checked by bin_count_kernel)
// Phases: counts per (b, t) -> [host offsets] -> k-run sizes per segment
// (atomicAdd) -> exclusive scan -> placement (atomic cursor per k-run) ->
// padding.  Inside one k-run rows are placed in atomic-cursor order rather
// than ascending; every product of a row still reaches the Sum in column
// order and no two entries of a k-run share a row, so y is bit-identical to
// the host-built plan's (tests/test_gpu_parity.py::test_bin_device_build).
#include <algorithm>
#include <vector>

#include "device.hpp"
#include "internal.hpp"

namespace spmv {

namespace {

inline unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65536)); }

// first index i in [lo, hi) with a[i] > v (a non-decreasing)
__device__ __forceinline__ int64_t upper_idx(const int64_t *__restrict__ a, int64_t lo, int64_t hi, int64_t v) {
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

struct EntryPos {
    int64_t b, r;
};

__device__ __forceinline__ EntryPos locate(int64_t j, const int64_t *__restrict__ rp, const int64_t *__restrict__ bstart,
                                           int64_t NB, const int32_t *__restrict__ row0) {
    EntryPos e;
    e.b = upper_idx(bstart, 0, NB + 1, j) - 1;
    e.r = upper_idx(rp, row0[e.b], (int64_t)row0[e.b + 1] + 1, j) - 1;
    return e;
}

__global__ __launch_bounds__(256) void bin_count_kernel(const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                        int64_t nnz, const int64_t *__restrict__ bstart, int64_t NB,
                                                        const int32_t *__restrict__ row0, int32_t C, int64_t S,
                                                        int32_t *__restrict__ cnt, unsigned *__restrict__ bad) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * 256) {
        const EntryPos e = locate(j, rp, bstart, NB, row0);
        const int32_t t = col[j] / C;
        atomicAdd(&cnt[e.b * S + t], 1);
        if (j > rp[e.r] && col[j - 1] / C > t) atomicOr(bad, 1u);
    }
}

// k of entry j in row r: j - (first entry of r with col >= t*C)
__device__ __forceinline__ int64_t entry_k(int64_t j, int64_t r, int32_t t, int32_t C, const int64_t *__restrict__ rp,
                                           const int32_t *__restrict__ col) {
    int64_t lo = rp[r], hi = j;
    const int32_t c0 = t * C;
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (col[mid] < c0) lo = mid + 1;
        else hi = mid;
    }
    return j - lo;
}

__global__ __launch_bounds__(256) void bin_khist_kernel(const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                        int64_t nnz, const int64_t *__restrict__ bstart, int64_t NB,
                                                        const int32_t *__restrict__ row0, int32_t C, int64_t S,
                                                        const int64_t *__restrict__ off2,
                                                        unsigned long long *__restrict__ kh) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * 256) {
        const EntryPos e = locate(j, rp, bstart, NB, row0);
        const int32_t t = col[j] / C;
        const int64_t k = entry_k(j, e.r, t, C, rp, col);
        atomicAdd(&kh[off2[e.b * S + t] + k], 1ull);
    }
}

__global__ __launch_bounds__(256) void bin_place_kernel(
    const int64_t *__restrict__ rp, const int32_t *__restrict__ col, const double *__restrict__ val, int64_t nnz,
    const int64_t *__restrict__ bstart, int64_t NB, const int32_t *__restrict__ row0, int32_t C, int64_t S,
    const int64_t *__restrict__ off1, const int64_t *__restrict__ off2, const int64_t *__restrict__ ks,
    unsigned long long *__restrict__ cur, const int64_t *__restrict__ pbb, int pad_log,
    const int64_t *__restrict__ run_off, const int64_t *__restrict__ srun_off, int64_t SB, int sum_u,
    double *__restrict__ val1, uint16_t *__restrict__ cs1, uint16_t *__restrict__ slot2, int32_t *__restrict__ dst1) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * 256) {
        const EntryPos e = locate(j, rp, bstart, NB, row0);
        const int32_t c = col[j];
        const int32_t t = c / C;
        const int64_t k = entry_k(j, e.r, t, C, rp, col);
        const int64_t seg = e.b * S + t;
        const int64_t o1 = off1[seg], o2 = off2[seg];
        const int64_t pos = (ks[o2 + k] - ks[o2]) + (int64_t)atomicAdd(&cur[o2 + k], 1ull);
        val1[o1 + pos] = val[j];
        cs1[o1 + pos] = (uint16_t)(c - t * C);
        const int64_t run = (t / SB) * NB + e.b;
        slot2[bin_slot_index(o2 + pos, run_off[run], srun_off[run], sum_u)] = (uint16_t)(e.r - row0[e.b]);
        // every 2^pad_log group of a segment starts with a real entry (Mul
        // order, dst1 == nullptr: no destinations)
        if (dst1 && (pos & ((1 << pad_log) - 1)) == 0)
            dst1[(o1 + pos) >> pad_log] = (int32_t)((o2 + pos - pbb[e.b]) >> pad_log);
    }
}

__global__ __launch_bounds__(256) void bin_pad_kernel(const int32_t *__restrict__ cnt, int64_t nseg,
                                                      const int64_t *__restrict__ off1,
                                                      int pad_log, double *__restrict__ val1,
                                                      uint16_t *__restrict__ cs1) {
    const int64_t PAD = (int64_t)1 << pad_log;
    for (int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x; s < nseg; s += (int64_t)gridDim.x * 256) {
        const int64_t n0 = cnt[s], n8 = (n0 + PAD - 1) & ~(PAD - 1);
        for (int64_t k = n0; k < n8; ++k) {
            val1[off1[s] + k] = 0.0;
            cs1[off1[s] + k] = 0;
        }
    }
}

__global__ __launch_bounds__(256) void fill_u16_kernel(uint16_t *__restrict__ a, int64_t n, uint16_t v) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) a[i] = v;
}

// hipMalloc'd scratch, freed (after the stream drains) on every exit path
struct Scratch {
    hipStream_t st;
    std::vector<void *> v;
    ~Scratch() {
        (void)hipStreamSynchronize(st);
        for (void *t : v) (void)hipFree(t);
    }
    template <typename T>
    int alloc(T **q, size_t count) {
        void *t = nullptr;
        if (hipMalloc(&t, sizeof(T) * std::max<size_t>(count, 1)) != hipSuccess) {
            (void)hipGetLastError();
            set_error("BIN device build: scratch allocation failed");
            return SPMV_ERROR_OUT_OF_MEMORY;
        }
        v.push_back(t);
        *q = (T *)t;
        return SPMV_SUCCESS;
    }
    template <typename T>
    int upload(T **q, const std::vector<T> &h) {
        SPMV_RETURN_IF(alloc(q, h.size()));
        if (!h.empty()) SPMV_HIP_TRY(hipMemcpyAsync(*q, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice, st));
        return SPMV_SUCCESS;
    }
};

int finish(hipStream_t st, const char *what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        set_error(std::string("BIN device build (") + what + "): " + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    return SPMV_SUCCESS;
}

}  // namespace

int bin_count_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const std::vector<int32_t> &row0,
                     const std::vector<int64_t> &bstart, int64_t S, std::vector<int32_t> &cnt) {
    const hipStream_t st = p->stream;
    const int64_t NB = (int64_t)row0.size() - 1;
    Scratch sc{st, {}};
    int32_t *d_row0, *d_cnt;
    int64_t *d_bstart;
    unsigned *d_bad;
    SPMV_RETURN_IF(sc.upload(&d_row0, row0));
    SPMV_RETURN_IF(sc.upload(&d_bstart, bstart));
    SPMV_RETURN_IF(sc.alloc(&d_cnt, (size_t)(NB * S)));
    SPMV_RETURN_IF(sc.alloc(&d_bad, 1));
    SPMV_HIP_TRY(hipMemsetAsync(d_cnt, 0, sizeof(int32_t) * (size_t)(NB * S), st));
    SPMV_HIP_TRY(hipMemsetAsync(d_bad, 0, sizeof(unsigned), st));
    hipLaunchKernelGGL(bin_count_kernel, dim3(grid_of(p->nnz)), dim3(256), 0, st, d_rp, d_col, p->nnz, d_bstart, NB,
                       d_row0, (int32_t)p->bin.strip, S, d_cnt, d_bad);
    SPMV_RETURN_IF(finish(st, "counts"));
    unsigned bad = 0;
    cnt.assign((size_t)(NB * S), 0);
    SPMV_HIP_TRY(hipMemcpy(cnt.data(), d_cnt, sizeof(int32_t) * cnt.size(), hipMemcpyDeviceToHost));
    SPMV_HIP_TRY(hipMemcpy(&bad, d_bad, sizeof(unsigned), hipMemcpyDeviceToHost));
    return bad ? kBinNeedHostBuild : SPMV_SUCCESS;
}

int bin_fill_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                    const std::vector<int32_t> &row0, const std::vector<int64_t> &bstart,
                    const std::vector<int32_t> &cnt, const std::vector<int64_t> &off1,
                    const std::vector<int64_t> &off2, const std::vector<int64_t> &run_off,
                    const std::vector<int64_t> &srun_off, int64_t S, int64_t E, int64_t ES) {
    BinDev &B = p->bin;
    const hipStream_t st = p->stream;
    const int64_t NB = (int64_t)row0.size() - 1, C = B.strip;
    // product offset of each bin's row group (nonzero only when groups
    // re-use one product buffer)
    std::vector<int64_t> pbb((size_t)NB, 0);
    if (B.reuse)
        for (int g = 0; g < B.G; ++g)
            for (int64_t b = B.g_bin[(size_t)g]; b < B.g_bin[(size_t)g + 1]; ++b) pbb[(size_t)b] = B.g_prod[(size_t)g];
    void *q;
    // val1 / cs1 / dst1 with the Mul's unclamped-batch slack (kBinMulSlack), zeroed
    // (Mul order: the entries fill [0, nnz) unpadded, the rest is slack)
    const int64_t Ez = B.mo ? p->nnz : E;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(double) * (size_t)(E + kBinMulSlack)));
    B.val1 = (double *)q;
    SPMV_HIP_TRY(hipMemsetAsync(B.val1 + Ez, 0, sizeof(double) * (size_t)(E - Ez + kBinMulSlack), st));
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(uint16_t) * (size_t)(E + kBinMulSlack)));
    B.cs1 = (uint16_t *)q;
    SPMV_HIP_TRY(hipMemsetAsync(B.cs1 + Ez, 0, sizeof(uint16_t) * (size_t)(E - Ez + kBinMulSlack), st));
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(uint16_t) * (size_t)std::max<int64_t>(ES, 1)));
    B.slot2 = (uint16_t *)q;
    if (!B.mo) {  // Mul-ordered products need no destinations
        SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(int32_t) * (size_t)std::max<int64_t>((E + kBinMulSlack) >> B.pad_log, 1)));
        B.dst1 = (int32_t *)q;
        SPMV_HIP_TRY(hipMemsetAsync(B.dst1 + (E >> B.pad_log), 0, sizeof(int32_t) * (size_t)(kBinMulSlack >> B.pad_log), st));
    }
    Scratch sc{st, {}};
    int32_t *d_row0, *d_cnt;
    int64_t *d_bstart, *d_off1, *d_off2, *d_pbb, *d_ks, *d_run, *d_srun;
    unsigned long long *d_kh;
    SPMV_RETURN_IF(sc.upload(&d_row0, row0));
    SPMV_RETURN_IF(sc.upload(&d_bstart, bstart));
    SPMV_RETURN_IF(sc.upload(&d_cnt, cnt));
    SPMV_RETURN_IF(sc.upload(&d_off1, off1));
    SPMV_RETURN_IF(sc.upload(&d_off2, off2));
    SPMV_RETURN_IF(sc.upload(&d_run, run_off));
    SPMV_RETURN_IF(sc.upload(&d_srun, srun_off));
    // every slot starts as the dummy slot (segment padding and the padding of
    // each slot run to whole Sum batches)
    hipLaunchKernelGGL(fill_u16_kernel, dim3(grid_of(ES)), dim3(256), 0, st, B.slot2, ES, (uint16_t)B.max_rows);
    SPMV_RETURN_IF(sc.upload(&d_pbb, pbb));
    SPMV_RETURN_IF(sc.alloc(&d_kh, (size_t)E));
    SPMV_RETURN_IF(sc.alloc(&d_ks, (size_t)E));
    SPMV_HIP_TRY(hipMemsetAsync(d_kh, 0, 8 * (size_t)E, st));
    const unsigned grid = grid_of(p->nnz);
    hipLaunchKernelGGL(bin_khist_kernel, dim3(grid), dim3(256), 0, st, d_rp, d_col, p->nnz, d_bstart, NB, d_row0,
                       (int32_t)C, S, d_off2, d_kh);
    SPMV_RETURN_IF(exclusive_scan_i64((const int64_t *)d_kh, d_ks, E, st, sc.v));
    SPMV_HIP_TRY(hipMemsetAsync(d_kh, 0, 8 * (size_t)E, st));  // now the k-run cursors
    hipLaunchKernelGGL(bin_place_kernel, dim3(grid), dim3(256), 0, st, d_rp, d_col, d_val, p->nnz, d_bstart, NB,
                       d_row0, (int32_t)C, S, d_off1, d_off2, d_ks, d_kh, d_pbb, B.pad_log, d_run, d_srun,
                       B.strip_block, B.sum_u, B.val1, B.cs1, B.slot2,
                       B.dst1);
    if (!B.mo)  // (Mul order: the Mul's segments are not padded)
        hipLaunchKernelGGL(bin_pad_kernel, dim3(grid_of(NB * S)), dim3(256), 0, st, d_cnt, NB * S, d_off1, B.pad_log,
                           B.val1, B.cs1);
    return finish(st, "fill");
}

}  // namespace spmv

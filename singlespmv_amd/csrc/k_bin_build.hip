// k_bin_build.hip -- BIN fill from a CSR already in HBM (build_bin_device in
// build_bin.cpp drives it).  The OptimizeProblem counterpart is opt_ss's
// host-side segment build (src/opt_ss.cpp:52-142); here a 1 G-entry matrix
// never round-trips through the host: only the row pointers (to cut the row
// bins), the (bin, strip) entry counts (to lay out the segments) and the long
// rows' runs visit it.
//
// One thread per CSR entry j:
//   bin   b = last bin whose first entry <= j     (binary search, NB + 1 starts)
//   row   r = last row of b whose first entry <= j (binary search in row_ptr)
//   strip t = col[j] / C
//   k       = ordinal of j among row r's entries in strip t
//             (= j - first entry of r in strip t; rows must have
//              non-decreasing strips, checked by bin_count_kernel -- a CSR
//              with rows out of strip order is first sorted by strip per
//              row, stably, bin_sort_rows_device)
// Phases: counts per (b, t) -> [host offsets] -> key off2(b, t) + k per
// entry -> stable radix sort of (key, j) -> placement: the i-th sorted entry
// sits at i - (entries of the earlier segments) in its segment -> padding.
// Within a segment that is the host fill's order exactly -- k-runs ascending,
// rows ascending inside a k-run (the sort is stable and j ascends with the
// row) -- so the arrays are byte-identical to the host-built plan's
// (spmv_plan_digest, tests/test_gpu_parity.py::test_bin_device_build).
#include <hipcub/hipcub.hpp>

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

// a long row (>= LL entries, LL > 0) takes the run path, not the segments
__device__ __forceinline__ bool is_long(const int64_t *__restrict__ rp, int64_t r, int64_t LL) {
    return LL > 0 && rp[r + 1] - rp[r] >= LL;
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
                                                        int64_t LL, int32_t *__restrict__ cnt,
                                                        unsigned *__restrict__ bad) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * 256) {
        const EntryPos e = locate(j, rp, bstart, NB, row0);
        const int32_t t = col[j] / C;
        if (!is_long(rp, e.r, LL)) atomicAdd(&cnt[e.b * S + t], 1);
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

// sort key of entry j: its (bin, strip) segment's Sum position + k (long
// rows: `none`, past every segment); value: j
template <typename K, typename V>
__global__ __launch_bounds__(256) void bin_key_kernel(const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                      int64_t nnz, const int64_t *__restrict__ bstart, int64_t NB,
                                                      const int32_t *__restrict__ row0, int32_t C, int64_t S,
                                                      const int64_t *__restrict__ off2, int64_t LL, K none,
                                                      K *__restrict__ keys, V *__restrict__ vals) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * 256) {
        const EntryPos e = locate(j, rp, bstart, NB, row0);
        K key = none;
        if (!is_long(rp, e.r, LL)) {
            const int32_t t = col[j] / C;
            key = (K)(off2[e.b * S + t] + entry_k(j, e.r, t, C, rp, col));
        }
        keys[j] = key;
        vals[j] = (V)j;
    }
}

// the i-th entry in key order (i < the segments' entries): position
// i - cbase(segment) in its segment
template <typename V>
__global__ __launch_bounds__(256) void bin_place_kernel(
    const int64_t *__restrict__ rp, const int32_t *__restrict__ col, const double *__restrict__ val,
    const V *__restrict__ order, int64_t n_seg_entries, const int64_t *__restrict__ bstart, int64_t NB,
    const int32_t *__restrict__ row0, int32_t C, int64_t S, const int64_t *__restrict__ off1,
    const int64_t *__restrict__ off2, const int64_t *__restrict__ cbase, const int64_t *__restrict__ pbb, int pad_log,
    const int64_t *__restrict__ run_off, const int64_t *__restrict__ srun_off, int64_t SB, int sum_u,
    double *__restrict__ val1, uint16_t *__restrict__ cs1, uint16_t *__restrict__ slot2, int32_t *__restrict__ dst1) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_seg_entries; i += (int64_t)gridDim.x * 256) {
        const int64_t j = (int64_t)order[i];
        const EntryPos e = locate(j, rp, bstart, NB, row0);
        const int32_t c = col[j];
        const int32_t t = c / C;
        const int64_t seg = e.b * S + t;
        const int64_t o1 = off1[seg], o2 = off2[seg];
        const int64_t pos = i - cbase[seg];
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

__global__ __launch_bounds__(256) void fill_i32_kernel(int32_t *__restrict__ a, int64_t n, int32_t v) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) a[i] = v;
}

// ---- rows whose strips are out of order: each row's entries stably sorted
// by strip (CSR order kept inside a strip, the order the host fill reads
// them in) -- key = row * S + strip, value = entry
template <typename V>
__global__ __launch_bounds__(256) void bin_row_strip_key_kernel(const int64_t *__restrict__ rp, int64_t m,
                                                                const int32_t *__restrict__ col, int64_t nnz,
                                                                int32_t C, int64_t S, uint64_t *__restrict__ keys,
                                                                V *__restrict__ vals) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * 256) {
        const int64_t r = upper_idx(rp, 0, m + 1, j) - 1;
        keys[j] = (uint64_t)r * (uint64_t)S + (uint64_t)(col[j] / C);
        vals[j] = (V)j;
    }
}

template <typename V>
__global__ __launch_bounds__(256) void bin_gather_entries_kernel(const V *__restrict__ order, int64_t nnz,
                                                                 const int32_t *__restrict__ col,
                                                                 const double *__restrict__ val,
                                                                 int32_t *__restrict__ col2, double *__restrict__ val2) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * 256) {
        const int64_t j = (int64_t)order[i];
        col2[i] = col[j];
        val2[i] = val[j];
    }
}

// ---- long rows (the run path, internal.hpp BinDev) ----------------------
// one wave per long row: its runs, the maximal ranges of entries in one
// strip (a row's strips are non-decreasing, so a (row, strip) pair is one
// contiguous range).  roff == nullptr: count them into nruns; else write
// each run's strip and first entry at the row's offset roff[i].
__global__ __launch_bounds__(256) void bin_long_runs_kernel(int64_t nl, const int32_t *__restrict__ lrows,
                                                            const int64_t *__restrict__ rp,
                                                            const int32_t *__restrict__ col, int32_t C,
                                                            const int64_t *__restrict__ roff,
                                                            int32_t *__restrict__ nruns,
                                                            int32_t *__restrict__ rstrip,
                                                            int64_t *__restrict__ rbeg) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= nl) return;
    const int64_t r = lrows[i], a = rp[r], z = rp[r + 1];
    int64_t k = roff ? roff[i] : 0;
    for (int64_t j0 = a; j0 < z; j0 += 64) {
        const int64_t j = j0 + lane;
        int32_t t = 0;
        bool st = false;
        if (j < z) {
            t = col[j] / C;
            st = j == a || col[j - 1] / C != t;
        }
        const uint64_t m = __ballot(st);
        if (roff && st) {
            const int64_t q = k + __popcll(m & ((1ull << lane) - 1));
            rstrip[q] = t;
            rbeg[q] = j;
        }
        k += __popcll(m);
    }
    if (!roff && lane == 0) nruns[i] = (int32_t)k;
}

// one wave per run (sorted [strip][row], BinLongRuns): its entries into the
// strip's long block, lcode = piece start bit | (last entry of its piece ?
// the piece's product position : 0x7FFFFFFF); pieces start at the run's
// first entry and at every 64-entry boundary of the block, and number on
// from the run's first piece (fpos); each piece's slot in its bin's long run
__global__ __launch_bounds__(256) void bin_long_fill_kernel(
    int64_t R, const int64_t *__restrict__ j0, const int32_t *__restrict__ len, const int32_t *__restrict__ strip,
    const int32_t *__restrict__ slot, const int32_t *__restrict__ bin, const int64_t *__restrict__ q0,
    const int64_t *__restrict__ fpos, const int32_t *__restrict__ col, const double *__restrict__ val, int32_t C,
    const int64_t *__restrict__ lstart, const int64_t *__restrict__ lcode_off, const int64_t *__restrict__ run_off,
    const int64_t *__restrict__ srun_off, int64_t lrun0, int sum_u, double *__restrict__ val1,
    uint16_t *__restrict__ cs1, int32_t *__restrict__ lcode, uint16_t *__restrict__ slot2) {
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (g >= R) return;
    const int64_t a = j0[g], q = q0[g], n = len[g], fp = fpos[g];
    const int32_t t = strip[g];
    const int64_t ms = lstart[t], cs = lcode_off[t], run = lrun0 + bin[g];
    for (int64_t i = lane; i < n; i += 64) {
        const int64_t p2 = q + i;
        const bool start = i == 0 || (p2 & 63) == 0;
        const bool end = i + 1 == n || ((p2 + 1) & 63) == 0;
        const int64_t pos = fp + (p2 >> 6) - (q >> 6);
        val1[ms + p2] = val[a + i];
        cs1[ms + p2] = (uint16_t)(col[a + i] - t * C);
        lcode[cs + p2] = (int32_t)((start ? 0x80000000u : 0u) | (end ? (uint32_t)pos : 0x7FFFFFFFu));
        if (start) slot2[bin_slot_index(pos, run_off[run], srun_off[run], sum_u)] = (uint16_t)slot[g];
    }
}

// padding lanes of each strip's long block: their own piece, to the trash line
__global__ __launch_bounds__(256) void bin_long_pad_kernel(int64_t S, const int64_t *__restrict__ lb_off,
                                                           const int64_t *__restrict__ lpad,
                                                           const int64_t *__restrict__ lcode_off, int32_t trash,
                                                           int32_t *__restrict__ lcode) {
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < S; t += (int64_t)gridDim.x * 256)
        for (int64_t p2 = lb_off[t + 1] - lb_off[t]; p2 < lpad[t]; ++p2)
            lcode[lcode_off[t] + p2] = (int32_t)(0x80000000u | (uint32_t)trash);
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

struct SortPlaceArgs {
    const int64_t *rp;
    const int32_t *col;
    const double *val;
    int64_t NB, S;
    const int32_t *row0;
    const int64_t *bstart, *off1, *off2, *cbase, *pbb, *run, *srun;
    int64_t E, LL, n_seg;
};

// keys, stable radix sort (the keys' significant bits only), placement
template <typename K, typename V>
int bin_sort_place(spmv_plan_s *p, Scratch &sc, const SortPlaceArgs &A) {
    BinDev &B = p->bin;
    const hipStream_t st = p->stream;
    const int64_t nnz = p->nnz;
    int bits = 1;  // none = 2^bits - 1 >= E > every key
    while (bits < (int)(8 * sizeof(K)) && (((uint64_t)1 << bits) - 1) < (uint64_t)A.E) ++bits;
    const K none = bits >= 64 ? (K)~0ull : (K)(((uint64_t)1 << bits) - 1);
    K *k0, *k1;
    V *v0, *v1;
    SPMV_RETURN_IF(sc.alloc(&k0, (size_t)nnz));
    SPMV_RETURN_IF(sc.alloc(&k1, (size_t)nnz));
    SPMV_RETURN_IF(sc.alloc(&v0, (size_t)nnz));
    SPMV_RETURN_IF(sc.alloc(&v1, (size_t)nnz));
    const unsigned grid = grid_of(nnz);
    hipLaunchKernelGGL((bin_key_kernel<K, V>), dim3(grid), dim3(256), 0, st, A.rp, A.col, nnz, A.bstart, A.NB, A.row0,
                       (int32_t)B.strip, A.S, A.off2, A.LL, none, k0, v0);
    hipcub::DoubleBuffer<K> dk(k0, k1);
    hipcub::DoubleBuffer<V> dv(v0, v1);
    size_t tb = 0;
    SPMV_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dv, nnz, 0, bits, st));
    char *tmp = nullptr;
    SPMV_RETURN_IF(sc.alloc(&tmp, tb));
    SPMV_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dv, nnz, 0, bits, st));
    hipLaunchKernelGGL((bin_place_kernel<V>), dim3(grid_of(A.n_seg)), dim3(256), 0, st, A.rp, A.col, A.val,
                       (const V *)dv.Current(), A.n_seg, A.bstart, A.NB, A.row0, (int32_t)B.strip, A.S, A.off1, A.off2,
                       A.cbase, A.pbb, B.pad_log, A.run, A.srun, B.strip_block, B.sum_u, B.val1, B.cs1, B.slot2,
                       B.dst1);
    return SPMV_SUCCESS;
}

template <typename V>
int bin_sort_rows_t(spmv_plan_s *p, Scratch &sc, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                    int32_t *col2, double *val2) {
    const hipStream_t st = p->stream;
    const int64_t m = p->m, nnz = p->nnz, C = p->bin.strip, S = std::max<int64_t>(1, (p->n + C - 1) / C);
    int bits = 1;
    while (bits < 64 && (((uint64_t)1 << bits) - 1) < (uint64_t)m * (uint64_t)S) ++bits;
    uint64_t *k0, *k1;
    V *v0, *v1;
    SPMV_RETURN_IF(sc.alloc(&k0, (size_t)nnz));
    SPMV_RETURN_IF(sc.alloc(&k1, (size_t)nnz));
    SPMV_RETURN_IF(sc.alloc(&v0, (size_t)nnz));
    SPMV_RETURN_IF(sc.alloc(&v1, (size_t)nnz));
    hipLaunchKernelGGL((bin_row_strip_key_kernel<V>), dim3(grid_of(nnz)), dim3(256), 0, st, d_rp, m, d_col, nnz,
                       (int32_t)C, S, k0, v0);
    hipcub::DoubleBuffer<uint64_t> dk(k0, k1);
    hipcub::DoubleBuffer<V> dv(v0, v1);
    size_t tb = 0;
    SPMV_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dv, nnz, 0, bits, st));
    char *tmp = nullptr;
    SPMV_RETURN_IF(sc.alloc(&tmp, tb));
    SPMV_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dv, nnz, 0, bits, st));
    hipLaunchKernelGGL((bin_gather_entries_kernel<V>), dim3(grid_of(nnz)), dim3(256), 0, st, (const V *)dv.Current(),
                       nnz, d_col, d_val, col2, val2);
    return finish(st, "row strip sort");
}

}  // namespace

int bin_count_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const std::vector<int32_t> &row0,
                     const std::vector<int64_t> &bstart, int64_t S, int64_t LL, std::vector<int32_t> &cnt) {
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
                       d_row0, (int32_t)p->bin.strip, S, LL, d_cnt, d_bad);
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
                    const std::vector<int64_t> &srun_off, int64_t S, int64_t E, int64_t ES, int64_t LL, int64_t E1,
                    int32_t dst_fill) {
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
    // val1 / cs1 / dst1 over the Mul positions [0, E1) with the Mul's
    // unclamped-batch slack (kBinMulSlack), zeroed past the entries (Mul
    // order: the entries fill [0, nnz) unpadded, the rest is slack).  With
    // long rows the Mul positions hold voids and long blocks too: all zeroed
    // first, and every destination group points at the trash line (dst_fill)
    // until a segment claims it -- as the host fill leaves them.
    const int64_t Ez = LL > 0 ? 0 : B.mo ? p->nnz : E;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(double) * (size_t)(E1 + kBinMulSlack)));
    B.val1 = (double *)q;
    SPMV_HIP_TRY(hipMemsetAsync(B.val1 + Ez, 0, sizeof(double) * (size_t)(E1 - Ez + kBinMulSlack), st));
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(uint16_t) * (size_t)(E1 + kBinMulSlack)));
    B.cs1 = (uint16_t *)q;
    SPMV_HIP_TRY(hipMemsetAsync(B.cs1 + Ez, 0, sizeof(uint16_t) * (size_t)(E1 - Ez + kBinMulSlack), st));
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(uint16_t) * (size_t)std::max<int64_t>(ES, 1)));
    B.slot2 = (uint16_t *)q;
    if (!B.mo) {  // Mul-ordered products need no destinations
        const int64_t nd = (E1 + kBinMulSlack) >> B.pad_log;
        SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(int32_t) * (size_t)std::max<int64_t>(nd, 1)));
        B.dst1 = (int32_t *)q;
        if (LL > 0)
            hipLaunchKernelGGL(fill_i32_kernel, dim3(grid_of(nd)), dim3(256), 0, st, B.dst1, nd, dst_fill);
        else
            SPMV_HIP_TRY(hipMemsetAsync(B.dst1 + (E >> B.pad_log), 0, sizeof(int32_t) * (size_t)(kBinMulSlack >> B.pad_log), st));
    }
    Scratch sc{st, {}};
    int32_t *d_row0, *d_cnt;
    int64_t *d_bstart, *d_off1, *d_off2, *d_cbase, *d_pbb, *d_run, *d_srun;
    // cbase: entries of the segments before each one in the Sum order
    // ([strip block][bin][strip], bin_offsets), i.e. the sorted index of its
    // first entry
    std::vector<int64_t> cbase((size_t)(NB * S));
    int64_t n_seg = 0;
    {
        const int64_t SB = B.strip_block > 0 ? B.strip_block : S;
        for (int64_t k = 0; k * SB < S; ++k)
            for (int64_t b = 0; b < NB; ++b)
                for (int64_t t = k * SB; t < std::min(S, (k + 1) * SB); ++t) {
                    cbase[(size_t)(b * S + t)] = n_seg;
                    n_seg += cnt[(size_t)(b * S + t)];
                }
    }
    SPMV_RETURN_IF(sc.upload(&d_row0, row0));
    SPMV_RETURN_IF(sc.upload(&d_bstart, bstart));
    SPMV_RETURN_IF(sc.upload(&d_cnt, cnt));
    SPMV_RETURN_IF(sc.upload(&d_off1, off1));
    SPMV_RETURN_IF(sc.upload(&d_off2, off2));
    SPMV_RETURN_IF(sc.upload(&d_cbase, cbase));
    SPMV_RETURN_IF(sc.upload(&d_run, run_off));
    SPMV_RETURN_IF(sc.upload(&d_srun, srun_off));
    // every slot starts as the dummy slot (segment padding and the padding of
    // each slot run to whole Sum batches)
    hipLaunchKernelGGL(fill_u16_kernel, dim3(grid_of(ES)), dim3(256), 0, st, B.slot2, ES, (uint16_t)B.max_rows);
    SPMV_RETURN_IF(sc.upload(&d_pbb, pbb));
    const SortPlaceArgs A{d_rp, d_col, d_val, NB, S, d_row0, d_bstart, d_off1, d_off2, d_cbase, d_pbb, d_run, d_srun,
                          E, LL, n_seg};
    if (E < ((int64_t)1 << 32) - 1 && p->nnz < ((int64_t)1 << 32))
        SPMV_RETURN_IF((bin_sort_place<uint32_t, uint32_t>(p, sc, A)));
    else
        SPMV_RETURN_IF((bin_sort_place<uint64_t, uint64_t>(p, sc, A)));
    if (!B.mo)  // (Mul order: the Mul's segments are not padded)
        hipLaunchKernelGGL(bin_pad_kernel, dim3(grid_of(NB * S)), dim3(256), 0, st, d_cnt, NB * S, d_off1, B.pad_log,
                           B.val1, B.cs1);
    return finish(st, "fill");
}

int bin_long_runs_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const std::vector<int32_t> &lrows,
                         std::vector<int64_t> &roff, std::vector<int32_t> &rstrip, std::vector<int64_t> &rbeg) {
    const hipStream_t st = p->stream;
    const int64_t nl = (int64_t)lrows.size();
    const unsigned grid = (unsigned)std::max<int64_t>(1, (nl + 3) / 4);
    Scratch sc{st, {}};
    int32_t *d_lrows, *d_n, *d_strip;
    int64_t *d_roff, *d_beg;
    SPMV_RETURN_IF(sc.upload(&d_lrows, lrows));
    SPMV_RETURN_IF(sc.alloc(&d_n, (size_t)nl));
    hipLaunchKernelGGL(bin_long_runs_kernel, dim3(grid), dim3(256), 0, st, nl, d_lrows, d_rp, d_col,
                       (int32_t)p->bin.strip, (const int64_t *)nullptr, d_n, (int32_t *)nullptr, (int64_t *)nullptr);
    SPMV_RETURN_IF(finish(st, "long-row runs"));
    std::vector<int32_t> n((size_t)nl);
    SPMV_HIP_TRY(hipMemcpy(n.data(), d_n, sizeof(int32_t) * (size_t)nl, hipMemcpyDeviceToHost));
    roff.assign((size_t)nl + 1, 0);
    for (int64_t i = 0; i < nl; ++i) roff[(size_t)i + 1] = roff[(size_t)i] + n[(size_t)i];
    const int64_t R = roff[(size_t)nl];
    SPMV_RETURN_IF(sc.upload(&d_roff, roff));
    SPMV_RETURN_IF(sc.alloc(&d_strip, (size_t)R));
    SPMV_RETURN_IF(sc.alloc(&d_beg, (size_t)R));
    hipLaunchKernelGGL(bin_long_runs_kernel, dim3(grid), dim3(256), 0, st, nl, d_lrows, d_rp, d_col,
                       (int32_t)p->bin.strip, (const int64_t *)d_roff, d_n, d_strip, d_beg);
    SPMV_RETURN_IF(finish(st, "long-row runs"));
    rstrip.resize((size_t)R);
    rbeg.resize((size_t)R);
    SPMV_HIP_TRY(hipMemcpy(rstrip.data(), d_strip, sizeof(int32_t) * (size_t)R, hipMemcpyDeviceToHost));
    SPMV_HIP_TRY(hipMemcpy(rbeg.data(), d_beg, sizeof(int64_t) * (size_t)R, hipMemcpyDeviceToHost));
    return SPMV_SUCCESS;
}

int bin_long_fill_device(spmv_plan_s *p, const int32_t *d_col, const double *d_val, const BinLongRuns &LR,
                         const std::vector<int64_t> &lb_off, const std::vector<int64_t> &lpad,
                         const std::vector<int64_t> &lstart, const std::vector<int64_t> &lcode_off,
                         const std::vector<int64_t> &run_off, const std::vector<int64_t> &srun_off, int64_t lrun0,
                         int64_t trash) {
    BinDev &B = p->bin;
    const hipStream_t st = p->stream;
    const int64_t S = (int64_t)lpad.size(), R = (int64_t)LR.j0.size();
    void *q;
    const int64_t ncode = lcode_off.back() + lpad.back();
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(int32_t) * (size_t)std::max<int64_t>(ncode, 1)));
    B.lcode = (int32_t *)q;
    Scratch sc{st, {}};
    int64_t *d_j0, *d_q0, *d_fpos, *d_lb, *d_lpad, *d_lstart, *d_lco, *d_run, *d_srun;
    int32_t *d_len, *d_strip, *d_slot, *d_bin;
    SPMV_RETURN_IF(sc.upload(&d_j0, LR.j0));
    SPMV_RETURN_IF(sc.upload(&d_q0, LR.q0));
    SPMV_RETURN_IF(sc.upload(&d_fpos, LR.fpos));
    SPMV_RETURN_IF(sc.upload(&d_len, LR.len));
    SPMV_RETURN_IF(sc.upload(&d_strip, LR.strip));
    SPMV_RETURN_IF(sc.upload(&d_slot, LR.slot));
    SPMV_RETURN_IF(sc.upload(&d_bin, LR.bin));
    SPMV_RETURN_IF(sc.upload(&d_lb, lb_off));
    SPMV_RETURN_IF(sc.upload(&d_lpad, lpad));
    SPMV_RETURN_IF(sc.upload(&d_lstart, lstart));
    SPMV_RETURN_IF(sc.upload(&d_lco, lcode_off));
    SPMV_RETURN_IF(sc.upload(&d_run, run_off));
    SPMV_RETURN_IF(sc.upload(&d_srun, srun_off));
    if (R > 0)
        hipLaunchKernelGGL(bin_long_fill_kernel, dim3((unsigned)std::max<int64_t>(1, (R + 3) / 4)), dim3(256), 0, st, R,
                           d_j0, d_len, d_strip, d_slot, d_bin, d_q0, d_fpos, d_col, d_val, (int32_t)B.strip, d_lstart,
                           d_lco, d_run, d_srun, lrun0, B.sum_u, B.val1, B.cs1, B.lcode, B.slot2);
    hipLaunchKernelGGL(bin_long_pad_kernel, dim3(grid_of(S)), dim3(256), 0, st, S, d_lb, d_lpad, d_lco, (int32_t)trash,
                       B.lcode);
    return finish(st, "long rows");
}

int bin_sort_rows_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                         int32_t *col2, double *val2) {
    Scratch sc{p->stream, {}};
    if (p->nnz < ((int64_t)1 << 32)) return bin_sort_rows_t<uint32_t>(p, sc, d_rp, d_col, d_val, col2, val2);
    return bin_sort_rows_t<uint64_t>(p, sc, d_rp, d_col, d_val, col2, val2);
}

}  // namespace spmv

// formats.cpp -- host-side OptimizeProblem counterparts: build each device
// layout from a CSR view and upload it once (the reference does this untimed
// in OptimizeProblem, src/main.cpp:36).  OpenMP-parallel, 64-bit counts.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <numeric>
#include <queue>
#include <vector>

#include "internal.hpp"

namespace spmv {

int DevArena::alloc(void **p, size_t n) {
    if (n == 0) n = 16;
    if (vmm_min > 0 && n >= vmm_min) return alloc_vmm(p, n, kVmmChunk, device, kVmmAlign);
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, n);
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc(") + std::to_string(n) + "): " + hipGetErrorString(e));
        (void)hipGetLastError();
        return e == hipErrorOutOfMemory ? SPMV_ERROR_OUT_OF_MEMORY : SPMV_ERROR_HIP;
    }
    ptrs.push_back(q);
    bytes += (int64_t)n;
    *p = q;
    return SPMV_SUCCESS;
}

// Physical memory in `chunk`-byte handles (hipMemCreate) mapped back to back
// into one reserved VA range.  chunk is rounded to the allocation granularity.
int DevArena::alloc_vmm(void **p, size_t n, size_t chunk, int device, size_t align) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    SPMV_HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    if (gran == 0) gran = (size_t)2 << 20;
    if (n == 0) n = 16;
    const size_t need = (n + gran - 1) / gran * gran;
    chunk = std::min(need, std::max(gran, (chunk + gran - 1) / gran * gran));
    const size_t total = (n + chunk - 1) / chunk * chunk;
    VmmMap m;
    m.bytes = total;
    m.chunk = chunk;
    auto undo = [&](hipError_t e, const char *what) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        (void)hipGetLastError();
        for (size_t k = 0; k < m.handles.size(); ++k) {
            (void)hipMemUnmap((char *)m.va + k * chunk, chunk);
            (void)hipMemRelease(m.handles[k]);
        }
        if (m.res) (void)hipMemAddressFree(m.res, m.res_bytes);
        return e == hipErrorOutOfMemory ? SPMV_ERROR_OUT_OF_MEMORY : SPMV_ERROR_HIP;
    };
    align = align > gran ? (align + gran - 1) / gran * gran : 0;
    m.res_bytes = total + align;
    hipError_t e = hipMemAddressReserve(&m.res, m.res_bytes, gran, nullptr, 0);
    if (e != hipSuccess) return undo(e, "hipMemAddressReserve");
    m.va = align ? (void *)(((uintptr_t)m.res + align - 1) / align * align) : m.res;
    // all handles first, then mapped -- in creation order, or (probe build,
    // SPMV_VMM_SHUFFLE) handle k at chunk slot k * P mod count
    const size_t cnt = total / chunk;
    // probe build, SPMV_VMM_STRIDE=K: create K times the handles and keep
    // every K-th (the others are released once the kept ones are mapped), so
    // physically consecutive blocks do not back consecutive chunks
    size_t K = 1;
    if (const char *st = probe_env("SPMV_VMM_STRIDE")) K = (size_t)std::max(1, std::min(8, std::atoi(st)));
    std::vector<hipMemGenericAllocationHandle_t> spare;
    for (size_t k = 0; k < cnt * K; ++k) {
        hipMemGenericAllocationHandle_t h;
        e = hipMemCreate(&h, chunk, &prop, 0);
        if (e != hipSuccess) {
            for (auto hs : spare) (void)hipMemRelease(hs);
            return undo(e, "hipMemCreate");
        }
        if (k % K == 0) m.handles.push_back(h);
        else spare.push_back(h);
    }
    size_t P = 1;
    if (const char *sh = probe_env("SPMV_VMM_SHUFFLE"))
        if (std::atoi(sh) && cnt > 2) {
            P = (size_t)(0.6180339887 * (double)cnt) | 1;
            while (std::gcd(P, cnt) != 1) P += 2;
        }
    std::vector<hipMemGenericAllocationHandle_t> slot(cnt);
    for (size_t k = 0; k < cnt; ++k) slot[(k * P) % cnt] = m.handles[k];
    m.handles = slot;  // handles[k] is mapped at chunk slot k
    for (size_t k = 0; k < cnt; ++k) {
        e = hipMemMap((char *)m.va + k * chunk, chunk, 0, m.handles[k], 0);
        if (e != hipSuccess) {
            for (size_t j = k; j < cnt; ++j) (void)hipMemRelease(m.handles[j]);
            for (auto hs : spare) (void)hipMemRelease(hs);
            m.handles.resize(k);
            return undo(e, "hipMemMap");
        }
    }
    for (auto hs : spare) (void)hipMemRelease(hs);
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(m.va, total, &acc, 1);
    if (e != hipSuccess) return undo(e, "hipMemSetAccess");
    maps.push_back(m);
    bytes += (int64_t)total;
    *p = m.va;
    return SPMV_SUCCESS;
}

static void vmm_release(const VmmMap &m) {
    (void)hipDeviceSynchronize();
    for (size_t k = 0; k < m.handles.size(); ++k) {
        (void)hipMemUnmap((char *)m.va + k * m.chunk, m.chunk);
        (void)hipMemRelease(m.handles[k]);
    }
    (void)hipMemAddressFree(m.res, m.res_bytes);
}

void DevArena::free(void *p) {
    for (size_t i = 0; i < maps.size(); ++i)
        if (maps[i].va == p) {
            vmm_release(maps[i]);
            bytes -= (int64_t)maps[i].bytes;
            maps.erase(maps.begin() + (long)i);
            return;
        }
    for (size_t i = 0; i < ptrs.size(); ++i)
        if (ptrs[i] == p) {
            size_t n = 0;
            (void)hipMemPtrGetInfo(p, &n);
            (void)hipFree(p);
            bytes -= (int64_t)n;
            ptrs.erase(ptrs.begin() + (long)i);
            return;
        }
}

void DevArena::release() {
    for (const VmmMap &m : maps) vmm_release(m);
    maps.clear();
    for (void *q : ptrs) (void)hipFree(q);
    ptrs.clear();
    bytes = 0;
}

// Allocate count+pad elements, copy count from host, zero the pad.
template <typename T>
static int upload(spmv_plan_s *p, T **dst, const T *src, int64_t count, int64_t pad = 0) {
    void *q = nullptr;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(T) * (size_t)(count + pad)));
    if (count > 0) SPMV_HIP_TRY(hipMemcpy(q, src, sizeof(T) * (size_t)count, hipMemcpyHostToDevice));
    if (pad > 0) SPMV_HIP_TRY(hipMemset((char *)q + sizeof(T) * count, 0, sizeof(T) * (size_t)pad));
    *dst = (T *)q;
    return SPMV_SUCCESS;
}

template <typename T>
static int dev_alloc(spmv_plan_s *p, T **dst, int64_t count) {
    void *q = nullptr;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(T) * (size_t)count));
    *dst = (T *)q;
    return SPMV_SUCCESS;
}

static inline int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

int auto_csr_lanes(double mean_row) {
    // one 4-entry chunk per lane per row on average
    int L = 1;
    while (L < 64 && 4.0 * L < mean_row) L <<= 1;
    return L;
}

int auto_ss_sigma(double mean_row) {
    // ~one row boundary per lane keeps the in-lane work low while each lane
    // keeps SIGMA*12 bytes of loads in flight.  Long rows: 32 since the
    // streamed kernel (round 5: a lane holds PF + 1 quads, not SIGMA
    // entries -- round 4's tile kernel needed 172 VGPRs at 32 and lost with
    // it); config 4, same plans: SIGMA 20 / 32 / 48 / 64 at PF 2 2.629 /
    // 2.537 / 2.542 / 2.635 ms (profiles/round5/probe/c4_ss_sigma_pf_sweep.jsonl)
    if (mean_row <= 6) return 8;
    if (mean_row <= 24) return 16;
    return 32;
}

// ---------------------------------------------------------------- CSR
void csr_finish_info(spmv_plan_s *p) {
    const CsrDev &c = p->csr;
    p->stored_slots = p->nnz;
    p->algo_bytes = 12 * p->nnz + (c.rp64 ? 8 : 4) * (p->m + 1) + 8 * p->n + 8 * p->m;
    p->n_kernels = 1;
    if (c.lanes > 0) {
        p->kernel_name = std::string(c.win0 ? "csr_slabx_kernel<" : "csr_slab2_kernel<") + std::to_string(c.lanes) + ">";
    } else {
        p->kernel_name = "csr_adaptive_kernel";
        p->algo_bytes += 4 * p->m;  // the bins' row lists
        p->n_kernels = 1;
    }
}

// Length bin of a row (adaptive CSR): L = smallest power of two with 4L >=
// len (capped at 64), a whole workgroup beyond 4096 entries.
static int csr_bin_of(int64_t len) {
    if (len > 4096) return kCsrBins - 1;
    int b = 0;
    while (b < kCsrBins - 2 && 4 * (int64_t)kCsrBinLanes[b] < len) ++b;
    return b;
}

// Rows 0..m-1 of a CSR grouped by length bin (ascending within a bin).
static void csr_bin_rows(const int64_t *row_ptr, int64_t m, std::vector<int32_t> &rows,
                         int64_t off[kCsrBins + 1]) {
    int64_t cnt[kCsrBins] = {0};
    for (int64_t r = 0; r < m; ++r) ++cnt[csr_bin_of(row_ptr[r + 1] - row_ptr[r])];
    off[0] = 0;
    for (int b = 0; b < kCsrBins; ++b) off[b + 1] = off[b] + cnt[b];
    int64_t pos[kCsrBins];
    for (int b = 0; b < kCsrBins; ++b) pos[b] = off[b];
    rows.resize((size_t)m);
    for (int64_t r = 0; r < m; ++r) rows[(size_t)pos[csr_bin_of(row_ptr[r + 1] - row_ptr[r])]++] = (int32_t)r;
}

// Lanes per row.  An explicit csr_lanes applies to every row.  AUTO bins the
// rows by length (L = smallest power of two with 4L >= len, capped at 64;
// rows beyond 4096 entries get a whole workgroup) and, unless one bin holds
// >= 99 % of the rows with no row needing more than 16 steps of its lanes
// (then that L serves every row, no row list), keeps per-bin row lists.
int csr_plan_lanes(spmv_plan_s *p, const int64_t *row_ptr, int64_t m, const spmv_options_t &o) {
    CsrDev &c = p->csr;
    // 32-bit offsets of the slab kernel: the widest 64-row slab (+ one chunk
    // of 64 lanes' overreach) in bytes of val < 2^31, and x below 4 GB
    int64_t slab_max = 0;
#pragma omp parallel for schedule(static) reduction(max : slab_max)
    for (int64_t r = 0; r < m; r += 64)
        slab_max = std::max<int64_t>(slab_max, row_ptr[std::min<int64_t>(r + 64, m)] - row_ptr[r]);
    c.off32 = slab_max + 512 < ((int64_t)1 << 28) && p->n < ((int64_t)1 << 29);
    c.slab_max = slab_max;
    if (o.csr_lanes > 0) {
        c.lanes = o.csr_lanes;
        if (c.lanes < 1 || c.lanes > 64 || (c.lanes & (c.lanes - 1))) {
            set_error("csr_lanes must be a power of two in [1, 64]");
            return SPMV_ERROR_INVALID_VALUE;
        }
        // the row-group kernels hold a slab's row starts and entry index in
        // 32 bits, measured from the slab's first entry
        if (slab_max + 512 >= (int64_t)INT32_MAX) {
            set_error("csr_lanes: a 64-row slab holds >= 2^31 entries; use csr_lanes = 0 (adaptive)");
            return SPMV_ERROR_NOT_SUPPORTED;
        }
        return SPMV_SUCCESS;
    }
    auto bin_of = [](int64_t len) {
        if (len > 4096) return kCsrBins - 1;
        int b = 0;
        while (b < kCsrBins - 2 && 4 * (int64_t)kCsrBinLanes[b] < len) ++b;
        return b;
    };
    std::vector<uint8_t> bin((size_t)std::max<int64_t>(m, 1));
    int64_t cnt[kCsrBins] = {0};
    int64_t maxlen = 0;
#pragma omp parallel
    {
        int64_t lc[kCsrBins] = {0}, lmax = 0;
#pragma omp for schedule(static)
        for (int64_t r = 0; r < m; ++r) {
            const int64_t len = row_ptr[r + 1] - row_ptr[r];
            const int b = bin_of(len);
            bin[(size_t)r] = (uint8_t)b;
            ++lc[b];
            lmax = std::max(lmax, len);
        }
#pragma omp critical
        {
            for (int b = 0; b < kCsrBins; ++b) cnt[b] += lc[b];
            maxlen = std::max(maxlen, lmax);
        }
    }
    int d = 0;
    for (int b = 1; b < kCsrBins; ++b)
        if (cnt[b] > cnt[d]) d = b;
    if (m == 0 || (d < kCsrBins - 1 && (double)cnt[d] >= 0.99 * (double)m && cnt[kCsrBins - 1] == 0 &&
                   maxlen <= 64 * (int64_t)kCsrBinLanes[d])) {
        c.lanes = m ? kCsrBinLanes[d] : 1;
        return SPMV_SUCCESS;
    }
    c.lanes = 0;
    c.bin_off[0] = 0;
    for (int b = 0; b < kCsrBins; ++b) c.bin_off[b + 1] = c.bin_off[b] + cnt[b];
    std::vector<int32_t> rows((size_t)m);
    int64_t pos[kCsrBins];
    for (int b = 0; b < kCsrBins; ++b) pos[b] = c.bin_off[b];
    for (int64_t r = 0; r < m; ++r) rows[(size_t)pos[bin[(size_t)r]]++] = (int32_t)r;
    return upload(p, &c.bin_rows, rows.data(), m);
}

// x windows of csr_slabx's workgroups (k_csr.hip): the column span of each
// kCsrWinGroup-row granule's entries; a workgroup of S granules reads the
// union of theirs.  Kept when the default workgroup's union fits
// kCsrMaxWin columns (banded matrices), else none.
int csr_windows_finish(spmv_plan_s *p, const std::vector<int32_t> &lo, const std::vector<int32_t> &hi) {
    CsrDev &c = p->csr;
    const int64_t ng = (int64_t)lo.size();
    if (ng == 0 || p->n == 0 || p->nnz == 0) return SPMV_SUCCESS;  // no x to stage
    for (int si = 0; si < 3; ++si) {
        const int64_t S = (int64_t)1 << si;
        int64_t span = 1;
#pragma omp parallel for schedule(static) reduction(max : span)
        for (int64_t b = 0; b < ng; b += S) {
            int32_t l = std::numeric_limits<int32_t>::max(), h = -1;
            for (int64_t g = b; g < std::min(ng, b + S); ++g) {
                if (hi[(size_t)g] < 0) continue;  // no entries
                l = std::min(l, lo[(size_t)g]);
                h = std::max(h, hi[(size_t)g]);
            }
            if (h >= 0) span = std::max<int64_t>(span, (int64_t)h - l + 1);
        }
        c.win_s[si] = span <= kCsrMaxWin ? (int32_t)span : 0;
    }
    const int sd = kCsrSlabsPerWave == 4 ? 2 : kCsrSlabsPerWave == 2 ? 1 : 0;
    if (!c.win_s[sd]) return SPMV_SUCCESS;
    c.win = c.win_s[sd];
    std::vector<int32_t> w0(lo);
    for (int64_t g = 0; g < ng; ++g)
        if (hi[(size_t)g] < 0) w0[(size_t)g] = std::numeric_limits<int32_t>::max();  // empty: no lower bound
    return upload(p, &c.win0, w0.data(), ng);
}

static int csr_x_windows(spmv_plan_s *p, const HostCsr &A) {
    const int64_t ng = (A.m + kCsrWinGroup - 1) / kCsrWinGroup;
    std::vector<int32_t> lo((size_t)ng), hi((size_t)ng);
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < ng; ++b) {
        const int64_t e0 = A.row_ptr[b * kCsrWinGroup];
        const int64_t e1 = A.row_ptr[std::min<int64_t>(A.m, (b + 1) * kCsrWinGroup)];
        int32_t l = std::numeric_limits<int32_t>::max(), h = -1;
        for (int64_t j = e0; j < e1; ++j) {
            l = std::min(l, A.col[j]);
            h = std::max(h, A.col[j]);
        }
        lo[(size_t)b] = h < 0 ? 0 : l;
        hi[(size_t)b] = h;
    }
    return csr_windows_finish(p, lo, hi);
}

int build_csr(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o) {
    CsrDev &c = p->csr;
    // 64-bit row pointers from 2^31 entries on; SPMV_CSR_FORCE_RP64 (internal)
    // exercises that kernel instance on small matrices in the tests
    c.rp64 = A.nnz >= (int64_t)std::numeric_limits<int32_t>::max() - 64 || o.csr_row_ptr64 != 0 || probe_env("SPMV_CSR_FORCE_RP64");
    if (c.rp64) {
        SPMV_RETURN_IF(upload(p, (int64_t **)&c.row_ptr, A.row_ptr, A.m + 1));
    } else {
        std::vector<int32_t> rp32((size_t)A.m + 1);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i <= A.m; ++i) rp32[i] = (int32_t)A.row_ptr[i];
        SPMV_RETURN_IF(upload(p, (int32_t **)&c.row_ptr, rp32.data(), A.m + 1));
    }
    SPMV_RETURN_IF(upload(p, &c.col, A.col, A.nnz, kPad));
    SPMV_RETURN_IF(csr_plan_lanes(p, A.row_ptr, A.m, o));
    c.val_halves = csr_val_halves_wanted(c);
    if (c.val_halves) {
        const int64_t total = (A.nnz + 255) / 256 * 256;
        std::vector<double> vh((size_t)total);
#pragma omp parallel for schedule(static)
        for (int64_t pos = 0; pos < total; ++pos) {
            const int64_t e = csr_val_halves_entry(pos);
            vh[(size_t)pos] = e < A.nnz ? A.val[e] : 0.0;
        }
        SPMV_RETURN_IF(upload(p, &c.val, vh.data(), total, kPad));
    } else {
        SPMV_RETURN_IF(upload(p, &c.val, A.val, A.nnz, kPad));
    }
    if (c.lanes > 0) SPMV_RETURN_IF(csr_x_windows(p, A));
    csr_finish_info(p);
    return SPMV_SUCCESS;
}

// ---------------------------------------------------------------- ELL
// Slice offsets of the sliced-ELL layout from the row pointers alone (shared
// by the host and the device builders): slice s of 64 rows (rows order[i] when
// order is given) has width round_up(min(longest row, cap), 4); off[s] is its
// first slot, off[n_slices] the total.  Returns the widest slice.
int ell_slice_offsets(const int64_t *row_ptr, int64_t m, int cap, const int32_t *order, std::vector<int64_t> &off) {
    auto src = [&](int64_t r) -> int64_t { return order ? (int64_t)order[r] : r; };
    const int64_t ns = (m + 63) / 64;
    off.assign((size_t)ns + 1, 0);
    int maxw = 0;
#pragma omp parallel for schedule(static) reduction(max : maxw)
    for (int64_t s = 0; s < ns; ++s) {
        int64_t w = 0;
        const int64_t r1 = std::min<int64_t>(m, (s + 1) * 64);
        for (int64_t r = s * 64; r < r1; ++r) w = std::max<int64_t>(w, row_ptr[src(r) + 1] - row_ptr[src(r)]);
        w = std::min<int64_t>(w, cap);
        w = round_up(w, 4);
        off[s + 1] = 64 * w;
        maxw = std::max<int>(maxw, (int)w);
    }
    for (int64_t s = 0; s < ns; ++s) off[s + 1] += off[s];
    return maxw;
}

void ell_finish_info(spmv_plan_s *p, int maxw, int64_t total) {
    p->ell.max_width = maxw;
    p->ell.slots = total;
    p->stored_slots = total;
    p->algo_bytes = 12 * p->nnz + 8 * p->n + 8 * p->m;
    p->n_kernels = 1;
    p->kernel_name = "ell_slice_kernel";
}

// cap: maximum slots per row kept in the ELL part (HYB); INT32_MAX for ELL.
// order (JDS): slice row i is matrix row order[i]; nullptr = identity.
int build_ell(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &, int cap, const int32_t *order) {
    EllDev &e = p->ell;
    if (const char *u = probe_env("SPMV_ELL_UNROLL")) e.unroll = std::atoi(u);
    auto src = [&](int64_t r) -> int64_t { return order ? (int64_t)order[r] : r; };
    e.n_slices = (A.m + 63) / 64;
    std::vector<int64_t> off;
    const int maxw = ell_slice_offsets(A.row_ptr, A.m, cap, order, off);
    const int64_t total = off[e.n_slices];
    std::vector<int32_t> col((size_t)total);
    std::vector<double> val((size_t)total);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t s = 0; s < e.n_slices; ++s) {
        const int64_t base = off[s];
        const int64_t w = (off[s + 1] - base) / 64;
        for (int li = 0; li < 64; ++li) {
            const int64_t r = s * 64 + li;
            int64_t len = 0, rs = 0;
            if (r < A.m) {
                rs = A.row_ptr[src(r)];
                len = std::min<int64_t>(A.row_ptr[src(r) + 1] - rs, w);
            }
            int32_t last = 0;
            for (int64_t k = 0; k < w; ++k) {
                // columns: lane li's 4 slots of quad k/4 contiguous (16 B);
                // values: slots 0-1 in the quad's first 1 KB, 2-3 in its
                // second, lane li's pair at 16 B * li (k_ell.hip)
                const int64_t pos = base + (k >> 2) * 256 + li * 4 + (k & 3);
                const int64_t vpos = base + (k >> 2) * 256 + ((k & 2) ? 128 : 0) + li * 2 + (k & 1);
                if (k < len) {
                    last = A.col[rs + k];
                    col[pos] = last;
                    val[vpos] = A.val[rs + k];
                } else {
                    col[pos] = last;  // repeat a real column: no new cache line
                    val[vpos] = 0.0;
                }
            }
        }
    }
    SPMV_RETURN_IF(upload(p, &e.slice_off, off.data(), e.n_slices + 1));
    SPMV_RETURN_IF(upload(p, &e.col, col.data(), total));
    SPMV_RETURN_IF(upload(p, &e.val, val.data(), total));
    ell_finish_info(p, maxw, total);
    return SPMV_SUCCESS;
}

// ---------------------------------------------------------------- HYB / JDS overflow
// The entries of rows longer than K beyond their first K go to a CSR over
// those rows only (finished by the adaptive CSR kernel in y += mode).  The
// row list and its row pointers come from the matrix's row pointers alone.
void overflow_layout(const int64_t *row_ptr, int64_t m, int K, std::vector<int32_t> &rows, std::vector<int64_t> &rp) {
    rows.clear();
    rp.assign(1, 0);
    for (int64_t r = 0; r < m; ++r) {
        const int64_t len = row_ptr[r + 1] - row_ptr[r];
        if (len > K) {
            rows.push_back((int32_t)r);
            rp.push_back(rp.back() + (len - K));
        }
    }
}

// the overflow rows' index arrays (rows, row pointers, length bins) to the device
int overflow_upload_index(spmv_plan_s *p, const std::vector<int32_t> &rows, const std::vector<int64_t> &rp) {
    HybDev &h = p->hyb;
    h.n_rows = (int64_t)rows.size();
    h.nnz = rp.back();
    SPMV_RETURN_IF(upload(p, &h.rows, rows.data(), h.n_rows));
    SPMV_RETURN_IF(upload(p, &h.row_ptr, rp.data(), h.n_rows + 1));
    std::vector<int32_t> binned;
    csr_bin_rows(rp.data(), h.n_rows, binned, h.bin_off);
    return upload(p, &h.bin_rows, binned.data(), h.n_rows);
}

static int build_overflow(spmv_plan_s *p, const HostCsr &A, int K) {
    HybDev &h = p->hyb;
    std::vector<int32_t> rows;
    std::vector<int64_t> rp;
    overflow_layout(A.row_ptr, A.m, K, rows, rp);
    h.n_rows = (int64_t)rows.size();
    h.nnz = rp.back();
    std::vector<int32_t> col((size_t)h.nnz);
    std::vector<double> val((size_t)h.nnz);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < h.n_rows; ++i) {
        const int64_t src = A.row_ptr[rows[i]] + K;
        std::memcpy(&col[rp[i]], A.col + src, sizeof(int32_t) * (size_t)(rp[i + 1] - rp[i]));
        std::memcpy(&val[rp[i]], A.val + src, sizeof(double) * (size_t)(rp[i + 1] - rp[i]));
    }
    // overflow rows binned by overflow length (adaptive kernel, y +=)
    SPMV_RETURN_IF(overflow_upload_index(p, rows, rp));
    SPMV_RETURN_IF(upload(p, &h.col, col.data(), h.nnz, kPad));
    SPMV_RETURN_IF(upload(p, &h.val, val.data(), h.nnz, kPad));
    return SPMV_SUCCESS;
}

// ---------------------------------------------------------------- JDS
// opt_jds (src/opt_jds.cpp:29-71, 75-104): rows sorted by decreasing length
// (stable -- std::stable_sort's order, by a counting sort over the lengths),
// jagged diagonals = sliced ELL over the sorted rows, y written back through
// the permutation.  Jagged diagonals are capped at K (default max(64, 4 x mean
// row length)); the entries of longer rows beyond K are finished by the
// overflow kernel, so the longest-row slices do not run as single waves.
// Rows of length <= K are the sequential sum, bit for bit.
// jds_layout: that row order and K.  Returns true when the order is the
// identity (rows already in non-increasing length order, config 4): the
// slices then store rows in matrix order and the kernel writes y directly (no
// perm[] load, coalesced y).
bool jds_layout(const int64_t *row_ptr, int64_t m, int64_t nnz, const spmv_options_t &o, std::vector<int32_t> &order,
                int *K) {
    order.assign((size_t)std::max<int64_t>(m, 1), 0);
    int64_t maxlen = 0;
    bool identity = true;
    for (int64_t r = 0; r < m; ++r) {
        const int64_t len = row_ptr[r + 1] - row_ptr[r];
        if (r && len > row_ptr[r] - row_ptr[r - 1]) identity = false;
        maxlen = std::max(maxlen, len);
    }
    if (identity) {
        std::iota(order.begin(), order.begin() + m, 0);
    } else if (maxlen <= ((int64_t)1 << 24)) {
        // bucket start of length L = rows longer than L (descending, stable)
        std::vector<int64_t> start((size_t)maxlen + 2, 0);
        for (int64_t r = 0; r < m; ++r) ++start[(size_t)(maxlen - (row_ptr[r + 1] - row_ptr[r]) + 1)];
        for (int64_t k = 1; k <= maxlen + 1; ++k) start[(size_t)k] += start[(size_t)k - 1];
        for (int64_t r = 0; r < m; ++r) order[(size_t)start[(size_t)(maxlen - (row_ptr[r + 1] - row_ptr[r]))]++] = (int32_t)r;
    } else {
        std::iota(order.begin(), order.begin() + m, 0);
        std::stable_sort(order.begin(), order.begin() + m, [&](int32_t a, int32_t b) {
            return row_ptr[a + 1] - row_ptr[a] > row_ptr[b + 1] - row_ptr[b];
        });
    }
    const double mean = m ? (double)nnz / (double)m : 0.0;
    *K = o.ell_width > 0 ? (int)round_up(o.ell_width, 4)
                         : (int)std::max<int64_t>(64, round_up((int64_t)std::ceil(4.0 * mean), 4));
    return identity;
}

void jds_finish_info(spmv_plan_s *p, bool identity, int64_t ell_slots) {
    p->stored_slots = ell_slots + p->hyb.nnz;
    p->algo_bytes = 12 * p->nnz + 8 * p->n + 8 * p->m + (identity ? 0 : 4 * p->m) + 12 * p->hyb.n_rows;
    p->n_kernels = p->hyb.n_rows ? 2 : 1;
    const std::string ek = identity ? "ell_slice_kernel" : "ell_slice_kernel<perm>";
    p->kernel_name = p->hyb.n_rows ? ek + "+csr_adaptive_kernel" : ek;
}

int build_jds(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o) {
    std::vector<int32_t> order;
    int K = 0;
    const bool identity = jds_layout(A.row_ptr, A.m, A.nnz, o, order, &K);
    SPMV_RETURN_IF(build_ell(p, A, o, K, identity ? nullptr : order.data()));
    const int64_t ell_slots = p->stored_slots;
    if (!identity) SPMV_RETURN_IF(upload(p, &p->ell.perm, order.data(), A.m));
    SPMV_RETURN_IF(build_overflow(p, A, K));
    jds_finish_info(p, identity, ell_slots);
    return SPMV_SUCCESS;
}

// ---------------------------------------------------------------- COO
// opt_coo (src/opt_coo.cpp:21-47): zero y, then y[row] += val*x[col] with
// atomics; here one f64 atomic per equal-row run of a wave instead of one
// per entry.
int build_coo(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &) {
    CooDev &c = p->coo;
    // padded to whole 128-entry units; padding rows are -1 (no atomic)
    c.n_units = (A.nnz + kCooUnit - 1) / kCooUnit;
    const int64_t total = c.n_units * kCooUnit;
    std::vector<int32_t> row((size_t)std::max<int64_t>(total, 1), -1);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t r = 0; r < A.m; ++r)
        for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) row[(size_t)j] = (int32_t)r;
    SPMV_RETURN_IF(upload(p, &c.row, row.data(), total));
    SPMV_RETURN_IF(upload(p, &c.col, A.col, A.nnz, total - A.nnz));
    SPMV_RETURN_IF(upload(p, &c.val, A.val, A.nnz, total - A.nnz));
    coo_finish_info(p);
    return SPMV_SUCCESS;
}

void coo_finish_info(spmv_plan_s *p) {
    p->stored_slots = p->coo.n_units * kCooUnit;
    p->algo_bytes = 16 * p->nnz + 8 * p->n + 8 * p->m;
    p->n_kernels = 2;
    p->kernel_name = "coo_pair_kernel";
}

// ---------------------------------------------------------------- HYB
int choose_hyb_width(const int64_t *row_ptr, int64_t m) {
    // minimise modelled bytes: ELL slots (incl. padding) + overflow entries
    // + per-overflow-row overhead, over K in {4, 8, ..., 256}
    const HostCsr A{m, 0, 0, row_ptr, nullptr, nullptr};
    const int64_t ns = (A.m + 63) / 64;
    std::vector<int64_t> smax((size_t)ns);
#pragma omp parallel for schedule(static)
    for (int64_t s = 0; s < ns; ++s) {
        int64_t w = 0;
        const int64_t r1 = std::min<int64_t>(A.m, (s + 1) * 64);
        for (int64_t r = s * 64; r < r1; ++r) w = std::max<int64_t>(w, A.row_ptr[r + 1] - A.row_ptr[r]);
        smax[s] = w;
    }
    int bestK = 4;
    double best = std::numeric_limits<double>::max();
    for (int K = 4; K <= 256; K += 4) {
        double slots = 0, ovf = 0, ovr = 0;
#pragma omp parallel for schedule(static) reduction(+ : slots)
        for (int64_t s = 0; s < ns; ++s) slots += 64.0 * (double)round_up(std::min<int64_t>(smax[s], K), 4);
#pragma omp parallel for schedule(static) reduction(+ : ovf, ovr)
        for (int64_t r = 0; r < A.m; ++r) {
            const int64_t len = A.row_ptr[r + 1] - A.row_ptr[r];
            if (len > K) { ovf += (double)(len - K); ovr += 1.0; }
        }
        const double cost = 12.0 * slots + 12.0 * ovf + 32.0 * ovr;
        if (cost < best) { best = cost; bestK = K; }
    }
    return bestK;
}

int hyb_width(const int64_t *row_ptr, int64_t m, const spmv_options_t &o) {
    return o.ell_width > 0 ? (int)round_up(o.ell_width, 4) : choose_hyb_width(row_ptr, m);
}

void hyb_finish_info(spmv_plan_s *p, int K, int64_t ell_slots) {
    const HybDev &h = p->hyb;
    p->ell.max_width = K;
    p->stored_slots = ell_slots + h.nnz;
    p->algo_bytes = 12 * p->nnz + 8 * p->n + 8 * p->m + 12 * h.n_rows;
    p->n_kernels = h.n_rows ? 2 : 1;
    // every kernel of one execute ("a+b": the PMC traffic of an execute sums them)
    p->kernel_name = h.n_rows ? "ell_slice_kernel+csr_adaptive_kernel" : "ell_slice_kernel";
}

int build_hyb(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o) {
    const int K = hyb_width(A.row_ptr, A.m, o);
    SPMV_RETURN_IF(build_ell(p, A, o, K));
    const int64_t ell_slots = p->stored_slots;
    SPMV_RETURN_IF(build_overflow(p, A, K));
    hyb_finish_info(p, K, ell_slots);
    return SPMV_SUCCESS;
}

// ---------------------------------------------------------------- SS
// x window of each tile for ss_stream_kernel: the column range of its 64 x
// SIGMA positions (padding positions read column 0, as they do in the kernel)
// when it spans <= kSsWinCols columns, else none
void ss_tile_windows(const int32_t *col, int64_t nnz, int64_t n_tiles, int sigma, std::vector<int32_t> &win) {
    const int64_t T = 64 * (int64_t)sigma;
    win.assign((size_t)(2 * std::max<int64_t>(n_tiles, 1)), 0);
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < n_tiles; ++t) {
        int32_t lo = std::numeric_limits<int32_t>::max(), hi = -1;
        for (int64_t i = t * T; i < (t + 1) * T; ++i) {
            const int32_t c = i < nnz ? col[i] : 0;
            lo = std::min(lo, c);
            hi = std::max(hi, c);
        }
        if (hi - lo < kSsWinCols) {
            win[(size_t)(2 * t)] = lo;
            win[(size_t)(2 * t + 1)] = hi - lo + 1;
        }
    }
}

int build_ss(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o) {
    SsDev &s = p->ss;
    const double mean = A.m ? (double)A.nnz / (double)A.m : 0.0;
    s.sigma = o.ss_sigma > 0 ? o.ss_sigma : auto_ss_sigma(mean);
    if (!ss_sigma_ok(s.sigma)) {
        set_error("ss_sigma must be one of 4,8,12,16,20,24,32,48,64");
        return SPMV_ERROR_INVALID_VALUE;
    }
    ss_probe_options(s);
    const int64_t T = 64 * (int64_t)s.sigma;
    const int W = ss_flag_words(s.sigma);
    s.n_tiles = (A.nnz + T - 1) / T;
    // ordinals of non-empty rows
    std::vector<int64_t> nzord((size_t)A.m + 1, 0);
    for (int64_t r = 0; r < A.m; ++r) nzord[r + 1] = nzord[r] + (A.row_ptr[r + 1] > A.row_ptr[r] ? 1 : 0);
    s.n_nonempty = nzord[A.m];
    s.n_empty = A.m - s.n_nonempty;
    if (s.n_empty > 0) {
        std::vector<int32_t> nzrow((size_t)std::max<int64_t>(s.n_nonempty, 1));
        std::vector<int32_t> empty((size_t)s.n_empty);
        int64_t a = 0, b = 0;
        for (int64_t r = 0; r < A.m; ++r) {
            if (A.row_ptr[r + 1] > A.row_ptr[r]) nzrow[a++] = (int32_t)r;
            else empty[b++] = (int32_t)r;
        }
        SPMV_RETURN_IF(upload(p, &s.nzrow, nzrow.data(), s.n_nonempty));
        SPMV_RETURN_IF(upload(p, &s.empty_rows, empty.data(), s.n_empty));
    }
    const int64_t total = s.n_tiles * T;
    std::vector<uint32_t> flags((size_t)s.n_tiles * 64 * W, 0u);
    std::vector<int32_t> tord((size_t)s.n_tiles);
    auto set_flag = [&](int64_t pos) {
        const int64_t t = pos / T, li = pos % T, k = li % s.sigma;
        uint32_t *w = &flags[(size_t)((t * W + k / 32) * 64 + li / s.sigma)];
        __atomic_fetch_or(w, 1u << (k % 32), __ATOMIC_RELAXED);
    };
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < A.m; ++r)
        if (A.row_ptr[r + 1] > A.row_ptr[r]) set_flag(A.row_ptr[r]);
    if (A.nnz % T) set_flag(A.nnz);  // dummy segment over the padding
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < s.n_tiles; ++t) {
        const int64_t r = std::lower_bound(A.row_ptr, A.row_ptr + A.m, t * T) - A.row_ptr;
        tord[t] = (int32_t)nzord[r];
    }
    std::vector<int32_t> col((size_t)total);
    std::vector<double> val((size_t)total);
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < s.n_tiles; ++t) {
        for (int64_t li = 0; li < T; ++li) {
            const int64_t i = t * T + li;
            const int64_t lane = li / s.sigma, k = li % s.sigma;
            const int64_t pos = t * T + (k >> 2) * 256 + lane * 4 + (k & 3);
            const int64_t vpos = t * T + (k >> 2) * 256 + ((k & 2) ? 128 : 0) + lane * 2 + (k & 1);
            col[pos] = i < A.nnz ? A.col[i] : 0;
            val[vpos] = i < A.nnz ? A.val[i] : 0.0;
        }
    }
    std::vector<int32_t> win;
    ss_tile_windows(A.col, A.nnz, s.n_tiles, s.sigma, win);
    SPMV_RETURN_IF(upload(p, &s.col, col.data(), total));
    SPMV_RETURN_IF(upload(p, &s.val, val.data(), total));
    SPMV_RETURN_IF(upload(p, &s.flags, flags.data(), s.n_tiles * 64 * W));
    SPMV_RETURN_IF(upload(p, &s.tile_ord, tord.data(), s.n_tiles));
    SPMV_RETURN_IF(upload(p, &s.win, win.data(), 2 * s.n_tiles));
    SPMV_RETURN_IF(dev_alloc(p, &s.ht, 2 * s.n_tiles));
    SPMV_RETURN_IF(dev_alloc(p, &s.tail_ord, s.n_tiles));
    SPMV_RETURN_IF(ss_plan_tail_ord(p));
    ss_finish_info(p);
    return SPMV_SUCCESS;
}

void ss_finish_info(spmv_plan_s *p) {
    const SsDev &s = p->ss;
    p->stored_slots = s.n_tiles * 64 * s.sigma;
    p->empty_rows = s.n_empty;
    p->algo_bytes = 12 * p->nnz + 8 * p->n + 8 * p->m;
    p->n_kernels = 2;
    p->kernel_name = std::string(s.kernel == 0 && s.sigma <= 32 ? "ss_tile_kernel<" : "ss_stream_kernel<") +
                     std::to_string(s.sigma) + ">+ss_fixup_kernel";
}

// probe build: SPMV_SS_KERNEL (0 = ss_tile_kernel), SPMV_SS_PF at plan build
void ss_probe_options(SsDev &s) {
    if (const char *e = probe_env("SPMV_SS_KERNEL")) s.kernel = std::atoi(e);
    if (const char *e = probe_env("SPMV_SS_PF")) s.pf = std::atoi(e);
    if (const char *e = probe_env("SPMV_SS_STAGE")) s.stage = std::atoi(e) != 0;
}

// ---------------------------------------------------------------- DIA
// Occupied diagonals (col - row), ascending.  Returns false when the matrix
// exceeds the limits (too many diagonals / too much zero fill).
static bool dia_offsets(const HostCsr &A, int max_diags, double max_fill, std::vector<int32_t> &offs) {
    const int64_t N = A.m + A.n - 1;
    if (N <= 0) return true;
    std::vector<uint8_t> occ((size_t)N, 0);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < A.m; ++r)
        for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) occ[(size_t)(A.col[j] - r + A.m - 1)] = 1;
    for (int64_t d = 0; d < N; ++d) {
        if (occ[(size_t)d]) {
            offs.push_back((int32_t)(d - (A.m - 1)));
            if ((int)offs.size() > max_diags) return false;
        }
    }
    return (double)offs.size() * (double)A.m <= max_fill * (double)std::max<int64_t>(A.nnz, 1);
}

// Value-buffer placement (as BIN's product buffer, build_bin.cpp): the same
// launch runs ~10 % slower from some physical regions of HBM (the first of
// three identical config-4 plans in a process: 1.76-1.81 vs 1.59-1.62 ms,
// profiles/round1/probe/dia_placement.jsonl).  Copies of the values in up to
// 8 allocations spread over the free device memory are timed with one
// launch each over a zero x; the fastest is kept.
int dia_placement(spmv_plan_s *p, int64_t m, int64_t n, size_t bytes, const spmv_options_t &o) {
    DiaDev &d = p->dia;
    int mode = o.placement;
    SPMV_RETURN_IF(placement_mode_check(mode));
    if (const char *e = probe_env("SPMV_PLACEMENT_MODE")) mode = std::atoi(e);
    if (mode == SPMV_PLACEMENT_AUTO) mode = SPMV_PLACEMENT_PLAIN;
    if (mode == SPMV_PLACEMENT_SEARCH && bytes < ((size_t)256 << 20)) mode = SPMV_PLACEMENT_PLAIN;
    d.placement = mode;
    if (mode == SPMV_PLACEMENT_PLAIN) return SPMV_SUCCESS;
    if (mode == SPMV_PLACEMENT_VMM) {  // move the values into a VMM mapping
        size_t chunk = kVmmChunk, align = kVmmAlign;
        if (const char *e = probe_env("SPMV_VMM_CHUNK_MB")) chunk = (size_t)std::max(1, std::atoi(e)) << 20;
        if (const char *e = probe_env("SPMV_VMM_ALIGN_MB")) align = (size_t)std::max(0, std::atoi(e)) << 20;
        void *q = nullptr;
        SPMV_RETURN_IF(p->arena.alloc_vmm(&q, bytes, chunk, p->device, align));
        SPMV_HIP_TRY(hipMemcpy(q, d.val, bytes, hipMemcpyDeviceToDevice));
        p->arena.free(d.val);
        d.val = (double *)q;
        return SPMV_SUCCESS;
    }
    int K = 8;
    if (const char *e = probe_env("SPMV_DIA_PLACEMENT")) K = std::max(1, std::min(8, std::atoi(e)));
    if (K <= 1) return SPMV_SUCCESS;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return SPMV_SUCCESS;
    }
    const size_t scratch = 8 * (size_t)(std::max<int64_t>(n, 1) + std::max<int64_t>(m, 1));
    auto need_for = [&](int k) { return (size_t)k * bytes + scratch + ((size_t)8 << 30); };
    while (K > 2 && free_b < need_for(K)) --K;
    const size_t need = need_for(K);
    if (free_b < need) return SPMV_SUCCESS;  // no room for a search
    const size_t gap = std::max<size_t>((size_t)16 << 30, (free_b - need) / (size_t)(K - 1));
    // the search's scratch (zero x, a y, two events), released on every exit
    struct SearchScratch {
        double *xz = nullptr, *yz = nullptr;
        hipEvent_t a = nullptr, b = nullptr;
        ~SearchScratch() {
            (void)hipDeviceSynchronize();
            if (xz) (void)hipFree(xz);
            if (yz) (void)hipFree(yz);
            if (a) (void)hipEventDestroy(a);
            if (b) (void)hipEventDestroy(b);
        }
    } sc;
    SPMV_RETURN_IF(scratch_malloc(&sc.xz, 8 * (size_t)std::max<int64_t>(n, 1), "xz"));
    SPMV_RETURN_IF(scratch_malloc(&sc.yz, 8 * (size_t)std::max<int64_t>(m, 1), "yz"));
    double *xz = sc.xz, *yz = sc.yz;
    SPMV_HIP_TRY(hipMemset(xz, 0, 8 * (size_t)std::max<int64_t>(n, 1)));
    SPMV_HIP_TRY(hipEventCreate(&sc.a));
    SPMV_HIP_TRY(hipEventCreate(&sc.b));
    hipEvent_t a = sc.a, b = sc.b;
    auto time_one = [&](float *ms) -> int {
        SPMV_RETURN_IF(launch_dia(p, xz, yz));  // warm
        SPMV_HIP_TRY(hipEventRecord(a, p->stream));
        SPMV_RETURN_IF(launch_dia(p, xz, yz));
        SPMV_HIP_TRY(hipEventRecord(b, p->stream));
        SPMV_HIP_TRY(hipEventSynchronize(b));
        SPMV_HIP_TRY(hipEventElapsedTime(ms, a, b));
        return SPMV_SUCCESS;
    };
    double *orig = d.val;
    std::vector<double *> cand{orig};
    std::vector<float> t(1, 0.0f);
    std::vector<void *> spacers;
    int st = time_one(&t[0]);
    for (int k = 1; k < K && st == SPMV_SUCCESS; ++k) {
        void *g = nullptr;
        if (hipMalloc(&g, gap) == hipSuccess) spacers.push_back(g);
        else (void)hipGetLastError();
        void *q = nullptr;
        if (p->arena.alloc(&q, bytes) != SPMV_SUCCESS) {
            (void)hipGetLastError();
            break;
        }
        if (hipMemcpy(q, orig, bytes, hipMemcpyDeviceToDevice) != hipSuccess) {
            (void)hipGetLastError();
            p->arena.free(q);
            break;
        }
        d.val = (double *)q;
        float ms = 0;
        st = time_one(&ms);
        cand.push_back((double *)q);
        t.push_back(ms);
        // the modes differ by ~10 %: once both have been seen, stop
        if (k >= 3 && *std::min_element(t.begin(), t.end()) < 0.93f * *std::max_element(t.begin(), t.end())) break;
    }
    for (void *g : spacers) (void)hipFree(g);
    (void)hipGetLastError();
    const size_t best = st == SPMV_SUCCESS ? (size_t)(std::min_element(t.begin(), t.end()) - t.begin()) : 0;
    for (size_t k = 0; k < cand.size(); ++k)
        if (k != best) p->arena.free(cand[k]);
    d.val = cand[best];
    d.placement_ms = t;
    if (d.dbg & 16) {
        std::fprintf(stderr, "[dia] placement ms:");
        for (float tt : t) std::fprintf(stderr, " %.4f", tt);
        std::fprintf(stderr, " -> %zu\n", best);
    }
    return st;
}

int build_dia(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o) {
    DiaDev &d = p->dia;
    const int maxd = o.dia_max_diags > 0 ? o.dia_max_diags : 1024;
    const double fill = o.dia_max_fill > 0 ? o.dia_max_fill : 3.0;
    std::vector<int32_t> offs;
    if (!dia_offsets(A, maxd, fill, offs)) {
        set_error("DIA: matrix has too many diagonals or too much zero fill for the DIA format");
        return SPMV_ERROR_NOT_SUPPORTED;
    }
    d.n_diags = (int)offs.size();
    d.off_host = offs;
    const int64_t N = A.m + A.n - 1;
    std::vector<int32_t> idx((size_t)std::max<int64_t>(N, 1), -1);
    for (int i = 0; i < d.n_diags; ++i) idx[(size_t)(offs[i] + A.m - 1)] = i;
    // row blocks of kDiaBlockRows (one workgroup), each holding its rows of
    // every diagonal contiguously: val[(blk*nd + d)*B + r%B]
    d.mp = round_up(A.m, kDiaBlockRows);
    const int64_t slots = (int64_t)d.n_diags * d.mp;
    std::vector<double> val((size_t)std::max<int64_t>(slots, 1), 0.0);
    const int64_t nd = d.n_diags;
    if (const char *e = probe_env("SPMV_DIA_GROUP")) d.group = std::max(0, std::atoi(e));
    const int64_t G = d.group, nblk = d.mp / kDiaBlockRows;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < A.m; ++r)
        for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) {
            const int di = idx[(size_t)(A.col[j] - r + A.m - 1)];
            const int64_t b = r / kDiaBlockRows;
            int64_t at = (b * nd + di) * kDiaBlockRows + r % kDiaBlockRows;
            if (G > 0) {  // interleaved groups (k_dia.hip)
                const int64_t t = b / G, g = b - t * G, gt = std::min(G, nblk - t * G);
                at = (t * G * nd + di * gt + g) * kDiaBlockRows + r % kDiaBlockRows;
            }
            val[(size_t)at] += A.val[j];  // duplicates are summed
        }
    SPMV_RETURN_IF(upload(p, &d.off, offs.data(), d.n_diags));
    if (const char *e = probe_env("SPMV_DIA_DEBUG")) d.dbg = std::atoi(e);
    if (const char *e = probe_env("SPMV_DIA_LDS_KB")) d.lds_kb = std::atoi(e);
    p->stored_slots = slots;
    // AUTO: values of >= 256 MB go straight into 2-MB VMM handles mapped at a
    // 1-GB-aligned VA (config 4: 1.537-1.61 ms against 1.665-1.677 with one
    // plain hipMalloc, profiles/round3/probe/dia_placement_vmm.jsonl; the
    // same placement as BIN's product buffer)
    const size_t vbytes = (size_t)std::max<int64_t>(slots, 1) * sizeof(double);
    spmv_options_t oo = o;
    SPMV_RETURN_IF(placement_mode_check(oo.placement));
    if (oo.placement == SPMV_PLACEMENT_AUTO)
        oo.placement = vbytes >= kDiaVmmMinBytes ? SPMV_PLACEMENT_VMM : SPMV_PLACEMENT_PLAIN;
    if (oo.placement == SPMV_PLACEMENT_VMM && !probe_env("SPMV_PLACEMENT_MODE")) {
        void *q = nullptr;
        SPMV_RETURN_IF(p->arena.alloc_vmm(&q, vbytes, kVmmChunk, p->device, kVmmAlign));
        SPMV_HIP_TRY(hipMemcpy(q, val.data(), vbytes, hipMemcpyHostToDevice));
        d.val = (double *)q;
        d.placement = SPMV_PLACEMENT_VMM;
    } else {
        SPMV_RETURN_IF(upload(p, &d.val, val.data(), slots));
        SPMV_RETURN_IF(dia_placement(p, A.m, A.n, vbytes, oo));
    }
    dia_finish_info(p);
    return SPMV_SUCCESS;
}

void dia_finish_info(spmv_plan_s *p) {
    p->stored_slots = (int64_t)p->dia.n_diags * p->dia.mp;
    p->algo_bytes = 8 * p->nnz + 4 * (int64_t)p->dia.n_diags + 8 * p->n + 8 * p->m;
    p->n_kernels = 1;
    p->kernel_name = "dia_kernel";
}

// ---------------------------------------------------------------- CSS
namespace {
struct CssEntry {
    int32_t col;
    uint16_t slot;
    double val;
};
}  // namespace

// Column-slab sweep (k_css.hip).  Rows are cut into nnz-balanced blocks, one
// per (pass, workgroup), each using <= kCssMaxRows LDS slots; a row longer
// than half a worker wave's share is split into pieces with their own slots
// (merged in piece order at pass end), pieces go to the 15 worker waves
// longest-first onto the least loaded wave (LPT), and each wave's entries are
// sorted by column.
//
// css_layout: every decision above from the row pointers alone (the host and
// the device builder share it); the entry fill -- each wave list's entries
// stably sorted by column into its chunks -- is css_fill_host below or
// css_fill_device (k_css_build.hip).
int css_layout(spmv_plan_s *p, const int64_t *row_ptr, int64_t m, int64_t n, int64_t nnz, const spmv_options_t &o,
               CssLayout &CL) {
    CssDev &c = p->css;
    struct {
        int64_t m, n, nnz;
        const int64_t *row_ptr;
    } A{m, n, nnz, row_ptr};
    int ncu = 0;
    SPMV_HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, p->device));
    c.nwg = ncu > 0 ? ncu : 256;
    if (const char *e = probe_env("SPMV_CSS_WGS")) {  // experiment: a subset of the CUs
        const int k = std::atoi(e);
        if (k >= 8 && k < c.nwg) c.nwg = k;
    }
    constexpr int W = kCssWorkers;
    const int64_t per_pass = (int64_t)c.nwg * kCssMaxRows;
    const int P_min = (int)std::max<int64_t>(1, (A.m + per_pass - 1) / per_pass);
    auto row_len = [&](int64_t r) { return A.row_ptr[r + 1] - A.row_ptr[r]; };
    // Row blocks.  Short rows keep matrix order in contiguous runs cut by
    // nnz; rows much longer than the mean ("long") are then dealt
    // longest-first to the block with the least nnz that still has LDS slots
    // (LPT), so one block does not inherit a cluster of heavy rows (with
    // ~19.5 K rows per block at config 3 the slot cap alone left blocks at
    // 0.8-1.3x the mean nnz).  rmap lists each block's rows, slot order.
    const double mean_len = A.m ? (double)A.nnz / (double)A.m : 0.0;
    const int64_t tau = std::max<int64_t>(64, (int64_t)(8.0 * mean_len));
    std::vector<int64_t> longs, shorts;
    for (int64_t r = 0; r < A.m; ++r) (row_len(r) > tau ? longs : shorts).push_back(r);
    std::stable_sort(longs.begin(), longs.end(), [&](int64_t a, int64_t b) { return row_len(a) > row_len(b); });
    int64_t short_nnz = 0;
    for (int64_t r : shorts) short_nnz += row_len(r);
    std::vector<int64_t> &roff = CL.roff;  // [nb + 1] into rmap
    std::vector<int32_t> &rmap = CL.rmap;  // block rows in slot order
    int64_t piece_cap = 0;
    int piece_div = 2;
    if (const char *d = probe_env("SPMV_CSS_PIECE_DIV")) piece_div = std::max(1, std::atoi(d));
    bool fitted = false;
    for (c.P = P_min; c.P <= P_min + 1024 && !fitted; ++c.P) {
        const int64_t nb = (int64_t)c.P * c.nwg;
        piece_cap = std::max<int64_t>(64, A.nnz / (nb * W) / piece_div);
        auto slots_of = [&](int64_t r) { return std::max<int64_t>(1, (row_len(r) + piece_cap - 1) / piece_cap); };
        int64_t long_slots = 0;
        for (int64_t r : longs) long_slots += slots_of(r);
        const int64_t ns = (int64_t)shorts.size();
        // every block keeps room for its share of the long-row slots
        const int64_t reserve = longs.empty() ? 0 : (long_slots + nb - 1) / nb + 8;
        const int64_t cap_short = kCssMaxRows - reserve;
        if (cap_short <= 0 || ns > cap_short * nb) continue;
        // contiguous short runs, cumulative nnz targets, slot-capped
        std::vector<int64_t> s_off((size_t)nb + 1, 0), b_nnz((size_t)nb, 0), b_slots((size_t)nb, 0);
        size_t i = 0;
        int64_t cum = 0;  // nnz of shorts[0, i)
        for (int64_t b = 0; b < nb; ++b) {
            const bool last = b == nb - 1;
            const int64_t tgt_nnz = (int64_t)((__int128)short_nnz * (b + 1) / nb);
            const int64_t tgt_cnt = (int64_t)((__int128)ns * (b + 1) / nb);
            // rows this block must take so the later blocks can hold the rest
            const int64_t must = std::max<int64_t>(0, (ns - (int64_t)i) - (nb - b - 1) * cap_short);
            while ((int64_t)i < ns && b_slots[(size_t)b] < cap_short) {
                const bool forced = b_slots[(size_t)b] < must;
                if (!last && !forced && (short_nnz > 0 ? cum >= tgt_nnz : (int64_t)i >= tgt_cnt)) break;
                const int64_t len = row_len(shorts[i]);
                b_slots[(size_t)b] += 1;
                b_nnz[(size_t)b] += len;
                cum += len;
                ++i;
            }
            s_off[(size_t)b + 1] = (int64_t)i;
        }
        if (i < shorts.size()) continue;  // short rows left over: more passes
        // LPT of the long rows over blocks with free slots
        std::vector<std::vector<int64_t>> blong((size_t)nb);
        typedef std::pair<int64_t, int64_t> NB;  // (nnz, block)
        std::priority_queue<NB, std::vector<NB>, std::greater<NB>> heap;
        for (int64_t b = 0; b < nb; ++b) heap.push({b_nnz[(size_t)b], b});
        bool ok = true;
        std::vector<NB> full;
        for (int64_t r : longs) {
            const int64_t k = slots_of(r);
            while (!heap.empty() && b_slots[(size_t)heap.top().second] + k > kCssMaxRows) {
                full.push_back(heap.top());
                heap.pop();
            }
            if (heap.empty()) {
                ok = false;
                break;
            }
            NB t = heap.top();
            heap.pop();
            blong[(size_t)t.second].push_back(r);
            b_slots[(size_t)t.second] += k;
            t.first += row_len(r);
            heap.push(t);
            for (const NB &f : full) heap.push(f);  // a shorter row may still fit there
            full.clear();
        }
        if (!ok) continue;
        roff.assign((size_t)nb + 1, 0);
        rmap.clear();
        rmap.reserve((size_t)A.m);
        for (int64_t b = 0; b < nb; ++b) {
            for (int64_t q = s_off[(size_t)b]; q < s_off[(size_t)b + 1]; ++q) rmap.push_back((int32_t)shorts[(size_t)q]);
            for (int64_t r : blong[(size_t)b]) rmap.push_back((int32_t)r);
            roff[(size_t)b + 1] = (int64_t)rmap.size();
        }
        fitted = true;
        break;
    }
    if (!fitted) {
        set_error("CSS: could not fit the rows into LDS row blocks");
        return SPMV_ERROR_NOT_SUPPORTED;
    }
    if (o.css_slab_shift > 0) {
        c.slab_shift = o.css_slab_shift;
    } else {
        // narrowest slab that still gives every worker wave ~384 entries per
        // slab: pacing finer than that is pure overhead (measured sweep,
        // profiles/round1/it2_css: 2^18 columns for config 2, wider as n grows)
        const double per_wave = (double)std::max<int64_t>(A.nnz, 1) / ((double)c.nwg * W * c.P * 384.0);
        c.slab_shift = 14;
        while (c.slab_shift < 24 && (double)((A.n + ((int64_t)1 << c.slab_shift) - 1) >> c.slab_shift) > per_wave)
            ++c.slab_shift;
    }
    if (c.slab_shift < 8 || c.slab_shift > 30) {
        set_error("css_slab_shift must be in [8, 30]");
        return SPMV_ERROR_INVALID_VALUE;
    }
    c.S = (int)std::max<int64_t>(1, (A.n + ((int64_t)1 << c.slab_shift) - 1) >> c.slab_shift);
    c.lag = o.css_lag == 0 ? 4 : (o.css_lag < 0 ? 0 : o.css_lag);
    c.pace_all = o.css_pace == 2 ? 0 : 1;
    const int64_t nblocks = (int64_t)c.P * c.nwg;
    const int64_t nlists = nblocks * W;
    std::vector<int64_t> &woff = CL.woff;
    std::vector<int64_t> &moff = CL.moff;
    woff.assign((size_t)nlists + 1, 0);
    moff.assign((size_t)nblocks + 1, 0);
    std::vector<std::vector<int32_t>> merges((size_t)nblocks);
    std::vector<std::vector<CssPiece>> &wave_pieces = CL.wave_pieces;
    wave_pieces.assign((size_t)nlists, {});
#pragma omp parallel
    {
        std::vector<CssPiece> pieces;
        std::vector<int> order;
#pragma omp for schedule(dynamic, 4)
        for (int64_t pb = 0; pb < nblocks; ++pb) {
            const int64_t r0 = roff[(size_t)pb];
            const int rows = (int)(roff[(size_t)pb + 1] - r0);
            pieces.clear();
            int extra = rows;
            for (int l = 0; l < rows; ++l) {
                const int64_t row = rmap[(size_t)(r0 + l)];
                const int64_t b0 = A.row_ptr[row], len = row_len(row);
                const int64_t k = std::max<int64_t>(1, (len + piece_cap - 1) / piece_cap);
                if (k > 1) {
                    merges[(size_t)pb].insert(merges[(size_t)pb].end(), {l, extra, (int32_t)(k - 1)});
                }
                for (int64_t i = 0; i < k; ++i)
                    pieces.push_back(CssPiece{b0 + len * i / k, b0 + len * (i + 1) / k, i == 0 ? l : extra + (int)i - 1});
                extra += (int)(k - 1);
            }
            order.resize(pieces.size());
            std::iota(order.begin(), order.end(), 0);
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
                return pieces[a].end - pieces[a].begin > pieces[b].end - pieces[b].begin;
            });
            int64_t load[W] = {0};
            for (int i : order) {
                int best = 0;
                for (int w = 1; w < W; ++w)
                    if (load[w] < load[best]) best = w;
                load[best] += pieces[i].end - pieces[i].begin;
                wave_pieces[(size_t)(pb * W + best)].push_back(pieces[i]);
            }
            for (int w = 0; w < W; ++w) woff[(size_t)(pb * W + w + 1)] = load[w];
            moff[(size_t)pb + 1] = (int64_t)merges[(size_t)pb].size() / 3;
        }
    }
    // list lengths -> physical layout.  Contiguous: list L at woff[L].
    // Interleaved (default): chunk k (256 entries) of list L of pass p at
    // pbase + (k * lists_per_pass + L_local) * 256, so at any time all waves of
    // the chip stream one contiguous band of the entry arrays (measured:
    // tools/gather_probe.hip e10 vs e13); lists are padded to the longest of
    // the pass with benign entries (col 0, dummy slot, val 0).
    std::vector<int32_t> &wlen = CL.wlen;
    wlen.assign((size_t)nlists, 0);
    for (int64_t L = 0; L < nlists; ++L) wlen[(size_t)L] = (int32_t)woff[(size_t)L + 1];
    for (int64_t b = 0; b < nblocks; ++b) moff[b + 1] += moff[b];
    const int64_t lists_per_pass = (int64_t)c.nwg * W;
    c.interleaved = true;
    if (const char *e = probe_env("SPMV_CSS_LAYOUT")) c.interleaved = std::atoi(e) != 0;
    int64_t total = 0;
    if (c.interleaved) {
        for (int pp = 0; pp < c.P; ++pp) {
            int64_t kmax = 0;
            for (int64_t Lq = 0; Lq < lists_per_pass; ++Lq)
                kmax = std::max<int64_t>(kmax, ((int64_t)wlen[(size_t)(pp * lists_per_pass + Lq)] + 255) / 256);
            for (int64_t Lq = 0; Lq < lists_per_pass; ++Lq)
                woff[(size_t)(pp * lists_per_pass + Lq)] = total + Lq * 256;
            total += kmax * lists_per_pass * 256;
        }
        c.chunk_stride = lists_per_pass * 256;
        woff[(size_t)nlists] = total;
    } else {
        woff[0] = 0;
        for (int64_t L = 0; L < nlists; ++L) woff[(size_t)L + 1] = woff[(size_t)L] + wlen[(size_t)L];
        total = woff[(size_t)nlists];
        c.chunk_stride = 256;
    }
    CL.merge.assign((size_t)std::max<int64_t>(3 * moff[nblocks], 1), 0);
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblocks; ++b)
        std::copy(merges[(size_t)b].begin(), merges[(size_t)b].end(), CL.merge.begin() + 3 * moff[b]);
    CL.total = total;
    CL.nlists = nlists;
    CL.nblocks = nblocks;
    CL.has_longs = !longs.empty();
    c.split_rows = moff[nblocks];
    return SPMV_SUCCESS;
}

// the host fill: each wave list's entries, stably sorted by column (a row's
// entries of one column keep their CSR order), into the list's chunks
int css_fill_host(spmv_plan_s *p, const HostCsr &A, CssLayout &CL) {
    CssDev &c = p->css;
    const int64_t total = CL.total;
    std::vector<int32_t> col((size_t)std::max<int64_t>(total, 1), 0);
    std::vector<uint16_t> slot((size_t)std::max<int64_t>(total, 1), (uint16_t)kCssMaxRows);
    std::vector<double> val((size_t)std::max<int64_t>(total, 1), 0.0);
#pragma omp parallel
    {
        std::vector<CssEntry> in;
#pragma omp for schedule(dynamic, 4)
        for (int64_t L = 0; L < CL.nlists; ++L) {
            in.clear();
            for (const CssPiece &pc : CL.wave_pieces[(size_t)L])
                for (int64_t j = pc.begin; j < pc.end; ++j) in.push_back(CssEntry{A.col[j], (uint16_t)pc.slot, A.val[j]});
            // column order = slab order; stable keeps a row's CSR order
            std::stable_sort(in.begin(), in.end(), [](const CssEntry &a, const CssEntry &b) { return a.col < b.col; });
            const int64_t base = CL.woff[L];
            for (size_t i = 0; i < in.size(); ++i) {
                const int64_t out = base + (int64_t)(i / 256) * c.chunk_stride + (int64_t)(i % 256);
                col[out] = in[i].col;
                slot[out] = in[i].slot;
                val[out] = in[i].val;
            }
        }
    }
    // +256 entries: a contiguous list's last chunk may read past the array
    // (masked lanes); zero col, val -- and slot 0, which masking overrides
    SPMV_RETURN_IF(upload(p, &c.col, col.data(), total, 256));
    SPMV_RETURN_IF(upload(p, &c.row, slot.data(), total, 256));
    SPMV_RETURN_IF(upload(p, &c.val, val.data(), total, 256));
    return SPMV_SUCCESS;
}

// the layout's host arrays, pacing counters and plan info (both builders)
int css_finish(spmv_plan_s *p, const CssLayout &CL, int64_t m, int64_t n, int64_t nnz) {
    CssDev &c = p->css;
    SPMV_RETURN_IF(upload(p, &c.woff, CL.woff.data(), CL.nlists + 1));
    SPMV_RETURN_IF(upload(p, &c.wlen, CL.wlen.data(), CL.nlists));
    SPMV_RETURN_IF(upload(p, &c.bstart, CL.roff.data(), CL.nblocks + 1));
    c.rmap = nullptr;  // identity (rows in matrix order) unless long rows were dealt out
    c.n_rmap = 0;
    if (CL.has_longs) {
        SPMV_RETURN_IF(upload(p, &c.rmap, CL.rmap.data(), (int64_t)CL.rmap.size()));
        c.n_rmap = (int64_t)CL.rmap.size();
    }
    SPMV_RETURN_IF(upload(p, &c.moff, CL.moff.data(), CL.nblocks + 1));
    SPMV_RETURN_IF(upload(p, &c.merge, CL.merge.data(), 3 * CL.moff[(size_t)CL.nblocks]));
    std::vector<uint64_t> zeros(8 * 16, 0);
    SPMV_RETURN_IF(upload(p, &c.prog, zeros.data(), (int64_t)zeros.size()));
    c.launches = 0;
    c.n_lists = CL.nlists;
    if (const char *d = probe_env("SPMV_CSS_DEBUG")) c.dbg = std::atoi(d);
    if (c.dbg & 32) SPMV_RETURN_IF(dev_alloc(p, &c.tstamp, (int64_t)c.P * c.nwg * (kCssWorkers + 2)));
    p->stored_slots = CL.total;
    p->algo_bytes = 12 * nnz + 8 * n + 8 * m;
    p->n_kernels = 1;
    p->kernel_name = "css_sweep_kernel";
    return SPMV_SUCCESS;
}

int build_css(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o) {
    CssLayout CL;
    SPMV_RETURN_IF(css_layout(p, A.row_ptr, A.m, A.n, A.nnz, o, CL));
    SPMV_RETURN_IF(css_fill_host(p, A, CL));
    return css_finish(p, CL, A.m, A.n, A.nnz);
}

// ---------------------------------------------------------------- AUTO
int choose_format(const HostCsr &A, const spmv_options_t &o) {
    return choose_format_rp(A.m, A.n, A.nnz, A.row_ptr, o, [&]() {
        std::vector<int32_t> offs;
        return dia_offsets(A, 256, 1.25, offs);
    });
}

int choose_crs_exact(const HostCsr &A, spmv_options_t &o) {
    return choose_crs_exact(
        A.m, A.n, A.nnz, A.row_ptr, o,
        [&]() {
            std::vector<int32_t> offs;
            return dia_offsets(A, 256, 1.25, offs);
        },
        [&]() {
            int64_t desc = 0, dup = 0;
#pragma omp parallel for schedule(static) reduction(+ : desc, dup)
            for (int64_t r = 0; r < A.m; ++r)
                for (int64_t j = A.row_ptr[r] + 1; j < A.row_ptr[r + 1]; ++j) {
                    desc += A.col[j] < A.col[j - 1];
                    dup += A.col[j] == A.col[j - 1];
                }
            return desc ? kRowsUnsorted : dup ? kRowsSorted : kRowsStrict;
        });
}

// opt_crs semantics for a CSR request (spmv_options_t.crs_exact): the
// fastest layout whose every row is the sequential column-order sum, bit for
// bit -- DIA where AUTO finds a band, BIN (no run path) where AUTO's wide-x
// rule holds, sliced ELL for near-uniform rows of <= 64 entries, else CSR
// with one lane per row.  `o` is rewritten for the chosen layout.
int choose_crs_exact(int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr, spmv_options_t &o,
                     const std::function<bool()> &dia_ok, const std::function<int()> &rows_order) {
    const int f = choose_format_rp(m, n, nnz, row_ptr, o, dia_ok);
    // DIA adds duplicate entries into one slot before the product: bit-exact
    // only when every row's columns are strictly ascending.  BIN sums a row
    // strip by strip, each strip's entries in CSR order: the CSR order
    // whenever the columns ascend (duplicates allowed).  Otherwise ELL /
    // one-lane CSR below.
    if (f == SPMV_FORMAT_DIA && rows_order() == kRowsStrict) return f;
    if (f == SPMV_FORMAT_BIN && rows_order() != kRowsUnsorted) {
        o.bin_long_len = -1;  // every row on the segment path: sequential sums
        return f;
    }
    int64_t maxlen = 0;
#pragma omp parallel for schedule(static) reduction(max : maxlen)
    for (int64_t r = 0; r < m; ++r) maxlen = std::max<int64_t>(maxlen, row_ptr[r + 1] - row_ptr[r]);
    const double mean = m ? (double)nnz / (double)m : 0.0;
    if (m > 0 && maxlen <= 64 && (double)maxlen <= 2.0 * mean + 8.0) return SPMV_FORMAT_ELL;
    o.csr_lanes = 1;
    return SPMV_FORMAT_CSR;
}

// AUTO from the row-length histogram (row pointers only) plus, for short
// rows, the diagonal census `dia_ok` (host: dia_offsets; a device CSR:
// dia_offsets_device) -- the same decision for a host and a device CSR.
int choose_format_rp(int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr, const spmv_options_t &o,
                     const std::function<bool()> &dia_ok) {
    const HostCsr A{m, n, nnz, row_ptr, nullptr, nullptr};
    if (A.m == 0 || A.nnz == 0) return SPMV_FORMAT_CSR;
    const double mean = (double)A.nnz / (double)A.m;
    int64_t maxlen = 0;
#pragma omp parallel for schedule(static) reduction(max : maxlen)
    for (int64_t r = 0; r < A.m; ++r) maxlen = std::max<int64_t>(maxlen, A.row_ptr[r + 1] - A.row_ptr[r]);
    // banded: few, well-filled diagonals -> DIA moves 8 instead of 12 B/nnz
    if (maxlen <= 512 && dia_ok()) return SPMV_FORMAT_DIA;
    (void)o;
    // x beyond one XCD's 4 MiB L2 and enough rows to fill every CU: random
    // gathers dominate -> column-slab sweep (L2-resident x slabs).  Measured
    // crossover (profiles/round1/probe/auto_sweep.jsonl): row-parallel formats
    // win at n = 0.5 M (x = 4 MB), CSS from n = 1 M (x = 8 MB) on uniform and
    // power-law rows alike.
    // The binned Mul/Sum (x strips in LDS, no gathers at all) beats the
    // column-slab sweep in that same range once it has ~8 M entries: with a
    // Sum bin per wave on small plans (bin_rows) it runs 1 M x 1 M uniform
    // 16 / row in 0.104 ms against CSS's 0.132, 2 M power-law (9.9 M nnz)
    // 0.084 vs 0.122, 1 M power-law (5 M nnz) 0.059 vs 0.061
    // (profiles/round2/bin_small/auto_cross.jsonl; round 1, with m / 5119
    // bins, it took ~3.5 M columns, bin_vs_css_sizes.jsonl), and its
    // advantage grows with n (1.2 vs 2.6 ms at 10 M x 80 M)
    // ... as long as its (bin, strip) segments stay long enough for the
    // 8/16-entry padding (expected segment >= 12 entries: 20 at the N = 8
    // rank shape, 128 at config 2)
    if (A.n * 8 > ((int64_t)6 << 20) && A.nnz >= 8000000 && mean >= 2.0) {
        const double bins = std::ceil((double)A.m / 5119.0), strips = std::ceil((double)A.n / 20480.0);
        if ((double)A.nnz / (bins * strips) >= 12.0 && bins * strips <= (double)(1 << 28)) return SPMV_FORMAT_BIN;
    }
    if (A.n * 8 > ((int64_t)6 << 20) && A.m >= 256 * 1024 && mean >= 2.0) return SPMV_FORMAT_CSS;
    // near-uniform rows -> CSR (one lane count fits every row; it matched or
    // beat sliced ELL at every measured size); skewed -> segmented sum
    if ((double)maxlen <= 2.0 * mean + 8.0) return SPMV_FORMAT_CSR;
    return SPMV_FORMAT_SS;
}

}  // namespace spmv

// internal.hpp -- plan layout, error plumbing and launcher declarations shared
// by the C-ABI (capi.cpp), the host format builders (formats.cpp) and the
// kernels (k_*.hip).  Not installed; the public surface is include/spmv_hip.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "spmv_hip.h"

namespace spmv {

// ---- error plumbing (the C-ABI returns codes; it never exit()s, unlike
//      src/util.h:48-55 CUDA_SAFE_CALL and src/util.cpp:32-35) -------------
void set_error(const std::string &msg);
const char *last_error();

#define SPMV_HIP_TRY(call)                                                      \
    do {                                                                        \
        hipError_t e_ = (call);                                                 \
        if (e_ != hipSuccess) {                                                 \
            ::spmv::set_error(std::string(#call) + ": " + hipGetErrorString(e_) + \
                              " (" __FILE__ ":" + std::to_string(__LINE__) + ")"); \
            return SPMV_ERROR_HIP;                                              \
        }                                                                       \
    } while (0)

#define SPMV_CHECK_ARG(cond, msg)                                               \
    do {                                                                        \
        if (!(cond)) {                                                          \
            ::spmv::set_error(msg);                                             \
            return SPMV_ERROR_INVALID_VALUE;                                    \
        }                                                                       \
    } while (0)

#define SPMV_RETURN_IF(status)                                                  \
    do {                                                                        \
        int s_ = (status);                                                      \
        if (s_ != SPMV_SUCCESS) return s_;                                      \
    } while (0)

// Transient device scratch of the plan builders (freed before create
// returns): a failed allocation clears HIP's sticky error (a later launch
// check must not see it) and reports SPMV_ERROR_OUT_OF_MEMORY, so the
// host-CSR routing falls back to the host builders (capi.cpp) instead of
// failing a plan the host path builds fine.
inline int scratch_malloc_bytes(void **q, size_t n, const char *what) {
    *q = nullptr;
    const hipError_t e = hipMalloc(q, n ? n : 16);
    if (e == hipSuccess) return SPMV_SUCCESS;
    (void)hipGetLastError();
    *q = nullptr;
    set_error(std::string("builder scratch ") + what + " (" + std::to_string(n) + " B): " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? SPMV_ERROR_OUT_OF_MEMORY : SPMV_ERROR_HIP;
}
template <typename T>
inline int scratch_malloc(T **q, size_t n, const char *what = "") {
    void *v = nullptr;
    const int s = scratch_malloc_bytes(&v, n, what);
    *q = static_cast<T *>(v);
    return s;
}

// ---- experiment switches ------------------------------------------------
// The probe build (`make probes`, -DSPMV_PROBES, probes_build/) reads the
// SPMV_<FORMAT>_* tuning and ablation variables the tools/ scripts set; the
// product library ignores them all, so no stray environment variable can
// change what spmv_execute computes or how fast it runs.
inline const char *probe_env(const char *name) {
#ifdef SPMV_PROBES
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// Probe build: SPMV_LAUNCH_DEBUG, read at every launch, replaces a plan's
// SPMV_*_DEBUG kernel-selection bits -- launch-time variants A/B'd on ONE
// plan, so on one placement (tools/bin_phase_ab.py --launch-variants).
inline int launch_dbg(int plan_dbg) {
    if (const char *e = probe_env("SPMV_LAUNCH_DEBUG")) return std::atoi(e);
    return plan_dbg;
}

// Placement modes.  AUTO (the default) holds no transient
// device memory at create and times nothing; SPMV_PLACEMENT_SEARCH is the
// caller's explicit opt-in to a build-time search (transient candidate
// buffers spread over free HBM, one timed launch each).
inline int placement_mode_check(int mode) {
    SPMV_CHECK_ARG(mode >= SPMV_PLACEMENT_AUTO && mode <= SPMV_PLACEMENT_VMM, "unknown placement mode");
    return SPMV_SUCCESS;
}
constexpr size_t kVmmChunk = (size_t)2 << 20;          // physical handle size
constexpr size_t kVmmAlign = (size_t)1 << 30;          // VA alignment of the mapping
constexpr size_t kBinVmmMinBytes = (size_t)32 << 20;   // AUTO: VMM from this product-buffer size
constexpr size_t kDiaVmmMinBytes = (size_t)256 << 20;  // AUTO: VMM from this DIA value size
constexpr size_t kStreamVmmMinBytes = (size_t)256 << 20;  // AUTO: VMM from this array size (CSR, ELL, ...)

// ---- device memory owned by a plan --------------------------------------
// Plain hipMalloc allocations, plus buffers mapped through the HIP virtual
// memory API (hipMemCreate + hipMemMap: the BIN product buffer, see
// build_bin.cpp, placement).
struct VmmMap {
    void *va = nullptr;      // mapped range (aligned inside the reservation)
    size_t bytes = 0;
    void *res = nullptr;     // the reservation, res_bytes long
    size_t res_bytes = 0;
    std::vector<hipMemGenericAllocationHandle_t> handles;  // one per mapped chunk
    size_t chunk = 0;
};
struct DevArena {
    std::vector<void *> ptrs;
    std::vector<VmmMap> maps;
    int64_t bytes = 0;
    int device = 0;
    size_t vmm_min = 0;  // > 0: alloc() of >= vmm_min bytes maps 2-MB VMM handles instead
    int alloc(void **p, size_t n);  // hipMalloc (or VMM, above), zero-size safe
    // n bytes of physical memory in `chunk`-byte handles mapped at one VA range
    // (align > 0: the mapping starts at a multiple of `align` inside a larger
    // reservation -- hipMemAddressReserve itself honours only the granularity)
    int alloc_vmm(void **p, size_t n, size_t chunk, int device, size_t align = 0);
    void free(void *p);             // hipFree one allocation of this arena
    void release();
};

// ---- per-format device layouts ------------------------------------------

// CSR (opt_crs, src/opt_crs.h:3-9): row_ptr (int32 when nnz < 2^31, else
// int64), col_idx int32, val f64.  col/val are padded by kPad entries so the
// 16-byte vector loads of the aligned-start kernel never leave the buffer.
constexpr int kPad = 8;
// Adaptive CSR (csr_lanes = AUTO on skewed rows): rows binned by length,
// bin b summed by kCsrBinLanes[b] lanes per row (256 = one workgroup per row).
constexpr int kCsrBins = 8;
constexpr int kCsrBinLanes[kCsrBins] = {1, 2, 4, 8, 16, 32, 64, 256};
constexpr int kCsrMaxWin = 4096;   // columns of a csr_slabx x window (32 KB of LDS)
constexpr int kCsrWinGroup = 256;  // rows of one x-window granule (4 waves x 1 slab of 64)
constexpr int kCsrSlabsPerWave = 1;  // csr_slabx default: a workgroup owns 1 granule (256 rows)
struct CsrDev {
    void *row_ptr = nullptr;  // int32 or int64 [m+1]
    bool rp64 = false;
    int32_t *col = nullptr;   // [nnz + kPad]
    double *val = nullptr;    // [nnz + kPad]; val_halves: [roundup(nnz, 256) + kPad], each
                              //   256-entry chunk as ELL slots (k_csr.hip csr_vpos)
    bool val_halves = false;  // = lanes > 0 (the row-group kernels); adaptive plans keep CSR order
    int lanes = 4;            // lanes per row (1..64); 0 = adaptive (bins)
    bool off32 = false;       // every 64-row slab spans < 2^28 entries and n < 2^29:
                              // 32-bit byte offsets in csr_slab2 (k_csr.hip)
    int64_t slab_max = 0;     // entries of the widest 64-row slab
    int32_t *win0 = nullptr;  // [ceil(m / kCsrWinGroup)]: first column of each 256-row granule's
    int32_t win = 0;          //   x window; win = the widest window of kCsrSlabsPerWave granules
    int32_t win_s[3] = {};    //   ... of 1, 2, 4 granules (0: wider than kCsrMaxWin); null: none fits
    int32_t *bin_rows = nullptr;        // rows of every bin, ascending within a bin
    int64_t bin_off[kCsrBins + 1] = {};  // host: bin b = bin_rows[bin_off[b], bin_off[b+1])
};

// the entry stored at position pos of a val_halves array (inverse of csr_vpos)
__host__ __device__ inline int64_t csr_val_halves_entry(int64_t pos) {
    const int64_t r = pos & 255;
    return (pos & ~(int64_t)255) + ((r & 127) >> 1) * 4 + (r >> 7) * 2 + (r & 1);
}
// row-group plans store their values in halves (probe build:
// SPMV_CSR_VAL_PLAIN=1 keeps CSR order, for A/Bs)
inline bool csr_val_halves_wanted(const CsrDev &c) {
    if (const char *e = probe_env("SPMV_CSR_VAL_PLAIN")) return c.lanes > 0 && std::atoi(e) == 0;
    return c.lanes > 0;
}

// Sliced ELL (opt_ell, src/opt_ell.cpp): slices of 64 consecutive rows (one
// wave); slice s has width w_s (multiple of 4) = max row length in the slice
// (capped at K for HYB).  Slot k of local row i lives at
//   slice_off[s] + (k/4)*256 + i*4 + (k%4)
// so one 16-byte load gives a lane 4 consecutive slots of its row and a wave
// instruction reads 1 KiB contiguous.  Padding: col = last real col of the
// row (0 for an empty row), val = 0 -> adds +0.0, no new cache line.
struct EllDev {
    int32_t *perm = nullptr;       // JDS: slice row i -> matrix row perm[i]
    int64_t n_slices = 0;
    int64_t *slice_off = nullptr;  // [n_slices + 1] in slots
    int32_t *col = nullptr;
    double *val = nullptr;
    int max_width = 0;
    int64_t slots = 0;             // stored slots of the ELL part (HYB / JDS: without the overflow)
    int unroll = 2;  // quads per lane per iteration (SPMV_ELL_UNROLL, internal;
                     // 2 beat 4 by 28 % at config 4, 5 % at config 2)
};

// HYB overflow: rows whose length exceeds K keep entries K.. in a CSR over
// those rows only; a second kernel adds them (one writer per row).
struct HybDev {
    int32_t *bin_rows = nullptr;          // overflow rows (local) binned by length
    int64_t bin_off[kCsrBins + 1] = {};   // host offsets per bin
    int64_t n_rows = 0;
    int32_t *rows = nullptr;     // [n_rows] global row ids
    int64_t *row_ptr = nullptr;  // [n_rows + 1]
    int32_t *col = nullptr;
    double *val = nullptr;
    int64_t nnz = 0;
    int lanes = 64;
};

// Segmented sum (opt_ss / CSR5): tiles of 64 lanes x sigma nnz.  Lane l of
// tile t owns nnz t*64*sigma + l*sigma + k, k in [0, sigma), its column
// stored at t*64*sigma + (k/4)*256 + l*4 + (k%4) and its value at
//   t*64*sigma + (k/4)*256 + (k%4/2)*128 + l*2 + (k%2).
// flags[t*64 + l] bit k: that nnz is the first entry of a non-empty row.
// tile_ord[t]: ordinal (among non-empty rows) of the first row that starts
// inside tile t.  Rows that cross tiles are finished by a fixup kernel from
// per-tile head/tail partials (deterministic, no atomics, β = 0).
constexpr int kSsWinCols = 512;  // widest per-tile x window (doubles of LDS per wave)
// flag words per lane of a tile: bit k of word k/32 (SIGMA <= 64)
__host__ __device__ inline int ss_flag_words(int sigma) { return sigma > 32 ? 2 : 1; }
inline bool ss_sigma_ok(int sigma) {
    return sigma >= 4 && sigma % 4 == 0 && (sigma <= 24 || sigma == 32 || sigma == 48 || sigma == 64);
}
struct SsDev {
    int sigma = 16;
    int64_t n_tiles = 0;
    int32_t *col = nullptr;
    double *val = nullptr;
    uint32_t *flags = nullptr;   // [n_tiles][words][64]
    int32_t *win = nullptr;      // [n_tiles][2]: x window (first column, length; 0 = none)
    int kernel = 1;              // 1 = ss_stream_kernel, 0 = ss_tile_kernel (SIGMA <= 32)
    int pf = 2;                  // ss_stream_kernel: quads loaded ahead
    bool stage = true;           // ss_stream_kernel: finished rows staged in LDS, stored after the stream
    int32_t *tile_ord = nullptr;
    double *ht = nullptr;        // scratch [n_tiles][2]: head partial, tail partial (one store per tile)
    int32_t *tail_ord = nullptr; // [n_tiles] plan-time: ordinal of the tile's last row start, -1 = none
    int32_t *nzrow = nullptr;    // ordinal -> row (null when no empty rows)
    int64_t n_nonempty = 0;
    int32_t *empty_rows = nullptr;
    int64_t n_empty = 0;
};

// COO (opt_coo, src/opt_coo.cpp): sorted (row, col, val), padded to whole
// units of kCooUnit entries (row -1, col 0, val 0); one wave handles a unit
// per step (lane l: entries 2l, 2l+1), reduces equal-row runs in registers
// and issues one f64 atomic add per run (y zeroed first).
constexpr int64_t kCooUnit = 128;
struct CooDev {
    int32_t *row = nullptr;
    int32_t *col = nullptr;
    double *val = nullptr;
    int64_t n_units = 0;
};

// DIA (opt_dia, src/opt_dia.cpp), row-indexed and blocked by workgroup:
// A[r, r+off[d]] at val[((r/B)*n_diags + d)*B + r%B], B = kDiaBlockRows
// (0 where absent / outside), offsets ascending -- each workgroup streams one
// contiguous n_diags*B*8-byte block.
constexpr int kDiaBlockRows = 512;

struct DiaDev {
    int n_diags = 0;
    int32_t *off = nullptr;  // device copy of offsets
    std::vector<int32_t> off_host;
    double *val = nullptr;   // [n_diags * mp]
    int64_t mp = 0;          // m rounded up to kDiaBlockRows
    int dbg = 0;             // SPMV_DIA_DEBUG (internal): 1 = x from global memory, no LDS window
    int group = 0;           // > 0: value blocks interleaved per group of blocks (k_dia.hip)
    int lds_kb = -1;         // SPMV_DIA_LDS_KB (probe): LDS per workgroup (0: window only); -1: kDiaLdsKb
    int placement = 0;       // SPMV_PLACEMENT_* used for val
    std::vector<float> placement_ms;
};

// Column-slab sweep (CSS, k_css.hip).  Per (pass p, workgroup b, worker wave
// w) a list of entries (global col int32, LDS slot uint16, val f64) sorted by
// column; woff[(p*nwg+b)*kCssWorkers+w] is the list start.  Slots 0..rows-1
// are the block's rows; rows split into pieces use extra slots, merged at
// pass end from merge[] triples (slot, first extra slot, count), moff[] per
// block.  prog: per-XCD-label pacing counters (uint64, 128 B apart).
constexpr int kCssMaxRows = 19968;
constexpr int kCssWorkers = 15;  // worker waves per workgroup (+1 pacer wave)
struct CssDev {
    int nwg = 0, R = 0, P = 0, S = 0, slab_shift = 17, lag = 2, pace_all = 0;
    int64_t *woff = nullptr;    // physical start of each list's chunk 0
    int32_t *wlen = nullptr;    // entries of each list
    int64_t chunk_stride = 256; // entries between a list's consecutive 256-entry chunks
    bool interleaved = true;    // chunks of all lists of a pass interleaved
    int64_t *bstart = nullptr;  // [P*nwg + 1] offsets of each (pass, workgroup) block's rows in rmap
    int32_t *rmap = nullptr;    // block rows in slot order; null = identity (contiguous blocks)
    int64_t *moff = nullptr;    // [P*nwg + 1] merge-triple offsets per block
    int32_t *merge = nullptr;   // (slot, first extra slot, n extra) triples
    int64_t split_rows = 0;
    int32_t *col = nullptr;
    uint16_t *row = nullptr;
    double *val = nullptr;
    uint64_t *prog = nullptr;
    uint64_t launches = 0;
    int dbg = 0;  // ablation switches (SPMV_CSS_DEBUG, internal)
    uint64_t *tstamp = nullptr;  // dbg & 32: [P*nwg][kCssWorkers + 2] s_memrealtime stamps
    int64_t n_lists = 0;         // worker-wave lists (P * nwg * kCssWorkers)
    int64_t n_rmap = 0;          // entries of rmap (0: identity)
};
// CSS layout decided from the row pointers (formats.cpp css_layout), shared by
// the host fill and the device fill (k_css_build.hip)
struct CssPiece {
    int64_t begin, end;  // CSR entry range
    int slot;            // LDS slot (row l -> slot l; extra pieces after the rows)
};
struct CssLayout {
    std::vector<int64_t> roff;                     // [nblocks + 1] into rmap
    std::vector<int32_t> rmap;                     // block rows in slot order
    std::vector<std::vector<CssPiece>> wave_pieces; // [nlists] pieces of each worker-wave list, list order
    std::vector<int64_t> woff, moff;               // physical list starts [nlists + 1]; merge offsets [nblocks + 1]
    std::vector<int32_t> wlen, merge;              // list lengths [nlists]; merge triples
    int64_t total = 0, nlists = 0, nblocks = 0;
    bool has_longs = false;
};

// Binned two-phase Mul/Sum (BIN, k_bin.hip) -- opt_ss's Mul -> val_buf ->
// Sum split (src/opt_ss.cpp:188-221) crossed with opt_css's column blocks
// (src/opt_css.cpp:33-45).  Columns are cut into strips of `strip` columns
// (the x strip sits in LDS), rows into bins of <= kBinMaxRows (one wave's
// LDS y slice).  Entries are grouped into segments (strip s, bin b), each
// sorted by (row, col) and padded to a multiple of 8:
//   Mul order  [group][s][b][k]: val1 f64, cs1 u16 (column - strip start),
//              dst1 int32 per 8 entries (8-entry index in the group's product buffer)
//   Sum order  [group][b][s][k]: slot2 u16 (row - bin start; kBinMaxRows = pad)
// Mul: prod[dst] = val1 * xs[cs1] (x strip in LDS, coalesced 64-B product lines);
// Sum: one wave per bin adds its products in order into its LDS slice with
// ds_add_f64 and writes y -> deterministic, and an unsplit row's sum is the
// sequential opt_crs sum (column order) bit for bit.  Row groups bound the
// product buffer (re-used by every group: it can stay in the Infinity Cache).
//
// Long rows (>= long_len entries; power-law rows with many entries per
// strip) leave the segments: each strip's Mul range ends with their runs in
// the strip, packed in 64-entry blocks (the strip's range is 64-aligned, a
// void of zero entries after the segments).  The Mul reduces a block's runs
// with a segmented wave scan and writes one partial per run piece (a run
// cut at a block boundary is two pieces) to the piece's place in the bin's
// long run, which the Sum adds after the bin's segments (one more run per
// bin).  lcode per long entry: bit 31 = first entry of a piece, bits 0-30 =
// the piece's product position on its last entry, else 0x7FFFFFFF.  A long
// row is the sum of its pieces in (strip, piece) order -- deterministic, not
// the sequential order (<= 1e-12 relative), like CSS's split rows.
constexpr int kBinLdsDoubles = 20480;  // Sum: 160 KB of LDS y slices per workgroup
constexpr int kBinMulThreads = 1024;
constexpr int kBinMaxStrip = 20480;  // Mul: x strip of 160 KB of LDS
// Sum waves per workgroup W2 (4 or 8): a wave's slice holds kBinLdsDoubles/W2
// doubles = bin rows + one dummy slot (padding entries add +0.0 there)
inline int bin_max_rows(int w2) { return kBinLdsDoubles / w2 - 1; }
// Row slots are stored in 8-entry lane groups per Sum batch (64 lanes x U
// entries, entry (u, lane) = product position base + u*64 + lane): the slot
// of product position e of a run starting at product r0 / slot s0 (a
// multiple of 64*U) sits at s0 + batch*64U + (u/8)*512 + lane*8 + u%8, so a
// lane reads its U slots as U/8 16-byte loads, each load instruction of the
// wave covering 1 KB contiguously.
__host__ __device__ inline int64_t bin_slot_index(int64_t e, int64_t r0, int64_t s0, int U) {
    const int64_t rel = e - r0, step = 64 * (int64_t)U;
    const int64_t i = rel / step, w = rel - i * step;
    const int64_t u = w >> 6, lane = w & 63;
    return s0 + i * step + (u >> 3) * 512 + lane * 8 + (u & 7);
}
// Mul-ordered products (BinDev::mo, SPMV_BIN_ORDER_MUL): the Mul writes entry
// e's product to prod[e] (its own order, segments unpadded), and the Sum
// reads the Sum order's positions through a chunk table.  Entry (u, lane) of
// a Sum batch lies in chunk c = 8u + lane/8 of the batch: 8 consecutive Sum
// positions of one segment = 8 consecutive Mul positions (segment padding in
// the Sum order reads on into the next segment's products, to the dummy
// slot).  A batch's 8U chunk bases sit at table index sbase/8 (sbase = the
// batch's slot block) in the order below: word r of lane l is chunk 64r + l,
// so a lane loads its U/8 words at once and ds_bpermute hands chunk c to the
// 8 lanes reading it.
__host__ __device__ inline int64_t bin_mo_tab_at(int64_t c, int U) { return (c & 63) * (U / 8) + (c >> 6); }
// The Sum reads whole batches of 64*U products without clamping at a run's
// end (the padded slot batches send those lanes to the dummy slot), so the
// product buffer carries one batch of slack past its last run.
constexpr int64_t kBinProdSlack = 64 * 32;
// Likewise the Mul loads a wave's batch (64 x 8 entries) of val1 / cs1 / dst1
// without clamping at its piece's end (the stores past it are masked), so
// those arrays carry one batch of slack.
constexpr int64_t kBinMulSlack = 64 * 8;
struct BinDev {
    int strip = 20480;     // x strip width in columns (<= kBinMaxStrip)
    int pad_log = 3;       // segments padded to 2^pad_log entries (8: 64-B product lines)
    int sum_waves = 8;     // W2
    int max_rows = 0;      // bin_max_rows(W2) = the dummy slot
    int G = 1;             // row groups: one Mul launch each (write locality)
    bool reuse = false;    // one product buffer re-used per group (Sum per group)
    int nwg1 = 0, nwg2 = 0;
    int64_t n_bins = 0, n_strips = 0, n_entries = 0;
    int32_t xburst = 0;           // Mul: stage x strips with several loads in flight (wide shapes)
    std::vector<int64_t> g_bin;    // host [G+1]: bin range of each group
    std::vector<int64_t> g_prod;   // host [G+1]: product (= Mul entry) range of each group
    int64_t *piece_off = nullptr;  // [G*nwg1 + 1]: pieces of (group, workgroup)
    int32_t *piece_strip = nullptr;
    int64_t *piece_begin = nullptr, *piece_end = nullptr;
    double *val1 = nullptr;
    uint16_t *cs1 = nullptr;
    int32_t *dst1 = nullptr;       // per 2^pad_log entries (Sum-ordered products only)
    int order_req = 0;             // spmv_options_t.bin_product_order (SPMV_BIN_ORDER_*)
    double seg_est = 0;            // expected entries per (bin, strip) segment (bin_params)
    bool mo = false;               // products in Mul order (SPMV_BIN_ORDER_MUL, bin_mo_tab_at)
    int32_t *mtab = nullptr;       // mo: [ES / 8] Mul position of every 8-entry Sum chunk
    uint16_t *slot2 = nullptr;
    int64_t n_blocks = 1;         // strip blocks of the product layout
    int64_t *run_off = nullptr;   // [n_blocks*n_bins + 1]: run (blk, b) of bin b's products
    int64_t *srun_off = nullptr;  // [n_blocks*n_bins + 1]: its slots (runs padded to 64*sum_u)
    int sum_u = 32;               // Sum entries per lane per batch (the slot layout's U)
    int64_t strip_block = 0;      // strips per block (SB)
    int32_t *bin_row0 = nullptr;  // [n_bins + 1]
    double *prod = nullptr;       // product buffer (largest group)
    int64_t prod_cap = 0;
    int placement = 0;            // how prod was allocated (spmv_options_t.placement, resolved)
    bool mul_perm = false;        // Mul visits a strip's bins in scrambled order (build_bin.cpp)
    int64_t long_len = 0;         // rows with >= long_len entries take the run path (0: none)
    int64_t long_rows = 0, long_pieces = 0, long_entries = 0;
    int64_t mul_entries = 0;      // Mul-order length (segments + voids + long blocks)
    int64_t slot_entries = 0;     // slot2 length (every slot run padded to whole Sum batches)
    int64_t *lstart = nullptr;    // [n_strips]: Mul position where the strip's long blocks start
    int64_t *lshift = nullptr;    // [n_strips]: lcode index - Mul position in those blocks
    int32_t *lcode = nullptr;     // per long-block entry: piece start bit | product position
    int dbg = 0;  // SPMV_BIN_DEBUG (probe build only)
    std::vector<float> placement_ms;  // Mul ms of each product-buffer candidate
};

}  // namespace spmv

struct spmv_plan_s {
    int format = SPMV_FORMAT_CSR;
    int device = 0;
    int built_on_device = 0;  // 1: the layout was built in HBM (spmv_plan_create_csr_device or build AUTO/DEVICE)
    int64_t m = 0, n = 0, nnz = 0;
    hipStream_t stream = nullptr;
    spmv::DevArena arena;
    spmv::CsrDev csr;
    spmv::EllDev ell;
    spmv::HybDev hyb;
    spmv::SsDev ss;
    spmv::DiaDev dia;
    spmv::CssDev css;
    spmv::CooDev coo;
    spmv::BinDev bin;
    double *x_stage = nullptr;  // host-x staging (opt_cusparse.cpp:44-45)
    double *y_stage = nullptr;
    bool y_staged = false;      // y_stage holds the y of an SPMV_Y_STAGED execute
    int64_t stored_slots = 0;
    int64_t empty_rows = 0;
    int64_t algo_bytes = 0;
    int n_kernels = 1;
    std::string kernel_name;
    // spmv_profile: per-phase events (the g_profile/PROF_BEGIN counterpart,
    // src/util.h:59-65); prof_k < 0 = not profiling
    mutable hipEvent_t prof_ev[9] = {};
    mutable int prof_k = -1;
};

namespace spmv {

// Host-side matrix view handed to the builders (CSR, 64-bit row pointers).
struct HostCsr {
    int64_t m, n, nnz;
    const int64_t *row_ptr;
    const int32_t *col;
    const double *val;
};

// formats.cpp -- build + upload one format into `p`.
int build_csr(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);
int build_ell(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o, int cap,
              const int32_t *order = nullptr);
int build_hyb(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);
int build_ss(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);
int build_dia(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);
int build_css(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);
int build_coo(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);
int build_jds(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);
int build_bin(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o);  // build_bin.cpp
// BIN from a device CSR (build_bin.cpp + k_bin_build.hip), long rows
// included; rows whose column strips are out of order are first sorted by
// strip on the device (bin_sort_rows_device).  kBinNeedHostBuild is then
// internal to the builder.
constexpr int kBinNeedHostBuild = -1000;
int build_bin_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                     const spmv_options_t &o);
// k_bin_build.hip: bstart[b] = row_ptr[row0[b]] (first entry of each bin)
// rows whose column strips are out of order: col2 / val2 (nnz each, the
// caller's) = the CSR's entries stably sorted by strip inside every row
int bin_sort_rows_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                         int32_t *col2, double *val2);
// LL > 0: rows of >= LL entries take the run path and stay out of the segments
int bin_count_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const std::vector<int32_t> &row0,
                     const std::vector<int64_t> &bstart, int64_t S, int64_t LL, std::vector<int32_t> &cnt);
int bin_fill_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                    const std::vector<int32_t> &row0, const std::vector<int64_t> &bstart,
                    const std::vector<int32_t> &cnt, const std::vector<int64_t> &off1,
                    const std::vector<int64_t> &off2, const std::vector<int64_t> &run_off,
                    const std::vector<int64_t> &srun_off, int64_t S, int64_t E, int64_t ES, int64_t LL, int64_t E1,
                    int32_t dst_fill);
// Long rows from a device CSR: each run is one long row's entries in one
// strip (contiguous, the row's strips being non-decreasing).  The runs'
// (strip, first entry) come to the host to lay out the long blocks; the
// entries never do.  BinLongRuns: the runs sorted [strip][row], with their
// offset in the strip's long block (q0), length, the row's slot in its bin,
// the bin and the product position of the run's first piece (fpos).
struct BinLongRuns {
    std::vector<int64_t> j0, q0, fpos;
    std::vector<int32_t> len, strip, slot, bin;
};
int bin_long_runs_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const std::vector<int32_t> &lrows,
                         std::vector<int64_t> &roff, std::vector<int32_t> &rstrip, std::vector<int64_t> &rbeg);
int bin_long_fill_device(spmv_plan_s *p, const int32_t *d_col, const double *d_val, const BinLongRuns &LR,
                         const std::vector<int64_t> &lb_off, const std::vector<int64_t> &lpad,
                         const std::vector<int64_t> &lstart, const std::vector<int64_t> &lcode_off,
                         const std::vector<int64_t> &run_off, const std::vector<int64_t> &srun_off, int64_t lrun0,
                         int64_t trash);
// k_convert.hip -- device-input builders (the CSR already lives in HBM).
int validate_csr_device(const int64_t *d_rp, int64_t m, const int32_t *d_col, int64_t nnz, int64_t n);
int widen_row_ptr_device(const int32_t *d_rp32, int64_t m, int64_t **d_rp64);  // hipMalloc'd; caller frees
int launch_scale(const spmv_plan_s *p, double *y, double alpha);              // y *= alpha on p->stream
int exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, hipStream_t st, std::vector<void *> &tmp);
int build_csr_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                     const spmv_options_t &o, double mean_row);
int build_ss_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                    const spmv_options_t &o, double mean_row);
int choose_format(const HostCsr &A, const spmv_options_t &o);
int choose_format_rp(int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr, const spmv_options_t &o,
                     const std::function<bool()> &dia_ok);
// spmv_options_t.crs_exact: the layout for a CSR request with opt_crs semantics
int choose_crs_exact(const HostCsr &A, spmv_options_t &o);
int choose_crs_exact(int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr, spmv_options_t &o,
                     const std::function<bool()> &dia_ok, const std::function<int()> &rows_order);
// layout decisions that need the row pointers only (host and device builders)
int ell_slice_offsets(const int64_t *row_ptr, int64_t m, int cap, const int32_t *order, std::vector<int64_t> &off);
void ell_finish_info(spmv_plan_s *p, int maxw, int64_t total);
void overflow_layout(const int64_t *row_ptr, int64_t m, int K, std::vector<int32_t> &rows, std::vector<int64_t> &rp);
int overflow_upload_index(spmv_plan_s *p, const std::vector<int32_t> &rows, const std::vector<int64_t> &rp);
bool jds_layout(const int64_t *row_ptr, int64_t m, int64_t nnz, const spmv_options_t &o, std::vector<int32_t> &order,
                int *K);
void jds_finish_info(spmv_plan_s *p, bool identity, int64_t ell_slots);
int hyb_width(const int64_t *row_ptr, int64_t m, const spmv_options_t &o);
void hyb_finish_info(spmv_plan_s *p, int K, int64_t ell_slots);
void coo_finish_info(spmv_plan_s *p);
void dia_finish_info(spmv_plan_s *p);
int dia_placement(spmv_plan_s *p, int64_t m, int64_t n, size_t bytes, const spmv_options_t &o);
// k_devbuild.hip -- the other formats from a device CSR (f2): only the row
// pointers visit the host (layout decisions); entries move HBM -> HBM.
struct DevCsr {
    int64_t m, n, nnz;
    const int64_t *h_rp;  // host copy of the row pointers
    const int64_t *d_rp;
    const int32_t *d_col;
    const double *d_val;
};
constexpr int kDiaRefused = -1001;  // dia_offsets_device: too many diagonals / too much fill
int dia_offsets_device(spmv_plan_s *p, const DevCsr &A, int max_diags, double max_fill, std::vector<int32_t> &offs);
int build_dia_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o);
int css_layout(spmv_plan_s *p, const int64_t *row_ptr, int64_t m, int64_t n, int64_t nnz, const spmv_options_t &o,
               CssLayout &CL);
int css_finish(spmv_plan_s *p, const CssLayout &CL, int64_t m, int64_t n, int64_t nnz);
int build_css_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o);
// every row's columns strictly ascending (no duplicates, no disorder)?
// column order of a CSR's rows (choose_crs_exact): kRowsStrict = every row
// strictly ascending, kRowsSorted = ascending with duplicates, kRowsUnsorted
constexpr int kRowsUnsorted = 0, kRowsSorted = 1, kRowsStrict = 2;
int rows_order_device(spmv_plan_s *p, const DevCsr &A, int *order);
int build_ell_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o);
int build_hyb_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o);
int build_jds_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o);
int build_coo_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o);
int auto_csr_lanes(double mean_row);
int csr_plan_lanes(spmv_plan_s *p, const int64_t *row_ptr, int64_t m, const spmv_options_t &o);
// x windows of csr_slabx from each granule's column range (lo, hi; hi < 0: no entries)
int csr_windows_finish(spmv_plan_s *p, const std::vector<int32_t> &lo, const std::vector<int32_t> &hi);
void csr_finish_info(spmv_plan_s *p);
int auto_ss_sigma(double mean_row);
void ss_tile_windows(const int32_t *col, int64_t nnz, int64_t n_tiles, int sigma, std::vector<int32_t> &win);
void ss_finish_info(spmv_plan_s *p);
void ss_probe_options(SsDev &s);
int ss_plan_tail_ord(spmv_plan_s *p);

// end of one phase of a multi-kernel launch (no-op unless profiling)
inline void phase_mark(const spmv_plan_s *p) {
    if (p->prof_k >= 0 && p->prof_k < 7) (void)hipEventRecord(p->prof_ev[++p->prof_k], p->stream);
}

// kernels -- launch y = A x on p->stream (device x, y).
int launch_csr(const spmv_plan_s *p, const double *x, double *y);
int launch_ell(const spmv_plan_s *p, const double *x, double *y);
int launch_hyb_overflow(const spmv_plan_s *p, const double *x, double *y);
int launch_ss(const spmv_plan_s *p, const double *x, double *y);
int launch_dia(const spmv_plan_s *p, const double *x, double *y);
int launch_css(const spmv_plan_s *p, const double *x, double *y);
int launch_coo(const spmv_plan_s *p, const double *x, double *y);
int launch_bin(const spmv_plan_s *p, const double *x, double *y);
int bin_time_mul(const spmv_plan_s *p, const double *x, float *ms);  // one timed Mul pass (build-time)

}  // namespace spmv

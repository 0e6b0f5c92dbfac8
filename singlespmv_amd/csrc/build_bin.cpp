// build_bin.cpp -- builders of the binned two-phase Mul/Sum format (BIN, see
// internal.hpp BinDev and k_bin.hip).  The OptimizeProblem counterpart
// (src/opt_ss.cpp:52-142 builds opt_ss's segments and val_buf, untimed, once).
//
//   build_bin        host CSR: OpenMP-parallel over bins, then one upload
//   build_bin_device device CSR (k_bin_build.hip): only the row pointers,
//                    the (bin, strip) counts and the long rows' runs (strip,
//                    first entry) visit the host; the entry arrays are
//                    filled in HBM
//
// Both share the phases: parameters -> row bins -> segment counts -> offsets
// (row groups, Mul / Sum orders) -> fill -> Mul pieces -> uploads and the
// product-buffer placement search.
#include <omp.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "internal.hpp"

namespace spmv {

template <typename T>
static int upload_vec(spmv_plan_s *p, T **dst, const std::vector<T> &src) {
    void *q = nullptr;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(T) * std::max<size_t>(src.size(), 1)));
    if (!src.empty()) SPMV_HIP_TRY(hipMemcpy(q, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice));
    *dst = (T *)q;
    return SPMV_SUCCESS;
}

// Host-side layout shared by the two builders.
struct BinLayout {
    int64_t S = 0, NB = 0, E = 0, PAD = 16;
    std::vector<int32_t> row0;          // [NB + 1]
    std::vector<int32_t> cnt;           // [NB * S] entries per (bin, strip)
    std::vector<int64_t> off1, off2;    // [NB * S] segment start, Mul / Sum order
    std::vector<int64_t> run_off;       // [NBK * NB + 1]
    std::vector<int64_t> srun_off;      // [NBK * NB + 1] slot runs, each padded to 64*sum_u
    int64_t ES = 0, SB = 1;             // slot entries; strips per block
    std::vector<int64_t> strip_start;   // [G * (S + 1)] Mul-order start of (group, strip)
    std::vector<int64_t> mul_bins;      // [NB] bins in Mul visiting order within each strip (per group)
    // long rows (internal.hpp BinDev, the run path); LL = 0: none
    int64_t LL = 0, NP = 0, E1 = 0, TRASH = 0;
    std::vector<int64_t> eff_rp;        // [m + 1] cumulative Sum entries per row (bin cut)
    std::vector<int64_t> lb_off;        // [S + 1] long entries of strip t in lb_j / lb_row
    std::vector<int64_t> lb_j;          // entry index, ordered [strip][row][CSR order]
    std::vector<int32_t> lb_row;
    std::vector<int32_t> lpc;           // [NB * S] run pieces of (bin, strip)
    std::vector<int64_t> lpoff;         // [NB * S] product position of (bin, strip)'s first piece
    std::vector<int64_t> lpad;          // [S] long entries of strip t, padded to 64
    std::vector<int64_t> lstart;        // [S] Mul position of strip t's first long block
    std::vector<int64_t> lcode_off;     // [S] lcode index of the same
    int64_t rpad(int64_t v) const { return (v + PAD - 1) & ~(PAD - 1); }
    bool is_long(const int64_t *rp, int64_t r) const { return LL > 0 && rp[r + 1] - rp[r] >= LL; }
};

// ---- parameters (strip width, workgroups, padding, Sum waves) -----------
static int bin_params(spmv_plan_s *p, const spmv_options_t &o, int64_t m, int64_t n, int64_t nnz) {
    BinDev &B = p->bin;
    if (const char *d = probe_env("SPMV_BIN_DEBUG")) B.dbg = std::atoi(d);
    int ncu = 0;
    SPMV_HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, p->device));
    if (ncu <= 0) ncu = 256;
    B.strip = o.bin_strip_cols ? o.bin_strip_cols : kBinMaxStrip;
    SPMV_CHECK_ARG(B.strip >= 64 && B.strip <= kBinMaxStrip, "bin_strip_cols must be in [64, 20480]");
    const int64_t C = B.strip;
    B.nwg1 = ncu;  // one 1024-thread workgroup per CU (the x strip fills the LDS)
    B.nwg2 = ncu;  // 160 KB of LDS y slices per workgroup
    if (const char *e = probe_env("SPMV_BIN_CUS")) {  // experiment: a subset of the CUs
        const int k = std::atoi(e);
        if (k > 0 && k < ncu) {
            B.nwg1 = k;
            B.nwg2 = k;
        }
    }
    // internal tuning knobs; defaults measured at config 2
    // (profiles/round1/probe/bin_probe_c2.jsonl): 16-entry (128-B) product
    // lines and 4 Sum waves (5119-row bins, ~1 KB segments) took Mul from
    // 0.72 to 0.56-0.66 ms
    B.pad_log = 4;
    B.sum_waves = 4;
    // 128-B product lines only when segments are long: the expected segment
    // (nnz per strip x bin) is ~128 entries at config 2 (pad 16 best) and
    // 16-64 on the N = 2..8 weak-scaling shapes (pad 8 best: 22 % padding
    // instead of 43 % at N = 8, profiles/round1/probe/bin_wide.jsonl)
    //
    // Short segments (the N = 4 and N = 8 rank shapes: 42 and 21 entries at
    // 4 waves) take 2 Sum waves per workgroup instead: 10239-row bins double
    // the segments, so the Mul streams less padding (N = 8 shape: Mul
    // 0.83 -> 0.74-0.77 ms, Sum 0.33 -> 0.35, total 1.155 -> 1.09-1.12 ms;
    // N = 4: 1.00 -> 0.97-1.00; N = 2 and config 2 stay faster with 4,
    // profiles/round1/probe/bin_sum_waves_wide.jsonl).  Since the Sum's
    // unclamped batches and one-cursor walk (round 2) the 2-wave Sum costs
    // less, and segments below 256 entries take it too: config 3 (92 at 4
    // waves) 0.166-0.177 -> 0.161-0.165 ms, rank 0 of the 2-GPU job (84)
    // 0.880-0.912 -> 0.833-0.835 ms, both then with 128-B lines
    // (profiles/round2/probe/sum_waves_pad*_*.jsonl); config 2 (167): four
    // plans each, 0.8235-0.8323 (mean 0.830) -> 0.811-0.834 ms (mean 0.824),
    // Mul 0.536-0.542 -> 0.519-0.536, Sum 0.296 -> 0.298-0.307
    // (sum_waves_c2_4plans.jsonl)
    {
        const int64_t S0 = std::max<int64_t>(1, (n + C - 1) / C);
        auto seg_for = [&](int w) {
            const int64_t NB0 = std::max<int64_t>(1, (m + bin_max_rows(w) - 1) / bin_max_rows(w));
            return (double)nnz / ((double)S0 * (double)NB0);
        };
        double seg = seg_for(4);
        if (seg < 256.0) {
            B.sum_waves = 2;
            seg = seg_for(2);
        }
        B.pad_log = seg >= 96.0 ? 4 : 3;
        B.seg_est = seg;
    }
    if (o.bin_sum_waves) {
        SPMV_CHECK_ARG(o.bin_sum_waves == 2 || o.bin_sum_waves == 4 || o.bin_sum_waves == 8,
                       "bin_sum_waves must be 0, 2, 4 or 8");
        B.sum_waves = o.bin_sum_waves;
    }
    if (o.bin_pad) {
        SPMV_CHECK_ARG(o.bin_pad == 8 || o.bin_pad == 16 || o.bin_pad == 32, "bin_pad must be 0, 8, 16 or 32");
        B.pad_log = o.bin_pad == 8 ? 3 : o.bin_pad == 16 ? 4 : 5;
    }
    if (const char *e = probe_env("SPMV_BIN_PADLOG")) B.pad_log = std::min(5, std::max(3, std::atoi(e)));
    if (const char *e = probe_env("SPMV_BIN_SUMWAVES")) {
        const int w = std::atoi(e);
        B.sum_waves = w == 2 || w == 4 ? w : 8;
    }
    // probe build: one product buffer re-used per row group (read here, before
    // bin_mo_resolve, which needs it)
    if (const char *e = probe_env("SPMV_BIN_REUSE")) B.reuse = std::atoi(e) != 0;
    // product order: the caller's bin_product_order; AUTO resolves it in
    // bin_mo_resolve (Mul order for segments of < kBinMulOrderMaxSeg expected
    // entries, when the layout allows it)
    SPMV_CHECK_ARG(o.bin_product_order >= SPMV_BIN_ORDER_AUTO && o.bin_product_order <= SPMV_BIN_ORDER_MUL,
                   "bin_product_order must be 0, 1 or 2");
    B.order_req = o.bin_product_order;
    if (const char *e = probe_env("SPMV_BIN_ORDER")) B.order_req = std::atoi(e);
    B.max_rows = bin_max_rows(B.sum_waves);
    B.sum_u = B.sum_waves == 8 ? 8 : 32;  // must match launch_sum's <W2, U> pairs
    p->algo_bytes = 12 * nnz + 8 * n + 8 * m;
    p->n_kernels = 2;
    p->kernel_name = "bin_mul_kernel+bin_sum_kernel";
    return SPMV_SUCCESS;
}

// ---- long rows: the threshold, and the Sum entries each row will need
// (its nnz; a long row: its run pieces, about one per strip it touches)
static int64_t bin_long_threshold(const spmv_options_t &o, const int64_t *rp, int64_t m, int64_t nnz, int64_t S) {
    if (o.bin_long_len < 0 || o.bin_groups > 1 || nnz == 0) return 0;
    // product positions are int31 in lcode: a cheap early out here, the
    // exact check on the finished layout in bin_layout
    if (nnz + nnz / 2 + ((int64_t)S << 6) >= ((int64_t)1 << 31)) return 0;
    const int64_t LL = o.bin_long_len > 0 ? o.bin_long_len : std::max<int64_t>(128, S);
    int64_t lnnz = 0;
#pragma omp parallel for schedule(static) reduction(+ : lnnz)
    for (int64_t r = 0; r < m; ++r) {
        const int64_t l = rp[r + 1] - rp[r];
        if (l >= LL) lnnz += l;
    }
    if (lnnz == 0) return 0;
    // auto: only when long rows carry a real share of the entries (config 3:
    // rows >= 245 entries hold 38 %)
    if (o.bin_long_len == 0 && lnnz * 20 < nnz) return 0;
    return LL;
}

// Sum entries per row for the bin cut, and the long entries bucketed by
// strip ([strip][row][CSR order], rows ascending).
static void bin_long_prep(const HostCsr &A, int64_t C, BinLayout &L) {
    const int64_t m = A.m, S = L.S;
    std::vector<int64_t> w((size_t)m);
#pragma omp parallel
    {
        std::vector<int32_t> ts;
#pragma omp for schedule(dynamic, 4096)
        for (int64_t r = 0; r < m; ++r) {
            const int64_t l = A.row_ptr[r + 1] - A.row_ptr[r];
            if (!L.is_long(A.row_ptr, r)) {
                w[(size_t)r] = l;
                continue;
            }
            ts.clear();
            for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) ts.push_back(A.col[j] / (int32_t)C);
            std::sort(ts.begin(), ts.end());
            w[(size_t)r] = (int64_t)(std::unique(ts.begin(), ts.end()) - ts.begin()) + l / 64;
        }
    }
    L.eff_rp.assign((size_t)m + 1, 0);
    for (int64_t r = 0; r < m; ++r) L.eff_rp[(size_t)r + 1] = L.eff_rp[(size_t)r] + w[(size_t)r];
    L.lb_off.assign((size_t)S + 1, 0);
    for (int64_t r = 0; r < m; ++r)
        if (L.is_long(A.row_ptr, r))
            for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) ++L.lb_off[(size_t)(A.col[j] / C) + 1];
    for (int64_t t = 0; t < S; ++t) L.lb_off[(size_t)t + 1] += L.lb_off[(size_t)t];
    std::vector<int64_t> cur(L.lb_off.begin(), L.lb_off.end() - 1);
    L.lb_j.resize((size_t)L.lb_off[(size_t)S]);
    L.lb_row.resize(L.lb_j.size());
    for (int64_t r = 0; r < m; ++r)
        if (L.is_long(A.row_ptr, r))
            for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) {
                const int64_t k = cur[(size_t)(A.col[j] / C)]++;
                L.lb_j[(size_t)k] = j;
                L.lb_row[(size_t)k] = (int32_t)r;
            }
}

// a long entry starts a piece at its row's first entry in the strip and at
// every 64-entry block boundary
static inline bool long_starts(const BinLayout &L, int64_t b0, int64_t p) {
    return p == 0 || (p & 63) == 0 || L.lb_row[(size_t)(b0 + p)] != L.lb_row[(size_t)(b0 + p - 1)];
}

// run pieces per (bin, strip) and each strip's padded long length
static void bin_long_count(BinLayout &L) {
    const int64_t S = L.S, NB = L.NB;
    L.lpc.assign((size_t)(NB * S), 0);
    L.lpad.assign((size_t)S, 0);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t t = 0; t < S; ++t) {
        const int64_t b0 = L.lb_off[(size_t)t], nt = L.lb_off[(size_t)t + 1] - b0;
        int64_t b = 0;
        for (int64_t p = 0; p < nt; ++p) {
            if (!long_starts(L, b0, p)) continue;
            const int32_t r = L.lb_row[(size_t)(b0 + p)];
            while (L.row0[(size_t)b + 1] <= r) ++b;
            ++L.lpc[(size_t)(b * S + t)];
        }
        L.lpad[(size_t)t] = (nt + 63) & ~(int64_t)63;
    }
}

// ---- product order.  Mul order (BinDev::mo) needs the plain layout: no run
// path (its partials have Sum positions), one row group, one strip block,
// grouped slots with 32-entry Sum batches, and Mul positions that fit the
// int32 chunk table.  Its Sum reads 8-entry chunks, so the segments' padding
// in the Sum order is 8 entries unless the caller set bin_pad.
// AUTO takes it for short segments (expected < 112 entries per (bin,
// strip)): in-process A/Bs on the same matrices (profiles/round3/probe/
// mulorder_*), execute ms Sum order -> Mul order: 10 M x 80 M rank shape
// (42 entries per segment) 1.008 -> 0.959 (Mul 0.70 -> 0.61, Sum 0.315 ->
// 0.352); 10 M x 40 M (84) 0.900 -> 0.880; 10 M x 20 M (168) 0.823 ->
// 0.832; config 2 (320) 0.809 -> 0.830.  The scattered product writes cost
// the Sum-ordered Mul more the shorter the segments; the chunk gathers cost
// the Sum about the same at any length.
constexpr double kBinMulOrderMaxSeg = 112.0;
static void bin_mo_resolve(BinDev &B, const spmv_options_t &o, int64_t LL, int64_t nnz) {
    const bool want = B.order_req == SPMV_BIN_ORDER_MUL ||
                      (B.order_req == SPMV_BIN_ORDER_AUTO && B.seg_est < kBinMulOrderMaxSeg);
    B.mo = want && LL == 0 && o.bin_groups <= 1 && !B.reuse && B.sum_u == 32 && nnz + kBinProdSlack < ((int64_t)1 << 31);
    if (B.mo && !o.bin_pad && !probe_env("SPMV_BIN_PADLOG")) B.pad_log = 3;
}

// ---- row bins: <= max_rows rows, cut at cumulative nnz targets; a multiple
// of the Sum kernel's wave count when there are enough rows
static int bin_rows(spmv_plan_s *p, const int64_t *row_ptr, int64_t m, int64_t n, BinLayout &L) {
    BinDev &B = p->bin;
    const int max_rows = B.max_rows;
    L.S = std::max<int64_t>(1, (n + B.strip - 1) / B.strip);
    L.PAD = (int64_t)1 << B.pad_log;
    B.n_strips = L.S;
    // (Register staging only: the Mul stages x by LDS-DMA wherever x is
    // 16-byte aligned, k_bin.hip launch_mul_p.)
    // x strips staged with several loads in flight per thread when each Mul
    // workgroup walks many strips (the N = 4, 8 rank shapes: 7.6 / 15 per
    // workgroup): N = 8 shape Mul 0.738 -> 0.719 ms; with ~2 strips per
    // workgroup (config 2) or pieces of one strip (1 M rows) the burst of x
    // loads costs 0.4-2.4 % instead (profiles/round2/probe/xstage_ab_*.jsonl)
    B.xburst = L.S >= 4 * (int64_t)B.nwg1 ? 1 : 0;
    if (B.dbg & 131072) B.xburst = 0;  // probe A/B: serial staging
    if (B.dbg & 262144) B.xburst = 1;  // probe A/B: burst staging
    const int64_t waves = (int64_t)B.nwg2 * B.sum_waves;
    // cut on the Sum entries per row (long rows: their run pieces)
    const int64_t *cum = L.LL > 0 ? L.eff_rp.data() : row_ptr;
    const int64_t total = cum[m];
    int64_t nb = std::max<int64_t>(1, (m + max_rows - 1) / max_rows);
    // small matrices: more (shorter) bins than m / max_rows, up to one per
    // Sum wave, while the expected (bin, strip) segment keeps >= 128
    // entries -- else a few waves sum everything (100 K x 100 K, 16 / row:
    // 20 bins for 1024 waves).  Configs 2, 3 and the rank shapes already
    // have a bin per wave.
    if (nb < waves) nb = std::max(nb, std::min<int64_t>(std::min<int64_t>(waves, m), total / (L.S * 128)));
    if (nb * 2 >= waves) nb = (nb + waves - 1) / waves * waves;
    L.row0.assign(1, 0);
    for (int64_t r = 0; r < m;) {
        const int64_t b = (int64_t)L.row0.size() - 1;
        int64_t r1;
        if (b >= nb - 1) {
            r1 = std::min<int64_t>(m, r + max_rows);
        } else {
            const int64_t tgt = (int64_t)((__int128)total * (b + 1) / nb);
            r1 = std::lower_bound(cum + r + 1, cum + m + 1, tgt) - cum;
            r1 = std::max<int64_t>(r + 1, std::min<int64_t>(r1, r + max_rows));
        }
        L.row0.push_back((int32_t)r1);
        r = r1;
    }
    L.NB = (int64_t)L.row0.size() - 1;
    B.n_bins = L.NB;
    // the (bin, strip) tables are dense: refuse shapes whose segment grid
    // would not fit (a huge, very sparse matrix -- BIN's padding would be
    // most of its traffic there anyway)
    if ((__int128)L.NB * L.S > ((__int128)1 << 28)) {
        set_error("BIN: " + std::to_string(L.NB) + " row bins x " + std::to_string(L.S) +
                  " column strips exceed the segment table limit (2^28); use CSS or CSR");
        return SPMV_ERROR_NOT_SUPPORTED;
    }
    return SPMV_SUCCESS;
}

// ---- offsets from the counts: row groups, Sum (product) order
// [block][b][s in block], Mul order [g][s][b]
static void bin_offsets(spmv_plan_s *p, const spmv_options_t &o, BinLayout &L) {
    BinDev &B = p->bin;
    const int64_t S = L.S, NB = L.NB;
    std::vector<int64_t> bprod((size_t)NB, 0);
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < NB; ++b) {
        int64_t t = 0;
        for (int64_t s = 0; s < S; ++s) t += L.rpad(L.cnt[(size_t)(b * S + s)]);
        bprod[(size_t)b] = t;
    }
    int64_t E = 0;
    for (int64_t b = 0; b < NB; ++b) E += bprod[(size_t)b];
    L.E = E;
    B.n_entries = E;

    // row groups: contiguous bins, balanced by products
    int G = o.bin_groups > 0 ? o.bin_groups : 1;
    if (G > NB) G = (int)NB;
    B.G = G;
    B.g_bin.assign((size_t)G + 1, NB);
    B.g_prod.assign((size_t)G + 1, E);
    B.g_bin[0] = 0;
    B.g_prod[0] = 0;
    {
        int64_t cum = 0, b = 0;
        for (int g = 1; g < G; ++g) {
            const int64_t tgt = (int64_t)((__int128)E * g / G);
            while (b < NB - (G - g) && (cum < tgt || b <= B.g_bin[(size_t)g - 1])) cum += bprod[(size_t)b++];
            B.g_bin[(size_t)g] = b;
            B.g_prod[(size_t)g] = cum;
        }
    }

    // The strips may be cut into blocks of SB strips, so a Mul workgroup's
    // product writes stay inside one block's region instead of spanning the
    // whole buffer, and a Sum wave reads its bin as one run per block.
    // Measured (profiles/round1/probe/bin_strip_blocks.jsonl): the Mul's
    // placement sensitivity is unchanged by SB and the Sum slows down (0.31
    // ms at SB = S, 0.37 at 32, 0.67 at 8), so the default is SB = S: one
    // block, the plain bin-major layout.
    int64_t SB = S;
    if (const char *e = probe_env("SPMV_BIN_SB")) SB = std::max<int64_t>(1, std::atoll(e));
    if (B.reuse || B.mo || SB > S) SB = S;
    const int64_t NBK = (S + SB - 1) / SB;
    // long rows: one more run per bin (its run pieces, [strip][row][piece])
    const int64_t NR = NBK + (L.LL > 0 ? 1 : 0);
    B.n_blocks = NR;
    L.off2.assign((size_t)(NB * S), 0);
    L.off1.assign((size_t)(NB * S), 0);
    L.run_off.assign((size_t)(NR * NB + 1), 0);
    {
        int64_t cur = 0;
        for (int64_t k = 0; k < NBK; ++k)
            for (int64_t b = 0; b < NB; ++b) {
                L.run_off[(size_t)(k * NB + b)] = cur;
                for (int64_t t = k * SB; t < std::min(S, (k + 1) * SB); ++t) {
                    L.off2[(size_t)(b * S + t)] = cur;
                    cur += L.rpad(L.cnt[(size_t)(b * S + t)]);
                }
            }
        if (L.LL > 0) {
            L.lpoff.assign((size_t)(NB * S), 0);
            for (int64_t b = 0; b < NB; ++b) {
                L.run_off[(size_t)(NBK * NB + b)] = cur;
                for (int64_t t = 0; t < S; ++t) {
                    L.lpoff[(size_t)(b * S + t)] = cur;
                    cur += L.lpc[(size_t)(b * S + t)];
                }
            }
            L.NP = cur - E;
            // padding lanes and voids write to a trash line past the Sum's runs
            L.TRASH = L.rpad(cur);
        }
        L.run_off[(size_t)(NR * NB)] = cur;
    }
    // slot runs: the same runs, each padded to whole Sum batches
    {
        const int64_t step = 64 * (int64_t)B.sum_u;
        L.srun_off.assign(L.run_off.size(), 0);
        int64_t sc = 0;
        for (size_t r = 0; r + 1 < L.run_off.size(); ++r) {
            L.srun_off[r] = sc;
            sc += (L.run_off[r + 1] - L.run_off[r] + step - 1) / step * step;
        }
        L.srun_off.back() = sc;
        L.ES = sc;
        L.SB = SB;
        B.strip_block = SB;
    }
    // The Mul visits the bins of a strip in a scrambled order (b -> b * P mod
    // bins, P coprime, near the golden ratio of the group's bin count), so the
    // product segments it writes one after the other land far apart and in no
    // regular stride in the Sum-ordered buffer (in bin order they sit one
    // bin's product run apart).
    L.mul_bins.resize((size_t)NB);
    if (const char *e = probe_env("SPMV_BIN_MUL_PERM")) B.mul_perm = std::atoi(e) != 0;
    for (int g = 0; g < G; ++g) {
        const int64_t g0 = B.g_bin[(size_t)g], nbg = B.g_bin[(size_t)g + 1] - g0;
        int64_t P = 1;
        if (B.mul_perm && nbg > 2) {
            P = std::max<int64_t>(1, (int64_t)(0.6180339887 * (double)nbg)) | 1;
            while (std::__gcd(P, nbg) != 1) P += 2;
        }
        for (int64_t i = 0; i < nbg; ++i) L.mul_bins[(size_t)(g0 + i)] = g0 + (int64_t)(((__int128)i * P) % nbg);
    }
    L.strip_start.assign((size_t)G * (S + 1), 0);
    if (L.LL > 0) L.lstart.assign((size_t)S, 0);
    for (int g = 0; g < G; ++g) {
        int64_t cur = B.g_prod[(size_t)g];
        const int64_t g0 = B.g_bin[(size_t)g], nbg = B.g_bin[(size_t)g + 1] - g0;
        for (int64_t t = 0; t < S; ++t) {
            L.strip_start[(size_t)(g * (S + 1) + t)] = cur;
            for (int64_t j = 0; j < nbg; ++j) {
                const int64_t b = L.mul_bins[(size_t)(g0 + j)];
                L.off1[(size_t)(b * S + t)] = cur;
                // Mul-ordered products: the Mul's segments are not padded
                cur += B.mo ? L.cnt[(size_t)(b * S + t)] : L.rpad(L.cnt[(size_t)(b * S + t)]);
            }
            if (L.LL > 0) {  // G == 1: void up to a 64-entry boundary, then the long blocks
                cur = (cur + 63) & ~(int64_t)63;
                L.lstart[(size_t)t] = cur;
                cur += L.lpad[(size_t)t];
            }
        }
        L.strip_start[(size_t)(g * (S + 1) + S)] = cur;
    }
    L.E1 = L.strip_start.back();
    if (L.LL > 0) {
        L.lcode_off.assign((size_t)S, 0);
        for (int64_t t = 1; t < S; ++t) L.lcode_off[(size_t)t] = L.lcode_off[(size_t)t - 1] + L.lpad[(size_t)t - 1];
    }
}

// ---- host fill.  Within a segment the entries are ordered k-major: the
// k-th entry (in column order) of every row of the segment, rows ascending,
// then the (k+1)-th ...  A row's products still reach the Sum in column order
// (the sequential opt_crs order), but consecutive lanes of one ds_add_f64 hit
// different rows instead of all landing on one slot (a banded or long row
// otherwise serialises the LDS atomics 64 ways).
// The entry arrays as the host builder lays them out (uploaded by
// bin_fill_host; tests/bin_layout_check.cpp emulates the kernels on them).
struct BinHostArrays {
    std::vector<double> val1;
    std::vector<uint16_t> cs1, slot2;
    std::vector<int32_t> dst1, lcode, mtab;
    std::vector<int64_t> lshift;
};

// Mul order: the chunk table (internal.hpp bin_mo_tab_at) from the layout
// alone -- every segment's 8-entry chunks, Sum position -> Mul position;
// chunks past a run's end keep base 0 (their slots are the dummy slot)
static void bin_mo_table(const BinDev &B, const BinLayout &L, std::vector<int32_t> &tab) {
    const int64_t S = L.S, NB = L.NB, U = B.sum_u, step = 64 * U;
    tab.assign((size_t)(L.ES / 8), 0);
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < NB; ++b) {
        const int64_t r0 = L.run_off[(size_t)b], s0 = L.srun_off[(size_t)b];
        for (int64_t t = 0; t < S; ++t) {
            const int64_t o1 = L.off1[(size_t)(b * S + t)], o2 = L.off2[(size_t)(b * S + t)];
            const int64_t c = L.cnt[(size_t)(b * S + t)];
            for (int64_t k = 0; k < c; k += 8) {
                const int64_t rel = o2 + k - r0, i = rel / step, w = rel - i * step;
                const int64_t at = bin_mo_tab_at(w >> 3, (int)U);
                tab[(size_t)((s0 + i * step) / 8 + at)] = (int32_t)(o1 + k);
            }
        }
    }
}

static void bin_fill_arrays(const BinDev &B, const HostCsr &A, const BinLayout &L, BinHostArrays &H) {
    const int64_t S = L.S, NB = L.NB, E1 = L.E1, C = B.strip, PAD = L.PAD;
    const int max_rows = B.max_rows;
    // voids between a strip's segments and its long blocks stay zero; their
    // destination groups (and the long blocks') point at the trash line
    std::vector<double> &val1 = H.val1;
    std::vector<uint16_t> &cs1 = H.cs1, &slot2 = H.slot2;
    std::vector<int32_t> &dst1 = H.dst1;
    val1.assign((size_t)(E1 + kBinMulSlack), 0.0);
    cs1.assign((size_t)(E1 + kBinMulSlack), 0);
    slot2.assign((size_t)L.ES, (uint16_t)max_rows);
    if (B.mo) dst1.clear();  // Mul order: no destinations, no Mul-side padding
    else dst1.assign((size_t)((E1 + kBinMulSlack) >> B.pad_log), (int32_t)(L.TRASH >> B.pad_log));
    std::vector<int> gof((size_t)NB);
    for (int g = 0; g < B.G; ++g)
        for (int64_t b = B.g_bin[(size_t)g]; b < B.g_bin[(size_t)g + 1]; ++b) gof[(size_t)b] = g;
#pragma omp parallel
    {
        std::vector<int64_t> segbase((size_t)S + 1);
        std::vector<int32_t> kpos, rowk((size_t)S, 0);
#pragma omp for schedule(dynamic, 8)
        for (int64_t b = 0; b < NB; ++b) {
            const int64_t *o1 = L.off1.data() + b * S, *o2 = L.off2.data() + b * S;
            // slot index of product position q of strip t's segment (its run: block t / SB)
            auto sidx = [&](int64_t t, int64_t q) {
                const size_t run = (size_t)((t / L.SB) * NB + b);
                return (size_t)bin_slot_index(q, L.run_off[run], L.srun_off[run], B.sum_u);
            };
            const int32_t *row0 = L.row0.data();
            segbase[0] = 0;
            for (int64_t t = 0; t < S; ++t) segbase[(size_t)t + 1] = segbase[(size_t)t] + L.cnt[(size_t)(b * S + t)];
            kpos.assign((size_t)segbase[(size_t)S], 0);
            // pass 1: per segment, how many rows have a k-th entry
            for (int64_t r = row0[b]; r < row0[b + 1]; ++r) {
                if (L.is_long(A.row_ptr, r)) continue;  // run path
                for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) {
                    const int64_t t = A.col[j] / C;
                    ++kpos[(size_t)(segbase[(size_t)t] + rowk[(size_t)t]++)];
                }
                for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) rowk[(size_t)(A.col[j] / C)] = 0;
            }
            // counts -> start of each k-run inside its segment
            for (int64_t t = 0; t < S; ++t) {
                int32_t run = 0;
                for (int64_t q = segbase[(size_t)t]; q < segbase[(size_t)t + 1]; ++q) {
                    const int32_t c = kpos[(size_t)q];
                    kpos[(size_t)q] = run;
                    run += c;
                }
            }
            // pass 2: place every entry
            for (int64_t r = row0[b]; r < row0[b + 1]; ++r) {
                if (L.is_long(A.row_ptr, r)) continue;
                const uint16_t slot = (uint16_t)(r - row0[b]);
                for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) {
                    const int32_t c = A.col[j];
                    const int64_t t = c / C;
                    const int64_t k = kpos[(size_t)(segbase[(size_t)t] + rowk[(size_t)t]++)]++;
                    val1[(size_t)(o1[t] + k)] = A.val[j];
                    cs1[(size_t)(o1[t] + k)] = (uint16_t)(c - t * C);
                    slot2[sidx(t, o2[t] + k)] = slot;
                }
                for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) rowk[(size_t)(A.col[j] / C)] = 0;
            }
            const int64_t pb = B.reuse ? B.g_prod[(size_t)gof[(size_t)b]] : 0;
            for (int64_t s = 0; s < S; ++s) {
                const int64_t n0 = L.cnt[(size_t)(b * S + s)], n8 = L.rpad(n0);
                for (int64_t k = n0; k < n8; ++k) {
                    if (!B.mo) {
                        val1[(size_t)(o1[s] + k)] = 0.0;
                        cs1[(size_t)(o1[s] + k)] = 0;
                    }
                    slot2[sidx(s, o2[s] + k)] = (uint16_t)max_rows;
                }
                if (!B.mo)
                    for (int64_t t = 0; t < n8; t += PAD)
                        dst1[(size_t)((o1[s] + t) >> B.pad_log)] = (int32_t)((o2[s] + t - pb) >> B.pad_log);
            }
        }
    }
    if (L.LL > 0) {
        // long blocks of every strip: entries in [row][CSR order], each lane's
        // lcode = piece start bit | (last entry of its piece ? the piece's
        // product position : 0x7FFFFFFF); the piece's slot in the bin's long run
        std::vector<int32_t> &lcode = H.lcode;
        lcode.assign((size_t)(L.lcode_off.back() + L.lpad.back()), 0);
        const int64_t NBK = B.n_blocks - 1;
#pragma omp parallel for schedule(dynamic, 4)
        for (int64_t t = 0; t < S; ++t) {
            const int64_t b0 = L.lb_off[(size_t)t], nt = L.lb_off[(size_t)t + 1] - b0;
            const int64_t ms = L.lstart[(size_t)t], cs = L.lcode_off[(size_t)t];
            int64_t b = 0, pos = -1, lastb = -1;
            for (int64_t p2 = 0; p2 < nt; ++p2) {
                const int32_t r = L.lb_row[(size_t)(b0 + p2)];
                const int64_t j = L.lb_j[(size_t)(b0 + p2)];
                const bool start = long_starts(L, b0, p2);
                if (start) {
                    while (L.row0[(size_t)b + 1] <= r) ++b;
                    if (b != lastb) {
                        pos = L.lpoff[(size_t)(b * S + t)];
                        lastb = b;
                    } else {
                        ++pos;
                    }
                    const size_t run = (size_t)(NBK * NB + b);
                    slot2[(size_t)bin_slot_index(pos, L.run_off[run], L.srun_off[run], B.sum_u)] =
                        (uint16_t)(r - L.row0[(size_t)b]);
                }
                const bool end = p2 + 1 == nt || long_starts(L, b0, p2 + 1);
                val1[(size_t)(ms + p2)] = A.val[j];
                cs1[(size_t)(ms + p2)] = (uint16_t)(A.col[j] - t * C);
                lcode[(size_t)(cs + p2)] = (int32_t)((start ? 0x80000000u : 0u) | (end ? (uint32_t)pos : 0x7FFFFFFFu));
            }
            for (int64_t p2 = nt; p2 < L.lpad[(size_t)t]; ++p2)  // padding lanes: own piece, to the trash line
                lcode[(size_t)(cs + p2)] = (int32_t)(0x80000000u | (uint32_t)L.TRASH);
        }
        H.lshift.resize((size_t)S);
        for (int64_t t = 0; t < S; ++t) H.lshift[(size_t)t] = L.lcode_off[(size_t)t] - L.lstart[(size_t)t];
    }
    if (B.mo) bin_mo_table(B, L, H.mtab);
}

static int bin_fill_host(spmv_plan_s *p, const HostCsr &A, const BinLayout &L) {
    BinDev &B = p->bin;
    BinHostArrays H;
    bin_fill_arrays(B, A, L, H);
    if (L.LL > 0) {
        SPMV_RETURN_IF(upload_vec(p, &B.lcode, H.lcode));
        SPMV_RETURN_IF(upload_vec(p, &B.lstart, L.lstart));
        SPMV_RETURN_IF(upload_vec(p, &B.lshift, H.lshift));
    }
    SPMV_RETURN_IF(upload_vec(p, &B.val1, H.val1));
    SPMV_RETURN_IF(upload_vec(p, &B.cs1, H.cs1));
    if (B.mo) SPMV_RETURN_IF(upload_vec(p, &B.mtab, H.mtab));
    else SPMV_RETURN_IF(upload_vec(p, &B.dst1, H.dst1));
    SPMV_RETURN_IF(upload_vec(p, &B.slot2, H.slot2));
    return SPMV_SUCCESS;
}

// ---- product buffer placement ---------------------------------------------
// The Mul writes 1-KB segments scattered over the whole product buffer; with
// some allocations of the same size it runs ~15 % slower (config 2: 0.66 vs
// 0.56 ms for ONE plan whose buffer was re-allocated between timings,
// profiles/round1/probe/bin_realloc.jsonl).

static int alloc_prod_plain(spmv_plan_s *p, size_t prod_bytes) {
    // (hipDeviceMallocContiguous was tried for the product buffer: plans built
    // after another plan was freed returned WRONG sums -- the buffer behaved
    // as if aliased -- so it is not used; tools/dbg_bin.py reproduces it.)
    void *q = nullptr;
    SPMV_RETURN_IF(p->arena.alloc(&q, prod_bytes));
    p->bin.prod = (double *)q;
    return SPMV_SUCCESS;
}

// SPMV_PLACEMENT_SEARCH: keep the fastest of up to K candidates, each timed
// with a Mul pass over a zero x at build time (results never depend on it).
// Up to 8 candidates: best-of-4 still left 5 of 9 config-2 plans in the slow
// mode, best-of-8 1 of 9 (profiles/round1/probe/bin_placement_k8.txt).
static int bin_place_search(spmv_plan_s *p, int64_t n, size_t prod_bytes) {
    BinDev &B = p->bin;
    int K = 8;
    if (const char *e = probe_env("SPMV_BIN_PLACEMENT")) K = std::max(1, std::min(12, std::atoi(e)));
    if (K == 1) return alloc_prod_plain(p, prod_bytes);
    double *xz = nullptr;
    SPMV_RETURN_IF(scratch_malloc(&xz, sizeof(double) * (size_t)std::max<int64_t>(n, 1), "xz"));
    if (const hipError_t e = hipMemset(xz, 0, sizeof(double) * (size_t)std::max<int64_t>(n, 1)); e != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(xz);
        set_error(std::string("BIN placement search: ") + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    std::vector<double *> cand;
    std::vector<float> t;
    int st = SPMV_SUCCESS;
    // Consecutive allocations tend to share the fast or the slow mode;
    // candidates spaced by 16 GB spacer allocations land in different
    // regions of device memory (all 6 unspaced candidates slow, 3 of 6
    // spaced ones fast, profiles/round1/probe/bin_placement_spacers.jsonl).
    // Spacers only when the device has room for them with 8 GB to spare.
    int64_t gap_mb = 16384;
    const char *gap_env = probe_env("SPMV_BIN_PLACEMENT_GAP_MB");
    if (gap_env) gap_mb = std::atoll(gap_env);
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();
            free_b = 0;
        }
        // spread the candidates over all free memory (gaps of at least
        // 16 GB): memory freed by an earlier plan's search tends to be
        // the slow kind, and equal 16 GB steps left every candidate of
        // a second plan inside it (bin_placement_k8_default.txt)
        if (!gap_env) {
            const size_t rest = (size_t)K * prod_bytes + ((size_t)8 << 30);
            if (free_b > rest) gap_mb = std::max<int64_t>(gap_mb, (int64_t)((free_b - rest) / (size_t)(K - 1) >> 20));
        }
        // as many spaced candidates as fit (at least 2), else 4 unspaced
        auto need = [&](int k) {
            return (size_t)(k - 1) * ((size_t)gap_mb << 20) + (size_t)k * prod_bytes + ((size_t)8 << 30);
        };
        while (K > 2 && free_b < need(K)) --K;
        if (free_b < need(K)) {
            gap_mb = 0;
            K = std::min(K, 4);
        }
    }
    std::vector<void *> spacers;
    for (int k = 0; k < K; ++k) {
        if (k > 0 && gap_mb > 0) {
            void *g = nullptr;
            if (hipMalloc(&g, (size_t)gap_mb << 20) == hipSuccess) spacers.push_back(g);
            else (void)hipGetLastError();
        }
        if (alloc_prod_plain(p, prod_bytes) != SPMV_SUCCESS) {
            // out of room for another candidate: rank the ones timed so far
            (void)hipGetLastError();
            break;
        }
        cand.push_back(B.prod);
        float ms = 0;
        st = bin_time_mul(p, xz, &ms);
        if (st != SPMV_SUCCESS) break;  // a failed timing is never ranked
        t.push_back(ms);
        // the modes differ by ~15 %: once both have been seen, stop
        if (k >= 3 && *std::min_element(t.begin(), t.end()) < 0.93f * *std::max_element(t.begin(), t.end()))
            break;
    }
    for (void *g : spacers) (void)hipFree(g);
    (void)hipFree(xz);
    if (st != SPMV_SUCCESS || t.empty()) {
        for (double *c : cand) p->arena.free(c);
        B.prod = nullptr;
        if (st == SPMV_SUCCESS) {
            set_error("BIN: no product buffer could be allocated");
            st = SPMV_ERROR_OUT_OF_MEMORY;
        }
        return st;
    }
    const size_t best = (size_t)(std::min_element(t.begin(), t.end()) - t.begin());
    for (size_t k = 0; k < cand.size(); ++k)
        if (k != best) p->arena.free(cand[k]);
    B.prod = cand[best];
    B.placement_ms.assign(t.begin(), t.end());
    return SPMV_SUCCESS;
}

static int bin_place_prod(spmv_plan_s *p, int64_t n, size_t prod_bytes, const spmv_options_t &o) {
    BinDev &B = p->bin;
    int mode = o.placement;
    SPMV_RETURN_IF(placement_mode_check(mode));
    if (const char *e = probe_env("SPMV_PLACEMENT_MODE")) mode = std::atoi(e);
    // AUTO: a product buffer of >= 32 MB is built from 2-MB physical handles
    // (hipMemCreate) mapped into one VA range aligned to 1 GB; smaller ones
    // are one plain allocation.  With one plain hipMalloc the Mul ran in a
    // slow mode on most plans (config 2 Mul 0.61-0.62 vs 0.53 ms; 10 M x 80 M
    // rank shape 0.84 vs 0.72-0.73), the 2-MB handles were fast in 8 of 8
    // plans, first plan of a fresh process included, for no transient memory
    // (profiles/round3/probe/placement_vmm_*.jsonl, profiles/round1/README.md §4a "Placement,
    // round 3").
    if (mode == SPMV_PLACEMENT_AUTO)
        mode = prod_bytes >= kBinVmmMinBytes ? SPMV_PLACEMENT_VMM : SPMV_PLACEMENT_PLAIN;
    // the Mul of a 184 MB product buffer (config 3 with long rows) varies 0.118-0.151 ms
    // by placement as much as config 2's does: search from 32 MB
    if (mode == SPMV_PLACEMENT_SEARCH && prod_bytes < ((size_t)32 << 20)) mode = SPMV_PLACEMENT_PLAIN;
    B.placement = mode;
    if (mode == SPMV_PLACEMENT_SEARCH) return bin_place_search(p, n, prod_bytes);
    if (mode == SPMV_PLACEMENT_VMM) {
        size_t chunk = kVmmChunk, align = kVmmAlign;
        if (const char *e = probe_env("SPMV_VMM_CHUNK_MB")) chunk = (size_t)std::max(1, std::atoi(e)) << 20;
        if (const char *e = probe_env("SPMV_VMM_ALIGN_MB")) align = (size_t)std::max(0, std::atoi(e)) << 20;
        void *q = nullptr;
        SPMV_RETURN_IF(p->arena.alloc_vmm(&q, prod_bytes, chunk, p->device, align));
        B.prod = (double *)q;
        return SPMV_SUCCESS;
    }
    return alloc_prod_plain(p, prod_bytes);
}

// ---- Mul pieces, small tables, product buffer -----------------------------
// Mul pieces: each workgroup takes an nnz-balanced range of its group's
// Mul-ordered entries (cut at 64-entry multiples), split at strips
struct BinPieces {
    std::vector<int64_t> off{0}, beg, end;
    std::vector<int32_t> strip;
};
static void bin_pieces(const BinDev &B, const BinLayout &L, BinPieces &P) {
    const int64_t S = L.S;
    // one workgroup's Mul-order range [a, z) of group g, split at strips
    auto add_range = [&](const int64_t *ss, int64_t a, int64_t z, int64_t &s) {
        while (s < S && ss[s + 1] <= a) ++s;
        for (int64_t t = s; t < S && ss[t] < z; ++t) {
            const int64_t lo = std::max(a, ss[t]), hi = std::min(z, ss[t + 1]);
            if (lo < hi) {
                P.strip.push_back((int32_t)t);
                P.beg.push_back(lo);
                P.end.push_back(hi);
            }
        }
    };
    for (int g = 0; g < B.G; ++g) {
        // Mul-order range of the group (with long rows, G == 1: segments,
        // voids and long blocks)
        // (Mul-ordered products: G == 1, the unpadded entries [0, E1))
        const int64_t g0 = B.g_prod[(size_t)g], g1 = L.LL > 0 || B.mo ? L.E1 : B.g_prod[(size_t)g + 1];
        const int64_t *ss = L.strip_start.data() + (size_t)g * (S + 1);
        int64_t s = 0;
        for (int k = 0; k < B.nwg1; ++k) {
            const int64_t a = g0 + (int64_t)(((__int128)(g1 - g0) * k / B.nwg1) & ~(__int128)63);
            const int64_t z = k + 1 == B.nwg1 ? g1 : g0 + (int64_t)(((__int128)(g1 - g0) * (k + 1) / B.nwg1) & ~(__int128)63);
            add_range(ss, a, z, s);
            P.off.push_back((int64_t)P.strip.size());
        }
    }
}

static int bin_finish(spmv_plan_s *p, int64_t n, const BinLayout &L, const spmv_options_t &o) {
    BinDev &B = p->bin;
    const int64_t E = L.E;
    BinPieces P;
    bin_pieces(B, L, P);
    std::vector<int64_t> &piece_off = P.off, &pbeg = P.beg, &pend = P.end;
    std::vector<int32_t> &pstrip = P.strip;
    B.prod_cap = B.reuse ? 0 : (L.LL > 0 ? L.TRASH + L.PAD : B.mo ? L.E1 : E);
    if (B.reuse)
        for (int g = 0; g < B.G; ++g) B.prod_cap = std::max(B.prod_cap, B.g_prod[(size_t)g + 1] - B.g_prod[(size_t)g]);
    const size_t prod_bytes = sizeof(double) * (size_t)(std::max<int64_t>(B.prod_cap, 1) + kBinProdSlack);
    SPMV_RETURN_IF(upload_vec(p, &B.piece_off, piece_off));
    SPMV_RETURN_IF(upload_vec(p, &B.piece_strip, pstrip));
    SPMV_RETURN_IF(upload_vec(p, &B.piece_begin, pbeg));
    SPMV_RETURN_IF(upload_vec(p, &B.piece_end, pend));
    SPMV_RETURN_IF(upload_vec(p, &B.run_off, L.run_off));
    SPMV_RETURN_IF(upload_vec(p, &B.srun_off, L.srun_off));
    SPMV_RETURN_IF(upload_vec(p, &B.bin_row0, L.row0));
    // the run path is part of the launch the placement search times
    B.long_len = L.LL;
    SPMV_RETURN_IF(bin_place_prod(p, n, prod_bytes, o));
    if (B.dbg & 16) {
        std::fprintf(stderr, "[bin] val1 %p cs1 %p dst1 %p slot2 %p prod %p (E %lld) placement ms:", (void *)B.val1,
                     (void *)B.cs1, (void *)B.dst1, (void *)B.slot2, (void *)B.prod, (long long)E);
        for (float tt : B.placement_ms) std::fprintf(stderr, " %.4f", tt);
        std::fprintf(stderr, "\n");
    }
    if (B.mo) p->kernel_name = "bin_mul_kernel+bin_sum_bin_kernel";  // the Mul-ordered Sum
    p->stored_slots = L.E1;
    B.mul_entries = L.E1;
    B.slot_entries = L.ES;
    B.long_pieces = L.NP;
    B.long_entries = 0;
    for (int64_t v : L.lpad) B.long_entries += v;
    p->n_kernels = B.reuse ? 2 * B.G : B.G + 1;
    return SPMV_SUCCESS;
}

// The run path packs a piece's product position into bits 0-30 of its
// lcode word (bit 31 = piece start), so every position -- the trash line
// past the runs included -- must stay below 2^31.  That is known exactly only
// once the layout exists: the segments' padding can be several times nnz
// when segments are short (up to PAD - 1 per 1-entry segment).
constexpr int64_t kBinLongPosLimit = (int64_t)1 << 31;

// The host layout of A (row bins, segment counts, offsets).  Long rows take
// the run path when their product positions fit lcode; otherwise the layout
// is redone without it (every row then stays in the segments, bit-exact).
static int bin_layout(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o, BinLayout &L,
                      int64_t pos_limit) {
    BinDev &B = p->bin;
    int64_t LL = bin_long_threshold(o, A.row_ptr, A.m, A.nnz, std::max<int64_t>(1, (A.n + B.strip - 1) / B.strip));
    for (;;) {
        L = BinLayout();
        L.S = std::max<int64_t>(1, (A.n + B.strip - 1) / B.strip);
        L.LL = LL;
        B.long_rows = 0;
        if (L.LL > 0) {
            bin_long_prep(A, B.strip, L);
            for (int64_t r = 0; r < A.m; ++r) B.long_rows += L.is_long(A.row_ptr, r) ? 1 : 0;
        }
        bin_mo_resolve(B, o, L.LL, A.nnz);
        SPMV_RETURN_IF(bin_rows(p, A.row_ptr, A.m, A.n, L));
        // segment sizes (bin b, strip s); long rows are not in the segments
        const int64_t S = L.S, NB = L.NB, C = B.strip;
        L.cnt.assign((size_t)(NB * S), 0);
#pragma omp parallel for schedule(dynamic, 16)
        for (int64_t b = 0; b < NB; ++b) {
            int32_t *cb = L.cnt.data() + b * S;
            for (int64_t r = L.row0[(size_t)b]; r < L.row0[(size_t)b + 1]; ++r) {
                if (L.is_long(A.row_ptr, r)) continue;
                for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) ++cb[A.col[j] / C];
            }
        }
        if (L.LL > 0) bin_long_count(L);
        bin_offsets(p, o, L);
        if (L.LL > 0 && L.TRASH + L.PAD > pos_limit) {
            LL = 0;  // positions would wrap in lcode: no run path
            continue;
        }
        return SPMV_SUCCESS;
    }
}

int build_bin(spmv_plan_s *p, const HostCsr &A, const spmv_options_t &o) {
    BinDev &B = p->bin;
    SPMV_RETURN_IF(bin_params(p, o, A.m, A.n, A.nnz));
    if (A.m == 0 || A.nnz == 0) {  // launch_bin only clears y
        B.G = 0;
        return SPMV_SUCCESS;
    }
    BinLayout L;
    SPMV_RETURN_IF(bin_layout(p, A, o, L, kBinLongPosLimit));
    SPMV_RETURN_IF(bin_fill_host(p, A, L));
    return bin_finish(p, A.n, L, o);
}

// ---- long rows from a device CSR: the same layout from the rows' runs (a
// row's entries in one strip, contiguous when its strips are non-decreasing,
// which bin_count_device checks) instead of its entries -- the run-based twin
// of bin_long_prep and bin_long_count
struct BinDevLong {
    std::vector<int32_t> lrows;         // long rows, ascending
    std::vector<int64_t> roff, rbeg;    // [nl + 1] runs per long row; each run's first entry
    std::vector<int32_t> rstrip, rlen;  // each run's strip and length
    std::vector<int64_t> order;         // the runs sorted [strip][row]
};

static int bin_long_prep_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col,
                                const std::vector<int64_t> &rp, BinLayout &L, BinDevLong &D) {
    const int64_t m = p->m, S = L.S;
    D = BinDevLong();
    for (int64_t r = 0; r < m; ++r)
        if (L.is_long(rp.data(), r)) D.lrows.push_back((int32_t)r);
    SPMV_RETURN_IF(bin_long_runs_device(p, d_rp, d_col, D.lrows, D.roff, D.rstrip, D.rbeg));
    const int64_t nl = (int64_t)D.lrows.size(), R = D.roff[(size_t)nl];
    D.rlen.resize((size_t)R);
    // Sum entries per row: a long row needs one per strip it touches and one
    // per 64 entries (bin_long_prep)
    std::vector<int64_t> w((size_t)m);
    for (int64_t r = 0; r < m; ++r) w[(size_t)r] = rp[(size_t)r + 1] - rp[(size_t)r];
    for (int64_t i = 0; i < nl; ++i) {
        const int64_t r = D.lrows[(size_t)i], k0 = D.roff[(size_t)i], k1 = D.roff[(size_t)i + 1];
        for (int64_t k = k0; k < k1; ++k)
            D.rlen[(size_t)k] = (int32_t)((k + 1 < k1 ? D.rbeg[(size_t)k + 1] : rp[(size_t)r + 1]) - D.rbeg[(size_t)k]);
        w[(size_t)r] = (k1 - k0) + w[(size_t)r] / 64;
    }
    L.eff_rp.assign((size_t)m + 1, 0);
    for (int64_t r = 0; r < m; ++r) L.eff_rp[(size_t)r + 1] = L.eff_rp[(size_t)r] + w[(size_t)r];
    // long entries per strip, and the runs in [strip][row] order (a stable
    // counting sort: the runs of a row come in strip order, rows ascending)
    L.lb_off.assign((size_t)S + 1, 0);
    std::vector<int64_t> rc((size_t)S + 1, 0);
    for (int64_t k = 0; k < R; ++k) {
        L.lb_off[(size_t)D.rstrip[(size_t)k] + 1] += D.rlen[(size_t)k];
        ++rc[(size_t)D.rstrip[(size_t)k] + 1];
    }
    for (int64_t t = 0; t < S; ++t) {
        L.lb_off[(size_t)t + 1] += L.lb_off[(size_t)t];
        rc[(size_t)t + 1] += rc[(size_t)t];
    }
    D.order.resize((size_t)R);
    for (int64_t k = 0; k < R; ++k) D.order[(size_t)rc[(size_t)D.rstrip[(size_t)k]]++] = k;
    return SPMV_SUCCESS;
}

// the long row of run k (runs are numbered in long-row order)
static inline int64_t run_row_index(const BinDevLong &D, int64_t k) {
    return std::upper_bound(D.roff.begin(), D.roff.end(), k) - D.roff.begin() - 1;
}

// Walk the runs of every strip in [strip][row] order: f(t, k, row, bin, q0,
// pieces).  A piece starts at each run's first entry and at every 64-entry
// boundary of the strip's long block (long_starts).
template <typename F>
static void bin_long_walk(const BinLayout &L, const BinDevLong &D, F &&f) {
    int64_t t = 0, q0 = 0, b = 0;
    for (size_t i = 0; i < D.order.size(); ++i) {
        const int64_t k = D.order[i];
        if (D.rstrip[(size_t)k] != t || i == 0) {
            t = D.rstrip[(size_t)k];
            q0 = 0;
            b = 0;
        }
        const int32_t r = D.lrows[(size_t)run_row_index(D, k)];
        while (L.row0[(size_t)b + 1] <= r) ++b;
        const int64_t len = D.rlen[(size_t)k];
        f(t, k, r, b, q0, 1 + ((q0 + len - 1) >> 6) - (q0 >> 6));
        q0 += len;
    }
}

static void bin_long_count_device(BinLayout &L, const BinDevLong &D) {
    const int64_t S = L.S, NB = L.NB;
    L.lpc.assign((size_t)(NB * S), 0);
    L.lpad.assign((size_t)S, 0);
    bin_long_walk(L, D, [&](int64_t t, int64_t, int32_t, int64_t b, int64_t, int64_t pieces) {
        L.lpc[(size_t)(b * S + t)] += (int32_t)pieces;
    });
    for (int64_t t = 0; t < S; ++t) L.lpad[(size_t)t] = (L.lb_off[(size_t)t + 1] - L.lb_off[(size_t)t] + 63) & ~(int64_t)63;
}

// the fill's per-run table (bin_fill_arrays' long blocks): the product
// position of each run's first piece -- the pieces of bin b in strip t number
// on from lpoff[b][t] in strip order
static void bin_long_runs_table(const BinLayout &L, const BinDevLong &D, BinLongRuns &LR) {
    const int64_t S = L.S, R = (int64_t)D.order.size();
    LR.j0.resize((size_t)R);
    LR.q0.resize((size_t)R);
    LR.fpos.resize((size_t)R);
    LR.len.resize((size_t)R);
    LR.strip.resize((size_t)R);
    LR.slot.resize((size_t)R);
    LR.bin.resize((size_t)R);
    size_t i = 0;
    int64_t pos = -1, lastb = -1, lastt = -1;
    bin_long_walk(L, D, [&](int64_t t, int64_t k, int32_t r, int64_t b, int64_t q0, int64_t pieces) {
        if (t != lastt) {
            lastt = t;
            lastb = -1;
        }
        if (b != lastb) {
            pos = L.lpoff[(size_t)(b * S + t)];
            lastb = b;
        } else {
            ++pos;
        }
        LR.j0[i] = D.rbeg[(size_t)k];
        LR.q0[i] = q0;
        LR.fpos[i] = pos;
        LR.len[i] = D.rlen[(size_t)k];
        LR.strip[i] = (int32_t)t;
        LR.slot[i] = r - L.row0[(size_t)b];
        LR.bin[i] = (int32_t)b;
        pos += pieces - 1;
        ++i;
    });
}

static int build_bin_device_impl(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                                 const spmv_options_t &o) {
    BinDev &B = p->bin;
    SPMV_RETURN_IF(bin_params(p, o, p->m, p->n, p->nnz));
    if (p->m == 0 || p->nnz == 0) {
        B.G = 0;
        return SPMV_SUCCESS;
    }
    std::vector<int64_t> rp((size_t)p->m + 1);
    SPMV_HIP_TRY(hipMemcpy(rp.data(), d_rp, 8 * (size_t)(p->m + 1), hipMemcpyDeviceToHost));
    const int64_t S = std::max<int64_t>(1, (p->n + B.strip - 1) / B.strip);
    int64_t LL = bin_long_threshold(o, rp.data(), p->m, p->nnz, S);
    // bin_layout's loop: long rows take the run path when their product
    // positions fit lcode, else the layout is redone without it
    BinLayout L;
    BinDevLong D;
    std::vector<int64_t> bstart;
    for (;;) {
        L = BinLayout();
        L.S = S;
        L.LL = LL;
        B.long_rows = 0;
        if (LL > 0) {
            SPMV_RETURN_IF(bin_long_prep_device(p, d_rp, d_col, rp, L, D));
            B.long_rows = (int64_t)D.lrows.size();
        }
        bin_mo_resolve(B, o, LL, p->nnz);
        SPMV_RETURN_IF(bin_rows(p, rp.data(), p->m, p->n, L));
        bstart.assign((size_t)L.NB + 1, 0);
        for (int64_t b = 0; b <= L.NB; ++b) bstart[(size_t)b] = rp[(size_t)L.row0[(size_t)b]];
        const int st = bin_count_device(p, d_rp, d_col, L.row0, bstart, L.S, LL, L.cnt);
        if (st != SPMV_SUCCESS) return st;  // kBinNeedHostBuild: unsorted rows
        if (LL > 0) bin_long_count_device(L, D);
        bin_offsets(p, o, L);
        if (LL > 0 && L.TRASH + L.PAD > kBinLongPosLimit) {
            LL = 0;
            continue;
        }
        break;
    }
    std::vector<int64_t>().swap(rp);
    SPMV_RETURN_IF(bin_fill_device(p, d_rp, d_col, d_val, L.row0, bstart, L.cnt, L.off1, L.off2, L.run_off,
                                   L.srun_off, L.S, L.E, L.ES, LL, L.E1,
                                   (int32_t)(L.TRASH >> B.pad_log)));
    if (LL > 0) {
        BinLongRuns LR;
        bin_long_runs_table(L, D, LR);
        D = BinDevLong();
        SPMV_RETURN_IF(bin_long_fill_device(p, d_col, d_val, LR, L.lb_off, L.lpad, L.lstart, L.lcode_off, L.run_off,
                                            L.srun_off, (B.n_blocks - 1) * L.NB, L.TRASH));
        std::vector<int64_t> lshift((size_t)S);
        for (int64_t t = 0; t < S; ++t) lshift[(size_t)t] = L.lcode_off[(size_t)t] - L.lstart[(size_t)t];
        SPMV_RETURN_IF(upload_vec(p, &B.lstart, L.lstart));
        SPMV_RETURN_IF(upload_vec(p, &B.lshift, lshift));
    }
    if (B.mo) {  // the chunk table needs only the layout
        std::vector<int32_t> tab;
        bin_mo_table(B, L, tab);
        SPMV_RETURN_IF(upload_vec(p, &B.mtab, tab));
    }
    return bin_finish(p, p->n, L, o);
}

int build_bin_device(spmv_plan_s *p, const int64_t *d_rp, const int32_t *d_col, const double *d_val,
                     const spmv_options_t &o) {
    const int st = build_bin_device_impl(p, d_rp, d_col, d_val, o);
    if (st != kBinNeedHostBuild) return st;
    // some row's column strips are out of order: sort every row's entries by
    // strip on the device (stable, so a strip's entries keep their CSR order
    // -- the order the host fill reads them in) and build from that copy: the
    // host builder's layout byte for byte.  No room for the copy: the caller
    // stages the CSR through the host builder.
    void *c2 = nullptr, *v2 = nullptr;
    const size_t nz = (size_t)std::max<int64_t>(p->nnz, 1);
    if (hipMalloc(&c2, 4 * nz) != hipSuccess || hipMalloc(&v2, 8 * nz) != hipSuccess) {
        (void)hipGetLastError();
        if (c2) (void)hipFree(c2);
        return kBinNeedHostBuild;
    }
    int st2 = bin_sort_rows_device(p, d_rp, d_col, d_val, (int32_t *)c2, (double *)v2);
    if (st2 == SPMV_SUCCESS) st2 = build_bin_device_impl(p, d_rp, (const int32_t *)c2, (const double *)v2, o);
    (void)hipStreamSynchronize(p->stream);
    (void)hipFree(c2);
    (void)hipFree(v2);
    return st2;
}

}  // namespace spmv

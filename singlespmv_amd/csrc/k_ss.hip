// k_ss.hip -- segmented-sum SpMV for gfx950: replaces opt_ss
// (src/opt_ss.cpp:222-350: Mul into val_buf, tree fold "Sum1", row "Sum2")
// and the vendored CSR5 (CSR5_cuda/detail/cuda/csr5_spmv_cuda.h:275-419:
// compute -> calibrate -> tail) with a fused, deterministic, idempotent
// wave64 design.
//
// ss_tile_kernel<SIGMA>: one wave = one tile of 64 lanes x SIGMA nnz.  Lane l
// owns SIGMA consecutive nnz (see SsDev layout: every wave load instruction is
// 1 KiB contiguous -- col as 4 ints per lane, val as two 1-KiB halves of 2
// doubles per lane, like ELL's values).  Products never touch memory (no val_buf: opt_ss's extra
// 16 B/nnz is gone).  Per lane: sequential segmented sums split by the row
// start bit-flags; rows that start and end in the lane are written directly.
// Across the wave: a segmented scan (fixed tree) carries open rows from lane
// to lane; the lane where a carried row ends writes it.  A row still open at
// the tile end leaves (tail partial, its ordinal); the partial of the tile's
// first row continuing from earlier tiles leaves as head partial.
//
// x window: when a tile's columns span fewer than kSsWin, the wave first
// copies x[lo, hi] into its own LDS slice (coalesced, mostly L2 hits) and
// reads its SIGMA values per lane from there; a gather per entry touches up to
// 64 lines per instruction (lanes own different rows).  Same values, same
// arithmetic: bit-identical.  Same plans: config 4 (SIGMA 20) -5 to -6 %,
// config 3 -4 %, config 2 -0.7 %; SIGMA 32 (172 VGPRs with the window)
// -1 to +1 % (profiles/round4/probe/ss_sigma_window_*, ss_window_default_c4).
//
// ss_fixup_kernel: one thread per tile whose tail is open adds the heads of
// the following tiles up to the next tile that starts a row (fixed order --
// no atomics, unlike the CAS atomicAdd calibrator of CSR5,
// csr5_spmv_cuda.h:313-382), and zeroes empty rows.  Every y entry is written
// exactly once per execute (β = 0), fixing the CSR5 non-idempotence noted in
// SURVEY §3.5.
#include <type_traits>

#include "device.hpp"
#include "internal.hpp"

namespace spmv {

__device__ __forceinline__ void ss_store(double *y, const int32_t *nzrow, int64_t n_nonempty,
                                         int64_t ord, double v) {
    if (ord < n_nonempty) y[nzrow ? (int64_t)nzrow[ord] : ord] = v;
}

constexpr int kSsWin = 512;  // x window per wave (doubles) of the WIN instance

template <int SIGMA, bool WIN>
__global__ __launch_bounds__(256) void ss_tile_kernel(
    int64_t n_tiles, const int32_t *__restrict__ col, const double *__restrict__ val,
    const uint32_t *__restrict__ flags, const int32_t *__restrict__ tile_ord,
    const int32_t *__restrict__ nzrow, int64_t n_nonempty, const double *__restrict__ x,
    double *__restrict__ y, double *__restrict__ head, double *__restrict__ tail,
    int32_t *__restrict__ tail_ord) {
    static_assert(SIGMA % 4 == 0 && SIGMA <= 32, "sigma");
    constexpr int Q = SIGMA / 4;
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (tile >= n_tiles) return;  // wave-uniform
    const int64_t base = tile * 64 * SIGMA;
    const uint32_t f = flags[tile * 64 + lane];
    const int32_t *cp = col + base + lane * 4;
    const double *vp = val + base + lane * 2;  // entries k%4 < 2 of step k/4, then k%4 >= 2 128 later

    i32x4 c[Q];
    f64x2 a[Q], b[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        c[q] = ld_stream4(cp + q * 256);
        a[q] = ld_stream2(vp + q * 256);
        b[q] = ld_stream2(vp + q * 256 + 128);
    }
    double g[SIGMA];
    bool gathered = false;
    if constexpr (WIN) {
        // the tile's column range; when it fits kSsWin, x comes through a
        // per-wave LDS window (coalesced loads, then LDS reads) instead of
        // SIGMA gathers that each touch up to 64 lines
        __shared__ double xs[4][kSsWin];
        int lo = INT32_MAX, hi = -1;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            lo = min(lo, min(min(c[q].x, c[q].y), min(c[q].z, c[q].w)));
            hi = max(hi, max(max(c[q].x, c[q].y), max(c[q].z, c[q].w)));
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, __shfl_xor(lo, o, 64));
            hi = max(hi, __shfl_xor(hi, o, 64));
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        hi = __builtin_amdgcn_readfirstlane(hi);
        if (hi - lo < kSsWin) {  // wave-uniform
            const int wv = threadIdx.x >> 6;
            for (int i = lane; i <= hi - lo; i += 64) xs[wv][i] = ld_x(x, lo + i);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                g[4 * q + 0] = xs[wv][c[q].x - lo];
                g[4 * q + 1] = xs[wv][c[q].y - lo];
                g[4 * q + 2] = xs[wv][c[q].z - lo];
                g[4 * q + 3] = xs[wv][c[q].w - lo];
            }
            gathered = true;
        }
    }
    if (!gathered) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            g[4 * q + 0] = ld_x(x, c[q].x);
            g[4 * q + 1] = ld_x(x, c[q].y);
            g[4 * q + 2] = ld_x(x, c[q].z);
            g[4 * q + 3] = ld_x(x, c[q].w);
        }
    }

    const int pc = __builtin_popcount(f);
    const int incl = wave_inclusive_sum(pc, lane);
    const int64_t ord0 = (int64_t)tile_ord[tile] + (incl - pc);  // this lane's first start

    double run = 0.0, head_l = 0.0;
    int seen = 0;
#pragma unroll
    for (int k = 0; k < SIGMA; ++k) {
        if ((f >> k) & 1u) {
            if (seen == 0) head_l = run;
            else ss_store(y, nzrow, n_nonempty, ord0 + seen - 1, run);
            run = 0.0;
            ++seen;
        }
        const double v = (k & 2) ? ((k & 1) ? b[k >> 2].y : b[k >> 2].x)
                                 : ((k & 1) ? a[k >> 2].y : a[k >> 2].x);
        run = madd(v, g[k], run);
    }

    const bool has = f != 0u;
    const double S = wave_seg_scan(run, has, lane);  // open-segment sum at lane end
    double C = __shfl_up(S, 1, 64);
    if (lane == 0) C = 0.0;
    const uint64_t ball = __ballot(has);
    const bool started_before = (ball & ((1ull << lane) - 1ull)) != 0ull;
    if (has) {
        const double tot = __dadd_rn(C, head_l);
        if (started_before) ss_store(y, nzrow, n_nonempty, ord0 - 1, tot);
        else head[tile] = tot;  // exactly one lane: the first lane with a start
    }
    if (lane == 63) {
        if (ball == 0ull) {
            head[tile] = S;  // the whole tile continues an earlier row
            tail_ord[tile] = -1;
        } else {
            tail[tile] = S;
            tail_ord[tile] = tile_ord[tile] + incl - 1;
        }
    }
}

// ss_stream_kernel<SIGMA, WIN, PF>: the same tile, sums and hand-off as
// ss_tile_kernel (bit-identical y), streamed: the quads of a lane are loaded
// PF ahead of the quad being summed (sched_barrier-fenced stages), so a lane
// holds PF + 1 quads instead of all SIGMA entries -- SIGMA up to 64 (two flag
// words per lane) at the register cost of SIGMA 12.  The x window of a tile is
// a plan-time descriptor (SsDev::win: first column, length), so the wave
// stages it while its first quads are still in flight instead of after its
// columns arrive.
constexpr int kSsStageRows = 256;  // rows a wave stages in LDS before writing them out

template <int SIGMA, bool WIN, int PF, bool STAGE>
__global__ __launch_bounds__(256) void ss_stream_kernel(
    int64_t n_tiles, const int32_t *__restrict__ col, const double *__restrict__ val,
    const uint32_t *__restrict__ flags, const int32_t *__restrict__ tile_ord, const int32_t *__restrict__ win,
    const int32_t *__restrict__ nzrow, int64_t n_nonempty, const double *__restrict__ x,
    double *__restrict__ y, double *__restrict__ head, double *__restrict__ tail,
    int32_t *__restrict__ tail_ord) {
    static_assert(SIGMA % 4 == 0 && SIGMA <= 64, "sigma");
    constexpr int Q = SIGMA / 4, W = SIGMA > 32 ? 2 : 1;
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (tile >= n_tiles) return;  // wave-uniform
    const int64_t base = tile * 64 * SIGMA;
    const int32_t *cp = col + base + lane * 4;
    const double *vp = val + base + lane * 2;
    i32x4 c[Q];
    f64x2 a[Q], b[Q];
    auto load = [&](int q) {
        c[q] = ld_stream4(cp + q * 256);
        a[q] = ld_stream2(vp + q * 256);
        b[q] = ld_stream2(vp + q * 256 + 128);
    };
#pragma unroll
    for (int q = 0; q < (PF < Q ? PF : Q); ++q) load(q);
    uint32_t f[W];
#pragma unroll
    for (int w = 0; w < W; ++w) f[w] = flags[(tile * W + w) * 64 + lane];
    __shared__ double xs[4][kSsWin];
    const int wv = threadIdx.x >> 6;
    int32_t lo = 0, len = 0;
    if constexpr (WIN) {
        lo = win[2 * tile];
        len = win[2 * tile + 1];
        if (len > 0) {  // wave-uniform
            for (int i = lane; i < len; i += 64) xs[wv][i] = ld_x(x, lo + i);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    int pc = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) pc += __builtin_popcount(f[w]);
    const int incl = wave_inclusive_sum(pc, lane);
    const int64_t ord_base = tile_ord[tile];  // rel ordinal r below = row ord_base + r
    // STAGE: the rows finished inside the tile (ordinals ord_base + [0,
    // total - 1)) go to an LDS slice and leave as coalesced stores after the
    // stream, so no y store sits between the tile's loads in the in-order
    // vmcnt queue; tiles finishing more rows than the slice store directly
    __shared__ double ys[STAGE ? 4 : 1][STAGE ? kSsStageRows : 1];
    const int total = __shfl(incl, 63, 64);
    const bool stage = STAGE && total <= kSsStageRows;  // wave-uniform
    auto finish = [&](int rel, double v) {
        if (STAGE && stage) ys[STAGE ? wv : 0][rel] = v;
        else ss_store(y, nzrow, n_nonempty, ord_base + rel, v);
    };
    const int rel0 = incl - pc;  // this lane's first start

    double run = 0.0, head_l = 0.0;
    int seen = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        if (q + PF < Q) load(q + PF);
        __builtin_amdgcn_sched_barrier(0);
        double g[4];
        if (WIN && len > 0) {
            g[0] = xs[wv][c[q].x - lo];
            g[1] = xs[wv][c[q].y - lo];
            g[2] = xs[wv][c[q].z - lo];
            g[3] = xs[wv][c[q].w - lo];
        } else {
            g[0] = ld_x(x, c[q].x);
            g[1] = ld_x(x, c[q].y);
            g[2] = ld_x(x, c[q].z);
            g[3] = ld_x(x, c[q].w);
        }
        const double v[4] = {a[q].x, a[q].y, b[q].x, b[q].y};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int k = 4 * q + kk;
            if ((f[k >> 5] >> (k & 31)) & 1u) {
                if (seen == 0) head_l = run;
                else finish(rel0 + seen - 1, run);
                run = 0.0;
                ++seen;
            }
            run = madd(v[kk], g[kk], run);
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    const bool has = pc != 0;
    const double S = wave_seg_scan(run, has, lane);  // open-segment sum at lane end
    double C = __shfl_up(S, 1, 64);
    if (lane == 0) C = 0.0;
    const uint64_t ball = __ballot(has);
    const bool started_before = (ball & ((1ull << lane) - 1ull)) != 0ull;
    if (has) {
        const double tot = __dadd_rn(C, head_l);
        if (started_before) finish(rel0 - 1, tot);
        else head[tile] = tot;  // exactly one lane: the first lane with a start
    }
    if constexpr (STAGE) {
        if (stage) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int i = lane; i < total - 1; i += 64) ss_store(y, nzrow, n_nonempty, ord_base + i, ys[wv][i]);
        }
    }
    if (lane == 63) {
        if (ball == 0ull) {
            head[tile] = S;  // the whole tile continues an earlier row
            tail_ord[tile] = -1;
        } else {
            tail[tile] = S;
            tail_ord[tile] = (int32_t)(ord_base + incl - 1);
        }
    }
}

// ss_run_kernel<SIGMA, PF, STAGE>: the tiles [t0, t0 + tpw) of one wave as ONE
// stream.  Quad g of the wave (tile t0 + g / Q, quad g % Q) sits at
// (t0 * Q + g) * 256 in the column array and likewise in the value halves, so
// the wave's loads are a contiguous 1-KiB-per-instruction stream across its
// tiles, kept PF quads deep (a quad is loaded right after the one PF earlier
// is summed, into the register slot it frees: slot g % Q, statically indexed
// because the tile loop is unrolled over Q).  Each tile's flags and first
// ordinal are loaded one tile ahead; the per-tile scan, hand-off and y writes
// are those of ss_tile_kernel (bit-identical y, same head / tail for
// ss_fixup_kernel).  x: the wave's tiles' plan-time windows (SsDev::win) are
// merged at the wave start; when all have one and their union spans fewer than
// kSsWin columns, that union is staged once into the wave's LDS slice and
// every tile reads x there, else x is gathered.
template <int SIGMA, int PF, bool STAGE>
__global__ __launch_bounds__(256) void ss_run_kernel(
    int64_t n_tiles, int tpw, const int32_t *__restrict__ col, const double *__restrict__ val,
    const uint32_t *__restrict__ flags, const int32_t *__restrict__ tile_ord, const int32_t *__restrict__ win,
    const int32_t *__restrict__ nzrow, int64_t n_nonempty, const double *__restrict__ x, double *__restrict__ y,
    double *__restrict__ head, double *__restrict__ tail, int32_t *__restrict__ tail_ord) {
    static_assert(SIGMA % 4 == 0 && SIGMA <= 64, "sigma");
    constexpr int Q = SIGMA / 4, W = SIGMA > 32 ? 2 : 1;
    static_assert(PF >= 1 && PF <= Q, "prefetch depth");
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t t0 = ((int64_t)blockIdx.x * 4 + wv) * tpw;
    if (t0 >= n_tiles) return;  // wave-uniform
    const int nt = (int)(n_tiles - t0 < tpw ? n_tiles - t0 : (int64_t)tpw);
    // the wave's window candidates first: they are waited on before the stream
    int32_t wlo = INT32_MAX, whi = -1, wok = 1;
    if (lane < nt) {
        const int32_t lo = win[2 * (t0 + lane)], len = win[2 * (t0 + lane) + 1];
        wok = len > 0;
        wlo = lo;
        whi = lo + len - 1;
    }
    uint32_t f[W];
#pragma unroll
    for (int w = 0; w < W; ++w) f[w] = flags[(t0 * W + w) * 64 + lane];
    int32_t ordb = tile_ord[t0];
    const int32_t *cp = col + t0 * 64 * SIGMA + lane * 4;
    const double *vp = val + t0 * 64 * SIGMA + lane * 2;
    i32x4 c[Q];
    f64x2 a[Q], b[Q];
    auto load = [&](int slot, int64_t g) {
        c[slot] = ld_stream4(cp + g * 256);
        a[slot] = ld_stream2(vp + g * 256);
        b[slot] = ld_stream2(vp + g * 256 + 128);
    };
#pragma unroll
    for (int q = 0; q < PF; ++q) load(q, q);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        wlo = min(wlo, __shfl_xor(wlo, o, 64));
        whi = max(whi, __shfl_xor(whi, o, 64));
        wok = min(wok, __shfl_xor(wok, o, 64));
    }
    wlo = __builtin_amdgcn_readfirstlane(wlo);
    whi = __builtin_amdgcn_readfirstlane(whi);
    const bool xwin = __builtin_amdgcn_readfirstlane(wok) && whi - wlo < kSsWin;  // wave-uniform
    __shared__ double xs[4][kSsWin];
    if (xwin) {
        for (int i = lane; i <= whi - wlo; i += 64) xs[wv][i] = ld_x(x, wlo + i);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __shared__ double ys[STAGE ? 4 : 1][STAGE ? kSsStageRows : 1];

    for (int it = 0; it < nt; ++it) {
        const int64_t t = t0 + it;
        const bool more = it + 1 < nt;  // wave-uniform
        uint32_t fn[W];
        int32_t ordn = 0;
        if (more) {
#pragma unroll
            for (int w = 0; w < W; ++w) fn[w] = flags[((t + 1) * W + w) * 64 + lane];
            ordn = tile_ord[t + 1];
        }
        int pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) pc += __builtin_popcount(f[w]);
        const int incl = wave_inclusive_sum(pc, lane);
        const int total = __shfl(incl, 63, 64);
        const bool stage = STAGE && total <= kSsStageRows;  // wave-uniform
        const int64_t ord_base = ordb;
        auto finish = [&](int rel, double v) {
            if (STAGE && stage) ys[STAGE ? wv : 0][rel] = v;
            else ss_store(y, nzrow, n_nonempty, ord_base + rel, v);
        };
        const int rel0 = incl - pc;
        double run = 0.0, head_l = 0.0;
        int seen = 0;
        const int64_t gq = (int64_t)it * Q;  // the tile's first quad in the wave stream
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            __builtin_amdgcn_sched_barrier(0);
            double g[4];
            if (xwin) {
                g[0] = xs[wv][c[q].x - wlo];
                g[1] = xs[wv][c[q].y - wlo];
                g[2] = xs[wv][c[q].z - wlo];
                g[3] = xs[wv][c[q].w - wlo];
            } else {
                g[0] = ld_x(x, c[q].x);
                g[1] = ld_x(x, c[q].y);
                g[2] = ld_x(x, c[q].z);
                g[3] = ld_x(x, c[q].w);
            }
            const double v[4] = {a[q].x, a[q].y, b[q].x, b[q].y};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int k = 4 * q + kk;
                if ((f[k >> 5] >> (k & 31)) & 1u) {
                    if (seen == 0) head_l = run;
                    else finish(rel0 + seen - 1, run);
                    run = 0.0;
                    ++seen;
                }
                run = madd(v[kk], g[kk], run);
            }
            // the slot just summed takes the quad PF ahead (this tile's or
            // the next tile's)
            if (q + PF < Q) load(q + PF, gq + q + PF);
            else if (more) load(q + PF - Q, gq + q + PF);
            __builtin_amdgcn_sched_barrier(0);
        }

        const bool has = pc != 0;
        const double S = wave_seg_scan(run, has, lane);
        double C = __shfl_up(S, 1, 64);
        if (lane == 0) C = 0.0;
        const uint64_t ball = __ballot(has);
        const bool started_before = (ball & ((1ull << lane) - 1ull)) != 0ull;
        if (has) {
            const double tot = __dadd_rn(C, head_l);
            if (started_before) finish(rel0 - 1, tot);
            else head[t] = tot;
        }
        if constexpr (STAGE) {
            if (stage) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int i = lane; i < total - 1; i += 64) ss_store(y, nzrow, n_nonempty, ord_base + i, ys[wv][i]);
                // the slice is rewritten by the next tile: every lane's reads first
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        if (lane == 63) {
            if (ball == 0ull) {
                head[t] = S;
                tail_ord[t] = -1;
            } else {
                tail[t] = S;
                tail_ord[t] = (int32_t)(ord_base + incl - 1);
            }
        }
        if (more) {
#pragma unroll
            for (int w = 0; w < W; ++w) f[w] = fn[w];
            ordb = ordn;
        }
    }
}

__global__ __launch_bounds__(256) void ss_fixup_kernel(int64_t n_tiles, const double *__restrict__ head,
                                                       const double *__restrict__ tail,
                                                       const int32_t *__restrict__ tail_ord,
                                                       const int32_t *__restrict__ nzrow,
                                                       int64_t n_nonempty,
                                                       const int32_t *__restrict__ empty_rows,
                                                       int64_t n_empty, double *__restrict__ y) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n_tiles) {
        const int32_t ord = tail_ord[t];
        if (ord >= 0 && ord < n_nonempty) {
            double s = tail[t];
            for (int64_t u = t + 1; u < n_tiles; ++u) {
                s = __dadd_rn(s, head[u]);
                if (tail_ord[u] >= 0) break;
            }
            y[nzrow ? (int64_t)nzrow[ord] : (int64_t)ord] = s;
        }
    }
    if (t < n_empty) y[empty_rows[t]] = 0.0;
}

template <int SIGMA>
static void launch_ss_t(const spmv_plan_s *p, const double *x, double *y) {
    const SsDev &s = p->ss;
    const int64_t blocks = (s.n_tiles + 3) / 4;
    // probe build: SPMV_LAUNCH_SS = 0 -> ss_tile_kernel (all SIGMA entries
    // loaded up front, window from the loaded columns, round 4), else the
    // streamed kernel with SPMV_LAUNCH_SS_PF quads ahead; SPMV_LAUNCH_SS_WIN=0
    // gathers x from memory always
    int kind = SIGMA > 32 && s.kernel == 0 ? 1 : s.kernel, pf = s.pf;
    size_t lds = 0;  // dynamic LDS per workgroup: caps workgroups per CU (probe: SPMV_LAUNCH_SS_LDS_KB)
    bool win = true, stage = s.stage;
    if (const char *v = probe_env("SPMV_LAUNCH_SS_STAGE")) stage = std::atoi(v) != 0;
    if (const char *v = probe_env("SPMV_LAUNCH_SS_LDS_KB")) lds = (size_t)std::atoi(v) * 1024;
    if (const char *v = probe_env("SPMV_LAUNCH_SS")) kind = SIGMA > 32 && std::atoi(v) == 0 ? 1 : std::atoi(v);
    if (const char *v = probe_env("SPMV_LAUNCH_SS_PF")) pf = std::atoi(v);
    if (const char *v = probe_env("SPMV_LAUNCH_SS_WIN")) win = std::atoi(v) != 0;
    auto go = [&](auto kern, bool stream) {
        if (stream)
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, p->stream, s.n_tiles, s.col, s.val, s.flags,
                               s.tile_ord, s.win, s.nzrow, s.n_nonempty, x, y, s.head, s.tail, s.tail_ord);
    };
    if (kind == 0 && SIGMA <= 32) {
        constexpr int S0 = SIGMA <= 32 ? SIGMA : 32;
        if (win)
            hipLaunchKernelGGL((ss_tile_kernel<S0, true>), dim3((unsigned)blocks), dim3(256), lds, p->stream,
                               s.n_tiles, s.col, s.val, s.flags, s.tile_ord, s.nzrow, s.n_nonempty, x, y,
                               s.head, s.tail, s.tail_ord);
        else
            hipLaunchKernelGGL((ss_tile_kernel<S0, false>), dim3((unsigned)blocks), dim3(256), lds, p->stream,
                               s.n_tiles, s.col, s.val, s.flags, s.tile_ord, s.nzrow, s.n_nonempty, x, y,
                               s.head, s.tail, s.tail_ord);
        return;
    }
    win = win && s.win;
    if (kind == 2) {  // ss_run_kernel: tpw tiles per wave as one stream
        int tpw = s.tpw;
        if (const char *v = probe_env("SPMV_LAUNCH_SS_TPW")) tpw = std::atoi(v);
        tpw = tpw < 1 ? 1 : (tpw > 64 ? 64 : tpw);
        const int64_t waves = (s.n_tiles + tpw - 1) / tpw;
        const unsigned rblocks = (unsigned)((waves + 3) / 4);
        auto run = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(rblocks), dim3(256), lds, p->stream, s.n_tiles, tpw, s.col, s.val, s.flags,
                               s.tile_ord, s.win, s.nzrow, s.n_nonempty, x, y, s.head, s.tail, s.tail_ord);
        };
        constexpr int P2 = SIGMA / 4 < 2 ? SIGMA / 4 : 2, P4 = SIGMA / 4 < 4 ? SIGMA / 4 : 4;
        if (pf >= 4) stage ? run(ss_run_kernel<SIGMA, P4, true>) : run(ss_run_kernel<SIGMA, P4, false>);
        else stage ? run(ss_run_kernel<SIGMA, P2, true>) : run(ss_run_kernel<SIGMA, P2, false>);
        return;
    }
    auto pick = [&](auto pfc) {
        constexpr int P = decltype(pfc)::value;
        if (stage) win ? go(ss_stream_kernel<SIGMA, true, P, true>, true) : go(ss_stream_kernel<SIGMA, false, P, true>, true);
        else win ? go(ss_stream_kernel<SIGMA, true, P, false>, true) : go(ss_stream_kernel<SIGMA, false, P, false>, true);
    };
    switch (pf) {
        case 1: pick(std::integral_constant<int, 1>{}); break;
        case 4: pick(std::integral_constant<int, 4>{}); break;
        default: pick(std::integral_constant<int, 2>{});
    }
}

int launch_ss(const spmv_plan_s *p, const double *x, double *y) {
    const SsDev &s = p->ss;
    if (s.n_tiles > 0) {
        switch (s.sigma) {
            case 4: launch_ss_t<4>(p, x, y); break;
            case 8: launch_ss_t<8>(p, x, y); break;
            case 12: launch_ss_t<12>(p, x, y); break;
            case 16: launch_ss_t<16>(p, x, y); break;
            case 20: launch_ss_t<20>(p, x, y); break;
            case 24: launch_ss_t<24>(p, x, y); break;
            case 32: launch_ss_t<32>(p, x, y); break;
            case 48: launch_ss_t<48>(p, x, y); break;
            case 64: launch_ss_t<64>(p, x, y); break;
            default: set_error("ss sigma must be one of 4,8,12,16,20,24,32,48,64"); return SPMV_ERROR_INVALID_VALUE;
        }
        SPMV_HIP_TRY(hipGetLastError());
    }
    phase_mark(p);  // tile | fixup
    const int64_t work = s.n_tiles > s.n_empty ? s.n_tiles : s.n_empty;
    if (work > 0) {
        hipLaunchKernelGGL(ss_fixup_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                           p->stream, s.n_tiles, s.head, s.tail, s.tail_ord, s.nzrow, s.n_nonempty,
                           s.empty_rows, s.n_empty, y);
        SPMV_HIP_TRY(hipGetLastError());
    }
    return SPMV_SUCCESS;
}

}  // namespace spmv

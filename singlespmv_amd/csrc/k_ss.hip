// k_ss.hip -- segmented-sum SpMV for gfx950: replaces opt_ss
// (src/opt_ss.cpp:222-350: Mul into val_buf, tree fold "Sum1", row "Sum2")
// and the vendored CSR5 (CSR5_cuda/detail/cuda/csr5_spmv_cuda.h:275-419:
// compute -> calibrate -> tail) with a fused, deterministic, idempotent
// wave64 design.
//
// The product launches ss_stream_kernel (below); ss_tile_kernel, its
// all-loads-first twin, is compiled into the probe build only (`make probes`,
// SPMV_SS_KERNEL=0), like the stream kernel's non-default PF / stage / window
// instances.
// The tile, common to both: one wave = 64 lanes x SIGMA nnz.  Lane l
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

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// The end of a tile, after the wave's segmented scan.  S: the lane's open
// segment sum at its end; tot: a starting lane's finished first row (C + its
// head run); ball: the lanes with a row start.  Lanes with a start after the
// tile's first finished rows (tot) already; the rest leave here:
//   head = tot of the first lane with a start (or the whole-tile S of lane 63
//          when no row starts: the tile continues an earlier row),
//   tail = S of lane 63 (the row still open at the tile end),
//   and, when `nrows` finished rows wait in the wave's LDS slice `ys`, those.
// All of them go out as ONE store instruction (lanes 0..nrows-1 the rows,
// lane 62 the head, lane 63 the tail) when nrows <= 62, instead of round 4's
// four (rows, head, tail, tail ordinal) -- neutral at config 4, where the
// time the y writes cost is spent at the memory, not in the store count
// (profiles/round5/README.md).  The tail's ordinal is a plan constant
// (SsDev::tail_ord), not stored here.
__device__ __forceinline__ void ss_tile_end(int lane, int64_t tile, uint64_t ball, double tot, double S, int nrows,
                                            const double *ys, int64_t ord_base, const int32_t *nzrow,
                                            int64_t n_nonempty, double *y, double *ht) {
    const double s63 = readlane_f64(S, 63);
    const double headv = ball ? readlane_f64(tot, (int)__builtin_ctzll(ball)) : s63;
    int rem = nrows;
    if (nrows > 62) {  // wide tile: the rows first, in whole waves
        for (int i = lane; i < nrows; i += 64) ss_store(y, nzrow, n_nonempty, ord_base + i, ys[i]);
        rem = 0;
    }
    double *a = nullptr;
    double v = 0.0;
    if (lane < rem) {
        const int64_t ord = ord_base + lane;
        if (ord < n_nonempty) a = y + (nzrow ? (int64_t)nzrow[ord] : ord);
        v = ys[lane];
    } else if (lane == 62) {
        a = ht + 2 * tile;
        v = headv;
    } else if (lane == 63 && ball) {
        a = ht + 2 * tile + 1;
        v = s63;
    }
    if (a) *a = v;
}

#ifdef SPMV_PROBES  // round 4's kernel: probe build only (launch_ss_probe)
template <int SIGMA, bool WIN>
__global__ __launch_bounds__(256) void ss_tile_kernel(
    int64_t n_tiles, const int32_t *__restrict__ col, const double *__restrict__ val,
    const uint32_t *__restrict__ flags, const int32_t *__restrict__ tile_ord,
    const int32_t *__restrict__ nzrow, int64_t n_nonempty, const double *__restrict__ x,
    double *__restrict__ y, double *__restrict__ ht) {
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
    const double tot = __dadd_rn(C, head_l);
    if (has && started_before) ss_store(y, nzrow, n_nonempty, ord0 - 1, tot);
    ss_tile_end(lane, tile, ball, tot, S, 0, nullptr, 0, nzrow, n_nonempty, y, ht);
}
#endif

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
    double *__restrict__ y, double *__restrict__ ht) {
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
    // total - 1)) go to the wave's LDS slice and leave in the tile's one store
    // instruction (ss_tile_end); tiles finishing more rows than the slice
    // holds store them directly.  Slice layout: [0] = rel -1 (a lane's head
    // segment parks at rel0 - 1 until the scan), [1, kSsStageRows] = rel 0..,
    // then one dump slot per lane.
    __shared__ double ys[STAGE ? 4 : 1][STAGE ? kSsStageRows + 1 + 64 : 1];
    const int total = __builtin_amdgcn_readlane(incl, 63);
    const bool stage = STAGE && total <= kSsStageRows;  // wave-uniform
    double *yl = &ys[STAGE ? wv : 0][STAGE ? 1 : 0];
    double *dump = &ys[STAGE ? wv : 0][STAGE ? kSsStageRows + 1 + lane : 0];
    const int rel0 = incl - pc;  // this lane's first start

    double run = 0.0, head_l = 0.0;
    auto sum_tile = [&](auto fastc) {
        // FAST (staged tiles): branch-free -- at every entry the run so far
        // is written to LDS, to the slot of the segment it closes when the
        // entry starts a row (its head segment to rel0 - 1, then rel0, ...)
        // and to the lane's dump slot otherwise, then reset by a select.
        // Same additions in the same order as the branchy form below (which
        // the direct-store tiles keep): bit-identical.
        constexpr bool FAST = decltype(fastc)::value;
        int seen = 0, sl = rel0 - 1;
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
                const bool st = (f[k >> 5] >> (k & 31)) & 1u;
                if constexpr (FAST) {
                    *(st ? yl + sl : dump) = run;
                    run = st ? 0.0 : run;
                    sl += st ? 1 : 0;
                } else if (st) {
                    if (seen == 0) head_l = run;
                    else ss_store(y, nzrow, n_nonempty, ord_base + rel0 + seen - 1, run);
                    run = 0.0;
                    ++seen;
                }
                run = madd(v[kk], g[kk], run);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (FAST) head_l = pc ? yl[rel0 - 1] : 0.0;
    };
    if (stage) sum_tile(std::true_type{});
    else sum_tile(std::false_type{});

    const bool has = pc != 0;
    const double S = wave_seg_scan(run, has, lane);  // open-segment sum at lane end
    double C = __shfl_up(S, 1, 64);
    if (lane == 0) C = 0.0;
    const uint64_t ball = __ballot(has);
    const bool started_before = (ball & ((1ull << lane) - 1ull)) != 0ull;
    const double tot = __dadd_rn(C, head_l);
    if (has && started_before) {
        if (stage) yl[rel0 - 1] = tot;
        else ss_store(y, nzrow, n_nonempty, ord_base + rel0 - 1, tot);
    }
    if constexpr (STAGE) {
        if (stage) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    ss_tile_end(lane, tile, ball, tot, S, stage ? total - 1 : 0, yl, ord_base, nzrow, n_nonempty, y, ht);
}

__global__ __launch_bounds__(256) void ss_fixup_kernel(int64_t n_tiles, const double *__restrict__ ht,
                                                       const int32_t *__restrict__ tail_ord,
                                                       const int32_t *__restrict__ nzrow,
                                                       int64_t n_nonempty,
                                                       const int32_t *__restrict__ empty_rows,
                                                       int64_t n_empty, double *__restrict__ y) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n_tiles) {
        const int32_t ord = tail_ord[t];
        if (ord >= 0 && ord < n_nonempty) {
            double s = ht[2 * t + 1];
            for (int64_t u = t + 1; u < n_tiles; ++u) {
                s = __dadd_rn(s, ht[2 * u]);
                if (tail_ord[u] >= 0) break;
            }
            y[nzrow ? (int64_t)nzrow[ord] : (int64_t)ord] = s;
        }
    }
    if (t < n_empty) y[empty_rows[t]] = 0.0;
}

// plan time: tail_ord[t] = ordinal of tile t's last row start (its first
// start's ordinal tile_ord[t] + the tile's flag count - 1; the dummy start
// over the padding counts, as the tile kernels count it), -1 when no row
// starts in the tile.  One wave per tile.
__global__ __launch_bounds__(256) void ss_tail_ord_kernel(int64_t n_tiles, int words,
                                                          const uint32_t *__restrict__ flags,
                                                          const int32_t *__restrict__ tile_ord,
                                                          int32_t *__restrict__ tail_ord) {
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= n_tiles) return;
    int pc = 0;
    for (int w = 0; w < words; ++w) pc += __builtin_popcount(flags[(t * words + w) * 64 + lane]);
    for (int o = 32; o > 0; o >>= 1) pc += __shfl_xor(pc, o, 64);
    if (lane == 0) tail_ord[t] = pc ? tile_ord[t] + pc - 1 : -1;
}

int ss_plan_tail_ord(spmv_plan_s *p) {
    const SsDev &s = p->ss;
    if (s.n_tiles > 0) {
        hipLaunchKernelGGL(ss_tail_ord_kernel, dim3((unsigned)((s.n_tiles + 3) / 4)), dim3(256), 0, p->stream,
                           s.n_tiles, ss_flag_words(s.sigma), s.flags, s.tile_ord, s.tail_ord);
        SPMV_HIP_TRY(hipGetLastError());
        SPMV_HIP_TRY(hipStreamSynchronize(p->stream));  // executes may run on another stream
    }
    return SPMV_SUCCESS;
}

#ifdef SPMV_PROBES
// Probe build only (`make probes`): the round-4 all-loads-first kernel
// (SPMV_LAUNCH_SS = 0 / SPMV_SS_KERNEL = 0), the other prefetch depths
// (SPMV_LAUNCH_SS_PF 1 / 4), unstaged rows (SPMV_LAUNCH_SS_STAGE = 0), no x
// window (SPMV_LAUNCH_SS_WIN = 0) and a dynamic-LDS cap on workgroups per CU
// (SPMV_LAUNCH_SS_LDS_KB).  None of these instances is in the product library.
template <int SIGMA>
static void launch_ss_probe(const spmv_plan_s *p, const double *x, double *y) {
    const SsDev &s = p->ss;
    const int64_t blocks = (s.n_tiles + 3) / 4;
    int kind = SIGMA > 32 && s.kernel == 0 ? 1 : s.kernel, pf = s.pf;
    size_t lds = 0;
    bool win = true, stage = s.stage;
    if (const char *v = probe_env("SPMV_LAUNCH_SS_STAGE")) stage = std::atoi(v) != 0;
    if (const char *v = probe_env("SPMV_LAUNCH_SS_LDS_KB")) lds = (size_t)std::atoi(v) * 1024;
    if (const char *v = probe_env("SPMV_LAUNCH_SS")) kind = SIGMA > 32 && std::atoi(v) == 0 ? 1 : std::atoi(v);
    if (const char *v = probe_env("SPMV_LAUNCH_SS_PF")) pf = std::atoi(v);
    if (const char *v = probe_env("SPMV_LAUNCH_SS_WIN")) win = std::atoi(v) != 0;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, p->stream, s.n_tiles, s.col, s.val, s.flags,
                           s.tile_ord, s.win, s.nzrow, s.n_nonempty, x, y, s.ht);
    };
    if (kind == 0 && SIGMA <= 32) {
        constexpr int S0 = SIGMA <= 32 ? SIGMA : 32;
        if (win)
            hipLaunchKernelGGL((ss_tile_kernel<S0, true>), dim3((unsigned)blocks), dim3(256), lds, p->stream,
                               s.n_tiles, s.col, s.val, s.flags, s.tile_ord, s.nzrow, s.n_nonempty, x, y, s.ht);
        else
            hipLaunchKernelGGL((ss_tile_kernel<S0, false>), dim3((unsigned)blocks), dim3(256), lds, p->stream,
                               s.n_tiles, s.col, s.val, s.flags, s.tile_ord, s.nzrow, s.n_nonempty, x, y, s.ht);
        return;
    }
    win = win && s.win;
    auto pick = [&](auto pfc) {
        constexpr int P = decltype(pfc)::value;
        if (stage) win ? go(ss_stream_kernel<SIGMA, true, P, true>) : go(ss_stream_kernel<SIGMA, false, P, true>);
        else win ? go(ss_stream_kernel<SIGMA, true, P, false>) : go(ss_stream_kernel<SIGMA, false, P, false>);
    };
    switch (pf) {
        case 1: pick(std::integral_constant<int, 1>{}); break;
        case 4: pick(std::integral_constant<int, 4>{}); break;
        default: pick(std::integral_constant<int, 2>{});
    }
}
#endif

// The product launch: the streamed kernel, 2 quads ahead, finished rows
// staged in LDS, x through the plan's per-tile windows (when the plan has any)
// -- two instances per SIGMA.
template <int SIGMA>
static void launch_ss_t(const spmv_plan_s *p, const double *x, double *y) {
#ifdef SPMV_PROBES
    launch_ss_probe<SIGMA>(p, x, y);
#else
    const SsDev &s = p->ss;
    const dim3 grid((unsigned)((s.n_tiles + 3) / 4));
    if (s.win)
        hipLaunchKernelGGL((ss_stream_kernel<SIGMA, true, 2, true>), grid, dim3(256), 0, p->stream, s.n_tiles, s.col,
                           s.val, s.flags, s.tile_ord, s.win, s.nzrow, s.n_nonempty, x, y, s.ht);
    else
        hipLaunchKernelGGL((ss_stream_kernel<SIGMA, false, 2, true>), grid, dim3(256), 0, p->stream, s.n_tiles, s.col,
                           s.val, s.flags, s.tile_ord, s.win, s.nzrow, s.n_nonempty, x, y, s.ht);
#endif
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
                           p->stream, s.n_tiles, s.ht, s.tail_ord, s.nzrow, s.n_nonempty,
                           s.empty_rows, s.n_empty, y);
        SPMV_HIP_TRY(hipGetLastError());
    }
    return SPMV_SUCCESS;
}

}  // namespace spmv

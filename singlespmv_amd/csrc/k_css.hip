// k_css.hip -- column-slab sweep SpMV ("CSS") for gfx950.
//
// Design ancestor: the reference's column-blocked segmented sum opt_css
// (src/opt_css.cpp:33-45 splits columns into N_BLOCK blocks so the x block
// stays cache resident).  Re-designed for the MI355X memory
// hierarchy, where a random 8-byte x gather that misses the XCD's 4 MiB L2
// costs a 64 B fabric request (~54 G gathers/s chip-wide, MALL or HBM alike)
// while an L2 hit runs at ~190 G/s (profiles/round1/it1_baseline/gather_probe.json).
//
// Geometry (see CssDev):
//  * one 1024-thread workgroup per CU: 15 WORKER waves + 1 PACER wave.  The
//    workgroup owns an nnz-balanced block of <= 19968 rows per pass and keeps their
//    y in LDS (160 KB), so y never round-trips through HBM between slabs;
//  * columns are cut into slabs of 2^slab_shift columns.  Each worker wave
//    owns a set of rows / row pieces (LPT-balanced by nnz) and streams its own
//    entry list, sorted by column, i.e. slab by slab, software-pipelined one
//    256-entry chunk ahead;
//  * pacing (speed only, never results): workers report finished slabs with
//    LDS atomics and wait, in LDS, for the slab to be allowed.  The pacer
//    wave alone talks to global memory: it publishes the workgroup's finished
//    slabs to a per-XCD-label counter (blockIdx % 8 labels the workgroups
//    that share an XCD under the observed round-robin placement) and turns
//    the label's (or every label's) progress into the LDS "allowed" slab, so
//    the workgroups of an XCD sweep within `lag` slabs of each other and the
//    XCD's L2 serves the x gathers.  Every wait is bounded.
//
// Determinism / exactness: a row (or row piece) is owned by one wave, which
// adds its entries in ascending column order (ds_add_f64 in program order;
// lanes of one instruction that hit the same slot are applied in lane = list
// order by the LDS unit -- observed; the named guard is tests/test_gpu_parity.py::
// test_lds_add_lane_order, and tests/test_guards.py checks the adds compile to
// ds_add_f64);
// the slot starts at +0.0.  An unsplit row is therefore the sequential
// opt_crs sum (src/opt_crs.cpp:61-66) bit for bit; a row longer than half a
// wave's share is split into pieces whose sums are added in piece order at
// the end of the pass (deterministic, different rounding order).
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

constexpr int kCssThreads = 64 * (kCssWorkers + 1);
constexpr int kCssRing = 512;  // slab arrival ring in LDS (aliasing only blurs pacing)

struct CssChunk {
    int32_t c[4];
    uint32_t r2[2];  // the four 16-bit LDS slots, two per register
    double v[4];
    __device__ __forceinline__ int slot(int u) const { return (int)((r2[u >> 1] >> (16 * (u & 1))) & 0xFFFFu); }
};

// One 256-entry chunk of a wave's list, branch-free (so the compiler's
// in-order vmcnt tracking stays exact across the pipeline).  Chunk kc of the
// list starts at base + kc * stride (stride 256: contiguous lists; lists x 256:
// interleaved layout); lanes past the list's end re-load the list's first
// entry and are redirected to the dummy slot kCssMaxRows by css_mask.
template <bool NT>
__device__ __forceinline__ void css_load(CssChunk &k, int64_t kc, int64_t base, int64_t stride, int64_t len,
                                         int lane, const int32_t *__restrict__ col,
                                         const uint16_t *__restrict__ row,
                                         const double *__restrict__ val) {
    uint32_t r[4];
    const int64_t cs = base + kc * stride;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t o = kc * 256 + u * 64 + lane;
        const int64_t jj = o < len ? cs + u * 64 + lane : base;
        if (NT) {
            k.c[u] = ld_stream(col + jj);
            r[u] = __builtin_nontemporal_load(row + jj);
            k.v[u] = ld_stream(val + jj);
        } else {
            k.c[u] = col[jj];
            r[u] = row[jj];
            k.v[u] = val[jj];
        }
    }
    k.r2[0] = r[0] | (r[1] << 16);
    k.r2[1] = r[2] | (r[3] << 16);
}

__device__ __forceinline__ void css_mask(CssChunk &k, int64_t kc, int64_t len, int lane) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const bool ok = kc * 256 + u * 64 + lane < len;
        const uint32_t keep = ok ? 0xFFFFu : 0u, dummy = ok ? 0u : (uint32_t)kCssMaxRows;
        const int sh = 16 * (u & 1);
        k.r2[u >> 1] = (k.r2[u >> 1] & ~(0xFFFFu << sh)) | ((((k.r2[u >> 1] >> sh) & keep) | dummy) << sh);
        k.v[u] = ok ? k.v[u] : 0.0;
    }
}

template <int DBG>
__device__ __forceinline__ void css_gather(double (&g)[4], const CssChunk &k, const double *__restrict__ x) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (DBG & 1) g[u] = (double)k.c[u];                   // ablation: no gathers
        else if (DBG & 16) g[u] = ld_x(x, k.c[u] & 0x1FFFF);  // ablation: all gathers in 1 MiB
        else g[u] = ld_x(x, k.c[u]);
    }
}

template <bool NT, int DBG>
__global__ __launch_bounds__(kCssThreads) void css_sweep_kernel(
    const int64_t *__restrict__ bstart, const int32_t *__restrict__ rmap, const int64_t *__restrict__ moff,
    const int32_t *__restrict__ merge, int32_t P, int32_t nwg, int32_t S, int32_t slab_shift, int32_t lag,
    const int64_t *__restrict__ woff, const int32_t *__restrict__ wlen, int64_t stride,
    const int32_t *__restrict__ col,
    const uint16_t *__restrict__ row, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, uint64_t *__restrict__ prog,
    uint64_t seq, int32_t pace_all, uint64_t *__restrict__ tstamp) {
    __shared__ double ylds[kCssMaxRows + 1];  // + dummy slot for masked lanes
    __shared__ int32_t arrive[kCssRing];
    __shared__ int32_t allowed;
    const int w = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x;
    const int label = b & 7;
    const bool pacing = lag > 0;
    const bool pacer = w == kCssWorkers;

    for (int p = 0; p < P; ++p) {
        // this workgroup's nnz-balanced row block of pass p (<= kCssMaxRows rows)
        const int64_t row0 = bstart[(int64_t)p * nwg + b];
        const int rows = (int)(bstart[(int64_t)p * nwg + b + 1] - row0);
        for (int i = threadIdx.x; i < kCssMaxRows; i += kCssThreads) ylds[i] = 0.0;  // rows + piece slots
        for (int i = threadIdx.x; i < kCssRing; i += kCssThreads) arrive[i] = 0;
        if (threadIdx.x == 0) allowed = pacing ? lag - 1 : S;
        __syncthreads();
        uint64_t *ts = tstamp ? tstamp + ((int64_t)p * nwg + b) * (kCssWorkers + 2) : nullptr;
        if (ts && threadIdx.x == 0) ts[0] = __builtin_amdgcn_s_memrealtime();

        if (pacer) {
            // ---------------- pacer wave: the only wave touching prog[] ----
            if (pacing && lane == 0) {
                int done = -1;  // highest slab of this pass finished by all workers
                int idle = 0;
                while (done < S - 1) {
                    bool moved = false;
                    while (done < S - 1 &&
                           __hip_atomic_load(&arrive[(done + 1) & (kCssRing - 1)], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP) >= kCssWorkers) {
                        ++done;
                        // consume exactly one slab's arrivals (a wave far ahead may
                        // already have added to the same ring slot)
                        __hip_atomic_fetch_add(&arrive[done & (kCssRing - 1)], -kCssWorkers, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(prog + label * 16, (uint64_t)1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        moved = true;
                        idle = 0;
                    }
                    // slowest label (or own label) progress -> allowed slab
                    int64_t lo = INT64_MAX;
                    const int l0 = pace_all ? 0 : label, l1 = pace_all ? 8 : label + 1;
                    for (int l = l0; l < l1; ++l) {
                        const uint64_t cnt = (uint64_t)((nwg - l + 7) / 8);
                        const uint64_t base = (seq * (uint64_t)P + (uint64_t)p) * (uint64_t)S * cnt;
                        const uint64_t v = __hip_atomic_load(prog + l * 16, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
                        const int64_t doneall = v > base ? (int64_t)((v - base) / cnt) : 0;
                        lo = doneall < lo ? doneall : lo;
                    }
                    const int64_t a = lo + lag - 1;
                    __hip_atomic_store(&allowed, (int32_t)(a < S ? a : S), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (!moved) {
                        if (++idle > 20000) {  // bound: ~4 ms without progress -> stop pacing this pass
                            __hip_atomic_store(&allowed, S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
                __hip_atomic_store(&allowed, S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else {
            // ---------------- worker waves ----------------------------------
            const int64_t list = ((int64_t)p * nwg + b) * kCssWorkers + w;
            const int64_t base = woff[list];
            const int64_t len = wlen[list];
            int cur = -1;       // slab this wave has entered
            int budget = 4000;  // bounded total waiting per pass
            double dsink = 0.0;
            auto enter = [&](int s) {
                // report slabs < s as finished, then wait until s is allowed
                while (cur < s) {
                    if (cur >= 0 && lane == 0)
                        __hip_atomic_fetch_add(&arrive[cur & (kCssRing - 1)], 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                    ++cur;
                }
                if (pacing && s < S) {
                    while (budget > 0 &&
                           __hip_atomic_load(&allowed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < s) {
                        --budget;
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            };
            // Software pipeline, issue order per iteration k: gathers(k+1) |
            // stream loads(k+3) | LDS atomics(k), the stream loads of k+1 and
            // k+2 already in flight.  The register rotation at the end of the
            // iteration waits for gathers(k+1); a statically rotated 4-way
            // unroll without that wait measured 6 % slower (more stream loads
            // queue ahead of the gathers).  Lanes past the list end are masked
            // (dummy slot, +0.0).
            CssChunk L0, L1, L2, L3;
            double g0[4], g1[4];
            css_load<NT>(L0, 0, base, stride, len, lane, col, row, val);
            css_load<NT>(L1, 1, base, stride, len, lane, col, row, val);
            if (len > 0) {
                const int s0 = __builtin_amdgcn_readfirstlane(L0.c[0]) >> slab_shift;
                if (s0 > cur) enter(s0);
            }
            css_gather<DBG>(g0, L0, x);
            css_load<NT>(L2, 2, base, stride, len, lane, col, row, val);
            const int64_t nchunks = (len + 255) / 256;
            for (int64_t kc = 0; kc < nchunks; ++kc) {
                __builtin_amdgcn_sched_barrier(0);
                if (kc + 1 < nchunks) {
                    const int s1 = __builtin_amdgcn_readfirstlane(L1.c[0]) >> slab_shift;
                    if (s1 > cur) enter(s1);
                }
                css_gather<DBG>(g1, L1, x);
                __builtin_amdgcn_sched_barrier(0);
                css_load<NT>(L3, kc + 3, base, stride, len, lane, col, row, val);
                __builtin_amdgcn_sched_barrier(0);
                css_mask(L0, kc, len, lane);
                if (DBG & 2) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) dsink += __dmul_rn(L0.v[u], g0[u]) * (double)L0.slot(u);
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) atomicAdd(&ylds[L0.slot(u)], __dmul_rn(L0.v[u], g0[u]));
                }
                L0 = L1;
                L1 = L2;
                L2 = L3;
#pragma unroll
                for (int u = 0; u < 4; ++u) g0[u] = g1[u];
            }
            enter(S);  // report every remaining slab
            if (ts && lane == 0) ts[1 + w] = __builtin_amdgcn_s_memrealtime();
            if ((DBG & 2) && dsink == 1.2345) y[0] = dsink;  // keep ablated work alive
        }
        __syncthreads();
        // rows split into pieces: add the extra pieces in piece order
        {
            const int64_t pb = (int64_t)p * nwg + b;
            for (int64_t i = moff[pb] + threadIdx.x; i < moff[pb + 1]; i += kCssThreads) {
                const int slot = merge[3 * i], first = merge[3 * i + 1], cnt = merge[3 * i + 2];
                double acc = ylds[slot];
                for (int t = 0; t < cnt; ++t) acc = __dadd_rn(acc, ylds[first + t]);
                ylds[slot] = acc;
            }
        }
        __syncthreads();
        if (rmap)
            for (int i = threadIdx.x; i < rows; i += kCssThreads) y[rmap[row0 + i]] = ylds[i];
        else
            for (int i = threadIdx.x; i < rows; i += kCssThreads) y[row0 + i] = ylds[i];
        __syncthreads();
        if (ts && threadIdx.x == 0) ts[kCssWorkers + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

template <bool NT, int DBG>
static void launch_css_t(const spmv_plan_s *p, const double *x, double *y, uint64_t seq) {
    const CssDev &c = p->css;
    hipLaunchKernelGGL((css_sweep_kernel<NT, DBG>), dim3((unsigned)c.nwg), dim3(kCssThreads), 0, p->stream,
                       c.bstart, c.rmap, c.moff, c.merge, c.P, c.nwg, c.S, c.slab_shift, c.lag, c.woff, c.wlen,
                       c.chunk_stride, c.col, c.row, c.val,
                       x, y, c.prog, seq, c.pace_all, c.tstamp);
}

int launch_css(const spmv_plan_s *p, const double *x, double *y) {
    const CssDev &c = p->css;
    if (p->m == 0) return SPMV_SUCCESS;
    if (p->nnz == 0) {  // no entries: y = 0 (and x may be empty)
        SPMV_HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * (size_t)p->m, p->stream));
        return SPMV_SUCCESS;
    }
    spmv_plan_s *mp = const_cast<spmv_plan_s *>(p);
    const uint64_t seq = mp->css.launches++;
#ifndef SPMV_PROBES
    (void)c;
    launch_css_t<true, 0>(p, x, y, seq);
#else
    // ablations (SPMV_CSS_DEBUG, probe build only): 1 no gathers, 2 no LDS
    // atomics, 8 default cache policy on the matrix stream, 16 all gathers in 1 MiB
    switch (c.dbg & 19) {
        case 18: launch_css_t<true, 18>(p, x, y, seq); break;
        case 3: launch_css_t<true, 3>(p, x, y, seq); break;
        case 1: launch_css_t<true, 1>(p, x, y, seq); break;
        case 2: launch_css_t<true, 2>(p, x, y, seq); break;
        case 16: launch_css_t<true, 16>(p, x, y, seq); break;
        default:
            if (c.dbg & 8) launch_css_t<false, 0>(p, x, y, seq);
            else launch_css_t<true, 0>(p, x, y, seq);
    }
#endif
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

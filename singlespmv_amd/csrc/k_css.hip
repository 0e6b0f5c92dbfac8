// k_css.hip -- column-slab sweep SpMV ("CSS") for gfx950.
//
// Design ancestor: the reference's column-blocked segmented sum opt_css
// (src/opt_css.cpp:33-45 splits columns into N_BLOCK blocks so the x block
// stays cache resident).  Re-designed for the MI355X memory
// hierarchy, where a random 8-byte x gather that misses the XCD's 4 MiB L2
// costs a 64 B fabric request (~54 G gathers/s chip-wide, MALL or HBM alike)
// while an L2 hit runs at ~190 G/s (profiles/r01_baseline/gather_probe.json).
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
// order by the LDS unit -- observed, and checked bit for bit by the tests);
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
    int32_t r[4];
    double v[4];
};

template <bool NT>
__device__ __forceinline__ void css_load(CssChunk &k, int64_t j0, int64_t e1, int lane,
                                         const int32_t *__restrict__ col,
                                         const uint16_t *__restrict__ row,
                                         const double *__restrict__ val) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t j = j0 + u * 64 + lane;
        const bool ok = j < e1;
        if (NT) {
            k.c[u] = ok ? ld_stream(col + j) : 0;
            k.r[u] = ok ? (int32_t)__builtin_nontemporal_load(row + j) : -1;
            k.v[u] = ok ? ld_stream(val + j) : 0.0;
        } else {
            k.c[u] = ok ? col[j] : 0;
            k.r[u] = ok ? (int32_t)row[j] : -1;
            k.v[u] = ok ? val[j] : 0.0;
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(kCssThreads) void css_sweep_kernel(
    const int64_t *__restrict__ bstart, const int64_t *__restrict__ moff,
    const int32_t *__restrict__ merge, int32_t P, int32_t nwg, int32_t S, int32_t slab_shift, int32_t lag,
    const int64_t *__restrict__ woff, const int32_t *__restrict__ col,
    const uint16_t *__restrict__ row, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, uint64_t *__restrict__ prog,
    uint64_t seq, int32_t pace_all, int32_t dbg) {
    __shared__ double ylds[kCssMaxRows];
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
            const int64_t e0 = woff[list];
            const int64_t e1 = woff[list + 1];
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
            CssChunk A, B;
            if (e0 < e1) css_load<NT>(A, e0, e1, lane, col, row, val);
            for (int64_t j0 = e0; j0 < e1; j0 += 256) {
                // slab of the chunk's first entry (wave-uniform: lane 0, u = 0)
                const int s0 = __builtin_amdgcn_readfirstlane(A.c[0]) >> slab_shift;
                if (s0 > cur) enter(s0);
                double g[4];
                if (dbg & 1) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) g[u] = (double)A.c[u];
                } else if (dbg & 16) {  // ablation: every gather inside one 1 MiB window (all L2 hits)
#pragma unroll
                    for (int u = 0; u < 4; ++u) g[u] = ld_x(x, A.c[u] & 0x1FFFF);
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) g[u] = ld_x(x, A.c[u]);
                }
                __builtin_amdgcn_sched_barrier(0);
                // prefetch the next chunk behind the gathers (in-order vmcnt:
                // waiting for the gathers leaves these 12 loads in flight)
                const int64_t j1 = j0 + 256;
                if (j1 < e1) css_load<NT>(B, j1, e1, lane, col, row, val);
                __builtin_amdgcn_sched_barrier(0);
                if (dbg & 2) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) dsink += __dmul_rn(A.v[u], g[u]) * (double)A.r[u];
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (A.r[u] >= 0) atomicAdd(&ylds[A.r[u]], __dmul_rn(A.v[u], g[u]));
                }
                A = B;
            }
            enter(S);  // report every remaining slab
            if ((dbg & 2) && dsink == 1.2345) y[0] = dsink;  // keep ablated work alive
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
        for (int i = threadIdx.x; i < rows; i += kCssThreads) y[row0 + i] = ylds[i];
        __syncthreads();
    }
}

int launch_css(const spmv_plan_s *p, const double *x, double *y) {
    const CssDev &c = p->css;
    if (p->m == 0) return SPMV_SUCCESS;
    spmv_plan_s *mp = const_cast<spmv_plan_s *>(p);
    const uint64_t seq = mp->css.launches++;
    if (c.dbg & 8)  // ablation: default cache policy on the matrix stream
        hipLaunchKernelGGL(css_sweep_kernel<false>, dim3((unsigned)c.nwg), dim3(kCssThreads), 0, p->stream,
                           c.bstart, c.moff, c.merge, c.P, c.nwg, c.S, c.slab_shift, c.lag, c.woff, c.col, c.row, c.val, x, y,
                           c.prog, seq, c.pace_all, c.dbg);
    else
        hipLaunchKernelGGL(css_sweep_kernel<true>, dim3((unsigned)c.nwg), dim3(kCssThreads), 0, p->stream,
                           c.bstart, c.moff, c.merge, c.P, c.nwg, c.S, c.slab_shift, c.lag, c.woff, c.col, c.row, c.val, x, y,
                           c.prog, seq, c.pace_all, c.dbg);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

// k_csr.hip -- CSR SpMV for gfx950: the opt_crs hot loop
// (src/opt_crs.cpp:57-69, `y[i] = sum_j val[j] * x[idx[j]]`) re-designed for
// wave64.
//
// The product kernels: csr_slab2 (near-uniform rows, below) and
// csr_adaptive (rows binned by length).  csr_vec4 is the round-3 kernel whose
// order of arithmetic both keep; the probe build still launches it for A/Bs
// (SPMV_LAUNCH_CSR=0).
//
// csr_vec4<L, RP>: a group of L lanes (L | 64) owns one row.  The group walks
// the row from its 16-byte-aligned start a = ptr[i] & ~3 in chunks of 4*L
// entries; each lane issues ONE 16-byte load of 4 column indices and TWO
// 16-byte loads of 4 values (non-temporal: streamed once), so a wave
// instruction covers 1 KiB contiguous when rows are contiguous.  Entries
// outside [ptr[i], ptr[i+1]) are masked (no gather).  Each lane sums its
// entries in order, then the group reduces with a fixed butterfly; lane 0
// writes y[i] (β = 0, idempotent).
//
// Algorithmic bytes per row: 12*nnz_i + rp bytes + 8 (y) and the
// x gathers (8*n total, counted once).
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

// Values of a row-group plan (CsrDev::val_halves, CsrDev::lanes > 0): every
// aligned 256-entry chunk is laid as ELL's slots -- entries 4t, 4t+1 of the
// chunk at 2t, entries 4t+2, 4t+3 at 128 + 2t -- so the two 16-byte value
// loads of a lane's aligned 4-entry group j (at csr_vpos(j) and 128 later)
// each read whole lines across the wave instead of every other 16 bytes of
// every line (config 4: SS's values the same way, 3.08-3.26 -> 2.59-2.70 ms).
template <typename I>
__device__ __forceinline__ I csr_vpos(I j) {  // j % 4 == 0
    return (j & ~(I)255) + ((j & 255) >> 1);
}

template <int L, typename RP>
__global__ __launch_bounds__(256) void csr_vec4_kernel(int64_t m,
                                                       const RP *__restrict__ rp,
                                                       const int32_t *__restrict__ col,
                                                       const double *__restrict__ val,
                                                       const double *__restrict__ x,
                                                       double *__restrict__ y, bool vh) {
    const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t g = gtid / L;
    const int lane = threadIdx.x & (L - 1);
    if (g >= m) return;  // whole groups exit together (L | 256)
    const int64_t row = g;
    const int64_t s = rp[row];
    const int64_t e = rp[row + 1];
    double acc = 0.0;
    for (int64_t j = (s & ~(int64_t)3) + 4 * lane; j < e; j += 4 * L) {
        const i32x4 c = ld_stream4(col + j);
        const int64_t vj = vh ? csr_vpos(j) : j;
        const f64x2 v01 = ld_stream2(val + vj);
        const f64x2 v23 = ld_stream2(val + vj + (vh ? 128 : 2));
        // masked gathers: only entries of this row
        const double x0 = (j + 0 >= s && j + 0 < e) ? ld_x(x, c.x) : 0.0;
        const double x1 = (j + 1 >= s && j + 1 < e) ? ld_x(x, c.y) : 0.0;
        const double x2 = (j + 2 >= s && j + 2 < e) ? ld_x(x, c.z) : 0.0;
        const double x3 = (j + 3 >= s && j + 3 < e) ? ld_x(x, c.w) : 0.0;
        if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, x0, acc);
        if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, x1, acc);
        if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, x2, acc);
        if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, x3, acc);
    }
    acc = group_sum<L>(acc);
    if (lane == 0) y[row] = acc;
}

// csr_slab2<L, U, O32> (the product CSR kernel for near-uniform rows): one
// wave per slab of 64 consecutive rows, the 64 / L rows of a step summed by
// L-lane groups exactly as csr_vec4<L> sums them (same chunks, same order,
// same butterfly: bit-identical y), U steps' col / val loads issued before
// their gathers.  A long-lived wave replaces 64 / (256 / L) short ones and y
// leaves in one coalesced store per wave (config 4, same plans: csr_vec4<16>
// 2.82 -> 2.48 ms, profiles/round4/probe/c4_csr_slab2_first.jsonl).  No divergent control flow on the
// common path.  Lanes past their row's end load the row's first chunk again (same
// lines, no new traffic) and every loaded column is a real column (plan
// creation validated them; the kPad tail is zero), so the col / val loads
// and the x gathers are unconditional.  When every row of a batch of U steps
// is one aligned chunk of its group (4L entries from a 16-byte boundary:
// configs 2 and 4) the adds run unmasked; otherwise an entry outside [s, e)
// is dropped by a select on its add (one 32-bit compare per entry) -- either
// way the arithmetic of csr_vec4.  Group sums by DPP (group_sum_dpp:
// bit-identical to group_sum), the row sums through a 512-B LDS slab per
// wave, then one coalesced store.  Row pointers are exchanged by ds_bpermute
// as 32-bit values relative to the slab's first entry.  O32 (CsrDev::off32:
// every slab's byte span and x's fit 31 / 32 bits): the col / val loads and
// the x gathers address a wave-uniform base plus a 32-bit byte offset (the
// global_load saddr form: no 64-bit address arithmetic per lane).
template <bool O32>
__device__ __forceinline__ const void *at_bytes(const void *base, int idx, int size) {
    if constexpr (O32) return (const char *)base + (uint32_t)idx * (uint32_t)size;
    else return (const char *)base + (int64_t)idx * size;
}

template <int L, typename RP, int U, bool O32>
__global__ __launch_bounds__(256) void csr_slab2_kernel(int64_t m, const RP *__restrict__ rp,
                                                        const int32_t *__restrict__ col,
                                                        const double *__restrict__ val,
                                                        const double *__restrict__ x, double *__restrict__ y, bool vh) {
    constexpr int R = 64 / L;  // rows per step
    __shared__ double ysl[4][64];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
    const int lane = threadIdx.x & 63;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + wv) * 64;
    if (r0 >= m) return;  // wave-uniform
    const int g = lane / L, gl = lane & (L - 1);
    const int64_t rl = r0 + lane;
    auto ldx = [&](int c) -> double { return *(const double *)at_bytes<O32>(x, c, 8); };
    // the slab's entries [base, end) (a slab of 64 rows holds < 2^31 entries:
    // its offsets are 32-bit)
    const int64_t base = (int64_t)rp[r0] & ~(int64_t)3;
    const int rpl = (int)((int64_t)rp[rl < m ? rl : m] - base);            // lane t: row r0 + t's start
    const int rpe = (int)((int64_t)rp[r0 + 64 < m ? r0 + 64 : m] - base);  // the slab's end
    const int32_t *cb = col + base;
    const int64_t vbase = vh ? base & ~(int64_t)255 : base;
    const double *vb = val + vbase;
    const int vo = (int)(base - vbase), vstep = vh ? 128 : 2;
    auto vpos = [&](int j) -> int { return vh ? csr_vpos(j + vo) : j; };
    for (int st = 0; st < L; st += U) {
        int j0[U], rel[U], len[U];
        bool full = true;
        i32x4 c[U];
        f64x2 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int li = (st + u) * R + g;
            const int s = __shfl(rpl, li, 64);
            const int nx = __shfl(rpl, (li + 1) & 63, 64);
            const int e = li == 63 ? rpe : nx;
            const int a0 = s & ~3;
            j0[u] = a0 + 4 * gl;
            rel[u] = j0[u] - s;
            len[u] = e - s;
            full = full && (s & 3) == 0 && len[u] == 4 * L;
            const int jl = j0[u] < e ? j0[u] : a0;
            c[u] = ld_stream4((const int32_t *)at_bytes<O32>(cb, jl, 4));
            const int vj = vpos(jl);
            a[u] = ld_stream2((const double *)at_bytes<O32>(vb, vj, 8));
            b[u] = ld_stream2((const double *)at_bytes<O32>(vb, vj + vstep, 8));
        }
        double gx[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            gx[u][0] = ldx(c[u].x);
            gx[u][1] = ldx(c[u].y);
            gx[u][2] = ldx(c[u].z);
            gx[u][3] = ldx(c[u].w);
        }
        if (__ballot(!full) == 0) {  // no lane with a partial row: unmasked adds
#pragma unroll
            for (int u = 0; u < U; ++u) {
                double acc = 0.0;
                acc = madd(a[u].x, gx[u][0], acc);
                acc = madd(a[u].y, gx[u][1], acc);
                acc = madd(b[u].x, gx[u][2], acc);
                acc = madd(b[u].y, gx[u][3], acc);
                acc = group_sum_dpp<L>(acc);
                if (gl == 0) ysl[wv][(st + u) * R + g] = acc;
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                double acc = 0.0, t;
                t = madd(a[u].x, gx[u][0], acc);
                acc = (unsigned)(rel[u] + 0) < (unsigned)len[u] ? t : acc;
                t = madd(a[u].y, gx[u][1], acc);
                acc = (unsigned)(rel[u] + 1) < (unsigned)len[u] ? t : acc;
                t = madd(b[u].x, gx[u][2], acc);
                acc = (unsigned)(rel[u] + 2) < (unsigned)len[u] ? t : acc;
                t = madd(b[u].y, gx[u][3], acc);
                acc = (unsigned)(rel[u] + 3) < (unsigned)len[u] ? t : acc;
                // rows longer than one chunk of the group: the rest in order
                const int e = j0[u] - rel[u] + len[u];  // the row's end
                for (int jj = j0[u] + 4 * L; jj < e; jj += 4 * L) {
                    const i32x4 cc = ld_stream4((const int32_t *)at_bytes<O32>(cb, jj, 4));
                    const int vj = vpos(jj);
                    const f64x2 v01 = ld_stream2((const double *)at_bytes<O32>(vb, vj, 8));
                    const f64x2 v23 = ld_stream2((const double *)at_bytes<O32>(vb, vj + vstep, 8));
                    const double x0 = ldx(cc.x), x1 = ldx(cc.y), x2 = ldx(cc.z), x3 = ldx(cc.w);
                    acc = madd(v01.x, x0, acc);
                    t = madd(v01.y, x1, acc);
                    acc = jj + 1 < e ? t : acc;
                    t = madd(v23.x, x2, acc);
                    acc = jj + 2 < e ? t : acc;
                    t = madd(v23.y, x3, acc);
                    acc = jj + 3 < e ? t : acc;
                }
                acc = group_sum_dpp<L>(acc);
                if (gl == 0) ysl[wv][(st + u) * R + g] = acc;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (rl < m) __builtin_nontemporal_store(ysl[wv][lane], y + rl);
}

// csr_slabx<L, U, S, O32>: csr_slab2 for matrices whose rows stay near the
// diagonal (banded, config 4).  A workgroup owns 256 S consecutive rows (each
// wave S consecutive 64-row slabs) and reads x over one column window
// [c0, c0 + win), the union of its S 256-row granules' windows
// (host- or device-computed, CsrDev::win0); it is staged into LDS once, so the x reads are LDS reads
// (lgkmcnt) and no longer share the in-order vmcnt queue with the col / val
// stream -- which lets the stream run one batch ahead: batch i + 1's loads
// (the next slab's first one included) are in flight while batch i's x reads
// and adds run (A / B ping-pong, as BIN's kernels), and the first batch is
// issued before the window is staged.  Same chunks, same order, same
// butterfly as csr_slab2: bit-identical y.  Lanes whose loaded entry lies
// outside the window (masked entries of a neighbouring row) read a clamped,
// in-window slot.
template <int L, int U>
struct CsrBatch {
    i32x4 c[U];
    f64x2 a[U], b[U];
    int s[U], len[U];  // the row's start (relative to the wave's base) and length
    bool full;
};

template <int L, typename RP, int U, int S, bool O32>
__device__ __forceinline__ void csr_slabx_body(int64_t m, const RP *__restrict__ rp, const int32_t *__restrict__ col,
                                               const double *__restrict__ val, const double *__restrict__ x,
                                               double *__restrict__ y, const int32_t *__restrict__ win0, int32_t win,
                                               int64_t n, bool vh, double *xs, double (*ysl)[64]) {
    constexpr int R = 64 / L;   // rows per step
    constexpr int NB = L / U;   // batches per slab
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int g = lane / L, gl = lane & (L - 1);
    // the wave's slabs: rows r0 + 64 k, k < S (r0 >= m: no rows, but the wave
    // still helps stage the window and meets the barrier)
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + wv) * 64 * S;
    const int64_t rbase = r0 < m ? r0 : m;
    const int64_t base = (int64_t)rp[rbase] & ~(int64_t)3;
    int rpl[S], rpe[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int64_t rk = r0 + 64 * k + lane, ek = r0 + 64 * (k + 1);
        rpl[k] = (int)((int64_t)rp[rk < m ? rk : m] - base);
        rpe[k] = (int)((int64_t)rp[ek < m ? ek : m] - base);
    }
    const int32_t *cb = col + base;
    const int64_t vbase = vh ? base & ~(int64_t)255 : base;
    const double *vb = val + vbase;
    const int vo = (int)(base - vbase), vstep = vh ? 128 : 2;
    auto vpos = [&](int j) -> int { return vh ? csr_vpos(j + vo) : j; };
    auto load = [&](CsrBatch<L, U> &B, int i) {  // batch i: slab i / NB, steps (i % NB) U ..
        const int k = i / NB, st = (i % NB) * U;
        B.full = true;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int li = (st + u) * R + g;
            const int s = __shfl(rpl[k], li, 64);
            const int nx = __shfl(rpl[k], (li + 1) & 63, 64);
            const int e = li == 63 ? rpe[k] : nx;
            const int a0 = s & ~3;
            B.s[u] = s;
            B.len[u] = e - s;
            B.full = B.full && (s & 3) == 0 && B.len[u] == 4 * L;
            const int j0 = a0 + 4 * gl;
            const int jl = j0 < e ? j0 : a0;
            B.c[u] = ld_stream4((const int32_t *)at_bytes<O32>(cb, jl, 4));
            const int vj = vpos(jl);
            B.a[u] = ld_stream2((const double *)at_bytes<O32>(vb, vj, 8));
            B.b[u] = ld_stream2((const double *)at_bytes<O32>(vb, vj + vstep, 8));
        }
    };
    // the workgroup's window: the union of its S granules' (win0: per
    // 256-row granule, INT32_MAX when a granule has no entries)
    const int64_t ng = (m + kCsrWinGroup - 1) / kCsrWinGroup;
    int64_t c0 = INT32_MAX;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int64_t gk = (int64_t)blockIdx.x * S + k;
        if (gk < ng) c0 = c0 < win0[gk] ? c0 : (int64_t)win0[gk];
    }
    if (c0 == INT32_MAX) c0 = 0;
    const uint32_t wmax = (uint32_t)win - 1;
    auto xw = [&](int c) -> double {
        const uint32_t i = (uint32_t)((int64_t)c - c0);
        return xs[i < wmax ? i : wmax];
    };
    auto compute = [&](const CsrBatch<L, U> &B, int i) {
        const int k = i / NB, st = (i % NB) * U;
        double gx[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            gx[u][0] = xw(B.c[u].x);
            gx[u][1] = xw(B.c[u].y);
            gx[u][2] = xw(B.c[u].z);
            gx[u][3] = xw(B.c[u].w);
        }
        const bool all_full = __ballot(!B.full) == 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            double acc = 0.0, t;
            if (all_full) {
                acc = madd(B.a[u].x, gx[u][0], acc);
                acc = madd(B.a[u].y, gx[u][1], acc);
                acc = madd(B.b[u].x, gx[u][2], acc);
                acc = madd(B.b[u].y, gx[u][3], acc);
            } else {
                // positions of the lane's 4 entries relative to the row start
                const int a0 = B.s[u] & ~3;
                const int ra = a0 + 4 * gl - B.s[u];
                const int rb = ra + 2;
                t = madd(B.a[u].x, gx[u][0], acc);
                acc = (unsigned)(ra + 0) < (unsigned)B.len[u] ? t : acc;
                t = madd(B.a[u].y, gx[u][1], acc);
                acc = (unsigned)(ra + 1) < (unsigned)B.len[u] ? t : acc;
                t = madd(B.b[u].x, gx[u][2], acc);
                acc = (unsigned)(rb + 0) < (unsigned)B.len[u] ? t : acc;
                t = madd(B.b[u].y, gx[u][3], acc);
                acc = (unsigned)(rb + 1) < (unsigned)B.len[u] ? t : acc;
                const int e = B.s[u] + B.len[u];  // the row's end
                // rows longer than one chunk of the group: the rest in order
                for (int jj = a0 + 4 * gl + 4 * L; jj < e; jj += 4 * L) {
                    const i32x4 cc = ld_stream4((const int32_t *)at_bytes<O32>(cb, jj, 4));
                    const int vj = vpos(jj);
                    const f64x2 v01 = ld_stream2((const double *)at_bytes<O32>(vb, vj, 8));
                    const f64x2 v23 = ld_stream2((const double *)at_bytes<O32>(vb, vj + vstep, 8));
                    const double x0 = xw(cc.x), x1 = xw(cc.y), x2 = xw(cc.z), x3 = xw(cc.w);
                    acc = madd(v01.x, x0, acc);
                    t = madd(v01.y, x1, acc);
                    acc = jj + 1 < e ? t : acc;
                    t = madd(v23.x, x2, acc);
                    acc = jj + 2 < e ? t : acc;
                    t = madd(v23.y, x3, acc);
                    acc = jj + 3 < e ? t : acc;
                }
            }
            acc = group_sum_dpp<L>(acc);
            if (gl == 0) ysl[wv][(st + u) * R + g] = acc;
        }
        if (i % NB == NB - 1) {  // the slab is done: its 64 sums leave in one coalesced store
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int64_t rl = r0 + 64 * k + lane;
            if (rl < m) __builtin_nontemporal_store(ysl[wv][lane], y + rl);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    };
    // the wave's batches: all S slabs while their rows exist
    const int nb = r0 >= m ? 0 : (int)std::min<int64_t>(S, (m - r0 + 63) / 64) * NB;
    CsrBatch<L, U> A, B;
    // window staging: its loads go out first, then the first batch's, so
    // both are in flight together
    constexpr int XT = 4;  // window values per thread held in flight (win <= 256 XT: one pass)
    double t[XT];
#pragma unroll
    for (int q = 0; q < XT; ++q) {
        const int i = threadIdx.x + q * 256;
        t[q] = i < win ? x[c0 + i < n ? c0 + i : n - 1] : 0.0;
    }
    if (nb > 0) load(A, 0);
#pragma unroll
    for (int q = 0; q < XT; ++q) {
        const int i = threadIdx.x + q * 256;
        if (i < win) xs[i] = t[q];
    }
    for (int i = threadIdx.x + XT * 256; i < win; i += 256) xs[i] = x[c0 + i < n ? c0 + i : n - 1];
    __syncthreads();
    for (int i = 0; i < nb; i += 2) {
        if (i + 1 < nb) load(B, i + 1);
        compute(A, i);
        if (i + 1 >= nb) break;
        if (i + 2 < nb) load(A, i + 2);
        compute(B, i + 1);
    }
}

template <int L, typename RP, int U, int S, bool O32>
__global__ __launch_bounds__(256) void csr_slabx_kernel(int64_t m, const RP *__restrict__ rp,
                                                        const int32_t *__restrict__ col,
                                                        const double *__restrict__ val,
                                                        const double *__restrict__ x, double *__restrict__ y,
                                                        const int32_t *__restrict__ win0, int32_t win, int64_t n,
                                                        bool vh) {
    extern __shared__ double xs[];  // [win]
    __shared__ double ysl[4][64];
    csr_slabx_body<L, RP, U, S, O32>(m, rp, col, val, x, y, win0, win, n, vh, xs, ysl);
}

// Adaptive CSR in ONE launch: workgroup ranges map to the length bins
// (blk_off), so all bins run concurrently instead of back to back; the bin
// test is workgroup-uniform (no divergence).  Bin b has L = kCsrBinLanes[b]
// lanes per row; the last bin is one workgroup per row.
struct CsrBinTable {
    int64_t blk_off[kCsrBins + 1];  // first workgroup of each bin, in launch order
    int64_t row_off[kCsrBins + 1];  // first row (in bin_rows) of each bin
};
// launch order: the longest rows first (their workgroups run longest), so
// the short-row bins fill in behind them instead of forming the tail
constexpr int kCsrLaunchOrder[kCsrBins] = {7, 6, 5, 4, 3, 2, 1, 0};

// ADD: y[yrow[row]] += sum (the HYB/JDS overflow, one writer per row);
// otherwise y[row] = sum
template <int L, typename RP, bool ADD>
__device__ __forceinline__ void csr_rows_body(int64_t wg, int64_t nrows, const int32_t *__restrict__ rows,
                                              const RP *__restrict__ rp, const int32_t *__restrict__ col,
                                              const double *__restrict__ val, const double *__restrict__ x,
                                              double *__restrict__ y, const int32_t *__restrict__ yrow) {
    const int64_t g = (wg * 256 + threadIdx.x) / L;
    const int lane = threadIdx.x & (L - 1);
    if (g >= nrows) return;
    const int64_t row = rows[g];
    const int64_t s = rp[row];
    const int64_t e = rp[row + 1];
    double acc = 0.0;
    for (int64_t j = (s & ~(int64_t)3) + 4 * lane; j < e; j += 4 * L) {
        const i32x4 c = ld_stream4(col + j);
        const f64x2 v01 = ld_stream2(val + j);
        const f64x2 v23 = ld_stream2(val + j + 2);
        const double x0 = (j + 0 >= s && j + 0 < e) ? ld_x(x, c.x) : 0.0;
        const double x1 = (j + 1 >= s && j + 1 < e) ? ld_x(x, c.y) : 0.0;
        const double x2 = (j + 2 >= s && j + 2 < e) ? ld_x(x, c.z) : 0.0;
        const double x3 = (j + 3 >= s && j + 3 < e) ? ld_x(x, c.w) : 0.0;
        if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, x0, acc);
        if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, x1, acc);
        if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, x2, acc);
        if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, x3, acc);
    }
    acc = group_sum<L>(acc);
    if (lane == 0) {
        if (ADD) {
            const int64_t yi = yrow[row];
            y[yi] = __dadd_rn(y[yi], acc);
        } else {
            y[row] = acc;
        }
    }
}

template <typename RP, bool ADD>
__global__ __launch_bounds__(256) void csr_adaptive_kernel(CsrBinTable t, const int32_t *__restrict__ rows,
                                                           const RP *__restrict__ rp,
                                                           const int32_t *__restrict__ col,
                                                           const double *__restrict__ val,
                                                           const double *__restrict__ x, double *__restrict__ y,
                                                           const int32_t *__restrict__ yrow) {
    __shared__ double part[4];
    const int64_t blk = blockIdx.x;
    int k = 0;
    while (k < kCsrBins - 1 && blk >= t.blk_off[k + 1]) ++k;  // uniform
    const int b = kCsrLaunchOrder[k];
    const int64_t wg = blk - t.blk_off[k];
    const int32_t *br = rows + t.row_off[b];
    const int64_t n = t.row_off[b + 1] - t.row_off[b];
    switch (b) {
        case 0: csr_rows_body<1, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 1: csr_rows_body<2, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 2: csr_rows_body<4, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 3: csr_rows_body<8, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 4: csr_rows_body<16, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 5: csr_rows_body<32, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        case 6: csr_rows_body<64, RP, ADD>(wg, n, br, rp, col, val, x, y, yrow); break;
        default: {
            // one workgroup per row: four wave sums added in wave order
            const int64_t row = br[wg];
            const int64_t s = rp[row];
            const int64_t e = rp[row + 1];
            double acc = 0.0;
            for (int64_t j = (s & ~(int64_t)3) + 4 * threadIdx.x; j < e; j += 4 * 256) {
                const i32x4 c = ld_stream4(col + j);
                const f64x2 v01 = ld_stream2(val + j);
                const f64x2 v23 = ld_stream2(val + j + 2);
                if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, ld_x(x, c.x), acc);
                if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, ld_x(x, c.y), acc);
                if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, ld_x(x, c.z), acc);
                if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, ld_x(x, c.w), acc);
            }
            acc = group_sum<64>(acc);
            if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
            __syncthreads();
            if (threadIdx.x == 0) {
                const double sum = __dadd_rn(__dadd_rn(part[0], part[1]), __dadd_rn(part[2], part[3]));
                if (ADD) {
                    const int64_t yi = yrow[row];
                    y[yi] = __dadd_rn(y[yi], sum);
                } else {
                    y[row] = sum;
                }
            }
        }
    }
}

// one launch of the adaptive kernel over length bins (bin_off: host offsets)
template <typename RP, bool ADD>
static int launch_adaptive(const spmv_plan_s *p, const int64_t *bin_off, const int32_t *bin_rows, const RP *rp,
                           const int32_t *col, const double *val, const double *x, double *y,
                           const int32_t *yrow) {
    CsrBinTable t;
    t.blk_off[0] = 0;
    for (int b = 0; b <= kCsrBins; ++b) t.row_off[b] = bin_off[b];
    for (int k = 0; k < kCsrBins; ++k) {
        const int b = kCsrLaunchOrder[k];
        const int64_t n = bin_off[b + 1] - bin_off[b];
        const int L = kCsrBinLanes[b];
        t.blk_off[k + 1] = t.blk_off[k] + (L >= 256 ? n : (n * L + 255) / 256);
    }
    if (t.blk_off[kCsrBins] == 0) return SPMV_SUCCESS;
    hipLaunchKernelGGL((csr_adaptive_kernel<RP, ADD>), dim3((unsigned)t.blk_off[kCsrBins]), dim3(256), 0, p->stream,
                       t, bin_rows, rp, col, val, x, y, yrow);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

// launch-time shape of the row-parallel CSR kernels: csr_slabx where the plan
// has x windows (banded rows), else csr_slab2, with U = min(4, L) steps per
// batch.  Config 4 (16 lanes), same plans: csr_vec4 2.80-2.87, csr_slab2 U =
// 1 / 2 / 4 / 8 2.64 / 2.55 / 2.49 / 2.54 ms, csr_slabx U = 4 2.41-2.54 ms
// against csr_slab2's 2.54-2.62 on the same plans; config 2 (gather-bound)
// within 1 % (profiles/round4/probe/c4_csr_slab2_first.jsonl,
// c4_csr_slabx_s1.jsonl, c4_csr_slabx_pairs.jsonl, c2_csr_slab2_slabx.jsonl).
// The probe build reads SPMV_LAUNCH_CSR (0: csr_vec4, the round-3 kernel; 2:
// csr_slab2), SPMV_LAUNCH_CSR_U and SPMV_LAUNCH_CSR_LDS_KB at every launch, so
// variants are A/B'd on one plan's memory.
struct CsrLaunch {
    int slab = 3;    // 3: csr_slabx where the plan has x windows, else csr_slab2; 2: csr_slab2;
                     // 0: csr_vec4 (probe A/B)
    int u = 4;       // slab: steps whose loads are issued together
    size_t lds = 0;  // dynamic LDS per workgroup (caps workgroups per CU; probe)
};
#ifdef SPMV_PROBES
static CsrLaunch csr_launch_shape() {
    CsrLaunch s;
    if (const char *e = probe_env("SPMV_LAUNCH_CSR")) s.slab = std::atoi(e);
    if (const char *e = probe_env("SPMV_LAUNCH_CSR_U")) s.u = std::atoi(e);
    if (const char *e = probe_env("SPMV_LAUNCH_CSR_LDS_KB")) s.lds = (size_t)std::atoi(e) * 1024;
    return s;
}
#endif

template <int L, typename RP, int U>
static void launch_slab_u(const spmv_plan_s *p, int kind, size_t lds, const double *x, double *y) {
    constexpr int UU = U < L ? U : L;
    const int64_t waves = (p->m + 63) / 64;
    const CsrDev &c = p->csr;
    if (kind >= 3 && c.win0) {  // x window in LDS, stream one batch ahead
        // S granules (64-row slabs per wave) per workgroup: kCsrSlabsPerWave;
        // probe build: SPMV_LAUNCH_CSR_S = 1, 2 or 4 where that window fits
        int S = kCsrSlabsPerWave;
#ifdef SPMV_PROBES
        if (const char *e = probe_env("SPMV_LAUNCH_CSR_S")) S = std::atoi(e);
        if (!c.win_s[S == 4 ? 2 : S == 1 ? 0 : 1]) S = kCsrSlabsPerWave;
#endif
        const int32_t win = c.win_s[S == 4 ? 2 : S == 1 ? 0 : 1];
        const size_t wl = std::max(lds, sizeof(double) * (size_t)win);
        const unsigned grid = (unsigned)((p->m + 256 * S - 1) / (256 * S));
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), wl, p->stream, p->m, (const RP *)c.row_ptr, c.col, c.val,
                               x, y, c.win0, win, p->n, c.val_halves);
        };
        // 32-bit offsets span the wave's S slabs (off32 is per single slab)
        auto go_s = [&](auto sc) {
            constexpr int SS = decltype(sc)::value;
            if (c.off32 && (SS == 1 || (int64_t)SS * c.slab_max + 512 < ((int64_t)1 << 28)))
                go(csr_slabx_kernel<L, RP, UU, SS, true>);
            else
                go(csr_slabx_kernel<L, RP, UU, SS, false>);
        };
#ifdef SPMV_PROBES
        if (S == 1) go_s(std::integral_constant<int, 1>{});
        else if (S == 4) go_s(std::integral_constant<int, 4>{});
        else go_s(std::integral_constant<int, 2>{});
#else
        go_s(std::integral_constant<int, kCsrSlabsPerWave>{});
#endif
        return;
    }
    if (p->csr.off32)
        hipLaunchKernelGGL((csr_slab2_kernel<L, RP, UU, true>), dim3((unsigned)((waves + 3) / 4)), dim3(256), lds,
                           p->stream, p->m, (const RP *)p->csr.row_ptr, p->csr.col, p->csr.val, x, y, c.val_halves);
    else
        hipLaunchKernelGGL((csr_slab2_kernel<L, RP, UU, false>), dim3((unsigned)((waves + 3) / 4)), dim3(256), lds,
                           p->stream, p->m, (const RP *)p->csr.row_ptr, p->csr.col, p->csr.val, x, y, c.val_halves);
}

// The product instantiates only the default shape (CsrLaunch{}: slab 3, U =
// 4, S = kCsrSlabsPerWave); the probe build adds csr_vec4 and U / S / LDS
// variants, read at every launch.
template <int L, typename RP>
static int launch_csr_t(const spmv_plan_s *p, int64_t nrows, const double *x, double *y) {
    const int64_t threads = nrows * L;
    const int64_t blocks = (threads + 255) / 256;
    if (blocks == 0) return SPMV_SUCCESS;
#ifdef SPMV_PROBES
    const CsrLaunch sh = csr_launch_shape();
    if (sh.slab) {
        switch (sh.u) {
            case 1: launch_slab_u<L, RP, 1>(p, sh.slab, sh.lds, x, y); break;
            case 2: launch_slab_u<L, RP, 2>(p, sh.slab, sh.lds, x, y); break;
            case 8: launch_slab_u<L, RP, 8>(p, sh.slab, sh.lds, x, y); break;
            default: launch_slab_u<L, RP, 4>(p, sh.slab, sh.lds, x, y);
        }
    } else {
        hipLaunchKernelGGL((csr_vec4_kernel<L, RP>), dim3((unsigned)blocks), dim3(256), sh.lds, p->stream, nrows,
                           (const RP *)p->csr.row_ptr, p->csr.col, p->csr.val, x, y, p->csr.val_halves);
    }
#else
    constexpr CsrLaunch sh{};
    launch_slab_u<L, RP, sh.u>(p, sh.slab, sh.lds, x, y);
#endif
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

template <typename RP>
static int launch_csr_lanes(const spmv_plan_s *p, int lanes, int64_t nrows, const double *x, double *y) {
    switch (lanes) {
        case 1: return launch_csr_t<1, RP>(p, nrows, x, y);
        case 2: return launch_csr_t<2, RP>(p, nrows, x, y);
        case 4: return launch_csr_t<4, RP>(p, nrows, x, y);
        case 8: return launch_csr_t<8, RP>(p, nrows, x, y);
        case 16: return launch_csr_t<16, RP>(p, nrows, x, y);
        case 32: return launch_csr_t<32, RP>(p, nrows, x, y);
        case 64: return launch_csr_t<64, RP>(p, nrows, x, y);
        default: set_error("csr lanes must be a power of two in [1,64]"); return SPMV_ERROR_INVALID_VALUE;
    }
}

template <typename RP>
static int launch_csr_rp(const spmv_plan_s *p, const double *x, double *y) {
    const CsrDev &c = p->csr;
    if (!c.bin_rows) return launch_csr_lanes<RP>(p, c.lanes, p->m, x, y);
    // adaptive: every bin in one launch (workgroup ranges per bin)
    return launch_adaptive<RP, false>(p, c.bin_off, c.bin_rows, (const RP *)c.row_ptr, c.col, c.val, x, y, nullptr);
}

int launch_csr(const spmv_plan_s *p, const double *x, double *y) {
    if (p->nnz == 0) {  // no entries: y = 0 without touching x (x may be NULL when n == 0)
        if (p->m) SPMV_HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * (size_t)p->m, p->stream));
        return SPMV_SUCCESS;
    }
    return p->csr.rp64 ? launch_csr_rp<int64_t>(p, x, y) : launch_csr_rp<int32_t>(p, x, y);
}

// ---- HYB overflow: CSR-vector over the overflow rows, y[row] += sum -------
template <int L>
__global__ __launch_bounds__(256) void hyb_overflow_kernel(int64_t nrows, const int32_t *__restrict__ rows,
                                                           const int64_t *__restrict__ rp,
                                                           const int32_t *__restrict__ col,
                                                           const double *__restrict__ val,
                                                           const double *__restrict__ x,
                                                           double *__restrict__ y) {
    const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = gtid / L;
    const int lane = threadIdx.x & (L - 1);
    if (r >= nrows) return;
    const int64_t s = rp[r];
    const int64_t e = rp[r + 1];
    double acc = 0.0;
    for (int64_t j = (s & ~(int64_t)3) + 4 * lane; j < e; j += 4 * L) {
        const i32x4 c = ld_stream4(col + j);
        const f64x2 v01 = ld_stream2(val + j);
        const f64x2 v23 = ld_stream2(val + j + 2);
        if (j + 0 >= s && j + 0 < e) acc = madd(v01.x, ld_x(x, c.x), acc);
        if (j + 1 >= s && j + 1 < e) acc = madd(v01.y, ld_x(x, c.y), acc);
        if (j + 2 >= s && j + 2 < e) acc = madd(v23.x, ld_x(x, c.z), acc);
        if (j + 3 >= s && j + 3 < e) acc = madd(v23.y, ld_x(x, c.w), acc);
    }
    acc = group_sum<L>(acc);
    if (lane == 0) {
        const int32_t row = rows[r];
        y[row] = __dadd_rn(y[row], acc);  // single writer per row
    }
}

int launch_hyb_overflow(const spmv_plan_s *p, const double *x, double *y) {
    const HybDev &h = p->hyb;
    if (h.n_rows == 0) return SPMV_SUCCESS;
    if (h.bin_rows)  // overflow rows binned by their overflow length
        return launch_adaptive<int64_t, true>(p, h.bin_off, h.bin_rows, h.row_ptr, h.col, h.val, x, y, h.rows);
    const int L = 64;
    const int64_t blocks = (h.n_rows * L + 255) / 256;
    hipLaunchKernelGGL((hyb_overflow_kernel<64>), dim3((unsigned)blocks), dim3(256), 0, p->stream,
                       h.n_rows, h.rows, h.row_ptr, h.col, h.val, x, y);
    SPMV_HIP_TRY(hipGetLastError());
    return SPMV_SUCCESS;
}

}  // namespace spmv

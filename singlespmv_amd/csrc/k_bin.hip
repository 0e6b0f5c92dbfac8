// k_bin.hip -- binned two-phase Mul/Sum SpMV ("BIN") for gfx950.
//
// Lineage: opt_ss splits SpMV into Mul (val_buf[i] = val[i] * x[col[i]],
// src/opt_ss.cpp:225-239) and Sum (per-row reduction of val_buf,
// src/opt_ss.cpp:241-303); opt_css cuts the columns into blocks so the x block
// stays cache resident (src/opt_css.cpp:33-45).  Re-designed for MI355X, where
// a random 8-byte gather costs one L1 line request (~0.9 G/s per CU even when
// it hits L2, profiles/round1/probe/gather_probe.json) but an LDS read of the
// same value costs a few clocks:
//
//  * Mul (bin_mul_kernel): a workgroup walks its nnz-balanced range of the
//    Mul-ordered entry stream strip by strip.  Per strip it stages the
//    x strip (<= kBinMaxStrip columns) in LDS, then every entry gathers x from LDS and
//    writes its product to the product buffer at the entry's place in Sum
//    order.  The entry stream is ordered [strip][bin][k-th entry, row] and
//    padded per (strip, bin) segment to 16 entries (8 when segments are
//    short), so 16 (8) consecutive lanes write one aligned 128-byte (64-byte)
//    product line;
//  * Sum (bin_sum_kernel): one wave per bin (<= bin_max_rows(W2) rows)
//    streams the bin's products -- contiguous, ordered [strip][k, row] -- and
//    adds them with ds_add_f64 into its own LDS y slice, then writes the
//    bin's y rows; each wave walks all of its bins with one batch cursor.
//  * Mul order (BinDev::mo, the wide multi-GPU rank shapes whose segments
//    are short): the Mul writes entry e's product to prod[e] instead, and
//    bin_sum_bin_kernel gathers each bin's Sum order back in 8-entry chunks
//    through a chunk table (same add order, same y; DESIGN §3.5, profiles/round3/README.md §4c).
//
// HBM bytes per nnz: Mul 8 (val) + 2 (column in strip) + 0.25-0.5
// (destination) + 8 (product), Sum 8 (product) + 2 (row in bin): ~28.5 B,
// streamed and fully coalesced, against 12 B + an uncoalesced gather for
// row-parallel kernels (profiles/round1/README.md §4a: the Infinity Cache gives the product
// round trip no re-read benefit, so row groups (G > 1) only bound the buffer).
//
// Determinism / exactness: a bin is owned by one wave, which adds its
// products in Sum order = column order within each row (strips ascending,
// columns ascending within a segment); lanes of one ds_add_f64 that hit the
// same slot are applied in lane order (as k_css.hip relies on) -- the named
// guard of that hardware behaviour is tests/test_gpu_parity.py::
// test_lds_add_lane_order (one ds_add_f64 on order-sensitive values), and
// tests/test_guards.py checks that these adds compile to ds_add_f64 with no
// CAS loop; slots start at +0.0 and products are rounded multiplies,
// so every row is the sequential opt_crs sum (src/opt_crs.cpp:61-66) bit for
// bit, and repeated calls are identical.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {

// One batch of U entries per lane (entry base + u*64 + lane), loaded ahead
// of its use: the kernels ping-pong two batches so a wave always has one
// batch of loads in flight while it consumes the other (the single-batch
// loop drained the memory pipe every iteration: BIN lost 25 % on 160 CUs
// instead of 256, profiles/round1/probe/bin_cus.jsonl).
typedef uint32_t bin_u32x4 __attribute__((ext_vector_type(4)));

template <int U>
struct MulBatch {
    double v[U];
    uint32_t c[U];
    int32_t d[U];
};

// MODE bits of the Mul (all give the same y): 1 nontemporal product stores
// (Sum-ordered products), 4 products in Mul order (BinDev::mo: prod[e], no
// destinations), 256 x strips by LDS-DMA.  PL: segments padded to 2^PL
// entries.  LONG: blocks at or past `ls` (the strip's long blocks,
// 64-aligned) load their lcode word instead of the segment destination.
template <int U, int PL, int MODE, bool LONG>
__device__ __forceinline__ void mul_load(MulBatch<U> &B, int64_t base, int64_t e0, int64_t e1, int lane,
                                         const double *__restrict__ val1, const uint16_t *__restrict__ cs1,
                                         const int32_t *__restrict__ dst1, int64_t ls, int64_t lsh,
                                         const int32_t *__restrict__ lcode) {
    if constexpr (!LONG) {
        // lanes past the piece load the next entries unclamped (the arrays
        // carry kBinMulSlack; their stores are masked): one base address per
        // array, the u offsets are immediates (64 entries = 64 >> PL groups).
        // (With long blocks the extra live addresses spill: clamped below.)
        const double *vb = val1 + base + lane;
        const uint16_t *cb = cs1 + base + lane;
        const int32_t *db = dst1 + ((base + lane) >> PL);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            B.v[u] = ld_stream(vb + u * 64);
            B.c[u] = (uint32_t)__builtin_nontemporal_load(cb + u * 64);
            if constexpr ((MODE & 4) == 0) B.d[u] = ld_stream(db + u * (64 >> PL));
        }
        (void)e0;
        (void)e1;
        (void)ls;
        (void)lsh;
        (void)lcode;
        (void)db;
    } else {  // every load clamped at the piece's end
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * 64 + lane;
            const int64_t ee = e < e1 ? e : e0;
            B.v[u] = ld_stream(val1 + ee);
            B.c[u] = (uint32_t)__builtin_nontemporal_load(cs1 + ee);
            // a lane past the piece (e >= e1, masked at the store) reads word 0:
            // its e may lie beyond the strip's long blocks
            if (base + u * 64 >= ls) B.d[u] = ld_stream(lcode + (e < e1 ? e + lsh : 0));
            else if constexpr ((MODE & 4) == 0) B.d[u] = ld_stream(dst1 + (ee >> PL));
        }
    }
}

// One 64-entry long block: inclusive segmented scan of the products over the
// lanes (pieces start where lcode's bit 31 is set), then the last lane of
// every piece writes its partial.  The scan is a fixed DPP tree -- row_shr
// 1/2/4/8 inside each 16-lane row, then row_bcast15 (rows 1, 3) and
// row_bcast31 (rows 2, 3) -- so a partial is deterministic; a lane adds a
// source only from its own piece (source lane >= the piece's first lane).
__device__ __forceinline__ void mul_long_block(double pr, int32_t code, bool ok, int lane,
                                               double *__restrict__ prod) {
    const bool start = code < 0 || !ok;
    const uint64_t starts = __ballot(start);
    const uint64_t upto = starts & (~0ull >> (63 - lane));
    const int seg = 63 - __clzll((long long)upto);
    const int r16 = lane & 15, row = lane >> 4;
    double v = ok ? pr : 0.0, t;
    t = dpp_f64<0x111, 0xF>(v);  // row_shr:1
    if (r16 >= 1 && lane - 1 >= seg) v = __dadd_rn(t, v);
    t = dpp_f64<0x112, 0xF>(v);  // row_shr:2
    if (r16 >= 2 && lane - 2 >= seg) v = __dadd_rn(t, v);
    t = dpp_f64<0x114, 0xF>(v);  // row_shr:4
    if (r16 >= 4 && lane - 4 >= seg) v = __dadd_rn(t, v);
    t = dpp_f64<0x118, 0xF>(v);  // row_shr:8
    if (r16 >= 8 && lane - 8 >= seg) v = __dadd_rn(t, v);
    t = dpp_f64<0x142, 0xA>(v);  // row_bcast:15 -> rows 1 and 3
    if ((row & 1) && seg <= row * 16 - 1) v = __dadd_rn(t, v);
    t = dpp_f64<0x143, 0xC>(v);  // row_bcast:31 -> rows 2 and 3
    if (row >= 2 && seg <= 31) v = __dadd_rn(t, v);
    const int32_t pos = code & 0x7FFFFFFF;
    // Plain stores: a piece's 8-byte partial shares its 128-B line with the
    // neighbouring pieces of its (bin, strip), written by the next lanes or
    // the next block -- kept in L2 they merge into whole lines.  Nontemporal
    // partial stores cost the Mul that follows a Sum 0.111 -> 0.137 ms at
    // config 3 (profiles/round2/probe/c3_long_store.jsonl).
    if (ok && pos != 0x7FFFFFFF) prod[pos] = v;
}

template <int U, int MODE, int PL, bool LONG>
__device__ __forceinline__ void mul_store(const MulBatch<U> &B, int64_t base, int64_t e1, int lane,
                                          const double *xs, double *__restrict__ prod, int64_t ls) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t e = base + u * 64 + lane;
        if (LONG && base + u * 64 >= ls) {
            mul_long_block(__dmul_rn(B.v[u], xs[B.c[u]]), B.d[u], e < e1, lane, prod);
        } else if (e < e1) {
            const double pr = __dmul_rn(B.v[u], xs[B.c[u]]);
            // MODE 4: products in Mul order (BinDev::mo: contiguous, no
            // destinations) instead of the Sum order's segments
            double *dp = (MODE & 4) ? prod + e : prod + ((int64_t)B.d[u] << PL) + (e & ((1 << PL) - 1));
            if (MODE & 1) __builtin_nontemporal_store(pr, dp);
            else *dp = pr;
        }
    }
}

template <int U, int MODE, int PL, bool LONG>
__global__ __launch_bounds__(kBinMulThreads) void bin_mul_kernel(
    const int64_t *__restrict__ piece_off, int64_t q_base, const int32_t *__restrict__ piece_strip,
    const int64_t *__restrict__ piece_begin, const int64_t *__restrict__ piece_end,
    const double *__restrict__ val1, const uint16_t *__restrict__ cs1, const int32_t *__restrict__ dst1,
    const double *__restrict__ x, int64_t n, int32_t strip, double *__restrict__ prod,
    const int64_t *__restrict__ lstart, const int64_t *__restrict__ lshift, const int32_t *__restrict__ lcode,
    int32_t xburst) {
    __shared__ double xs[kBinMaxStrip];
    constexpr int NW = kBinMulThreads / 64;
    constexpr int64_t STEP = (int64_t)NW * 64 * U;
    // the wave index as a wave-uniform (SGPR) value: the compiler cannot
    // prove threadIdx.x >> 6 uniform, and the cursor's table loads then
    // become vector loads whose s_waitcnt vmcnt(0) drains the batch in flight
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t q0 = piece_off[q_base + blockIdx.x], q1 = piece_off[q_base + blockIdx.x + 1];
    for (int64_t q = q0; q < q1; ++q) {
        // consecutive pieces of a workgroup are consecutive strips: stage x
        const int32_t st = piece_strip[q];
        const int64_t c0 = (int64_t)st * strip;
        const int64_t e0 = piece_begin[q], e1 = piece_end[q];
        const int64_t ls = LONG ? lstart[st] : INT64_MAX, lsh = LONG ? lshift[st] : 0;
        const int cw = (int)(n - c0 < strip ? n - c0 : strip);
        __syncthreads();  // the previous strip's readers are done
        // xburst (wide shapes, build_bin.cpp): XL loads in flight per thread
        // before their LDS writes (3 round trips for a 20480-column strip
        // instead of 20); else, and always with long rows (their run path's
        // live registers would spill), one load per round trip
        constexpr int XL = 8;
        if constexpr ((MODE & 256) != 0) {
            // LDS-DMA (global_load_lds_dwordx4): each wave instruction copies
            // 1 KB of x straight into the strip, no VGPRs, all in flight at
            // once; the launch checks that x + c0 is 16-byte aligned.  The
            // tail past whole KB: plain loads.
            const int full = cw & ~127;
            for (int k = w; k * 128 < full; k += NW)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(x + c0 + k * 128 + lane * 2),
                    (__attribute__((address_space(3))) void *)(xs + k * 128), 16, 0, 0);
            for (int i = full + threadIdx.x; i < cw; i += kBinMulThreads) xs[i] = x[c0 + i];
            // other waves read these LDS bytes after the barrier: every DMA
            // load of this wave must have landed first (vmcnt(0); expcnt and
            // lgkmcnt left at their maxima), whatever the compiler's barrier
            // lowering does (the CK block_sync_lds_direct_load idiom)
            __builtin_amdgcn_s_waitcnt(0x0F70);
        } else if (LONG || !xburst) {
            for (int i = threadIdx.x; i < cw; i += kBinMulThreads) xs[i] = x[c0 + i];
        } else for (int i0 = threadIdx.x; i0 < cw; i0 += XL * kBinMulThreads) {
            double t[XL];
#pragma unroll
            for (int k = 0; k < XL; ++k) {
                const int i = i0 + k * kBinMulThreads;
                t[k] = i < cw ? x[c0 + i] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < XL; ++k) {
                const int i = i0 + k * kBinMulThreads;
                if (i < cw) xs[i] = t[k];
            }
        }
        __syncthreads();
        const int64_t first = e0 + (int64_t)w * 64 * U;
        const int64_t nit = first < e1 ? (e1 - first + STEP - 1) / STEP : 0;
        auto bat = [&](int64_t j) { return first + j * STEP; };
        MulBatch<U> A, B;
        if (nit > 0) mul_load<U, PL, MODE, LONG>(A, bat(0), e0, e1, lane, val1, cs1, dst1, ls, lsh, lcode);
        for (int64_t it = 0; it < nit; it += 2) {
            const int64_t ba = bat(it), bb = bat(it + 1);
            if (it + 1 < nit) mul_load<U, PL, MODE, LONG>(B, bb, e0, e1, lane, val1, cs1, dst1, ls, lsh, lcode);
            mul_store<U, MODE, PL, LONG>(A, ba, e1, lane, xs, prod, ls);
            if (it + 1 < nit) {
                if (it + 2 < nit)
                    mul_load<U, PL, MODE, LONG>(A, bat(it + 2), e0, e1, lane, val1, cs1, dst1, ls, lsh, lcode);
                mul_store<U, MODE, PL, LONG>(B, bb, e1, lane, xs, prod, ls);
            }
        }
    }
}

// two 16-bit row slots per word, unpacked at the add
template <int U>
struct SumBatch {
    double v[U];
    uint32_t w[U / 2];
    __device__ __forceinline__ uint32_t slot(int u) const { return (w[u >> 1] >> (16 * (u & 1))) & 0xFFFFu; }
};

// sbase: the batch's slot block (bin_slot_index): this lane's slots u..u+7
// are one 16-byte word, the wave's word q one contiguous KB.  The whole batch
// is loaded unclamped: lanes past the run's end read the next run's products
// (or the buffer's slack, kBinProdSlack) and their slots -- the padding of
// the batch's slot block -- are the dummy slot, so nothing but +x reaches a
// real row.  One base address, the u offsets are immediates: no per-entry
// clamp or 64-bit address math.  Products nontemporal (config 2 Sum 0.308 ->
// 0.298 ms, neutral at config 3 and the N = 8 shape,
// profiles/round1/probe/bin_sum_nt_loads.jsonl).
template <int U>
__device__ __forceinline__ void sum_load(SumBatch<U> &B, int64_t base, int lane, int64_t pbase, int64_t sbase,
                                         const uint16_t *__restrict__ slot2, const double *__restrict__ prod) {
    static_assert(U % 8 == 0, "slots are read 8 per 16-byte load");
    // slots first: the adds consume slot word q before product u >= 8q, and
    // loads complete in issue order
    const bin_u32x4 *sp = reinterpret_cast<const bin_u32x4 *>(slot2 + sbase + (int64_t)lane * 8);
#pragma unroll
    for (int q = 0; q < U / 8; ++q) {
        const bin_u32x4 w = __builtin_nontemporal_load(sp + q * 64);
#pragma unroll
        for (int h = 0; h < 4; ++h) B.w[4 * q + h] = w[h];
    }
    const double *pp = prod + (base - pbase) + lane;
#pragma unroll
    for (int u = 0; u < U; ++u) B.v[u] = ld_stream(pp + u * 64);
}

template <int U>
__device__ __forceinline__ void sum_add(const SumBatch<U> &B, double *ys) {
#pragma unroll
    for (int u = 0; u < U; ++u) atomicAdd(&ys[B.slot(u)], B.v[u]);  // past the run: the dummy slot
}

// The Sum of Sum-ordered products.  W2 waves per workgroup, each owning a
// slice of kBinLdsDoubles / W2 doubles.  A bin's products are NBK runs (one
// per strip block, run_off[blk*nbins + b]); the batches walk them in order
// (a batch never crosses a run), ping-ponged so one batch is always in
// flight -- across the wave's bins too: the next bin's first batches are
// already loading while the finished bin's y is written from LDS (its
// write-back and the loads overlap instead of alternating).  y leaves with
// nontemporal stores (not re-read by the kernel: config 2 Sum 0.302 -> 0.292
// ms, N = 8 shape 0.318 -> 0.308, profiles/round2/probe/sum_nt_y_*.jsonl).
template <int W2, int U>
__global__ __launch_bounds__(64 * W2) void bin_sum_kernel(
    int64_t b0, int64_t b1, int64_t nbins, int64_t nblk, const int64_t *__restrict__ run_off,
    const int64_t *__restrict__ srun_off, const int32_t *__restrict__ bin_row0, int64_t pbase,
    const uint16_t *__restrict__ slot2,
    const double *__restrict__ prod, double *__restrict__ y) {
    constexpr int SLICE = kBinLdsDoubles / W2;
    constexpr int64_t STEP = 64 * U;
    __shared__ double ylds[kBinLdsDoubles];
    // the wave index as a wave-uniform (SGPR) value: the compiler cannot
    // prove threadIdx.x >> 6 uniform, and the cursor's table loads then
    // become vector loads whose s_waitcnt vmcnt(0) drains the batch in flight
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    double *ys = ylds + w * SLICE;
    const int64_t bfirst = b0 + (int64_t)blockIdx.x * W2 + w, bstride = (int64_t)gridDim.x * W2;
    if (bfirst >= b1) return;
    // one cursor over all of the wave's bins: bin cb, its run k, the
    // batch [pos, min(pos + STEP, end)); products from rs, slots from ss
    int64_t cb = bfirst, k = 0, pos = run_off[cb], end = run_off[cb + 1], rs = pos, ss = srun_off[cb];
    auto next = [&](int64_t &lo, int64_t &sb, int64_t &bb) -> bool {
        while (pos >= end) {
            if (++k >= nblk) {  // bin cb exhausted: the wave's next bin
                cb += bstride;
                if (cb >= b1) return false;
                k = 0;
                pos = rs = run_off[cb];
                end = run_off[cb + 1];
                ss = srun_off[cb];
                continue;
            }
            pos = rs = run_off[k * nbins + cb];
            end = run_off[k * nbins + cb + 1];
            ss = srun_off[k * nbins + cb];
        }
        lo = pos;
        sb = ss + (lo - rs);
        bb = cb;
        pos = pos + STEP < end ? pos + STEP : end;
        return true;
    };
    // acc: the bin in the LDS slice; done: the wave's first bin whose y
    // is not written yet (bins without products get zeros)
    int64_t acc = -1, done = bfirst;
    auto write_zero = [&](int64_t bz) {
        const int64_t r0 = bin_row0[bz];
        const int rows = (int)(bin_row0[bz + 1] - r0);
        for (int i = lane; i < rows; i += 64) __builtin_nontemporal_store(0.0, y + r0 + i);
    };
    auto finish = [&]() {  // the slice's bin: LDS adds done -> y
        const int64_t r0 = bin_row0[acc];
        const int rows = (int)(bin_row0[acc + 1] - r0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (int i = lane; i < rows; i += 64) __builtin_nontemporal_store(ys[i], y + r0 + i);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        done = acc + bstride;
    };
    auto begin = [&](int64_t nb) {  // the next batch belongs to bin nb
        if (nb == acc) return;
        if (acc >= 0) finish();
        for (; done < nb; done += bstride) write_zero(done);
        const int rows = (int)(bin_row0[nb + 1] - bin_row0[nb]);
        for (int i = lane; i < rows; i += 64) ys[i] = 0.0;
        acc = nb;
        done = nb + bstride;
    };
    SumBatch<U> A, B;
    int64_t alo, asb, ab, blo, bsb, bbn;
    bool has_a = next(alo, asb, ab);
    if (has_a) sum_load<U>(A, alo, lane, pbase, asb, slot2, prod);
    while (has_a) {
        const bool has_b = next(blo, bsb, bbn);
        if (has_b) sum_load<U>(B, blo, lane, pbase, bsb, slot2, prod);
        begin(ab);
        sum_add<U>(A, ys);
        if (!has_b) break;
        has_a = next(alo, asb, ab);
        if (has_a) sum_load<U>(A, alo, lane, pbase, asb, slot2, prod);
        begin(bbn);
        sum_add<U>(B, ys);
    }
    if (acc >= 0) finish();
    for (; done < b1; done += bstride) write_zero(done);
}

// ---- Mul-ordered products (BinDev::mo, internal.hpp bin_mo_tab_at) -------
// The Sum's walk is bin_sum_kernel's (one cursor over a wave's bins, the next
// batch loading while the current one is added, y written per bin), but a
// batch's products are gathered in 8-entry chunks: lane l loads the batch's
// table words r = 0..U/8-1 (chunks 64r + l) with one 16-byte load, and load
// instruction u takes chunk 8u + l/8's base from lane 8(u%8) + l/8 by
// ds_bpermute.  Each wave instruction still reads 64 products -- 8 runs of
// 64 B.  The table is loaded one batch ahead of the products it addresses,
// so waiting for it never drains the batch of products in flight (loads
// complete in issue order).
template <int U>
struct SumTab {
    int32_t t[U / 8];
};

template <int U>
__device__ __forceinline__ void sum_mo_tab(SumTab<U> &T, int64_t sb, int lane, const int32_t *__restrict__ mtab) {
    static_assert(U == 32, "U/8 = 4 table words per lane: one 16-byte load");
    const bin_u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const bin_u32x4 *>(mtab + (sb >> 3)) + lane);
#pragma unroll
    for (int h = 0; h < 4; ++h) T.t[h] = (int32_t)w[h];
}

// ordinary (cached) product loads: a chunk's 64 B start at any 8-byte
// offset, so most chunks share a 128-B line with the next one -- kept in L2
// it is read from HBM once.  Nontemporal loads (the Sum order's choice) cost
// the rank shape's Sum 0.310 -> 0.342 ms on the same plan
// (profiles/round3/probe/mulorder_store_load_policy_*.jsonl)
template <int U>
__device__ __forceinline__ void sum_mo_load(SumBatch<U> &B, const SumTab<U> &T, int64_t sb, int lane,
                                            const uint16_t *__restrict__ slot2, const double *__restrict__ prod) {
    const bin_u32x4 *sp = reinterpret_cast<const bin_u32x4 *>(slot2 + sb + (int64_t)lane * 8);
#pragma unroll
    for (int q = 0; q < U / 8; ++q) {
        const bin_u32x4 w = __builtin_nontemporal_load(sp + q * 64);
#pragma unroll
        for (int h = 0; h < 4; ++h) B.w[4 * q + h] = w[h];
    }
    const double *pl = prod + (lane & 7);
    // all U bases first, then the U loads: a load right behind its own
    // ds_bpermute waits out the LDS latency, U times per batch
    int c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = __builtin_amdgcn_ds_bpermute((((u & 7) << 3) + (lane >> 3)) << 2, T.t[u >> 3]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) B.v[u] = pl[c[u]];
}

// ---- the Mul-ordered Sum: its pipeline kept inside one bin ---------------
// LLVM's s_waitcnt insertion is conservative around vector stores issued in
// a loop of unknown trip count (bin_sum_kernel's flat walk writes a finished
// bin's y and the zeros of empty bins inside its batch loop) and around
// conditionally issued loads: the ISA of such a walk waits for vmcnt(0) (or a
// few) before a batch's adds or table reads, draining the batch in flight.
// Here each bin's batch loop issues its loads unconditionally (the batches
// past the bin's end re-load its last batch and are dropped) and stores
// nothing, so its waits count only its own pipeline; the bin's y is written
// after the loop, while the next bin's first batches already load (the
// loop's batches past its bin's end are the next bin's).  Mul-ordered plans
// have no long rows (build_bin.cpp bin_mo_resolve): one run per bin.
template <int W2, int U>
__global__ __launch_bounds__(64 * W2) void bin_sum_bin_kernel(
    int64_t b0, int64_t b1, const int64_t *__restrict__ run_off, const int64_t *__restrict__ srun_off,
    const int32_t *__restrict__ bin_row0, const uint16_t *__restrict__ slot2, const int32_t *__restrict__ mtab,
    const double *__restrict__ prod, double *__restrict__ y) {
    constexpr int SLICE = kBinLdsDoubles / W2;
    constexpr int64_t STEP = 64 * U;
    __shared__ double ylds[kBinLdsDoubles];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    double *ys = ylds + w * SLICE;
    // a bin's rows, its batch count and batch j's slot block
    struct BinRun {
        int64_t r0 = 0, nb = 0, ss0 = 0;
        int rows = 0;
        __device__ int64_t s(int64_t j) const { return ss0 + j * STEP; }
    };
    auto bin_at = [&](int64_t b) {
        BinRun R;
        R.r0 = bin_row0[b];
        R.rows = (int)(bin_row0[b + 1] - R.r0);
        R.ss0 = srun_off[b];
        R.nb = (run_off[b + 1] - run_off[b] + STEP - 1) / STEP;
        return R;
    };
    const int64_t bstride = (int64_t)gridDim.x * W2;
    int64_t b = b0 + (int64_t)blockIdx.x * W2 + w;
    if (b >= b1) return;
    BinRun R = bin_at(b);
    for (int i = lane; i < R.rows; i += 64) ys[i] = 0.0;
    SumBatch<U> PA, PB;
    SumTab<U> TA, TB;
    bool pre = false;  // R's batch 0 (PA) and batch 1's table (TB) are in flight
    for (;;) {
        const int64_t bn = b + bstride;
        const bool more = bn < b1;
        const BinRun N = more ? bin_at(bn) : R;
        // batches past R's end are the next bin's first ones (its pipeline
        // starts while R's y is written), or R's last batch again (dropped)
        const bool pfn = more && N.nb > 0;
        auto sbat = [&](int64_t j) -> int64_t {
            if (j < R.nb) return R.s(j);
            return pfn ? N.s(j - R.nb < N.nb ? j - R.nb : N.nb - 1) : R.s(R.nb - 1);
        };
        bool swapped = false;
        if (R.nb > 0) {
            if (!pre) {
                sum_mo_tab<U>(TA, sbat(0), lane, mtab);
                sum_mo_tab<U>(TB, sbat(1), lane, mtab);
                sum_mo_load<U>(PA, TA, sbat(0), lane, slot2, prod);
            }
            for (int64_t j = 0;; j += 2) {
                // batch j (PA) is added while j+1's products (table TB) and
                // j+2's table (into TA: PA's loads are issued) are in flight
                sum_mo_tab<U>(TA, sbat(j + 2), lane, mtab);
                sum_mo_load<U>(PB, TB, sbat(j + 1), lane, slot2, prod);
                sum_add<U>(PA, ys);
                if (j + 1 >= R.nb) {
                    swapped = true;  // the next bin's batch 0 is in PB, its batch 1's table in TA
                    break;
                }
                sum_mo_tab<U>(TB, sbat(j + 3), lane, mtab);
                sum_mo_load<U>(PA, TA, sbat(j + 2), lane, slot2, prod);
                sum_add<U>(PB, ys);
                if (j + 2 >= R.nb) break;
            }
        }
        pre = R.nb > 0 && pfn;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (int i = lane; i < R.rows; i += 64) __builtin_nontemporal_store(ys[i], y + R.r0 + i);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (!more) break;
        for (int i = lane; i < N.rows; i += 64) ys[i] = 0.0;
        if (pre && swapped) {
            PA = PB;
            TB = TA;
        }
        b = bn;
        R = N;
    }
}

template <int W2>
static void launch_sum_mo(const spmv_plan_s *p, double *y) {
    const BinDev &B = p->bin;
    hipLaunchKernelGGL((bin_sum_bin_kernel<W2, 32>), dim3((unsigned)B.nwg2), dim3(64 * W2), 0, p->stream,
                       (int64_t)0, B.n_bins, B.run_off, B.srun_off, B.bin_row0, B.slot2, B.mtab, B.prod, y);
}

template <int MODE, int PL, int U = 8>
static void launch_mul_t(const spmv_plan_s *p, int g, const double *x) {
    const BinDev &B = p->bin;
    if (B.long_len > 0)
        hipLaunchKernelGGL((bin_mul_kernel<U, MODE, PL, true>), dim3((unsigned)B.nwg1), dim3(kBinMulThreads), 0,
                           p->stream, B.piece_off, (int64_t)g * B.nwg1, B.piece_strip, B.piece_begin, B.piece_end,
                           B.val1, B.cs1, B.dst1, x, p->n, (int32_t)B.strip, B.prod, B.lstart, B.lshift, B.lcode,
                           B.xburst);
    else
        hipLaunchKernelGGL((bin_mul_kernel<U, MODE, PL, false>), dim3((unsigned)B.nwg1), dim3(kBinMulThreads), 0,
                           p->stream, B.piece_off, (int64_t)g * B.nwg1, B.piece_strip, B.piece_begin, B.piece_end,
                           B.val1, B.cs1, B.dst1, x, p->n, (int32_t)B.strip, B.prod, nullptr, nullptr, nullptr,
                           B.xburst);
}

template <int PL>
static void launch_mul_p(const spmv_plan_s *p, int g, const double *x) {
    // Sum-ordered products: nontemporal stores (measured 0.81 -> 0.71 ms at
    // config 2, profiles/round1/probe/bin_probe_c2.jsonl).  Mul-ordered
    // products (BinDev::mo): ordinary stores -- the contiguous write streams
    // of all workgroups ran the rank shape's Mul at 0.593-0.660 instead of
    // 0.642-0.733 ms on two boxes, the Sum after them (cached loads)
    // 0.307-0.310 -> 0.346-0.363: execute 0.944 -> 0.933 and 1.039 -> 1.017
    // ms (profiles/round3/probe/mulorder_store_load_policy_*).  x strips by
    // LDS-DMA wherever x + c0 is 16-byte aligned (config 2 Mul 0.536 ->
    // 0.520 ms, N = 8 rank shape 0.738 -> 0.717, config 3 -1 %, same plans,
    // profiles/round3/probe/mul_glds_*.jsonl), else through registers.
    bool dma = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && p->bin.strip % 2 == 0;
    // probe build, SPMV_LAUNCH_DEBUG bit 24: registers instead of LDS-DMA
    if (launch_dbg(p->bin.dbg) & (1 << 24)) dma = false;
    if (p->bin.mo) {
        if (dma) launch_mul_t<256 | 4, PL>(p, g, x);
        else launch_mul_t<4, PL>(p, g, x);
    } else {
        if (dma) launch_mul_t<256 | 1, PL>(p, g, x);
        else launch_mul_t<1, PL>(p, g, x);
    }
}

static void launch_mul(const spmv_plan_s *p, int g, const double *x) {
    if (p->bin.pad_log == 5) launch_mul_p<5>(p, g, x);
    else if (p->bin.pad_log == 4) launch_mul_p<4>(p, g, x);
    else launch_mul_p<3>(p, g, x);
}

// Sum over the bins of group g (g < 0: every bin, product buffer = all products)
template <int W2, int U>
static void launch_sum_w(const spmv_plan_s *p, int g, double *y) {
    const BinDev &B = p->bin;
    const int64_t b0 = g < 0 ? 0 : B.g_bin[g], b1 = g < 0 ? B.n_bins : B.g_bin[g + 1];
    const int64_t pbase = g < 0 ? 0 : B.g_prod[g];
    hipLaunchKernelGGL((bin_sum_kernel<W2, U>), dim3((unsigned)B.nwg2), dim3(64 * W2), 0, p->stream, b0, b1,
                       B.n_bins, B.n_blocks, B.run_off, B.srun_off, B.bin_row0, pbase, B.slot2, B.prod, y);
}

int bin_time_mul(const spmv_plan_s *p, const double *x, float *ms) {
    const BinDev &B = p->bin;
    hipEvent_t a, b;
    SPMV_HIP_TRY(hipEventCreate(&a));
    SPMV_HIP_TRY(hipEventCreate(&b));
    for (int rep = 0; rep < 2; ++rep) {  // the second pass is timed
        if (rep == 1) SPMV_HIP_TRY(hipEventRecord(a, p->stream));
        for (int g = 0; g < B.G; ++g) {
            launch_mul(p, g, x);
        }
    }
    SPMV_HIP_TRY(hipEventRecord(b, p->stream));
    SPMV_HIP_TRY(hipEventSynchronize(b));
    SPMV_HIP_TRY(hipEventElapsedTime(ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return SPMV_SUCCESS;
}

int launch_bin(const spmv_plan_s *p, const double *x, double *y) {
    const BinDev &B = p->bin;
    if (p->m == 0) return SPMV_SUCCESS;
    if (p->nnz == 0) {  // no entries: y = 0 (and x may be empty)
        SPMV_HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * (size_t)p->m, p->stream));
        return SPMV_SUCCESS;
    }
    auto sum = [&](int g) {
        if (B.mo) {  // Mul-ordered products (G == 1, 32-entry batches)
            if (B.sum_waves == 2) launch_sum_mo<2>(p, y);
            else launch_sum_mo<4>(p, y);
            return;
        }
        if (B.sum_waves == 2) launch_sum_w<2, 32>(p, g, y);
        // 4 waves: 32-entry batches per lane (0.313 -> 0.295 ms against 16,
        // profiles/round1/probe/bin_sum_depth.jsonl; 231 VGPRs, 1 wave/SIMD)
        else if (B.sum_waves == 4) launch_sum_w<4, 32>(p, g, y);
        else launch_sum_w<8, 8>(p, g, y);
    };
    // Mul per row group (all groups' writes go to one product buffer unless
    // it is re-used per group), then Sum
    for (int g = 0; g < B.G; ++g) {
        launch_mul(p, g, x);
        SPMV_HIP_TRY(hipGetLastError());
        if (B.reuse) {
            phase_mark(p);  // mul | sum
            sum(g);
            SPMV_HIP_TRY(hipGetLastError());
            if (g + 1 < B.G) phase_mark(p);
        }
    }
    if (!B.reuse) {
        phase_mark(p);  // mul | sum
        sum(-1);
        SPMV_HIP_TRY(hipGetLastError());
    }
    return SPMV_SUCCESS;
}

}  // namespace spmv

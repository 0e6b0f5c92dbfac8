// Host-only check of the BIN layout (build_bin.cpp's bin_rows / bin_offsets
// and bin_slot_index), no GPU: for random CSRs and every strip width / Sum
// wave count / padding it
//   * cuts the row bins and counts (bin, strip) segments like build_bin,
//   * checks the Sum-order segments tile [0, E) bin-major, each padded to PAD,
//   * checks the Mul-order segments tile [0, E) strip-major with the same sizes,
//   * checks the slot layout: bin_slot_index maps every product position of a
//     run into that run's padded slot block without collisions, and the Sum
//     kernel's load formula (k_bin.hip sum_load: word q of lane l at
//     sbase + q*512 + l*8) finds entry (u, l) of every batch there;
//   * with long rows (the run path): segments hold only the short rows, the
//     long runs of every bin follow the segments in the Sum order and tile
//     [E, E + pieces), every strip's Mul range is 64-aligned with its long
//     blocks after its segments, and the trash line lies past every run.
//   * emulates both kernels (k_bin.hip bin_mul_kernel / bin_sum_kernel: the
//     same workgroup pieces, wave batches, lane clamps, long-block scan and
//     unclamped Sum batches) on the host builder's arrays, checking every index a lane
//     forms against its array's bounds, that the Sum reads only products the
//     Mul wrote, and that y is the sequential row sum -- bit for bit on
//     short rows, within 1e-12 of sum |a x| on long rows.
// Built and run by tests/test_bin_layout.py.  Prints "ok" or the failure.
#include "build_bin.cpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <random>

using namespace spmv;

static int fail(const char *what, long long a = 0, long long b = 0) {
    std::printf("FAIL %s %lld %lld\n", what, a, b);
    return 1;
}


// ---- host emulation of the two kernels on the host builder's arrays -------
static int emulate(const BinDev &B, const HostCsr &A, const BinLayout &L, const BinHostArrays &H,
                   const std::vector<double> &x) {
    const int64_t S = L.S, NB = L.NB, C = B.strip, PL = B.pad_log, PADE = (int64_t)1 << PL;
    const int64_t prod_cap = L.LL > 0 ? L.TRASH + L.PAD : B.mo ? L.E1 : L.E;
    std::vector<double> prod((size_t)prod_cap, 0.0);
    std::vector<char> written((size_t)prod_cap, 0);
    BinPieces P;
    bin_pieces(B, L, P);
    const int U = 8, NW = kBinMulThreads / 64;
    const int64_t STEP = (int64_t)NW * 64 * U;
    for (int k = 0; k < B.nwg1; ++k)
        for (int64_t q = P.off[(size_t)k]; q < P.off[(size_t)k + 1]; ++q) {
            const int32_t st = P.strip[(size_t)q];
            const int64_t e0 = P.beg[(size_t)q], e1 = P.end[(size_t)q], c0 = (int64_t)st * C;
            const int64_t ls = L.LL > 0 ? L.lstart[(size_t)st] : INT64_MAX, lsh = L.LL > 0 ? H.lshift[(size_t)st] : 0;
            const int64_t cw = std::min<int64_t>(A.n - c0, C);
            for (int w = 0; w < NW; ++w) {
                const int64_t first = e0 + (int64_t)w * 64 * U;
                const int64_t nit = first < e1 ? (e1 - first + STEP - 1) / STEP : 0;
                for (int64_t it = 0; it < nit; ++it)
                    for (int u = 0; u < U; ++u) {
                        const int64_t bs = first + it * STEP + u * 64;
                        const bool lng = L.LL > 0 && bs >= ls;
                        double v[64];
                        int32_t d[64];
                        bool ok[64];
                        for (int lane = 0; lane < 64; ++lane) {
                            // mul_load: unclamped -- lanes past the piece read on
                            // into the slack (their stores are masked)
                            const int64_t e = bs + lane, ee = e;
                            ok[lane] = e < e1;
                            if (ee < 0 || ee >= (int64_t)H.val1.size() || ee >= (int64_t)H.cs1.size())
                                return fail("mul val1/cs1 index", ee, H.val1.size());
                            const int64_t c = H.cs1[(size_t)ee];
                            if (c >= C) return fail("mul LDS strip index", c, C);
                            if (ok[lane] && c >= cw) return fail("mul x strip index", c, cw);
                            v[lane] = ok[lane] ? H.val1[(size_t)ee] * x[(size_t)(c0 + c)] : 0.0;
                            if (lng) {
                                const int64_t i = e < e1 ? e + lsh : 0;
                                if (i < 0 || i >= (int64_t)H.lcode.size()) return fail("mul lcode index", i, H.lcode.size());
                                d[lane] = H.lcode[(size_t)i];
                            } else if (!B.mo) {
                                const int64_t i = ee >> PL;
                                if (i < 0 || i >= (int64_t)H.dst1.size()) return fail("mul dst1 index", i, H.dst1.size());
                                d[lane] = H.dst1[(size_t)i];
                            }
                        }
                        if (lng) {  // mul_long_block
                            uint64_t starts = 0;
                            for (int lane = 0; lane < 64; ++lane)
                                if (d[lane] < 0 || !ok[lane]) starts |= 1ull << lane;
                            if (!(starts & 1)) return fail("long block without a start on lane 0", bs);
                            double s2[64];
                            for (int lane = 0; lane < 64; ++lane) s2[lane] = ok[lane] ? v[lane] : 0.0;
                            // the DPP tree: row_shr 1/2/4/8, row_bcast15 (rows 1, 3), row_bcast31 (rows 2, 3)
                            for (int step = 0; step < 6; ++step) {
                                double nv[64];
                                for (int lane = 0; lane < 64; ++lane) {
                                    const uint64_t upto = starts & (~0ull >> (63 - lane));
                                    const int seg = 63 - __builtin_clzll(upto), r16 = lane & 15, row = lane >> 4;
                                    int src = -1;
                                    if (step < 4) {
                                        const int dd = 1 << step;
                                        if (r16 >= dd && lane - dd >= seg) src = lane - dd;
                                    } else if (step == 4) {
                                        if ((row & 1) && seg <= row * 16 - 1) src = row * 16 - 1;
                                    } else if (row >= 2 && seg <= 31) {
                                        src = 31;
                                    }
                                    nv[lane] = src >= 0 ? s2[src] + s2[lane] : s2[lane];
                                }
                                std::memcpy(s2, nv, sizeof(nv));
                            }
                            for (int lane = 0; lane < 64; ++lane) {
                                const int64_t pos = d[lane] & 0x7FFFFFFF;
                                if (!ok[lane] || pos == 0x7FFFFFFF) continue;
                                if (pos >= prod_cap) return fail("long partial position", pos, prod_cap);
                                prod[(size_t)pos] = s2[lane];
                                written[(size_t)pos] = 1;
                            }
                        } else {
                            for (int lane = 0; lane < 64; ++lane) {
                                if (!ok[lane]) continue;
                                // Mul order (B.mo): the product of entry e goes to prod[e]
                                const int64_t pos = B.mo ? bs + lane : ((int64_t)d[lane] << PL) + ((bs + lane) & (PADE - 1));
                                if (pos < 0 || pos >= prod_cap) return fail("product position", pos, prod_cap);
                                prod[(size_t)pos] = v[lane];
                                written[(size_t)pos] = 1;
                            }
                        }
                    }
            }
        }
    // Sum
    const int W2 = B.sum_waves, U2 = B.sum_u, SLICE = kBinLdsDoubles / W2;
    const int64_t STEP2 = 64 * (int64_t)U2, nblk = B.n_blocks;
    std::vector<double> y((size_t)A.m, 0.0), ys((size_t)SLICE);
    for (int64_t b = 0; b < NB; ++b) {
        const int64_t r0 = L.row0[(size_t)b], rows = L.row0[(size_t)b + 1] - r0;
        if (rows > SLICE - 1) return fail("bin rows > slice", b, rows);
        std::fill(ys.begin(), ys.end(), 0.0);
        for (int64_t kk = 0; kk < nblk; ++kk) {
            const size_t run = (size_t)(kk * NB + b);
            const int64_t lo = L.run_off[run], hi = L.run_off[run + 1], ss = L.srun_off[run];
            for (int64_t pos = lo; pos < hi; pos += STEP2) {
                const int64_t bhi = std::min(pos + STEP2, hi), sbase = ss + (pos - lo);
                for (int u = 0; u < U2; ++u)
                    for (int lane = 0; lane < 64; ++lane) {
                        const int64_t e = pos + u * 64 + lane;
                        const int64_t si = sbase + (u / 8) * 512 + lane * 8 + (u % 8);
                        if (si >= L.ES) return fail("slot index", si, L.ES);
                        // the product read: position e, or (Mul order) lane
                        // l/8's chunk base from the table + l % 8 (sum_mo_load)
                        int64_t pe = e;
                        if (B.mo) {
                            const int64_t ti = sbase / 8 + bin_mo_tab_at((u * 64 + lane) >> 3, U2);
                            if (sbase % 8 || ti >= (int64_t)H.mtab.size()) return fail("chunk table index", ti, H.mtab.size());
                            pe = H.mtab[(size_t)ti] + (lane & 7);
                        }
                        if (pe < 0) return fail("negative product position", pe);
                        if (e >= bhi) {
                            // sum_load reads the whole batch unclamped: past the
                            // run it must stay inside the buffer (with its slack)
                            // and hit the dummy slot
                            if (pe >= prod_cap + kBinProdSlack) return fail("sum reads past the product buffer", pe, prod_cap);
                            if (H.slot2[(size_t)si] != SLICE - 1) return fail("slot past a run is not the dummy", e, H.slot2[(size_t)si]);
                            continue;
                        }
                        const int slot = H.slot2[(size_t)si];
                        if (B.mo && slot == SLICE - 1) {  // segment padding: the next segment's products
                            if (pe >= prod_cap + kBinProdSlack) return fail("padding read past the product buffer", pe, prod_cap);
                            continue;
                        }
                        if (pe >= prod_cap || !written[(size_t)pe]) return fail("sum reads an unwritten product", pe);
                        if (slot > SLICE - 1) return fail("slot past the dummy", slot);
                        if (slot < SLICE - 1 && slot >= rows) return fail("slot past the bin", slot, rows);
                        ys[(size_t)slot] += prod[(size_t)pe];
                    }
            }
        }
        for (int64_t i = 0; i < rows; ++i) y[(size_t)(r0 + i)] = ys[(size_t)i];
    }
    for (int64_t r = 0; r < A.m; ++r) {
        double t = 0.0, mag = 0.0;
        for (int64_t j = A.row_ptr[r]; j < A.row_ptr[r + 1]; ++j) {
            t = t + A.val[j] * x[(size_t)A.col[j]];
            mag += std::fabs(A.val[j] * x[(size_t)A.col[j]]);
        }
        if (L.is_long(A.row_ptr, r)) {
            if (!(std::fabs(y[(size_t)r] - t) <= 1e-12 * mag)) return fail("long row sum", r);
        } else if (y[(size_t)r] != t) {
            return fail("short row not bit-exact", r);
        }
    }
    return 0;
}

int main(int argc, char **argv) {
    std::mt19937_64 rng(7);
    int cases = 0;
    const int trials = argc > 1 ? std::atoi(argv[1]) : 60;  // the ASan run takes fewer (tests/test_guards.py)
    for (int trial = 0; trial < trials; ++trial) {
        const int64_t m = 1 + (int64_t)(rng() % 60000), n = 1 + (int64_t)(rng() % 300000);
        const int kind = trial % 3;  // uniform short rows / long rows / many empty rows
        std::vector<int64_t> rp(m + 1, 0);
        std::vector<int32_t> col;
        for (int64_t r = 0; r < m; ++r) {
            int64_t len = kind == 0 ? (int64_t)(rng() % 24) : kind == 1 ? ((rng() % 50 == 0) ? (int64_t)(rng() % 3000) : (int64_t)(rng() % 8)) : ((rng() % 3 == 0) ? (int64_t)(rng() % 40) : 0);
            std::vector<int32_t> c(len);
            for (auto &v : c) v = (int32_t)(rng() % n);
            std::sort(c.begin(), c.end());
            col.insert(col.end(), c.begin(), c.end());
            rp[r + 1] = rp[r] + len;
        }
        const int64_t nnz = rp[m];
        std::vector<double> val((size_t)nnz), x((size_t)n);
        for (auto &v : val) v = (double)(rng() >> 11) * 0x1.0p-53 - 0.25;
        for (auto &v : x) v = (double)(rng() >> 11) * 0x1.0p-53;
        const bool emu = m <= 20000;  // kernel emulation on the smaller CSRs
        const int strips[] = {20480, 3001, 64};
        const int waves[] = {2, 4, 8};
        for (int si = 0; si < 3; ++si)
            for (int wi = 0; wi < 3; ++wi)
                for (int pl = 3; pl <= 4; ++pl)
                for (int mo = 0; mo < (waves[wi] == 8 ? 1 : 2); ++mo) {
                    spmv_plan_s p;
                    BinDev &B = p.bin;
                    B.mo = mo == 1;  // products in Mul order (build_bin.cpp bin_mo_resolve)
                    B.strip = strips[si];
                    B.sum_waves = waves[wi];
                    B.max_rows = bin_max_rows(B.sum_waves);
                    B.sum_u = B.sum_waves == 8 ? 8 : 32;
                    B.pad_log = pl;
                    B.nwg1 = B.nwg2 = 256;
                    B.mul_perm = (si + wi + pl) % 2 == 0;  // both Mul bin orders
                    spmv_options_t o;
                    std::memset(&o, 0, sizeof(o));
                    BinLayout L;
                    if (bin_rows(&p, rp.data(), m, n, L) != SPMV_SUCCESS) return fail("bin_rows");
                    const int64_t S = L.S, NB = L.NB, C = B.strip;
                    for (int64_t b = 0; b < NB; ++b)
                        if (L.row0[b + 1] - L.row0[b] > B.max_rows || L.row0[b + 1] < L.row0[b])
                            return fail("bin rows", b, L.row0[b + 1] - L.row0[b]);
                    if (L.row0[NB] != m) return fail("bins cover rows", L.row0[NB], m);
                    L.cnt.assign((size_t)(NB * S), 0);
                    for (int64_t b = 0; b < NB; ++b)
                        for (int64_t j = rp[L.row0[b]]; j < rp[L.row0[b + 1]]; ++j) ++L.cnt[(size_t)(b * S + col[j] / C)];
                    bin_offsets(&p, o, L);
                    const int64_t E = L.E, PAD = L.PAD;
                    // Sum order: bin-major, strips ascending, contiguous, padded
                    int64_t cur = 0;
                    for (int64_t b = 0; b < NB; ++b) {
                        if (L.run_off[(size_t)b] != cur) return fail("run_off", b, cur);
                        for (int64_t t = 0; t < S; ++t) {
                            if (L.off2[(size_t)(b * S + t)] != cur) return fail("off2", b * S + t, cur);
                            if (cur % PAD) return fail("off2 alignment", cur, PAD);
                            cur += L.rpad(L.cnt[(size_t)(b * S + t)]);
                        }
                    }
                    if (cur != E) return fail("E", cur, E);
                    // Mul order: strip-major, the bins of a strip in L.mul_bins
                    // order (a permutation of the bins), same padded sizes
                    // (Mul-ordered products: unpadded, nnz in all)
                    {
                        std::vector<char> hit((size_t)NB, 0);
                        for (int64_t i = 0; i < NB; ++i) {
                            const int64_t b = L.mul_bins[(size_t)i];
                            if (b < 0 || b >= NB || hit[(size_t)b]++) return fail("mul_bins permutation", i, b);
                        }
                    }
                    cur = 0;
                    for (int64_t t = 0; t < S; ++t) {
                        if (L.strip_start[(size_t)t] != cur) return fail("strip_start", t, cur);
                        for (int64_t i = 0; i < NB; ++i) {
                            const int64_t b = L.mul_bins[(size_t)i];
                            if (L.off1[(size_t)(b * S + t)] != cur) return fail("off1", b * S + t, cur);
                            cur += B.mo ? L.cnt[(size_t)(b * S + t)] : L.rpad(L.cnt[(size_t)(b * S + t)]);
                        }
                    }
                    if (cur != (B.mo ? nnz : E) || L.E1 != cur) return fail("Mul E", cur, E);
                    // slots: padded runs, bijective index, kernel formula
                    const int U = B.sum_u;
                    const int64_t step = 64 * (int64_t)U;
                    std::vector<unsigned char> seen((size_t)std::max<int64_t>(L.ES, 1), 0);
                    for (int64_t b = 0; b < NB; ++b) {
                        const int64_t r0 = L.run_off[(size_t)b], r1 = L.run_off[(size_t)b + 1], s0 = L.srun_off[(size_t)b];
                        if (s0 % step) return fail("srun alignment", b, s0);
                        if (L.srun_off[(size_t)b + 1] - s0 != (r1 - r0 + step - 1) / step * step) return fail("srun size", b);
                        for (int64_t e = r0; e < r1; ++e) {
                            const int64_t k = bin_slot_index(e, r0, s0, U);
                            if (k < s0 || k >= L.srun_off[(size_t)b + 1]) return fail("slot range", e, k);
                            if (seen[(size_t)k]++) return fail("slot collision", e, k);
                            const int64_t lo = r0 + (e - r0) / step * step, w = e - lo;
                            const int u = (int)(w / 64), lane = (int)(w % 64);
                            const int64_t sbase = s0 + (lo - r0);
                            if (sbase + (u / 8) * 512 + lane * 8 + (u % 8) != k) return fail("kernel slot formula", e, k);
                        }
                    }
                    ++cases;
                    if (emu && (wi == 1 || mo)) {  // emulate the kernels on the exact (no long rows) layout
                        HostCsr A0{m, n, nnz, rp.data(), col.data(), val.data()};
                        BinHostArrays H0;
                        bin_fill_arrays(B, A0, L, H0);
                        if (emulate(B, A0, L, H0, x)) return fail("emulation (exact layout)", trial, si);
                        ++cases;
                    }
                    if (mo || kind == 0 || (kind == 2 && !emu) || si == 0) continue;
                    // ---- the same CSR with long rows on the run path: the
                    // auto threshold (long-row CSRs), or 6 entries (many short
                    // long rows, pieces cut at block boundaries)
                    HostCsr A{m, n, nnz, rp.data(), col.data(), val.data()};
                    BinLayout K;
                    K.S = std::max<int64_t>(1, (n + C - 1) / C);
                    o.bin_long_len = kind == 1 ? 0 : 6;
                    K.LL = bin_long_threshold(o, rp.data(), m, nnz, K.S);
                    o.bin_long_len = 0;
                    if (K.LL == 0) continue;  // too few long entries for auto
                    bin_long_prep(A, C, K);
                    if (bin_rows(&p, rp.data(), m, n, K) != SPMV_SUCCESS) return fail("long bin_rows");
                    const int64_t KB = K.NB;
                    K.cnt.assign((size_t)(KB * S), 0);
                    int64_t nlong = 0, runs = 0;
                    for (int64_t r = 0; r < m; ++r) {
                        if (K.is_long(rp.data(), r)) {
                            nlong += rp[r + 1] - rp[r];
                            int64_t last = -1;
                            for (int64_t j = rp[r]; j < rp[r + 1]; ++j)
                                if (col[j] / C != last) ++runs, last = col[j] / C;
                            continue;
                        }
                        int64_t b = std::upper_bound(K.row0.begin(), K.row0.end(), (int32_t)r) - K.row0.begin() - 1;
                        for (int64_t j = rp[r]; j < rp[r + 1]; ++j) ++K.cnt[(size_t)(b * S + col[j] / C)];
                    }
                    if (K.lb_off[(size_t)S] != nlong) return fail("long entries bucketed", K.lb_off[(size_t)S], nlong);
                    bin_long_count(K);
                    bin_offsets(&p, o, K);
                    const int64_t NBK = B.n_blocks - 1;
                    int64_t np = 0;
                    for (int64_t k = 0; k < KB * S; ++k) np += K.lpc[(size_t)k];
                    if (np != K.NP || np < runs) return fail("pieces", np, runs);
                    cur = K.E;
                    for (int64_t b = 0; b < KB; ++b) {
                        if (K.run_off[(size_t)(NBK * KB + b)] != cur) return fail("long run_off", b, cur);
                        for (int64_t t = 0; t < S; ++t) {
                            if (K.lpoff[(size_t)(b * S + t)] != cur) return fail("lpoff", b * S + t, cur);
                            cur += K.lpc[(size_t)(b * S + t)];
                        }
                    }
                    if (cur != K.E + K.NP || K.run_off.back() != cur) return fail("long runs end", cur, K.E + K.NP);
                    if (K.TRASH < cur || K.TRASH % K.PAD) return fail("trash line", K.TRASH, cur);
                    for (int64_t t = 0; t < S; ++t) {
                        int64_t reg = 0;
                        for (int64_t b = 0; b < KB; ++b) reg += K.rpad(K.cnt[(size_t)(b * S + t)]);
                        const int64_t s0 = K.strip_start[(size_t)t];
                        if (s0 % 64 || K.lstart[(size_t)t] % 64 || K.lstart[(size_t)t] < s0 + reg ||
                            K.lstart[(size_t)t] >= s0 + reg + 64)
                            return fail("long blocks start", t, K.lstart[(size_t)t]);
                        if (K.strip_start[(size_t)t + 1] != K.lstart[(size_t)t] + K.lpad[(size_t)t])
                            return fail("strip end", t);
                        if (K.lpad[(size_t)t] != (K.lb_off[(size_t)t + 1] - K.lb_off[(size_t)t] + 63) / 64 * 64)
                            return fail("lpad", t);
                    }
                    if (K.E1 != K.strip_start[(size_t)S]) return fail("E1", K.E1);
                    ++cases;
                    if (emu) {
                        BinHostArrays H;
                        bin_fill_arrays(B, A, K, H);
                        if (emulate(B, A, K, H, x)) return fail("emulation (long rows)", trial, si);
                        ++cases;
                    }
                }
    }
    // ---- the run path's positions must fit lcode's 31 bits (build_bin.cpp
    // bin_layout): a very sparse power-law shape (mostly 1-2 entry rows, so
    // short padded segments, plus long rows) laid out once with the
    // real limit and once with a limit just below its trash line's end --
    // the second must drop the run path (LL = 0) and stay a valid layout.
    {
        const int64_t m = 20000, n = 300000;
        std::vector<int64_t> rp(m + 1, 0);
        std::vector<int32_t> col;
        for (int64_t r = 0; r < m; ++r) {
            const int64_t len = (rng() % 100 == 0) ? 300 + (int64_t)(rng() % 1700) : 1 + (int64_t)(rng() % 2);
            std::vector<int32_t> c(len);
            for (auto &v : c) v = (int32_t)(rng() % n);
            std::sort(c.begin(), c.end());
            col.insert(col.end(), c.begin(), c.end());
            rp[r + 1] = rp[r] + len;
        }
        const int64_t nnz = rp[m];
        std::vector<double> val((size_t)nnz), x((size_t)n);
        for (auto &v : val) v = (double)(rng() >> 11) * 0x1.0p-53;
        for (auto &v : x) v = (double)(rng() >> 11) * 0x1.0p-53;
        HostCsr A{m, n, nnz, rp.data(), col.data(), val.data()};
        spmv_plan_s p;
        BinDev &B = p.bin;
        B.strip = 3001;
        B.sum_waves = 4;
        B.max_rows = bin_max_rows(B.sum_waves);
        B.sum_u = 32;
        B.pad_log = 4;
        B.nwg1 = B.nwg2 = 256;
        spmv_options_t o;
        std::memset(&o, 0, sizeof(o));
        o.bin_long_len = 64;
        BinLayout L;
        if (bin_layout(&p, A, o, L, kBinLongPosLimit) != SPMV_SUCCESS) return fail("bin_layout");
        if (L.LL != 64) return fail("run path expected", L.LL);
        const int64_t end = L.TRASH + L.PAD;
        BinLayout K;
        if (bin_layout(&p, A, o, K, end - 1) != SPMV_SUCCESS) return fail("bin_layout (limit)");
        if (K.LL != 0 || K.E < nnz || p.bin.long_rows != 0) return fail("run path not dropped", K.LL, K.E);
        BinHostArrays H;
        bin_fill_arrays(B, A, K, H);
        if (emulate(B, A, K, H, x)) return fail("emulation (run path dropped)");
        BinLayout J;  // exactly at the limit: kept
        if (bin_layout(&p, A, o, J, end) != SPMV_SUCCESS || J.LL != 64) return fail("limit boundary", J.LL);
        cases += 3;
    }
    std::printf("ok %d\n", cases);
    return 0;
}

// Host-only check of the BIN layout (build_bin.cpp's bin_rows / bin_offsets
// and bin_slot_index), no GPU: for random CSRs and every strip width / Sum
// wave count / padding it
//   * cuts the row bins and counts (bin, strip) segments like build_bin,
//   * checks the Sum-order segments tile [0, E) bin-major, each padded to PAD,
//   * checks the Mul-order segments tile [0, E) strip-major with the same sizes,
//   * checks the slot layout: bin_slot_index maps every product position of a
//     run into that run's padded slot block without collisions, and the Sum
//     kernel's load formula (k_bin.hip sum_load: word q of lane l at
//     sbase + q*512 + l*8) finds entry (u, l) of every batch there.
// Built and run by tests/test_bin_layout.py.  Prints "ok" or the failure.
#include "build_bin.cpp"

#include <cstdio>
#include <cstring>
#include <random>

using namespace spmv;

static int fail(const char *what, long long a = 0, long long b = 0) {
    std::printf("FAIL %s %lld %lld\n", what, a, b);
    return 1;
}

int main() {
    std::mt19937_64 rng(7);
    int cases = 0;
    for (int trial = 0; trial < 60; ++trial) {
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
        const int strips[] = {20480, 3001, 64};
        const int waves[] = {2, 4, 8};
        for (int si = 0; si < 3; ++si)
            for (int wi = 0; wi < 3; ++wi)
                for (int pl = 3; pl <= 4; ++pl) {
                    spmv_plan_s p;
                    BinDev &B = p.bin;
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
                    if (bin_rows(&p, rp.data(), m, n, nnz, L) != SPMV_SUCCESS) return fail("bin_rows");
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
                            cur += L.rpad(L.cnt[(size_t)(b * S + t)]);
                        }
                    }
                    if (cur != E) return fail("Mul E", cur, E);
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
                }
    }
    std::printf("ok %d\n", cases);
    return 0;
}

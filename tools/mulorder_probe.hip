// mulorder_probe.hip -- what would BIN's Sum cost if the Mul wrote its
// products in Mul order ([strip][bin], contiguous, no segment padding) and the
// Sum gathered each bin's segments back in 8-entry chunks?
//
// profiles/round3/README.md (round-3 open items): at the 10 M x 80 M rank shape ~100 us of the Mul is the scatter
// of its product writes into the Sum-ordered (bin, strip) segments (336-B
// runs); products written in Mul order would also drop the segment padding
// (174.0 M stored entries -> 160 M) and the destination array.  The price is
// on the Sum side: its batches no longer read one contiguous run per bin.
// This probe builds the same geometry synthetically (S strips x NB bins,
// Poisson segment lengths) and times the Sum's loop (two 64xU-entry batches in
// flight, slots 8 per 16-byte load, ds_add_f64 into an LDS y slice, y written
// per bin) over four product layouts:
//   var 0  today: Sum-ordered products, each bin one contiguous run
//   var 1  Mul order, instruction u reads 8 chunks (8 lanes each), every
//          lane loads the 32 (U) chunk bases of its lane group
//   var 2  Mul order, same lane mapping, one 16-byte table load per lane and
//          the bases redistributed by ds_bpermute
//   var 3  Mul order, lane-major: lane l owns 4 chunks of the batch (one
//          16-byte table load), so one instruction touches 64 chunks
// The chunk table is loaded one batch ahead of the products (so the in-order
// load counter never makes a table wait drain the batch in flight).  y is
// checked against the exact sum (integer-valued products) for every variant.
//   hipcc -O3 --offload-arch=gfx950 -o bin/mulorder_probe tools/mulorder_probe.hip
//   bin/mulorder_probe S NB mean m [mulpad]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

constexpr int W2 = 2, SLICE = 10240, DUMMY = SLICE - 1;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct Geo {
    const int64_t *bat_off;  // [NB+1] global batch index of each bin's first batch
    const int64_t *pstart;   // var 0: product start of each bin's run
    const int32_t *tab;      // var > 0: 8U chunk bases per batch, layout per var
    const uint16_t *slot;    // 64U slots per batch (16-byte lane words)
    const double *prod;
    double *y;
    int64_t nbins, rows_per_bin, m;
};

template <int V, int U>
struct Tab {
    int32_t t[V == 0 ? 1 : (V == 1 ? U : U / 8)];
};
template <int U>
struct Bat {
    double v[U];
    uint32_t s[U / 2];
};

template <int V, int U>
__device__ __forceinline__ void ldtab(Tab<V, U> &T, const Geo &g, int64_t gb, int lane) {
    if constexpr (V == 1) {
        const u32x4 *p = reinterpret_cast<const u32x4 *>(g.tab + gb * 8 * U + (lane >> 3) * U);
#pragma unroll
        for (int q = 0; q < U / 4; ++q) {
            const u32x4 w = __builtin_nontemporal_load(p + q);
#pragma unroll
            for (int h = 0; h < 4; ++h) T.t[4 * q + h] = (int32_t)w[h];
        }
    } else if constexpr (V >= 2 && U == 32) {
        const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(g.tab + gb * 8 * U) + lane);
#pragma unroll
        for (int h = 0; h < 4; ++h) T.t[h] = (int32_t)w[h];
    } else if constexpr (V >= 2 && U == 16) {
        const u32x2 w = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(g.tab + gb * 8 * U) + lane);
        T.t[0] = (int32_t)w[0];
        T.t[1] = (int32_t)w[1];
    }
}

template <int V, int U>
__device__ __forceinline__ void ldprod(Bat<U> &B, const Tab<V, U> &T, const Geo &g, int64_t gb, int64_t pb,
                                       int lane) {
    const u32x4 *sp = reinterpret_cast<const u32x4 *>(g.slot + gb * 64 * U + lane * 8);
#pragma unroll
    for (int q = 0; q < U / 8; ++q) {
        const u32x4 w = __builtin_nontemporal_load(sp + q * 64);
#pragma unroll
        for (int h = 0; h < 4; ++h) B.s[4 * q + h] = w[h];
    }
    if constexpr (V == 0) {
        const double *pp = g.prod + pb + lane;
#pragma unroll
        for (int u = 0; u < U; ++u) B.v[u] = __builtin_nontemporal_load(pp + u * 64);
    } else if constexpr (V == 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) B.v[u] = __builtin_nontemporal_load(g.prod + T.t[u] + (lane & 7));
    } else if constexpr (V == 2) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int base = __builtin_amdgcn_ds_bpermute((((u & 7) << 3) + (lane >> 3)) << 2, T.t[u >> 3]);
            B.v[u] = __builtin_nontemporal_load(g.prod + base + (lane & 7));
        }
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) B.v[u] = __builtin_nontemporal_load(g.prod + T.t[u >> 3] + (u & 7));
    }
}

template <int V, int U>
__global__ __launch_bounds__(64 * W2) void sum_probe(Geo g) {
    __shared__ double ylds[W2 * SLICE];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double *ys = ylds + w * SLICE;
    const int64_t nw = (int64_t)gridDim.x * W2, wid = (int64_t)blockIdx.x * W2 + w;
    int64_t cb = wid, gb = 0, ge = 0;
    if (cb < g.nbins) {
        gb = g.bat_off[cb];
        ge = g.bat_off[cb + 1];
    }
    auto next = [&](int64_t &ob, int64_t &ogb, int64_t &opb) -> bool {
        while (gb >= ge) {
            cb += nw;
            if (cb >= g.nbins) return false;
            gb = g.bat_off[cb];
            ge = g.bat_off[cb + 1];
        }
        ob = cb;
        ogb = gb;
        opb = V == 0 ? g.pstart[cb] + (gb - g.bat_off[cb]) * 64 * U : 0;
        ++gb;
        return true;
    };
    int64_t acc = -1;
    auto rows_of = [&](int64_t b) {
        const int64_t r0 = b * g.rows_per_bin;
        return (int)(r0 + g.rows_per_bin < g.m ? g.rows_per_bin : g.m - r0);
    };
    auto finish = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const int rows = rows_of(acc);
        for (int i = lane; i < rows; i += 64) __builtin_nontemporal_store(ys[i], g.y + acc * g.rows_per_bin + i);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    };
    auto begin = [&](int64_t nb) {
        if (nb == acc) return;
        if (acc >= 0) finish();
        for (int i = lane; i < SLICE; i += 64) ys[i] = 0.0;
        acc = nb;
    };
    auto add = [&](const Bat<U> &B) {
#pragma unroll
        for (int u = 0; u < U; ++u) atomicAdd(&ys[(B.s[u >> 1] >> (16 * (u & 1))) & 0xFFFFu], B.v[u]);
    };
    Bat<U> PA, PB;
    Tab<V, U> TA, TB;
    int64_t b0 = 0, g0 = 0, p0 = 0, b1 = 0, g1 = 0, p1 = 0, b2 = 0, g2 = 0, p2 = 0, b3 = 0, g3 = 0, p3 = 0;
    bool h0 = next(b0, g0, p0);
    bool h1 = h0 && next(b1, g1, p1);
    if (h0) ldtab<V, U>(TA, g, g0, lane);
    if (h1) ldtab<V, U>(TB, g, g1, lane);
    if (h0) ldprod<V, U>(PA, TA, g, g0, p0, lane);
    while (h0) {
        const bool h2 = h1 && next(b2, g2, p2);
        if (h2) ldtab<V, U>(TA, g, g2, lane);
        if (h1) ldprod<V, U>(PB, TB, g, g1, p1, lane);
        begin(b0);
        add(PA);
        if (!h1) break;
        const bool h3 = h2 && next(b3, g3, p3);
        if (h3) ldtab<V, U>(TB, g, g3, lane);
        if (h2) ldprod<V, U>(PA, TA, g, g2, p2, lane);
        begin(b1);
        add(PB);
        h0 = h2;
        b0 = b2;
        g0 = g2;
        p0 = p2;
        h1 = h3;
        b1 = b3;
        g1 = g3;
        p1 = p3;
    }
    if (acc >= 0) finish();
}

static inline int64_t pad8(int64_t v) { return (v + 7) & ~7LL; }

int main(int argc, char **argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s S NB mean m [mulpad]\n", argv[0]);
        return 2;
    }
    const int64_t S = atoll(argv[1]), NB = atoll(argv[2]), m = atoll(argv[4]);
    const double mean = atof(argv[3]);
    const int mulpad = argc > 5 ? atoi(argv[5]) : 0;
    const int64_t rpb = (m + NB - 1) / NB;
    if (rpb > DUMMY) {
        std::fprintf(stderr, "rows per bin %lld > %d\n", (long long)rpb, DUMMY);
        return 2;
    }
    std::mt19937_64 rng(1);
    std::poisson_distribution<int> pd(mean);
    std::vector<int32_t> L((size_t)(S * NB));
    int64_t nnz = 0;
    for (auto &l : L) nnz += (l = pd(rng));
    // Mul order [s][b]; Sum order [b][s] with 8-entry segment padding
    std::vector<int64_t> Bpos((size_t)(S * NB)), Vb((size_t)NB, 0), pstart((size_t)NB + 1, 0);
    int64_t mo = 0;
    for (int64_t s = 0; s < S; ++s)
        for (int64_t b = 0; b < NB; ++b) {
            Bpos[(size_t)(s * NB + b)] = mo;
            mo += mulpad ? pad8(L[(size_t)(s * NB + b)]) : L[(size_t)(s * NB + b)];
            Vb[(size_t)b] += pad8(L[(size_t)(s * NB + b)]);
        }
    for (int64_t b = 0; b < NB; ++b) pstart[(size_t)b + 1] = pstart[(size_t)b] + Vb[(size_t)b];
    const int64_t VA = pstart[(size_t)NB], slack = 4096;
    std::fprintf(stderr, "nnz %lld, Sum-order entries %lld, Mul-order entries %lld\n", (long long)nnz, (long long)VA,
                 (long long)mo);
    auto f = [](int64_t mp) { return (double)(mp % 13 + 1); };
    // row slot of every real entry, drawn once (the same rows for every layout)
    std::vector<uint16_t> rowof((size_t)nnz);
    {
        std::mt19937_64 r2(7);
        int64_t i = 0;
        for (int64_t b = 0; b < NB; ++b) {
            const int rows = (int)std::min<int64_t>(rpb, m - b * rpb);
            for (int64_t s = 0; s < S; ++s)
                for (int k = 0; k < L[(size_t)(s * NB + b)]; ++k) rowof[(size_t)i++] = (uint16_t)(r2() % rows);
        }
    }
    // exact y
    std::vector<double> yref((size_t)m, 0.0);
    {
        int64_t i = 0;
        for (int64_t b = 0; b < NB; ++b)
            for (int64_t s = 0; s < S; ++s)
                for (int k = 0; k < L[(size_t)(s * NB + b)]; ++k)
                    yref[(size_t)(b * rpb + rowof[(size_t)i++])] += f(Bpos[(size_t)(s * NB + b)] + k);
    }
    double *dA, *dB, *dy;
    CHECK(hipMalloc(&dA, (VA + slack) * 8));
    CHECK(hipMalloc(&dB, (mo + slack) * 8));
    CHECK(hipMalloc(&dy, m * 8));
    {
        std::vector<double> hA((size_t)(VA + slack), 0.0), hB((size_t)(mo + slack), 0.0);
        for (int64_t b = 0; b < NB; ++b) {
            int64_t v = pstart[(size_t)b];
            for (int64_t s = 0; s < S; ++s) {
                const int l = L[(size_t)(s * NB + b)];
                for (int k = 0; k < l; ++k) {
                    hA[(size_t)(v + k)] = f(Bpos[(size_t)(s * NB + b)] + k);
                    hB[(size_t)(Bpos[(size_t)(s * NB + b)] + k)] = f(Bpos[(size_t)(s * NB + b)] + k);
                }
                v += pad8(l);
            }
        }
        CHECK(hipMemcpy(dA, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dB, hB.data(), hB.size() * 8, hipMemcpyHostToDevice));
    }
    hipEvent_t ea, eb;
    CHECK(hipEventCreate(&ea));
    CHECK(hipEventCreate(&eb));
    auto run = [&](int V, int U, auto kern) {
        const int64_t BS = 64 * U;
        std::vector<int64_t> bat_off((size_t)NB + 1, 0);
        for (int64_t b = 0; b < NB; ++b) bat_off[(size_t)b + 1] = bat_off[(size_t)b] + (Vb[(size_t)b] + BS - 1) / BS;
        const int64_t G = bat_off[(size_t)NB];
        std::vector<uint16_t> slot((size_t)(G * BS), (uint16_t)DUMMY);
        std::vector<int32_t> tab((size_t)(G * 8 * U), 0);
        int64_t i = 0;
        for (int64_t b = 0; b < NB; ++b) {
            int64_t v = 0;
            for (int64_t s = 0; s < S; ++s) {
                const int l = L[(size_t)(s * NB + b)];
                for (int k = 0; k < pad8(l); ++k, ++v) {
                    const int64_t gb = bat_off[(size_t)b] + v / BS, r = v % BS;
                    const int u = V == 3 ? (int)(r % U) : (int)(r / 64), ln = V == 3 ? (int)(r / U) : (int)(r % 64);
                    if (k < l) slot[(size_t)(gb * BS + (u >> 3) * 512 + ln * 8 + (u & 7))] = rowof[(size_t)i++];
                    if (k % 8 == 0) {
                        const int64_t c = r / 8, base = Bpos[(size_t)(s * NB + b)] + k;
                        size_t at;
                        if (V == 1) at = (size_t)(c % 8) * U + (size_t)(c / 8);
                        else if (V == 2) at = (size_t)(c % 64) * (U / 8) + (size_t)(c / 64);
                        else at = (size_t)c;
                        tab[(size_t)(gb * 8 * U) + at] = (int32_t)base;
                    }
                }
            }
        }
        int64_t *dbo, *dps;
        uint16_t *ds;
        int32_t *dt;
        CHECK(hipMalloc(&dbo, bat_off.size() * 8));
        CHECK(hipMalloc(&dps, pstart.size() * 8));
        CHECK(hipMalloc(&ds, slot.size() * 2));
        CHECK(hipMalloc(&dt, tab.size() * 4));
        CHECK(hipMemcpy(dbo, bat_off.data(), bat_off.size() * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dps, pstart.data(), pstart.size() * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(ds, slot.data(), slot.size() * 2, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dt, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
        Geo g{dbo, dps, dt, ds, V == 0 ? dA : dB, dy, NB, rpb, m};
        CHECK(hipMemset(dy, 0xFF, m * 8));
        kern<<<256, 64 * W2>>>(g);
        CHECK(hipDeviceSynchronize());
        std::vector<double> yh((size_t)m);
        CHECK(hipMemcpy(yh.data(), dy, m * 8, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t r = 0; r < m; ++r) bad += yh[(size_t)r] != yref[(size_t)r];
        float best = 1e30f, sum = 0;
        for (int r = 0; r < 7; ++r) {
            CHECK(hipEventRecord(ea));
            kern<<<256, 64 * W2>>>(g);
            CHECK(hipEventRecord(eb));
            CHECK(hipEventSynchronize(eb));
            float ms;
            CHECK(hipEventElapsedTime(&ms, ea, eb));
            best = std::min(best, ms);
            sum += ms;
        }
        std::printf(
            "{\"var\": %d, \"U\": %d, \"S\": %lld, \"NB\": %lld, \"mean\": %.1f, \"mulpad\": %d, \"nnz\": %lld, "
            "\"sum_entries\": %lld, \"mul_entries\": %lld, \"ms\": %.4f, \"mean_ms\": %.4f, \"y_mismatch\": %lld}\n",
            V, U, (long long)S, (long long)NB, mean, mulpad, (long long)nnz, (long long)VA, (long long)mo, best,
            sum / 7, (long long)bad);
        std::fflush(stdout);
        CHECK(hipFree(dbo));
        CHECK(hipFree(dps));
        CHECK(hipFree(ds));
        CHECK(hipFree(dt));
    };
    for (int rep = 0; rep < 2; ++rep) {
        run(0, 32, sum_probe<0, 32>);
        run(1, 16, sum_probe<1, 16>);
        run(1, 32, sum_probe<1, 32>);
        run(2, 32, sum_probe<2, 32>);
        run(3, 32, sum_probe<3, 32>);
        run(2, 16, sum_probe<2, 16>);
    }
    CHECK(hipFree(dA));
    CHECK(hipFree(dB));
    CHECK(hipFree(dy));
    return 0;
}

// sum1w_probe.hip -- can ONE wave per CU run BIN's Sum at stream speed?
// The wide rank shapes (10 M x N*10 M, N >= 4) get short Mul segments from
// the two-wave Sum's 10239-row bins; one wave per workgroup would allow
// 20479-row bins (segments twice as long), but that Sum ran 0.57 ms against
// 0.35 (profiles/round1/README.md §4a).  This probe streams products (8 B) + row slots (2 B, read
// 8 per 16-byte load) per wave, two 64x32-entry batches in flight, and adds
// each product into a 20479-double LDS slice with ds_add_f64:
//   slots "random"  : uniform over the slice (bank conflicts as in the Sum)
//   slots "lane"    : slot = 64*k + lane (every lane its own bank pair)
//   slots "none"    : no adds (stream only)
// (slots < 5120 so every slice size fits them; banks depend on slot mod 32.)
// Output: one JSON line per (waves per CU, slot pattern): GB/s of the
// product + slot bytes.
//   hipcc -O3 --offload-arch=gfx950 -o bin/sum1w_probe tools/sum1w_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

constexpr int U = 32;
constexpr int LDSD = 20480;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int W, bool ADD>
__global__ __launch_bounds__(64 * W) void sum1w(const double *__restrict__ prod, const uint16_t *__restrict__ slot,
                                              long long n, double *__restrict__ out) {
    __shared__ double ylds[LDSD];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int SLICE = LDSD / W;
    double *ys = ylds + w * SLICE;
    for (int i = lane; i < SLICE; i += 64) ys[i] = 0.0;
    const long long waves = (long long)gridDim.x * W, wid = blockIdx.x * (long long)W + w;
    const long long step = 64LL * U, nb = n / (waves * step);
    double A[U], B[U];
    uint32_t sa[U / 2], sb[U / 2];
    auto load = [&](double *v, uint32_t *sw, long long j) {
        const long long base = (wid * nb + j) * step;
        const u32x4 *sp = reinterpret_cast<const u32x4 *>(slot + base + lane * 8);
#pragma unroll
        for (int q = 0; q < U / 8; ++q) {
            const u32x4 t = __builtin_nontemporal_load(sp + q * 64);
            sw[4 * q] = t.x;
            sw[4 * q + 1] = t.y;
            sw[4 * q + 2] = t.z;
            sw[4 * q + 3] = t.w;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(prod + base + u * 64 + lane);
    };
    double sink = 0;
    auto add = [&](const double *v, const uint32_t *sw) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t s = (sw[u >> 1] >> (16 * (u & 1))) & 0xFFFFu;
            if (ADD) atomicAdd(&ys[s], v[u]);
            else sink += v[u] * (double)s;
        }
    };
    load(A, sa, 0);
    for (long long j = 0; j < nb; j += 2) {
        if (j + 1 < nb) load(B, sb, j + 1);
        add(A, sa);
        if (j + 1 < nb) {
            if (j + 2 < nb) load(A, sa, j + 2);
            add(B, sb);
        }
    }
    if (sink == 1.2345) ys[0] = sink;
    __syncthreads();
    double s = 0;
    for (int i = lane; i < SLICE; i += 64) s += ys[i];
    if (s == 1.2345) out[0] = s;
}

int main() {
    const long long n = 7LL << 25;  // 235 M entries: 1.75 GB of products, 0.44 GB of slots
    double *prod, *out;
    uint16_t *slot;
    CHECK(hipMalloc(&prod, n * 8));
    CHECK(hipMalloc(&slot, n * 2));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(prod, 0, n * 8));
    std::vector<uint16_t> h((size_t)n);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int pat = 0; pat < 2; ++pat) {
        // slot words are read 8 per lane per 16-byte load: entry (u, lane) of a
        // batch sits at base + (u/8)*512 + lane*8 + u%8, so "lane" = slot
        // 64*k + lane for the entry's lane, "random" = a hash
        uint64_t z = 12345;
        for (long long i = 0; i < n; ++i) {
            const long long r = i % (64LL * U), lane = (r % 512) / 8;
            z = z * 6364136223846793005ull + 1442695040888963407ull;
            h[(size_t)i] = pat == 0 ? (uint16_t)((z >> 33) % 5119) : (uint16_t)(((z >> 33) % 79) * 64 + lane);
        }
        CHECK(hipMemcpy(slot, h.data(), n * 2, hipMemcpyHostToDevice));
        auto run = [&](const char *name, int wpc, auto launch) {
            launch();
            CHECK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int r = 0; r < 5; ++r) {
                CHECK(hipEventRecord(a));
                launch();
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            std::printf("{\"slots\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.4f, \"gbs\": %.0f}\n", name, wpc, best,
                        n * 10.0 / best / 1e6);
            std::fflush(stdout);
        };
        const char *nm = pat == 0 ? "random" : "lane";
        run(nm, 1, [&] { sum1w<1, true><<<256, 64>>>(prod, slot, n, out); });
        run(nm, 2, [&] { sum1w<2, true><<<256, 128>>>(prod, slot, n, out); });
        run(nm, 4, [&] { sum1w<4, true><<<256, 256>>>(prod, slot, n, out); });
        if (pat == 0) {
            run("none", 1, [&] { sum1w<1, false><<<256, 64>>>(prod, slot, n, out); });
            run("none", 4, [&] { sum1w<4, false><<<256, 256>>>(prod, slot, n, out); });
        }
    }
    CHECK(hipFree(prod));
    CHECK(hipFree(slot));
    CHECK(hipFree(out));
    return 0;
}

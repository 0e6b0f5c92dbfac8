// mall_probe.hip -- does the MI355X Infinity Cache (MALL, 256 MB) serve
// re-reads and read-after-write of a buffer that fits in it?  Decides whether
// the BIN format's product round trip (Mul writes, Sum reads) can be kept off
// HBM by cutting the rows into groups whose products fit in the MALL.
//
//   e1: read GB/s vs buffer size (16 MB .. 2 GB), 10 back-to-back launches,
//       default and nontemporal loads
//   e2: write S bytes (default / nontemporal stores), then read them; read
//       time vs the same read after a 2 GB flush read
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void rd(const f64x2 *__restrict__ a, long long n2, double *__restrict__ out) {
    double s = 0;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
        f64x2 v = NT ? __builtin_nontemporal_load(a + i) : a[i];
        s += v.x + v.y;
    }
    if (s == 1.2345) out[0] = s;
}

template <bool NT>
__global__ __launch_bounds__(256) void wr(f64x2 *__restrict__ a, long long n2, double v) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
        f64x2 t = {v, v + i};
        if (NT) __builtin_nontemporal_store(t, a + i);
        else a[i] = t;
    }
}

int main() {
    const long long big = 2LL << 30;
    f64x2 *buf, *flush;
    double *out;
    CHECK(hipMalloc(&buf, big));
    CHECK(hipMalloc(&flush, big));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 0, big));
    CHECK(hipMemset(flush, 0, big));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int grid = 256 * 16;
    auto t_of = [&](auto launch, int reps) {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms / reps;
    };
    const long long sizes[] = {16LL << 20, 32LL << 20, 64LL << 20, 128LL << 20, 192LL << 20, 256LL << 20,
                               512LL << 20, 2LL << 30};
    for (long long S : sizes) {
        const long long n2 = S / 16;
        float t0 = t_of([&] { rd<false><<<grid, 256>>>(buf, n2, out); }, 10);
        float t1 = t_of([&] { rd<true><<<grid, 256>>>(buf, n2, out); }, 10);
        std::printf("{\"e\": 1, \"mb\": %lld, \"read_gbs\": %.0f, \"read_nt_gbs\": %.0f}\n", S >> 20, S / t0 / 1e6,
                    S / t1 / 1e6);
    }
    for (long long S : sizes) {
        const long long n2 = S / 16;
        for (int mode = 0; mode < 4; ++mode) {  // bit0: NT store, bit1: NT load
            const bool nts = mode & 1, ntl = mode & 2;
            float tw = 0, tr = 0, trc = 0;
            const int reps = 5;
            for (int r = 0; r < reps; ++r) {
                CHECK(hipEventRecord(a));
                if (nts) wr<true><<<grid, 256>>>(buf, n2, 1.0 + r);
                else wr<false><<<grid, 256>>>(buf, n2, 1.0 + r);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                tw += ms;
                CHECK(hipEventRecord(a));
                if (ntl) rd<true><<<grid, 256>>>(buf, n2, out);
                else rd<false><<<grid, 256>>>(buf, n2, out);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                CHECK(hipEventElapsedTime(&ms, a, b));
                tr += ms;
                rd<true><<<grid, 256>>>(flush, big / 16, out);  // evict
                CHECK(hipEventRecord(a));
                if (ntl) rd<true><<<grid, 256>>>(buf, n2, out);
                else rd<false><<<grid, 256>>>(buf, n2, out);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                CHECK(hipEventElapsedTime(&ms, a, b));
                trc += ms;
            }
            std::printf("{\"e\": 2, \"mb\": %lld, \"nt_store\": %d, \"nt_load\": %d, \"write_gbs\": %.0f, "
                        "\"read_after_write_gbs\": %.0f, \"read_cold_gbs\": %.0f}\n",
                        S >> 20, (int)nts, (int)ntl, S / (tw / reps) / 1e6, S / (tr / reps) / 1e6,
                        S / (trc / reps) / 1e6);
        }
    }
    return 0;
}

// copy_probe.hip -- the HBM's mixed read + write rate: a copy kernel (16-byte
// loads, 16-byte stores, grid-stride) over R bytes read and W bytes written,
// W/R = 1 (copy) and 0.75 (BIN's Mul: 1.71 GB read, 1.31 GB written at
// config 2), with nontemporal or plain stores.  Output: GB/s of R + W.
//   hipcc -O3 --offload-arch=gfx950 -o bin/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

typedef double f64x2 __attribute__((ext_vector_type(2)));

// every thread reads 4 vectors of `a` and writes `wr` of them (of 4) to `b`
template <bool NT, int WR>
__global__ __launch_bounds__(256) void copyk(const f64x2 *__restrict__ a, f64x2 *__restrict__ b, long long n2,
                                             double *__restrict__ sink) {
    const long long G = (long long)gridDim.x * 256;
    double acc = 0.0;  // keeps the loads that are not stored live
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += G * 4) {
        f64x2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long long j = i + u * G;
            v[u] = j < n2 ? __builtin_nontemporal_load(a + j) : f64x2{0.0, 0.0};
        }
#pragma unroll
        for (int u = WR; u < 4; ++u) acc += v[u].x + v[u].y;
#pragma unroll
        for (int u = 0; u < WR; ++u) {
            const long long j = i + u * G;
            if (j < n2) {
                if (NT) __builtin_nontemporal_store(v[u], b + j);
                else b[j] = v[u];
            }
        }
    }
    if (acc == 1.2345) sink[0] = acc;
}

int main() {
    const long long bytes = 1792LL << 20;
    const long long n2 = bytes / 16;
    f64x2 *a, *b;
    double *sink;
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMemset(a, 0, bytes));
    CHECK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](const char *name, int wr, auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < 4; ++k) launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms / 4 < best) best = ms / 4;
        }
        const double moved = bytes * (1.0 + wr / 4.0);
        std::printf("{\"kernel\": \"%s\", \"write_frac\": %.2f, \"ms\": %.4f, \"gbs\": %.0f}\n", name, wr / 4.0, best,
                    moved / best / 1e6);
        std::fflush(stdout);
    };
    for (int g : {256 * 8, 256 * 32}) {
        run("copy_nt", 4, [&] { copyk<true, 4><<<g, 256>>>(a, b, n2, sink); });
        run("copy_plain", 4, [&] { copyk<false, 4><<<g, 256>>>(a, b, n2, sink); });
        run("mulmix_nt", 3, [&] { copyk<true, 3><<<g, 256>>>(a, b, n2, sink); });
        run("read_only", 0, [&] { copyk<true, 0><<<g, 256>>>(a, b, n2, sink); });
    }
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    return 0;
}

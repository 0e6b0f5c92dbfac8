// region_probe.hip -- is the BIN Mul / DIA "slow placement"  a
// property of physical HBM regions, and which access patterns feel it?
//
// Allocates the device memory in equal chunks (hipMalloc, in order, until
// `keep_free` GB remain) and measures each chunk with three kernels:
//   read     16-byte nontemporal loads, grid-stride (the DIA / Sum shape)
//   write    16-byte nontemporal stores, grid-stride
//   scatter  128-byte lines written by 16 lanes of 8 B (the Mul's product
//            lines) at line index (i * P) mod lines -- every line once, in
//            no regular stride
// One JSON line per chunk: {"chunk", "va", "read_gbs", "write_gbs",
// "scatter_gbs"}, best of `reps` launches each.
//
//   region_probe [chunk_mb=1024] [keep_free_gb=16] [reps=3] [max_chunks=400]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

__global__ __launch_bounds__(256) void rd(const f64x2 *__restrict__ a, long long n2, double *__restrict__ out) {
    double s = 0;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
        const f64x2 v = __builtin_nontemporal_load(a + i);
        s += v.x + v.y;
    }
    if (s == 1.2345) out[0] = s;
}

__global__ __launch_bounds__(256) void wr(f64x2 *__restrict__ a, long long n2, double v) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
        const f64x2 t = {v, v + (double)i};
        __builtin_nontemporal_store(t, a + i);
    }
}

// lines of 16 doubles; thread t handles line (t / 16) of each step, lane t % 16
__global__ __launch_bounds__(256) void scat(double *__restrict__ a, long long lines, long long P, double v) {
    const long long nthr = (long long)gridDim.x * 256;
    for (long long i = (blockIdx.x * 256LL + threadIdx.x) >> 4; i < lines; i += nthr >> 4) {
        const long long L = (long long)(((unsigned __int128)i * (unsigned long long)P) % (unsigned long long)lines);
        __builtin_nontemporal_store(v, a + L * 16 + (threadIdx.x & 15));
    }
}

int main(int argc, char **argv) {
    const long long chunk = (argc > 1 ? std::atoll(argv[1]) : 1024) << 20;
    const long long keep = (argc > 2 ? std::atoll(argv[2]) : 16) << 30;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 3;
    const int maxc = argc > 4 ? std::atoi(argv[4]) : 400;
    double *out;
    CHECK(hipMalloc(&out, 64));
    std::vector<void *> ch;
    for (int i = 0; i < maxc; ++i) {
        size_t fr = 0, tot = 0;
        CHECK(hipMemGetInfo(&fr, &tot));
        if ((long long)fr < chunk + keep) break;
        void *p = nullptr;
        if (hipMalloc(&p, chunk) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        ch.push_back(p);
    }
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int grid = 256 * 16;
    auto best = [&](auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        float bms = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (ms < bms) bms = ms;
        }
        return bms;
    };
    const long long n2 = chunk / 16, lines = chunk / 128;
    long long P = (long long)(0.6180339887 * (double)lines) | 1;
    while (lines % P == 0) P += 2;  // lines is a power of two for MB-sized chunks: any odd P is coprime
    for (size_t i = 0; i < ch.size(); ++i) {
        f64x2 *c = (f64x2 *)ch[i];
        const float tw = best([&] { wr<<<grid, 256>>>(c, n2, 1.0); });
        const float tr = best([&] { rd<<<grid, 256>>>(c, n2, out); });
        const float ts = best([&] { scat<<<grid, 256>>>((double *)c, lines, P, 2.0); });
        std::printf("{\"chunk\": %zu, \"mb\": %lld, \"va\": \"%p\", \"read_gbs\": %.0f, \"write_gbs\": %.0f, "
                    "\"scatter_gbs\": %.0f}\n",
                    i, chunk >> 20, ch[i], chunk / tr / 1e6, chunk / tw / 1e6, chunk / ts / 1e6);
        std::fflush(stdout);
    }
    for (void *p : ch) CHECK(hipFree(p));
    return 0;
}

// stream_shape_probe.hip -- does it matter for HBM read bandwidth whether the
// waves of a kernel read ONE moving window (grid-stride, like the STREAM probe
// and DIA's blocked layout) or each wave its own contiguous region (like
// BIN's Sum: one wave per bin, the bins' product runs far apart)?
//
// Every shape reads the same 1.75 GB of doubles with nontemporal loads:
//   grid   : grid-stride over the whole buffer, 8-B loads, U in flight per lane
//   region : W waves (256-thread workgroups x 4), wave w reads its own
//            contiguous 1/W of the buffer in batches of 64*U entries
//            (entry base + u*64 + lane) -- the Sum's access pattern
//   chunk  : the same per-wave batches, but batch j of wave w sits at
//            (j*W + w)*64*U: all waves read one moving window of W batches
// Output: one JSON line per (shape, U, waves).
//   hipcc -O3 --offload-arch=gfx950 -o bin/stream_shape_probe tools/stream_shape_probe.hip
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

// SHAPE 0 grid, 1 region, 2 chunk.  n = doubles in the buffer (a multiple of
// W*64*U for shapes 1 and 2).
template <int SHAPE, int U>
__global__ __launch_bounds__(256) void rd(const double *__restrict__ a, long long n, double *__restrict__ out) {
    double s = 0;
    if (SHAPE == 0) {
        const long long G = (long long)gridDim.x * 256;
        for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += G * U) {
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long long j = i + u * G;
                v[u] = j < n ? __builtin_nontemporal_load(a + j) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) s += v[u];
        }
    } else {
        const long long W = (long long)gridDim.x * 4;
        const long long w = blockIdx.x * 4LL + (threadIdx.x >> 6);
        const int lane = threadIdx.x & 63;
        const long long step = 64LL * U, nb = n / (W * step);  // batches per wave
        for (long long j = 0; j < nb; ++j) {
            const long long base = SHAPE == 1 ? (w * nb + j) * step : (j * W + w) * step;
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + base + u * 64 + lane);
#pragma unroll
            for (int u = 0; u < U; ++u) s += v[u];
        }
    }
    if (s == 1.2345) out[0] = s;
}

// one wave per workgroup (one per CU), its own region, two batches in flight
// (ping-pong, like the Sum); VEC: 16-byte loads (lane l reads entries 2l, 2l+1
// of every 128-entry block) instead of 8-byte ones
template <int U, bool VEC>
__global__ __launch_bounds__(64) void rd1(const double *__restrict__ a, long long n, double *__restrict__ out) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    const long long W = gridDim.x, w = blockIdx.x;
    const int lane = threadIdx.x;
    const long long step = 64LL * U, nb = n / (W * step);
    double s = 0;
    double A[U], B[U];
    auto load = [&](double *v, long long j) {
        const long long base = (w * nb + j) * step;
        if (VEC) {
#pragma unroll
            for (int u = 0; u < U; u += 2) {
                const f64x2 t = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(a + base + (u / 2) * 128 + 2 * lane));
                v[u] = t.x;
                v[u + 1] = t.y;
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + base + u * 64 + lane);
        }
    };
    load(A, 0);
    for (long long j = 0; j < nb; j += 2) {
        if (j + 1 < nb) load(B, j + 1);
#pragma unroll
        for (int u = 0; u < U; ++u) s += A[u];
        if (j + 1 < nb) {
            if (j + 2 < nb) load(A, j + 2);
#pragma unroll
            for (int u = 0; u < U; ++u) s += B[u];
        }
    }
    if (s == 1.2345) out[0] = s;
}

int main() {
    const long long bytes = 1792LL << 20;  // 1.75 GB: 7 * 2^28, divisible by every W*64*U below
    const long long n = bytes / 8;
    double *buf, *out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 0, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto t_of = [&](auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CHECK(hipEventRecord(a));
            for (int k = 0; k < 4; ++k) launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (ms / 4 < best) best = ms / 4;
        }
        return best;
    };
    auto report = [&](const char *shape, int U, long long waves, float ms) {
        std::printf("{\"shape\": \"%s\", \"U\": %d, \"waves\": %lld, \"ms\": %.4f, \"gbs\": %.0f}\n", shape, U, waves,
                    ms, bytes / ms / 1e6);
        std::fflush(stdout);
    };
    report("grid", 4, 256 * 16 * 4, t_of([&] { rd<0, 4><<<256 * 16, 256>>>(buf, n, out); }));
    report("grid", 8, 256 * 16 * 4, t_of([&] { rd<0, 8><<<256 * 16, 256>>>(buf, n, out); }));
    report("grid", 32, 256 * 4, t_of([&] { rd<0, 32><<<256, 256>>>(buf, n, out); }));
    for (int wg : {256, 512}) {
        const long long W = wg * 4LL;
        report("region", 32, W, t_of([&] { rd<1, 32><<<wg, 256>>>(buf, n, out); }));
        report("chunk", 32, W, t_of([&] { rd<2, 32><<<wg, 256>>>(buf, n, out); }));
        report("region", 16, W, t_of([&] { rd<1, 16><<<wg, 256>>>(buf, n, out); }));
        report("chunk", 16, W, t_of([&] { rd<2, 16><<<wg, 256>>>(buf, n, out); }));
    }
    // one wave per CU (the one-wave Sum of 20479-row bins)
    report("region1w", 32, 256, t_of([&] { rd1<32, false><<<256, 64>>>(buf, n, out); }));
    report("region1w_vec", 32, 256, t_of([&] { rd1<32, true><<<256, 64>>>(buf, n, out); }));
    report("region1w", 64, 256, t_of([&] { rd1<64, false><<<256, 64>>>(buf, n, out); }));
    report("region1w_vec", 64, 256, t_of([&] { rd1<64, true><<<256, 64>>>(buf, n, out); }));
    report("region2w_vec", 32, 512, t_of([&] { rd1<32, true><<<512, 64>>>(buf, n, out); }));
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}

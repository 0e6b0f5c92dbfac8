// k_probe.hip -- the measured STREAM-read ceiling SURVEY §8(d) asks bench.py
// to report beside the 8 TB/s spec: a nontemporal 16-byte-per-lane read of
// a buffer far larger than the 256 MB MALL, timed with HIP events.
#include "device.hpp"
#include "internal.hpp"

namespace spmv {
namespace {

__global__ __launch_bounds__(256) void stream_read_kernel(const f64x2 *__restrict__ a, int64_t n2,
                                                          double *__restrict__ sink) {
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += G * 4) {
        f64x2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t j = i + u * G;
            v[u] = j < n2 ? __builtin_nontemporal_load(a + j) : f64x2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x + v[u].y;
    }
    if (acc == 12345.678) *sink = acc;  // keeps the loads live; never true for a zeroed buffer
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void gather_idx_kernel(int32_t *__restrict__ idx, int64_t n, int64_t tab_elems) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        idx[i] = (int32_t)(mix64((uint64_t)i) % (uint64_t)tab_elems);
}

// the same read, one 16-byte load per thread per step (the faster shape on
// some boxes: tools/mall_probe.hip e1 read 2 GB at 6.8 TB/s this way)
__global__ __launch_bounds__(256) void stream_read1_kernel(const f64x2 *__restrict__ a, int64_t n2,
                                                           double *__restrict__ sink) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        const f64x2 v = __builtin_nontemporal_load(a + i);
        acc += v.x + v.y;
    }
    if (acc == 1.2345) sink[0] = acc;
}

// streamed 4-byte indices, 8-byte gathers, 8 in flight per lane
__global__ __launch_bounds__(256) void gather_rate_kernel(const int32_t *__restrict__ idx, const double *__restrict__ tab,
                                                          int64_t n, double *__restrict__ sink) {
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += G * 8) {
        int32_t c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t j = i + u * G;
            c[u] = j < n ? __builtin_nontemporal_load(idx + j) : 0;
        }
        double g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) g[u] = tab[c[u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += g[u];
    }
    if (acc == 12345.678) *sink = acc;
}

}  // namespace
}  // namespace spmv

using namespace spmv;

// Measured ceiling of random 8-byte gathers from an L2-resident table (the
// best case a gather-bound SpMV can reach; tools/gather_probe.hip e1).
extern "C" int spmv_gather_probe(int32_t device, int64_t n, int64_t table_bytes, double *g_per_s) {
    SPMV_CHECK_ARG(g_per_s != nullptr && n >= (1 << 20) && n < INT32_MAX && table_bytes >= 4096, "bad arguments");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible");
        return SPMV_ERROR_NO_DEVICE;
    }
    SPMV_CHECK_ARG(device >= 0 && device < count, "device ordinal out of range");
    SPMV_HIP_TRY(hipSetDevice(device));
    const int64_t te = table_bytes / 8;
    int32_t *idx = nullptr;
    double *tab = nullptr, *sink = nullptr;
    SPMV_HIP_TRY(hipMalloc(&idx, 4 * (size_t)n));
    if (hipMalloc(&tab, 8 * (size_t)te) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) {
        (void)hipFree(idx);
        (void)hipFree(tab);
        set_error("hipMalloc failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    (void)hipMemset(tab, 0, 8 * (size_t)te);
    hipLaunchKernelGGL(gather_idx_kernel, dim3(4096), dim3(256), 0, 0, idx, n, te);
    const unsigned blocks = 256 * 8;
    hipLaunchKernelGGL(gather_rate_kernel, dim3(blocks), dim3(256), 0, 0, idx, tab, n, sink);  // warm-up
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    hipError_t e = hipSuccess;
    for (int r = 0; r < 5 && e == hipSuccess; ++r) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(gather_rate_kernel, dim3(blocks), dim3(256), 0, 0, idx, tab, n, sink);
        (void)hipEventRecord(e1, 0);
        e = hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(idx);
    (void)hipFree(tab);
    (void)hipFree(sink);
    if (e != hipSuccess) {
        set_error(std::string("gather probe: ") + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    *g_per_s = (double)n / (best * 1e-3);
    return SPMV_SUCCESS;
}

extern "C" int spmv_stream_probe(int32_t device, int64_t bytes, int32_t iters, double *read_gbs) {
    SPMV_CHECK_ARG(read_gbs != nullptr && bytes >= (1 << 20) && iters > 0, "bad arguments");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible");
        return SPMV_ERROR_NO_DEVICE;
    }
    SPMV_CHECK_ARG(device >= 0 && device < count, "device ordinal out of range");
    SPMV_HIP_TRY(hipSetDevice(device));
    const int64_t n2 = bytes / 16;
    f64x2 *a = nullptr;
    double *sink = nullptr;
    SPMV_HIP_TRY(hipMalloc(&a, (size_t)n2 * 16));
    if (hipMalloc(&sink, 8) != hipSuccess) {
        (void)hipFree(a);
        set_error("hipMalloc failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    (void)hipMemset(a, 0, (size_t)n2 * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const unsigned blocks = 256 * 16;
    // the ceiling is the faster of two read shapes (4 strided loads in flight
    // per thread / one contiguous load per thread)
    float ms = 0;
    hipError_t e = hipSuccess;
    for (int shape = 0; shape < 2 && e == hipSuccess; ++shape) {
        auto launch = [&]() {
            if (shape == 0) hipLaunchKernelGGL(stream_read_kernel, dim3(blocks), dim3(256), 0, 0, a, n2, sink);
            else hipLaunchKernelGGL(stream_read1_kernel, dim3(blocks), dim3(256), 0, 0, a, n2, sink);
        };
        launch();  // warm-up
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < iters; ++i) launch();
        (void)hipEventRecord(e1, 0);
        e = hipEventSynchronize(e1);
        float t = 0;
        (void)hipEventElapsedTime(&t, e0, e1);
        if (shape == 0 || t < ms) ms = t;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(sink);
    if (e != hipSuccess) {
        set_error(std::string("stream probe: ") + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    *read_gbs = (double)n2 * 16 * iters / (ms * 1e-3) / 1e9;
    return SPMV_SUCCESS;
}

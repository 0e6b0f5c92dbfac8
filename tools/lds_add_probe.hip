// lds_add_probe.hip -- how fast does a CU add f64 values into LDS slots?
// BIN's Sum adds every product into its wave's LDS y slice with ds_add_f64
// (167.5 M adds per execute at config 2, ~0.92 adds per clock per CU at the
// Sum's 0.298 ms).  Each workgroup = 4 waves, each owning a 5120-double slice
// (160 KB, one workgroup per CU, the Sum's shape); every wave issues ITERS x
// 32 instructions over slots from a hash (no memory traffic).
//   atomic      : atomicAdd(&ys[slot], v)  -> ds_add_f64
//   rmw         : ys[slot] = ys[slot] + v  -> ds_read_b64 + v_add_f64 + ds_write_b64
//                 (loses updates when lanes collide; timing only)
//   atomic_lane : ds_add_f64 with slot = 64*k + lane (no two lanes on one bank pair)
//   read        : ds_read_b64 only
// Output: one JSON line per variant: adds/s per CU and cycles per instruction.
//   hipcc -O3 --offload-arch=gfx950 -o bin/lds_add_probe tools/lds_add_probe.hip
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

constexpr int SLICE = 5120;
constexpr int ITERS = 2048;

__device__ __forceinline__ uint32_t hash32(uint32_t z) {
    z ^= z >> 16;
    z *= 0x7feb352dU;
    z ^= z >> 15;
    z *= 0x846ca68bU;
    z ^= z >> 16;
    return z;
}

template <int V>
__global__ __launch_bounds__(256) void lds_add(double *__restrict__ out, uint32_t seed) {
    __shared__ double ylds[4 * SLICE];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double *ys = ylds + w * SLICE;
    for (int i = lane; i < SLICE; i += 64) ys[i] = 0.0;
    uint32_t h = hash32(seed ^ (blockIdx.x * 256 + threadIdx.x));
    double v = 1.0 + lane * 1e-3, acc = 0.0;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            h = h * 1664525u + 1013904223u;
            const uint32_t slot = V == 2 ? (((h >> 8) & 63) * 64 + lane) : ((h >> 8) & 4095);
            if (V == 0 || V == 2) atomicAdd(&ys[slot], v);
            else if (V == 1) ys[slot] = ys[slot] + v;
            else acc += ys[slot];
        }
    }
    __syncthreads();
    double s = acc;
    for (int i = lane; i < SLICE; i += 64) s += ys[i];
    if (s == 1.2345) out[0] = s;
}

int main() {
    int dev = 0, cus = 0, clk_khz = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
    double *out;
    CHECK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const char *names[] = {"atomic", "rmw", "atomic_lane", "read"};
    for (int v = 0; v < 4; ++v) {
        auto launch = [&] {
            switch (v) {
                case 0: lds_add<0><<<cus * 4, 256>>>(out, 7); break;
                case 1: lds_add<1><<<cus * 4, 256>>>(out, 7); break;
                case 2: lds_add<2><<<cus * 4, 256>>>(out, 7); break;
                default: lds_add<3><<<cus * 4, 256>>>(out, 7); break;
            }
        };
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
        // cus*4 workgroups (4 rounds of one per CU), 4 waves, ITERS*32 instructions of 64 lanes
        const double instr_per_cu = 4.0 * 4 * ITERS * 32;
        const double adds_per_cu = instr_per_cu * 64;
        const double clk_hz = clk_khz * 1e3;
        std::printf("{\"variant\": \"%s\", \"ms\": %.4f, \"adds_per_s_per_cu\": %.3e, \"cycles_per_instr\": %.1f, "
                    "\"clock_mhz\": %.0f, \"cus\": %d}\n",
                    names[v], best, adds_per_cu / (best * 1e-3), best * 1e-3 * clk_hz / instr_per_cu, clk_hz / 1e6,
                    cus);
        std::fflush(stdout);
    }
    CHECK(hipFree(out));
    return 0;
}

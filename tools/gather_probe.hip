// gather_probe.hip -- micro-benchmark of the x-gather that bounds SpMV on
// MI355X (SURVEY §7 hard part 1: "measure first").
//
// Every experiment streams N int32 indices (like col_idx) and gathers 8-byte
// doubles from a table of T bytes (like x), one gather per index, 8 in
// flight per lane, grid-stride so concurrently resident waves sit at nearby
// stream positions.  Reports G gathers/s and the streamed GB/s.
//
//   e1: uniform random indices over T  (T = 1 MB .. 2 GB)
//   e2: T = 80 MB, indices confined to a W-byte window that slides across the
//       table with the stream position (a synchronised column sweep)
//   e3: HBM streaming read ceiling (dwordx4), for calibration
//   e4: small tables (4 KB .. 1 MB): is an L1 (TCP) hit cheaper than an L2 hit?
//   e5: 1 MB table, fewer workgroups: per-CU or chip-wide (L2) bound?
//   e6: 64 MB table, groups of k consecutive lanes read the same 128 B line:
//       does the vector memory path merge same-line lanes of one instruction?
//   e8: 1 MB table, gathers + the CSS entry stream (4 B col + 2 B slot + 8 B
//       value per gather) vs the 4 B index stream alone
//   e9: 1 MB table, gathers issued through the SCALAR cache (readlane + s_load)
//       alone and mixed 1:3 with vector gathers: is it a second request path?
//   e10: e8 with every wave streaming its OWN contiguous segment of the entry
//       arrays (CSS's per-wave lists) instead of the grid-strided layout, in
//       1024-thread workgroups pinned one per CU
//   e7: 1 MB table, one 1024-thread workgroup per CU (LDS-pinned), 256 .. 16
//       CUs: does the per-CU rate rise when fewer CUs share the L2?
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// idx[i] = base(i) + hash(i) % W  where base slides from 0 to T-W over the stream
__global__ void make_idx(int *idx, long long n, long long tab_elems, long long win_elems) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n; i += (long long)gridDim.x * blockDim.x) {
        long long base = (win_elems >= tab_elems) ? 0 : (long long)((double)i / (double)n * (double)(tab_elems - win_elems));
        idx[i] = (int)(base + (long long)(mix((unsigned long long)i) % (unsigned long long)win_elems));
    }
}

// gather<8> in 1024-thread workgroups pinned one per CU by 96 KB of LDS
__global__ __launch_bounds__(1024) void gather_cu(const int *__restrict__ idx, const double *__restrict__ tab,
                                                  double *__restrict__ out, long long n) {
    extern __shared__ double pin[];
    const long long G = (long long)gridDim.x * blockDim.x;
    long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0;
    for (long long i = t; i < n; i += G * 8) {
        int c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            long long j = i + u * G;
            c[u] = j < n ? __builtin_nontemporal_load(idx + j) : 0;
        }
        double g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) g[u] = tab[c[u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += g[u];
    }
    if (threadIdx.x == 0) pin[0] = acc;
    if (acc == 1.2345) out[t] = acc + pin[0];
}

// gather<4> plus an extra 2 B + 8 B stream per gather (the CSS entry shape)
__global__ __launch_bounds__(256) void gather_css_shape(const int *__restrict__ idx, const unsigned short *__restrict__ slot,
                                                        const double *__restrict__ vals, const double *__restrict__ tab,
                                                        double *__restrict__ out, long long n, int with_stream) {
    const long long G = (long long)gridDim.x * blockDim.x;
    long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0;
    for (long long i = t; i < n; i += G * 4) {
        int c[4];
        double v[4];
        int r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            long long j = i + u * G;
            j = j < n ? j : 0;
            c[u] = __builtin_nontemporal_load(idx + j);
            if (with_stream) {
                r[u] = __builtin_nontemporal_load(slot + j);
                v[u] = __builtin_nontemporal_load(vals + j);
            } else {
                r[u] = 1;
                v[u] = 1.0;
            }
        }
        double g[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] = tab[c[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += g[u] * v[u] + r[u];
    }
    if (acc == 1.2345) out[t] = acc;
}

// scalar-path gathers: every lane's index is read into an SGPR and gathered
// with a scalar load; SCAL_OF_4 of every 4 index groups go the scalar way
template <int SCAL_OF_4>
__global__ __launch_bounds__(256) void gather_scalar(const int *__restrict__ idx, const double *__restrict__ tab,
                                                     double *__restrict__ out, long long n) {
    const long long G = (long long)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0;
    for (long long i = t; i < n; i += G * 4) {
        int c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            long long j = i + u * G;
            c[u] = __builtin_nontemporal_load(idx + (j < n ? j : 0));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (u < SCAL_OF_4) {
                double mine = 0;
                for (int k0 = 0; k0 < 64; k0 += 16) {
                    double v[16];
#pragma unroll
                    for (int k = 0; k < 16; ++k) v[k] = tab[__builtin_amdgcn_readlane(c[u], k0 + k)];  // s_load
#pragma unroll
                    for (int k = 0; k < 16; ++k) mine = lane == k0 + k ? v[k] : mine;
                }
                acc += mine;
            } else {
                acc += tab[c[u]];
            }
        }
    }
    if (acc == 1.2345) out[t] = acc;
}

// e10: per-wave contiguous segments, 4 entries per lane per step (CSS shape)
__global__ __launch_bounds__(1024) void gather_segments(const int *__restrict__ idx, const unsigned short *__restrict__ slot,
                                                        const double *__restrict__ vals, const double *__restrict__ tab,
                                                        double *__restrict__ out, long long n) {
    extern __shared__ double pin[];
    const long long waves = (long long)gridDim.x * (blockDim.x / 64);
    const long long w = (long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long long seg = (n + waves - 1) / waves;
    const long long b = w * seg, e = b + seg < n ? b + seg : n;
    double acc = 0;
    for (long long j0 = b; j0 < e; j0 += 256) {
        int c[4], r[4];
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            long long j = j0 + u * 64 + lane;
            j = j < e ? j : b;
            c[u] = __builtin_nontemporal_load(idx + j);
            r[u] = __builtin_nontemporal_load(slot + j);
            v[u] = __builtin_nontemporal_load(vals + j);
        }
        double g[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] = tab[c[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += g[u] * v[u] + r[u];
    }
    if (threadIdx.x == 0) pin[0] = acc;
    if (acc == 1.2345) out[w & 2047] = acc + pin[0];
}

// e11: per-WORKGROUP contiguous segments, the 16 waves taking interleaved
// 256-entry chunks (wave w: chunks w, w+16, ...), 1 WG of 1024 per CU
__global__ __launch_bounds__(1024) void gather_wg_interleaved(const int *__restrict__ idx,
                                                              const unsigned short *__restrict__ slot,
                                                              const double *__restrict__ vals,
                                                              const double *__restrict__ tab, double *__restrict__ out,
                                                              long long n) {
    extern __shared__ double pin[];
    const int nw = blockDim.x / 64;
    const int w = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const long long seg = (n + gridDim.x - 1) / gridDim.x;
    const long long b = (long long)blockIdx.x * seg, e = b + seg < n ? b + seg : n;
    double acc = 0;
    for (long long j0 = b + (long long)w * 256; j0 < e; j0 += (long long)nw * 256) {
        int c[4], r[4];
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            long long j = j0 + u * 64 + lane;
            j = j < e ? j : b;
            c[u] = __builtin_nontemporal_load(idx + j);
            r[u] = __builtin_nontemporal_load(slot + j);
            v[u] = __builtin_nontemporal_load(vals + j);
        }
        double g[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] = tab[c[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += g[u] * v[u] + r[u];
    }
    if (threadIdx.x == 0) pin[0] = acc;
    if (acc == 1.2345) out[blockIdx.x * 16 + w] = acc + pin[0];
}

// e13: chunks interleaved across EVERY wave of the chip (chunk k of wave g at
// (k*W + g)*256): all waves stream one contiguous band, as in e8, but with
// CSS's wave-owned 256-entry chunks; 1 WG of 1024 per CU
__global__ __launch_bounds__(1024) void gather_chip_interleaved(const int *__restrict__ idx,
                                                                const unsigned short *__restrict__ slot,
                                                                const double *__restrict__ vals,
                                                                const double *__restrict__ tab,
                                                                double *__restrict__ out, long long n) {
    extern __shared__ double pin[];
    const long long W = (long long)gridDim.x * (blockDim.x / 64);
    const long long g = (long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    double acc = 0;
    for (long long j0 = g * 256; j0 < n; j0 += W * 256) {
        int c[4], r[4];
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            long long j = j0 + u * 64 + lane;
            j = j < n ? j : 0;
            c[u] = __builtin_nontemporal_load(idx + j);
            r[u] = __builtin_nontemporal_load(slot + j);
            v[u] = __builtin_nontemporal_load(vals + j);
        }
        double gg[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) gg[u] = tab[c[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += gg[u] * v[u] + r[u];
    }
    if (threadIdx.x == 0) pin[0] = acc;
    if (acc == 1.2345) out[g & 2047] = acc + pin[0];
}

// groups of k consecutive indices share one random 128 B line
__global__ void make_idx_lines(int *idx, long long n, long long tab_elems, int k) {
    const long long lines = tab_elems / 16;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n; i += (long long)gridDim.x * blockDim.x)
        idx[i] = (int)((long long)(mix((unsigned long long)(i / k)) % (unsigned long long)lines) * 16 + (i % k));
}

template <int U>
__global__ __launch_bounds__(256) void gather(const int *__restrict__ idx, const double *__restrict__ tab,
                                              double *__restrict__ out, long long n) {
    const long long G = (long long)gridDim.x * blockDim.x;
    long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0;
    for (long long i = t; i < n; i += G * U) {
        int c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long long j = i + u * G;
            c[u] = j < n ? __builtin_nontemporal_load(idx + j) : 0;
        }
        double g[U];
#pragma unroll
        for (int u = 0; u < U; ++u) g[u] = tab[c[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += g[u];
    }
    out[t] = acc;
}

__global__ __launch_bounds__(256) void stream_read(const f64x2 *__restrict__ a, double *__restrict__ out, long long n2) {
    const long long G = (long long)gridDim.x * blockDim.x;
    long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0;
    for (long long i = t; i < n2; i += G * 4) {
        f64x2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            long long j = i + u * G;
            v[u] = j < n2 ? __builtin_nontemporal_load(a + j) : f64x2{0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x + v[u].y;
    }
    out[t] = acc;
}

static float time_gather(const int *idx, const double *tab, double *out, long long n, int blocks) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(gather<8>, dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(gather<8>, dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char **argv) {
    const long long N = argc > 1 ? atoll(argv[1]) : 160000000LL;
    const long long TMAX = 2048LL << 20;
    int *idx;
    double *tab, *out;
    const int blocks = 256 * 8;
    CK(hipMalloc(&idx, sizeof(int) * N));
    CK(hipMalloc(&tab, TMAX));
    CK(hipMalloc(&out, sizeof(double) * blocks * 256));
    CK(hipMemset(tab, 0, TMAX));
    std::printf("{\"N\": %lld, \"e1\": [", N);
    const long long mbs[] = {1, 2, 4, 8, 16, 32, 64, 80, 128, 192, 256, 384, 512, 1024, 2048};
    bool first = true;
    for (long long mb : mbs) {
        const long long te = (mb << 20) / 8;
        hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, N, te, te);
        CK(hipDeviceSynchronize());
        const float ms = time_gather(idx, tab, out, N, blocks);
        std::printf("%s{\"table_MB\": %lld, \"ms\": %.4f, \"Ggather_s\": %.2f}", first ? "" : ", ", mb, ms,
                    N / (ms * 1e-3) / 1e9);
        first = false;
        std::fflush(stdout);
    }
    std::printf("], \"e2\": [");
    first = true;
    const long long te80 = (80LL << 20) / 8;
    const double wins[] = {0.25, 0.5, 1, 2, 4, 8, 16, 80};
    for (double w : wins) {
        const long long we = (long long)(w * (1 << 20)) / 8;
        hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, N, te80, we);
        CK(hipDeviceSynchronize());
        const float ms = time_gather(idx, tab, out, N, blocks);
        std::printf("%s{\"window_MB\": %.2f, \"ms\": %.4f, \"Ggather_s\": %.2f}", first ? "" : ", ", w, ms,
                    N / (ms * 1e-3) / 1e9);
        first = false;
        std::fflush(stdout);
    }
    // e3: streaming read of 2 GB
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const long long n2 = TMAX / 16;
    hipLaunchKernelGGL(stream_read, dim3(blocks), dim3(256), 0, 0, (const f64x2 *)tab, out, n2);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(stream_read, dim3(blocks), dim3(256), 0, 0, (const f64x2 *)tab, out, n2);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    std::printf("], \"e3_stream_GBs\": %.1f", TMAX / (best * 1e-3) / 1e9);
    std::printf(", \"e4\": [");
    first = true;
    const long long kbs[] = {4, 16, 32, 64, 128, 256, 1024};
    for (long long kb : kbs) {
        const long long te = (kb << 10) / 8;
        hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, N, te, te);
        CK(hipDeviceSynchronize());
        const float ms = time_gather(idx, tab, out, N, blocks);
        std::printf("%s{\"table_KB\": %lld, \"ms\": %.4f, \"Ggather_s\": %.2f}", first ? "" : ", ", kb, ms,
                    N / (ms * 1e-3) / 1e9);
        first = false;
        std::fflush(stdout);
    }
    std::printf("], \"e5\": [");
    first = true;
    {
        const long long te = (1LL << 20) / 8;
        hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, N, te, te);
        CK(hipDeviceSynchronize());
        const int bl[] = {256 * 8, 256 * 4, 256, 128, 64, 32};
        for (int nb : bl) {
            const float ms = time_gather(idx, tab, out, N / 4, nb);
            std::printf("%s{\"blocks\": %d, \"ms\": %.4f, \"Ggather_s\": %.2f}", first ? "" : ", ", nb, ms,
                        N / 4 / (ms * 1e-3) / 1e9);
            first = false;
            std::fflush(stdout);
        }
    }
    std::printf("], \"e6\": [");
    first = true;
    {
        const long long te = (64LL << 20) / 8;
        const int ks[] = {1, 2, 4, 8, 16};
        for (int k : ks) {
            hipLaunchKernelGGL(make_idx_lines, dim3(4096), dim3(256), 0, 0, idx, N, te, k);
            CK(hipDeviceSynchronize());
            const float ms = time_gather(idx, tab, out, N, blocks);
            std::printf("%s{\"lanes_per_line\": %d, \"ms\": %.4f, \"Ggather_s\": %.2f}", first ? "" : ", ", k,
                        ms, N / (ms * 1e-3) / 1e9);
            first = false;
            std::fflush(stdout);
        }
    }
    std::printf("], \"e8\": [");
    {
        const long long te = (1LL << 20) / 8;
        const long long n = N;
        hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, n, te, te);
        CK(hipDeviceSynchronize());
        unsigned short *slot;
        double *vals;
        CK(hipMalloc(&slot, 2 * n));
        CK(hipMalloc(&vals, 8 * n));
        CK(hipMemset(slot, 0, 2 * n));
        CK(hipMemset(vals, 0, 8 * n));
        for (int ws = 0; ws < 2; ++ws) {
            hipEvent_t a2, b2;
            CK(hipEventCreate(&a2));
            CK(hipEventCreate(&b2));
            float bm = 1e30f;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a2));
                hipLaunchKernelGGL(gather_css_shape, dim3(blocks), dim3(256), 0, 0, idx, slot, vals, tab, out, n, ws);
                CK(hipEventRecord(b2));
                CK(hipEventSynchronize(b2));
                float ms;
                CK(hipEventElapsedTime(&ms, a2, b2));
                if (r && ms < bm) bm = ms;
            }
            std::printf("%s{\"entry_stream\": %d, \"ms\": %.4f, \"Ggather_s\": %.2f}", ws ? ", " : "", ws, bm,
                        n / (bm * 1e-3) / 1e9);
            std::fflush(stdout);
        }
        // e10: same arrays, per-wave contiguous segments, 1 WG of 1024 per CU
        CK(hipFuncSetAttribute((const void *)gather_segments, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
        {
            hipEvent_t a2, b2;
            CK(hipEventCreate(&a2));
            CK(hipEventCreate(&b2));
            float bm = 1e30f;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a2));
                hipLaunchKernelGGL(gather_segments, dim3(256), dim3(1024), 96 * 1024, 0, idx, slot, vals, tab, out, n);
                CK(hipEventRecord(b2));
                CK(hipEventSynchronize(b2));
                float ms;
                CK(hipEventElapsedTime(&ms, a2, b2));
                if (r && ms < bm) bm = ms;
            }
            std::printf(", {\"per_wave_segments\": 1, \"ms\": %.4f, \"Ggather_s\": %.2f}", bm, n / (bm * 1e-3) / 1e9);
        }
        CK(hipFuncSetAttribute((const void *)gather_wg_interleaved, hipFuncAttributeMaxDynamicSharedMemorySize,
                               96 * 1024));
        {
            hipEvent_t a2, b2;
            CK(hipEventCreate(&a2));
            CK(hipEventCreate(&b2));
            float bm = 1e30f;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a2));
                hipLaunchKernelGGL(gather_wg_interleaved, dim3(256), dim3(1024), 96 * 1024, 0, idx, slot, vals, tab,
                                   out, n);
                CK(hipEventRecord(b2));
                CK(hipEventSynchronize(b2));
                float ms;
                CK(hipEventElapsedTime(&ms, a2, b2));
                if (r && ms < bm) bm = ms;
            }
            std::printf(", {\"per_wg_interleaved\": 1, \"ms\": %.4f, \"Ggather_s\": %.2f}", bm,
                        n / (bm * 1e-3) / 1e9);
        }
        // e12: per-wave segments with TWO 1024-thread workgroups per CU (64 KB LDS each)
        {
            hipEvent_t a2, b2;
            CK(hipEventCreate(&a2));
            CK(hipEventCreate(&b2));
            float bm = 1e30f;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a2));
                hipLaunchKernelGGL(gather_segments, dim3(512), dim3(1024), 64 * 1024, 0, idx, slot, vals, tab, out, n);
                CK(hipEventRecord(b2));
                CK(hipEventSynchronize(b2));
                float ms;
                CK(hipEventElapsedTime(&ms, a2, b2));
                if (r && ms < bm) bm = ms;
            }
            std::printf(", {\"per_wave_segments_2wg_per_cu\": 1, \"ms\": %.4f, \"Ggather_s\": %.2f}", bm,
                        n / (bm * 1e-3) / 1e9);
        }
        CK(hipFuncSetAttribute((const void *)gather_chip_interleaved, hipFuncAttributeMaxDynamicSharedMemorySize,
                               96 * 1024));
        {
            hipEvent_t a2, b2;
            CK(hipEventCreate(&a2));
            CK(hipEventCreate(&b2));
            float bm = 1e30f;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a2));
                hipLaunchKernelGGL(gather_chip_interleaved, dim3(256), dim3(1024), 96 * 1024, 0, idx, slot, vals, tab,
                                   out, n);
                CK(hipEventRecord(b2));
                CK(hipEventSynchronize(b2));
                float ms;
                CK(hipEventElapsedTime(&ms, a2, b2));
                if (r && ms < bm) bm = ms;
            }
            std::printf(", {\"chip_interleaved_chunks\": 1, \"ms\": %.4f, \"Ggather_s\": %.2f}", bm,
                        n / (bm * 1e-3) / 1e9);
        }
        CK(hipFree(slot));
        CK(hipFree(vals));
    }
    std::printf("], \"e9\": [");
    {
        const long long te = (1LL << 20) / 8;
        const long long n = N / 4;
        hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, n, te, te);
        CK(hipDeviceSynchronize());
        for (int mode = 0; mode < 4; ++mode) {
            hipEvent_t a2, b2;
            CK(hipEventCreate(&a2));
            CK(hipEventCreate(&b2));
            float bm = 1e30f;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a2));
                if (mode == 0) hipLaunchKernelGGL(gather_scalar<0>, dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
                else if (mode == 1) hipLaunchKernelGGL(gather_scalar<1>, dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
                else if (mode == 2) hipLaunchKernelGGL(gather_scalar<2>, dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
                else hipLaunchKernelGGL(gather_scalar<4>, dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
                CK(hipEventRecord(b2));
                CK(hipEventSynchronize(b2));
                float ms;
                CK(hipEventElapsedTime(&ms, a2, b2));
                if (r && ms < bm) bm = ms;
            }
            std::printf("%s{\"scalar_of_4\": %d, \"ms\": %.4f, \"Ggather_s\": %.2f}", mode ? ", " : "",
                        mode == 3 ? 4 : mode, bm, n / (bm * 1e-3) / 1e9);
            std::fflush(stdout);
        }
    }
    std::printf("], \"e7\": [");
    first = true;
    {
        const long long te = (1LL << 20) / 8;
        hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, N, te, te);
        CK(hipDeviceSynchronize());
        CK(hipFuncSetAttribute((const void *)gather_cu, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
        const int cus[] = {256, 128, 64, 32, 16};
        for (int nc : cus) {
            const long long n = N / 16;
            hipEvent_t a2, b2;
            CK(hipEventCreate(&a2));
            CK(hipEventCreate(&b2));
            hipLaunchKernelGGL(gather_cu, dim3(nc), dim3(1024), 96 * 1024, 0, idx, tab, out, n);
            CK(hipDeviceSynchronize());
            float bm = 1e30f;
            for (int r = 0; r < 3; ++r) {
                CK(hipEventRecord(a2));
                hipLaunchKernelGGL(gather_cu, dim3(nc), dim3(1024), 96 * 1024, 0, idx, tab, out, n);
                CK(hipEventRecord(b2));
                CK(hipEventSynchronize(b2));
                float ms;
                CK(hipEventElapsedTime(&ms, a2, b2));
                if (ms < bm) bm = ms;
            }
            std::printf("%s{\"cus\": %d, \"ms\": %.4f, \"Ggather_s\": %.2f, \"per_cu_G\": %.3f}",
                        first ? "" : ", ", nc, bm, n / (bm * 1e-3) / 1e9, n / (bm * 1e-3) / 1e9 / nc);
            first = false;
            std::fflush(stdout);
        }
    }
    std::printf("]}\n");
    return 0;
}

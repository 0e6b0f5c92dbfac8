// gather_policy_probe.hip -- does the cache policy of an 8-byte x gather
// change the rate at which L2 (or the Infinity Cache) serves it?
//
// gather_probe.hip e1/e7 measured ~190 G random 8-B gathers/s from an
// L2-resident table with plain loads, i.e. ~0.38 128-B lines per clock per
// CU -- close to a 64 B/clk L2->L1 return path moving whole 128-B lines.
// Loads that bypass L1 (sc1, sc0 sc1, nt: MI355X_MICROARCH.md "stores/loads
// of each flavour") might be served at a smaller granule.  This probe times
// the same random gather with each policy, and with 4-byte gathers, over
// tables of 1, 4, 16, 80 and 512 MB.
//
//   policy 0 plain      global_load_dwordx2
//   policy 1 nt         global_load_dwordx2 ... nt
//   policy 2 sc1        __hip_atomic_load relaxed, agent scope
//   policy 3 sc0 sc1    __hip_atomic_load relaxed, system scope
//   policy 4 plain, 4-byte gathers (float table)
//   policy 5 sc1,  4-byte gathers
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

__global__ void make_idx(int *idx, long long n, long long tab_elems) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n; i += (long long)gridDim.x * blockDim.x)
        idx[i] = (int)(mix((unsigned long long)i) % (unsigned long long)tab_elems);
}

template <int P>
__device__ __forceinline__ double ld(const double *p) {
    if constexpr (P == 1) return __builtin_nontemporal_load(p);
    else if constexpr (P == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if constexpr (P == 3) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else return *p;
}

template <int P>
__device__ __forceinline__ float ldf(const float *p) {
    if constexpr (P == 5) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}

// U gathers in flight per lane, grid-stride over the index stream
template <int P, int U>
__global__ __launch_bounds__(256) void gather(const int *__restrict__ idx, const void *__restrict__ tab,
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
        for (int u = 0; u < U; ++u) {
            if constexpr (P >= 4) g[u] = ldf<P>((const float *)tab + c[u]);
            else g[u] = ld<P>((const double *)tab + c[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += g[u];
    }
    if (acc == 1.2345) out[t] = acc;
}

template <int P, int U>
static float run(const int *idx, const void *tab, double *out, long long n, int blocks) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((gather<P, U>), dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 4; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((gather<P, U>), dim3(blocks), dim3(256), 0, 0, idx, tab, out, n);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return best;
}

int main(int argc, char **argv) {
    const long long N = argc > 1 ? atoll(argv[1]) : 80000000LL;
    const long long TMAX = 512LL << 20;
    int *idx;
    void *tab;
    double *out;
    const int blocks = 256 * 8;
    CK(hipMalloc(&idx, sizeof(int) * N));
    CK(hipMalloc(&tab, TMAX));
    CK(hipMalloc(&out, sizeof(double) * blocks * 256));
    CK(hipMemset(tab, 0, TMAX));
    const long long mbs[] = {1, 4, 16, 80, 512};
    const char *names[] = {"plain", "nt", "sc1", "sc0sc1", "plain_f32", "sc1_f32"};
    std::printf("{\"N\": %lld, \"rows\": [", N);
    bool first = true;
    for (long long mb : mbs) {
        for (int p = 0; p < 6; ++p) {
            const long long te = (mb << 20) / (p >= 4 ? 4 : 8);
            hipLaunchKernelGGL(make_idx, dim3(4096), dim3(256), 0, 0, idx, N, te);
            CK(hipDeviceSynchronize());
            float ms8 = 0, ms16 = 0;
            switch (p) {
            case 0: ms8 = run<0, 8>(idx, tab, out, N, blocks); ms16 = run<0, 16>(idx, tab, out, N, blocks); break;
            case 1: ms8 = run<1, 8>(idx, tab, out, N, blocks); ms16 = run<1, 16>(idx, tab, out, N, blocks); break;
            case 2: ms8 = run<2, 8>(idx, tab, out, N, blocks); ms16 = run<2, 16>(idx, tab, out, N, blocks); break;
            case 3: ms8 = run<3, 8>(idx, tab, out, N, blocks); ms16 = run<3, 16>(idx, tab, out, N, blocks); break;
            case 4: ms8 = run<4, 8>(idx, tab, out, N, blocks); ms16 = run<4, 16>(idx, tab, out, N, blocks); break;
            default: ms8 = run<5, 8>(idx, tab, out, N, blocks); ms16 = run<5, 16>(idx, tab, out, N, blocks); break;
            }
            std::printf("%s\n {\"table_MB\": %lld, \"policy\": \"%s\", \"ms_u8\": %.4f, \"G_s_u8\": %.1f, "
                        "\"ms_u16\": %.4f, \"G_s_u16\": %.1f}",
                        first ? "" : ",", mb, names[p], ms8, N / (ms8 * 1e-3) / 1e9, ms16, N / (ms16 * 1e-3) / 1e9);
            first = false;
            std::fflush(stdout);
        }
    }
    std::printf("]}\n");
    CK(hipFree(idx));
    CK(hipFree(tab));
    CK(hipFree(out));
    return 0;
}

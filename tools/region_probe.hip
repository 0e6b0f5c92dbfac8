// region_probe.hip -- is the BIN Mul / DIA "slow placement" (profiles/round1/README.md §4a) a
// property of physical HBM regions, and which access patterns feel it?
//
// Allocates the device memory in equal chunks (hipMalloc, in order, until
// `keep_free` GB remain) and measures each chunk with three kernels:
//   read     16-byte nontemporal loads, grid-stride (the DIA / Sum shape)
//   write    16-byte nontemporal stores, grid-stride
//   scatter  128-byte lines written by 16 lanes of 8 B (the Mul's product
//            lines) at line index (i * P) mod lines -- every line once, in
//            no regular stride
//   blocked  256 / 1024 workgroups, each streaming its own contiguous share
//            (the DIA / BIN Mul shape) with 16-byte nontemporal loads
// One JSON line per chunk: {"chunk", "va", "read_gbs", "write_gbs",
// "scatter_gbs"}, best of `reps` launches each.
//
//   region_probe [chunk_mb=1024] [keep_free_gb=16] [reps=3] [max_chunks=400]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
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
// (lines is a power of two: i * P mod lines, P odd, is a bijection)
__global__ __launch_bounds__(256) void scat(double *__restrict__ a, long long lines, long long P, double v) {
    const long long nthr = (long long)gridDim.x * 256;
    for (long long i = (blockIdx.x * 256LL + threadIdx.x) >> 4; i < lines; i += nthr >> 4) {
        const long long L = (long long)(((unsigned long long)i * (unsigned long long)P) & (unsigned long long)(lines - 1));
        __builtin_nontemporal_store(v, a + L * 16 + (threadIdx.x & 15));
    }
}

// blocked: workgroup w streams its own contiguous 1/grid of the chunk (the
// DIA / BIN Mul shape: many concurrent streams far apart), 16-byte loads
__global__ __launch_bounds__(256) void rd_blocked(const f64x2 *__restrict__ a, long long n2, double *__restrict__ out) {
    const long long per = n2 / gridDim.x, b0 = (long long)blockIdx.x * per;
    double s = 0;
    for (long long i = threadIdx.x; i < per; i += 256) {
        const f64x2 v = __builtin_nontemporal_load(a + b0 + i);
        s += v.x + v.y;
    }
    if (s == 1.2345) out[0] = s;
}

// "frag" mode: the same kernels on a 1 GB buffer allocated (A) first,
// (B) after the last ~9 GB were filled with 2 MB allocations and every other
// one freed, (C) the same with 64 KB allocations -- B and C can only be
// backed by the holes (small physical pieces, so small page-table fragments)
// once the rest of memory is held.  A TLB-bound access pattern slows down
// from A to C; a bandwidth-bound one does not.
static int frag_mode(int reps);
static int alloc_mode(int reps);
static int dia_mode(int nalloc, long long gb);

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "frag") return frag_mode(argc > 2 ? std::atoi(argv[2]) : 3);
    if (argc > 1 && std::string(argv[1]) == "alloc") return alloc_mode(argc > 2 ? std::atoi(argv[2]) : 3);
    if (argc > 1 && std::string(argv[1]) == "dia")
        return dia_mode(argc > 2 ? std::atoi(argv[2]) : 6, argc > 3 ? std::atoll(argv[3]) : 10);
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
        const float tb = best([&] { rd_blocked<<<256, 256>>>(c, n2, out); });
        const float tb2 = best([&] { rd_blocked<<<1024, 256>>>(c, n2, out); });
        std::printf("{\"chunk\": %zu, \"mb\": %lld, \"va\": \"%p\", \"read_gbs\": %.0f, \"write_gbs\": %.0f, "
                    "\"scatter_gbs\": %.0f, \"blocked256_gbs\": %.0f, \"blocked1024_gbs\": %.0f}\n",
                    i, chunk >> 20, ch[i], chunk / tr / 1e6, chunk / tw / 1e6, chunk / ts / 1e6, chunk / tb / 1e6,
                    chunk / tb2 / 1e6);
        std::fflush(stdout);
    }
    for (void *p : ch) CHECK(hipFree(p));
    return 0;
}

static int frag_mode(int reps) {
    double *out;
    CHECK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
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
    const long long bytes = 1024LL << 20, n2 = bytes / 16, lines = bytes / 128;
    // lines = 12 Mi: not a power of two -- use the largest power of two below
    long long pl = 1;
    while (pl * 2 <= lines) pl *= 2;
    const long long P = (long long)(0.6180339887 * (double)pl) | 1;
    auto measure = [&](const char *name, void *p) {
        f64x2 *c = (f64x2 *)p;
        const float tw = best([&] { wr<<<4096, 256>>>(c, n2, 1.0); });
        const float tr = best([&] { rd<<<4096, 256>>>(c, n2, out); });
        const float ts = best([&] { scat<<<4096, 256>>>((double *)c, pl, P, 2.0); });
        const float tb = best([&] { rd_blocked<<<256, 256>>>(c, n2, out); });
        const float tb2 = best([&] { rd_blocked<<<1024, 256>>>(c, n2, out); });
        std::printf("{\"frag\": \"%s\", \"va\": \"%p\", \"read_gbs\": %.0f, \"write_gbs\": %.0f, \"scatter_gbs\": %.0f, "
                    "\"blocked256_gbs\": %.0f, \"blocked1024_gbs\": %.0f}\n",
                    name, p, bytes / tr / 1e6, bytes / tw / 1e6, pl * 128.0 / ts / 1e6, bytes / tb / 1e6, bytes / tb2 / 1e6);
        std::fflush(stdout);
    };
    void *A = nullptr;
    CHECK(hipMalloc(&A, bytes));
    measure("A_first", A);
    // hold everything but ~9 GB, so later buffers must come from the holes
    std::vector<void *> hold;
    for (;;) {
        size_t fr = 0, tot = 0;
        CHECK(hipMemGetInfo(&fr, &tot));
        if ((long long)fr < (9LL << 30) + (1LL << 30)) break;
        void *p = nullptr;
        if (hipMalloc(&p, 1LL << 30) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        hold.push_back(p);
    }
    // fill all free memory (down to 64 MB) with `piece`-sized buffers, then
    // free every other one
    auto holes = [&](long long piece, long long total) {
        std::vector<void *> v;
        for (long long t = 0; t < total; t += piece) {
            size_t f2 = 0, t2 = 0;
            CHECK(hipMemGetInfo(&f2, &t2));
            if ((long long)f2 < (64LL << 20) + piece) break;
            void *p = nullptr;
            if (hipMalloc(&p, piece) != hipSuccess) {
                (void)hipGetLastError();
                break;
            }
            v.push_back(p);
        }
        std::vector<void *> keep;
        for (size_t i = 0; i < v.size(); ++i) {
            if (i % 2) CHECK(hipFree(v[i]));
            else keep.push_back(v[i]);
        }
        return keep;
    };
    // B: ~9 GB in 2 MB pieces, every other freed: ~4.5 GB of 2 MB holes
    std::vector<void *> k2 = holes(2LL << 20, 16LL << 30);
    size_t fr = 0, tot = 0;
    CHECK(hipMemGetInfo(&fr, &tot));
    std::printf("{\"free_after_2mb_holes_gb\": %.2f}\n", fr / 1073741824.0);
    void *Bf = nullptr;
    if (hipMalloc(&Bf, bytes) == hipSuccess) measure("B_2mb_holes", Bf);
    else (void)hipGetLastError();
    // C: the rest (~3.5 GB) in 64 KB pieces, every other freed
    std::vector<void *> k64 = holes(64LL << 10, 16LL << 30);
    CHECK(hipMemGetInfo(&fr, &tot));
    std::printf("{\"free_after_64kb_holes_gb\": %.2f}\n", fr / 1073741824.0);
    void *Cf = nullptr;
    if (hipMalloc(&Cf, bytes) == hipSuccess) measure("C_64kb_holes", Cf);
    else (void)hipGetLastError();
    measure("A_again", A);
    for (void *p : k64) CHECK(hipFree(p));
    for (void *p : k2) CHECK(hipFree(p));
    for (void *p : hold) CHECK(hipFree(p));
    if (Cf) CHECK(hipFree(Cf));
    if (Bf) CHECK(hipFree(Bf));
    void *D = nullptr;
    CHECK(hipMalloc(&D, bytes));
    measure("D_after_all_freed", D);
    CHECK(hipFree(D));
    CHECK(hipFree(A));
    return 0;
}

// "alloc" mode: which allocation method gives a buffer the fast mode?  Each
// method allocates 4 buffers of 1.5 GB (kept, so each is new memory) and
// measures them like frag mode; then 20 GB of 2 MB pieces with every other
// one freed fragment the free memory, and the methods run again.
//   plain        hipMalloc
//   vmm1g_one    hipMemAddressReserve aligned to 1 GB + ONE hipMemCreate handle
//   vmm1g_chunks the same with 512 MB handles
//   contig       hipExtMallocWithFlags(hipDeviceMallocContiguous)
static int alloc_mode(int reps) {
    double *out;
    CHECK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
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
    const long long bytes = 1536LL << 20, n2 = bytes / 16;
    long long pl = 1;
    while (pl * 2 <= bytes / 128) pl *= 2;
    const long long P = (long long)(0.6180339887 * (double)pl) | 1;
    auto measure = [&](const char *phase, const char *name, int rep, void *p) {
        f64x2 *c = (f64x2 *)p;
        const float tw = best([&] { wr<<<4096, 256>>>(c, n2, 1.0); });
        const float tr = best([&] { rd<<<4096, 256>>>(c, n2, out); });
        const float ts = best([&] { scat<<<4096, 256>>>((double *)c, pl, P, 2.0); });
        const float tb2 = best([&] { rd_blocked<<<1024, 256>>>(c, n2, out); });
        std::printf("{\"phase\": \"%s\", \"method\": \"%s\", \"rep\": %d, \"va\": \"%p\", \"va_mod_1g_mb\": %lld, "
                    "\"read_gbs\": %.0f, \"write_gbs\": %.0f, \"scatter_gbs\": %.0f, \"blocked1024_gbs\": %.0f}\n",
                    phase, name, rep, p, (long long)(((uintptr_t)p) & ((1ULL << 30) - 1)) >> 20, bytes / tr / 1e6,
                    bytes / tw / 1e6, pl * 128.0 / ts / 1e6, bytes / tb2 / 1e6);
        std::fflush(stdout);
    };
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    struct Vmm {
        void *va;
        size_t size;
        std::vector<hipMemGenericAllocationHandle_t> h;
        size_t chunk;
    };
    std::vector<void *> plain;
    std::vector<Vmm> vmms;
    auto vmm = [&](size_t chunk) -> void * {
        Vmm v;
        v.size = (size_t)bytes;
        v.chunk = std::min(chunk, v.size);
        CHECK(hipMemAddressReserve(&v.va, v.size, 1ULL << 30, nullptr, 0));
        for (size_t o = 0; o < v.size; o += v.chunk) {
            hipMemGenericAllocationHandle_t h;
            CHECK(hipMemCreate(&h, v.chunk, &prop, 0));
            CHECK(hipMemMap((char *)v.va + o, v.chunk, 0, h, 0));
            v.h.push_back(h);
        }
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CHECK(hipMemSetAccess(v.va, v.size, &acc, 1));
        vmms.push_back(v);
        return v.va;
    };
    auto run = [&](const char *phase, int nr) {
        for (int r = 0; r < nr; ++r) {
            void *p = nullptr;
            CHECK(hipMalloc(&p, bytes));
            plain.push_back(p);
            measure(phase, "plain", r, p);
        }
        for (int r = 0; r < nr; ++r) measure(phase, "vmm1g_one", r, vmm((size_t)bytes));
        for (int r = 0; r < nr; ++r) measure(phase, "vmm1g_chunks", r, vmm(512ULL << 20));
        for (int r = 0; r < nr; ++r) {
            void *p = nullptr;
            if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous) != hipSuccess) {
                (void)hipGetLastError();
                std::printf("{\"phase\": \"%s\", \"method\": \"contig\", \"rep\": %d, \"error\": 1}\n", phase, r);
                continue;
            }
            plain.push_back(p);
            measure(phase, "contig", r, p);
        }
    };
    run("fresh", 4);
    // fragment: 20 GB of 2 MB pieces, every other one freed
    std::vector<void *> pieces, keep;
    for (int i = 0; i < 10240; ++i) {
        void *p = nullptr;
        if (hipMalloc(&p, 2LL << 20) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        pieces.push_back(p);
    }
    for (size_t i = 0; i < pieces.size(); ++i) {
        if (i % 2) CHECK(hipFree(pieces[i]));
        else keep.push_back(pieces[i]);
    }
    run("after_2mb_holes", 4);
    // squeezed: hold all but 16 GB, fragment those, one buffer per method
    std::vector<void *> hold;
    for (;;) {
        size_t fr = 0, tot = 0;
        CHECK(hipMemGetInfo(&fr, &tot));
        if ((long long)fr < (17LL << 30)) break;
        void *p = nullptr;
        if (hipMalloc(&p, 1LL << 30) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        hold.push_back(p);
    }
    std::vector<void *> p2;
    for (;;) {
        size_t fr = 0, tot = 0;
        CHECK(hipMemGetInfo(&fr, &tot));
        if ((long long)fr < (256LL << 20)) break;
        void *p = nullptr;
        if (hipMalloc(&p, 2LL << 20) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        p2.push_back(p);
    }
    for (size_t i = 0; i < p2.size(); ++i) {
        if (i % 2) CHECK(hipFree(p2[i]));
        else keep.push_back(p2[i]);
    }
    run("squeezed_2mb_holes", 1);
    for (void *p : hold) CHECK(hipFree(p));
    for (void *p : keep) CHECK(hipFree(p));
    for (void *p : plain) CHECK(hipFree(p));
    for (auto &v : vmms) {
        for (size_t k = 0; k < v.h.size(); ++k) {
            CHECK(hipMemUnmap((char *)v.va + k * v.chunk, v.chunk));
            CHECK(hipMemRelease(v.h[k]));
        }
        CHECK(hipMemAddressFree(v.va, v.size));
    }
    return 0;
}

// "dia" mode: the DIA kernel's value stream alone -- workgroup b (256
// threads, 16-byte loads, 8 in flight per lane) streams its own contiguous
// 256 KB block (the blocked layout, 64 diagonals x 512 rows) -- over
// `nalloc` separate allocations of `gb` GB each, kept (so each is new
// memory), three times each; next to the same bytes read grid-stride.
// Does the rate vary from allocation to allocation like dia_kernel's
// (1.51-1.68 ms at config 4, profiles/round1/README.md §4a), and which pattern is immune?
__global__ __launch_bounds__(256) void rd_dia(const f64x2 *__restrict__ a, long long blk2, double *__restrict__ out) {
    const f64x2 *b = a + (long long)blockIdx.x * blk2 + threadIdx.x;
    double s = 0;
    for (long long i = 0; i < blk2; i += 256 * 8) {
        f64x2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(b + i + u * 256);
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u].x + v[u].y;
    }
    if (s == 1.2345) out[0] = s;
}

static int dia_mode(int nalloc, long long gb) {
    double *out;
    CHECK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const long long bytes = gb << 30, n2 = bytes / 16, blk2 = (256LL << 10) / 16, nblk = n2 / blk2;
    auto time = [&](auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        float bms = 1e30f;
        for (int r = 0; r < 3; ++r) {
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
    std::vector<void *> keep;
    for (int k = 0; k < nalloc; ++k) {
        void *p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        keep.push_back(p);
        CHECK(hipMemset(p, 0, bytes));
        const float td = time([&] { rd_dia<<<(unsigned)nblk, 256>>>((const f64x2 *)p, blk2, out); });
        const float tg = time([&] { rd<<<4096, 256>>>((const f64x2 *)p, n2, out); });
        std::printf("{\"alloc\": %d, \"gb\": %lld, \"va\": \"%p\", \"dia_blocked_ms\": %.4f, \"dia_blocked_gbs\": %.0f, "
                    "\"gridstride_ms\": %.4f, \"gridstride_gbs\": %.0f}\n",
                    k, gb, p, td, bytes / td / 1e6, tg, bytes / tg / 1e6);
        std::fflush(stdout);
    }
    for (void *p : keep) CHECK(hipFree(p));
    return 0;
}

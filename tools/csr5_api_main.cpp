// csr5_api_main.cpp -- the CSR5 benchmark's driver flow
// (opt/Benchmark_SpMV_using_CSR5/CSR5_cuda/main.cu: call_anonymouslib and the
// check at :330-360) against include/csr5_hip.h: device CSR in, inputCSR ->
// setX -> setSigma(auto) -> asCSR5 -> spmv(alpha, y) x3 -> asCSR -> destroy.
// y is compared with the benchmark's own check, sum += x[col] * val * alpha.
//
//   csr5_api [matrix.mtx] [alpha] [sigma]      (no matrix: 300 K-row power law)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "csr5_hip.h"

#define HIPCHK(x)                                                              \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 2;                                                          \
        }                                                                      \
    } while (0)

int main(int argc, char **argv) {
    int64_t m = 0, n = 0, nnz = 0;
    int64_t *rp64 = nullptr;
    int32_t *col = nullptr;
    double *val = nullptr;
    if (argc > 1 && argv[1][0] != '-') {
        uint32_t info = 0;
        if (spmv_load_mtx_csr(argv[1], 0, &m, &n, &nnz, &rp64, &col, &val, &info) != SPMV_SUCCESS) {
            std::fprintf(stderr, "load: %s\n", spmv_last_error());
            return 2;
        }
    } else {
        spmv_gen_spec_t s{};
        s.kind = SPMV_GEN_POWERLAW;
        s.m = s.n = 300000;
        s.max_len = 3000;
        s.alpha = 2.0;
        s.seed = 7;
        m = s.m;
        n = s.n;
        spmv_gen_count(&s, 0, m, &nnz);
        rp64 = (int64_t *)std::malloc(8 * (m + 1));
        col = (int32_t *)std::malloc(4 * (nnz + 1));
        val = (double *)std::malloc(8 * (nnz + 1));
        spmv_gen_fill(&s, 0, m, rp64, col, val);
    }
    const double alpha = argc > 2 ? std::atof(argv[2]) : 1.5;
    const int sigma = argc > 3 ? std::atoi(argv[3]) : ANONYMOUSLIB_AUTO_TUNED_SIGMA;
    std::vector<int> rp((size_t)m + 1);
    for (int64_t i = 0; i <= m; ++i) rp[(size_t)i] = (int)rp64[i];
    std::vector<double> x((size_t)std::max<int64_t>(n, 1));
    srand(3);
    for (auto &v : x) v = rand() / (double)RAND_MAX;

    int *d_rp, *d_col;
    double *d_val, *d_x, *d_y;
    HIPCHK(hipMalloc(&d_rp, 4 * (m + 1)));
    HIPCHK(hipMalloc(&d_col, 4 * std::max<int64_t>(nnz, 1)));
    HIPCHK(hipMalloc(&d_val, 8 * std::max<int64_t>(nnz, 1)));
    HIPCHK(hipMalloc(&d_x, 8 * std::max<int64_t>(n, 1)));
    HIPCHK(hipMalloc(&d_y, 8 * std::max<int64_t>(m, 1)));
    HIPCHK(hipMemcpy(d_rp, rp.data(), 4 * (m + 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_col, col, 4 * nnz, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_val, val, 8 * nnz, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_x, x.data(), 8 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(d_y, 0, 8 * m));
    std::vector<int> col_before(col, col + nnz);

    int bad = 0;
    {
        anonymouslibHandle<int, unsigned int, double> A((int)m, (int)n);
        int err = A.inputCSR((int)nnz, d_rp, d_col, d_val);
        err |= A.setX(d_x);
        if (A.spmv(alpha, d_y) != ANONYMOUSLIB_UNSUPPORTED_CSR_SPMV) {  // CSR mode refuses, as the reference
            std::fprintf(stderr, "spmv before asCSR5 should be refused\n");
            bad = 1;
        }
        A.setSigma(sigma);
        A.warmup();
        err |= A.asCSR5();
        std::vector<double> y((size_t)m), y1((size_t)m);
        for (int call = 0; call < 3; ++call) {
            err |= A.spmv(alpha, d_y);
            HIPCHK(hipMemcpy(call ? y1.data() : y.data(), d_y, 8 * m, hipMemcpyDeviceToHost));
            if (call && std::memcmp(y.data(), y1.data(), 8 * m) != 0) {
                std::fprintf(stderr, "call %d differs from call 0\n", call);
                bad = 1;
            }
        }
        spmv_plan_info_t info;
        spmv_plan_info(A.plan(), &info);
        // the benchmark's check (main.cu:340-356): sum += x[col] * val * alpha
        double max_rel = 0;
        for (int64_t i = 0; i < m; ++i) {
            double sum = 0;
            for (int64_t j = rp64[i]; j < rp64[i + 1]; ++j) sum += x[(size_t)col[j]] * val[j] * alpha;
            const double rel = std::fabs(y[(size_t)i] - sum) / std::max(std::fabs(sum), 1e-300);
            if (std::fabs(y[(size_t)i] - sum) > 1e-300) max_rel = std::max(max_rel, rel);
        }
        err |= A.destroy();
        std::vector<int> col_after((size_t)nnz);
        HIPCHK(hipMemcpy(col_after.data(), d_col, 4 * nnz, hipMemcpyDeviceToHost));
        if (col_after != col_before) {
            std::fprintf(stderr, "caller's column array was modified\n");
            bad = 1;
        }
        if (err != ANONYMOUSLIB_SUCCESS || max_rel > 1e-10) bad = 1;
        std::printf("csr5_api: m=%ld n=%ld nnz=%ld sigma=%d alpha=%g max_rel=%.3e err=%d -> %s\n", (long)m, (long)n,
                    (long)nnz, info.ss_sigma, alpha, max_rel, err, bad ? "FAIL" : "OK");
    }
    (void)hipFree(d_rp);
    (void)hipFree(d_col);
    (void)hipFree(d_val);
    (void)hipFree(d_x);
    (void)hipFree(d_y);
    spmv_free_host(rp64);
    spmv_free_host(col);
    spmv_free_host(val);
    return bad;
}

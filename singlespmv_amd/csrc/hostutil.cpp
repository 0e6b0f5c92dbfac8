// hostutil.cpp -- host side of the path around the kernels (the Matrix Market
// loader lives in mmio.cpp): CreateRandomVector (src/util.cpp:92-102),
// VerifyResult (src/util.cpp:67-83), and the seeded
// synthetic generators for the BASELINE configs (built in memory: a 1.28 G-nnz
// .mtx would be ~38 GB of text, SURVEY §7 hard part 5).
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "internal.hpp"

using namespace spmv;

namespace {

// ---- counter-based generator ----------------------------------------------
inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// one 64-bit draw per (seed, stream, i, j); independent of thread count
inline uint64_t draw(uint64_t seed, uint64_t stream, uint64_t i, uint64_t j) {
    return splitmix64(splitmix64(splitmix64(seed ^ (stream * 0xD6E8FEB86659FD93ull)) ^ i) ^ j);
}
inline double u01_open_closed(uint64_t h) { return (double)((h >> 11) + 1) * 0x1.0p-53; }  // (0,1]
inline double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }                    // [0,1)
inline int64_t below(uint64_t h, int64_t n) { return (int64_t)(((unsigned __int128)h * (uint64_t)n) >> 64); }

enum : uint64_t { S_COL = 1, S_VAL = 2, S_LEN = 3, S_VEC = 4 };

struct PowerLaw {
    std::vector<double> cdf;  // cdf[k-1] = P(len <= k)
    PowerLaw(int max_len, double alpha) : cdf((size_t)max_len) {
        double s = 0;
        for (int k = 1; k <= max_len; ++k) s += std::pow((double)k, -alpha);
        double c = 0;
        for (int k = 1; k <= max_len; ++k) {
            c += std::pow((double)k, -alpha) / s;
            cdf[(size_t)k - 1] = c;
        }
        cdf.back() = 1.0;
    }
    int64_t len(double u) const {
        return (int64_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()) + 1;
    }
};

int check_spec(const spmv_gen_spec_t *s, int64_t rb, int64_t re) {
    SPMV_CHECK_ARG(s != nullptr, "spec is NULL");
    SPMV_CHECK_ARG(s->m >= 0 && s->n > 0 && s->n < INT32_MAX, "bad m/n");
    SPMV_CHECK_ARG(0 <= rb && rb <= re && re <= s->m, "bad row range");
    switch (s->kind) {
        case SPMV_GEN_UNIFORM: SPMV_CHECK_ARG(s->per_row >= 0, "per_row < 0"); break;
        case SPMV_GEN_POWERLAW: SPMV_CHECK_ARG(s->max_len >= 1 && s->alpha > 0, "bad power law"); break;
        case SPMV_GEN_BANDED: SPMV_CHECK_ARG(s->band_lo <= s->band_hi, "band_lo > band_hi"); break;
        default: SPMV_CHECK_ARG(false, "unknown generator kind");
    }
    return SPMV_SUCCESS;
}

inline int64_t banded_len(const spmv_gen_spec_t *s, int64_t r) {
    const int64_t lo = std::max<int64_t>(0, r + s->band_lo);
    const int64_t hi = std::min<int64_t>(s->n - 1, r + s->band_hi);
    return hi >= lo ? hi - lo + 1 : 0;
}

}  // namespace

extern "C" {

void spmv_srand(uint32_t seed) { srand(seed); }
void spmv_rand_vector(int32_t n, double *out) {
    for (int32_t i = 0; i < n; ++i) out[i] = double(rand()) / RAND_MAX;
}

int64_t spmv_verify_coo(int32_t m, int32_t nnz, const int32_t *row_idx, const int32_t *col_idx,
                        const double *val, const double *x, const double *y) {
    std::vector<double> res((size_t)std::max(m, 1), 0.0);
    for (int32_t i = 0; i < nnz; ++i) res[row_idx[i]] += val[i] * x[col_idx[i]];
    for (int32_t i = 0; i < m; ++i) {
        const double rel = std::fabs(std::fabs(res[i] - y[i]) / res[i]);
        const double ab = std::fabs(res[i] - y[i]);
        if (ab > 1e-6 && rel > 1e-6) return i;
    }
    return -1;
}

int spmv_gen_count(const spmv_gen_spec_t *s, int64_t rb, int64_t re, int64_t *nnz) {
    SPMV_RETURN_IF(check_spec(s, rb, re));
    SPMV_CHECK_ARG(nnz != nullptr, "nnz is NULL");
    int64_t total = 0;
    if (s->kind == SPMV_GEN_UNIFORM) {
        total = (re - rb) * (int64_t)s->per_row;
    } else if (s->kind == SPMV_GEN_BANDED) {
#pragma omp parallel for schedule(static) reduction(+ : total)
        for (int64_t r = rb; r < re; ++r) total += banded_len(s, r);
    } else {
        const PowerLaw pl(s->max_len, s->alpha);
#pragma omp parallel for schedule(static) reduction(+ : total)
        for (int64_t r = rb; r < re; ++r) total += pl.len(u01(draw(s->seed, S_LEN, (uint64_t)r, 0)));
    }
    *nnz = total;
    return SPMV_SUCCESS;
}

int spmv_gen_fill(const spmv_gen_spec_t *s, int64_t rb, int64_t re, int64_t *row_ptr,
                  int32_t *col_idx, double *val) {
    SPMV_RETURN_IF(check_spec(s, rb, re));
    SPMV_CHECK_ARG(row_ptr != nullptr, "row_ptr is NULL");
    const int64_t rows = re - rb;
    const PowerLaw *pl = s->kind == SPMV_GEN_POWERLAW ? new PowerLaw(s->max_len, s->alpha) : nullptr;
    row_ptr[0] = 0;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < rows; ++i) {
        const int64_t r = rb + i;
        int64_t len;
        if (s->kind == SPMV_GEN_UNIFORM) len = s->per_row;
        else if (s->kind == SPMV_GEN_BANDED) len = banded_len(s, r);
        else len = pl->len(u01(draw(s->seed, S_LEN, (uint64_t)r, 0)));
        row_ptr[i + 1] = len;
    }
    for (int64_t i = 0; i < rows; ++i) row_ptr[i + 1] += row_ptr[i];
    if (col_idx == nullptr && val == nullptr) {  // row pointers only (nnz-balanced shard cuts)
        delete pl;
        return SPMV_SUCCESS;
    }
    SPMV_CHECK_ARG(col_idx != nullptr && val != nullptr, "col_idx / val is NULL");
    const bool intv = s->integer_values != 0;
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t i = 0; i < rows; ++i) {
        const int64_t r = rb + i;
        const int64_t b = row_ptr[i], e = row_ptr[i + 1];
        int32_t *c = col_idx + b;
        if (s->kind == SPMV_GEN_BANDED) {
            const int64_t lo = std::max<int64_t>(0, r + s->band_lo);
            for (int64_t k = 0; k < e - b; ++k) c[k] = (int32_t)(lo + k);
        } else {
            for (int64_t k = 0; k < e - b; ++k) c[k] = (int32_t)below(draw(s->seed, S_COL, (uint64_t)r, (uint64_t)k), s->n);
            std::sort(c, c + (e - b));  // sorted within the row, duplicates kept
        }
        for (int64_t k = 0; k < e - b; ++k) {
            const uint64_t h = draw(s->seed, S_VAL, (uint64_t)r, (uint64_t)k);
            val[b + k] = intv ? (double)(h % 10) : u01_open_closed(h);
        }
    }
    delete pl;
    return SPMV_SUCCESS;
}

int spmv_gen_vector(uint64_t seed, int32_t integer_values, int64_t begin, int64_t count, double *out) {
    SPMV_CHECK_ARG(out != nullptr || count == 0, "out is NULL");
    SPMV_CHECK_ARG(begin >= 0 && count >= 0, "bad range");
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < count; ++i) {
        const uint64_t h = draw(seed, S_VEC, (uint64_t)(begin + i), 0);
        out[i] = integer_values ? (double)(h % 10) : u01(h);
    }
    return SPMV_SUCCESS;
}

}  // extern "C"

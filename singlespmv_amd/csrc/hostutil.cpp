// hostutil.cpp -- host side of the path around the kernels: the Matrix Market
// loader (LoadSparseMatrix semantics, src/util.cpp:30-66), CreateRandomVector
// (src/util.cpp:92-102), VerifyResult (src/util.cpp:67-83), and the seeded
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

// ---- Matrix Market text ---------------------------------------------------
struct Cursor {
    const char *p, *end;
    void skip_ws() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\f' || *p == '\v')) ++p;
    }
    bool read_long(long long &v) {
        skip_ws();
        if (p >= end) return false;
        char *q;
        char buf[64];
        size_t n = std::min<size_t>(63, (size_t)(end - p));
        std::memcpy(buf, p, n);
        buf[n] = 0;
        v = std::strtoll(buf, &q, 10);
        if (q == buf) return false;
        p += (q - buf);
        return true;
    }
    bool read_double(double &v) {
        skip_ws();
        if (p >= end) return false;
        char *q;
        char buf[128];
        size_t n = std::min<size_t>(127, (size_t)(end - p));
        std::memcpy(buf, p, n);
        buf[n] = 0;
        v = std::strtod(buf, &q);
        if (q == buf) return false;
        p += (q - buf);
        return true;
    }
};

struct Trip {
    int32_t r, c;
    double v;
};

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

void spmv_free_host(void *p) { std::free(p); }

int spmv_load_mtx(const char *path, int32_t *m, int32_t *n, int32_t *nnz, int32_t **row_idx,
                  int32_t **col_idx, double **val) {
    SPMV_CHECK_ARG(path && m && n && nnz && row_idx && col_idx && val, "NULL argument");
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
        set_error(std::string("File not Found: ") + path);  // util.cpp:32-35
        return SPMV_ERROR_IO;
    }
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        set_error("fstat failed");
        return SPMV_ERROR_IO;
    }
    const size_t size = (size_t)st.st_size;
    const char *base = size ? (const char *)mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0) : "";
    close(fd);
    if (base == MAP_FAILED) {
        set_error("mmap failed");
        return SPMV_ERROR_IO;
    }
    Cursor cur{base, base + size};
    // util.cpp:37-39: skip lines whose first character is '%'
    while (cur.p < cur.end && *cur.p == '%') {
        const char *nl = (const char *)std::memchr(cur.p, '\n', (size_t)(cur.end - cur.p));
        cur.p = nl ? nl + 1 : cur.end;
    }
    long long M, N, L;
    int status = SPMV_SUCCESS;
    std::vector<Trip> t;
    if (!cur.read_long(M) || !cur.read_long(N) || !cur.read_long(L) || M < 0 || N < 0 || L < 0 ||
        M >= INT32_MAX || N >= INT32_MAX || L >= INT32_MAX) {
        set_error("bad Matrix Market header");
        status = SPMV_ERROR_IO;
    } else {
        t.resize((size_t)L);
        // util.cpp:44-50: exactly L triplets, 1 -> 0 based
        for (long long i = 0; i < L; ++i) {
            long long r, c;
            double v;
            if (!cur.read_long(r) || !cur.read_long(c) || !cur.read_double(v)) {
                set_error("truncated triplet list (fewer than L entries)");
                status = SPMV_ERROR_IO;
                break;
            }
            if (r < 1 || r > M || c < 1 || c > N) {
                set_error("entry outside the declared shape");
                status = SPMV_ERROR_IO;
                break;
            }
            t[(size_t)i] = Trip{(int32_t)(r - 1), (int32_t)(c - 1), v};
        }
    }
    if (size) munmap((void *)base, size);
    if (status != SPMV_SUCCESS) return status;
    // util.cpp:51: sort row-major by (row, col); stable keeps duplicates in
    // file order (std::sort leaves them unspecified)
    std::stable_sort(t.begin(), t.end(), [](const Trip &a, const Trip &b) {
        return a.r != b.r ? a.r < b.r : a.c < b.c;
    });
    const size_t k = t.size() ? t.size() : 1;
    int32_t *ri = (int32_t *)std::malloc(sizeof(int32_t) * k);
    int32_t *ci = (int32_t *)std::malloc(sizeof(int32_t) * k);
    double *vv = (double *)std::malloc(sizeof(double) * k);
    if (!ri || !ci || !vv) {
        std::free(ri);
        std::free(ci);
        std::free(vv);
        set_error("host allocation failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    for (size_t i = 0; i < t.size(); ++i) {
        ri[i] = t[i].r;
        ci[i] = t[i].c;
        vv[i] = t[i].v;
    }
    *m = (int32_t)M;
    *n = (int32_t)N;
    *nnz = (int32_t)L;
    *row_idx = ri;
    *col_idx = ci;
    *val = vv;
    return SPMV_SUCCESS;
}

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

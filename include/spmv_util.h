/*
 * spmv_util.h -- host types and helpers for C++ callers of the drop-in
 * (include/opt_hip.h).  The structs reproduce the reference's binary layout so
 * OptimizeProblem/SpMV keep the reference signatures and mangled names:
 *   SpMat  = sorted COO, int indices          (reference src/util.h:7-19)
 *   Vec    = {int size; double *val;}          (reference src/util.h:20-28)
 * The helpers wrap the C-ABI utilities of spmv_hip.h with the reference
 * function names (src/util.h:40-45).  Header-only.
 *
 * Build inside the reference tree instead by defining
 * OPT_HIP_USE_REFERENCE_TYPES and including the reference util.h first
 * (see INTEGRATION.md).
 */
#ifndef SPMV_UTIL_H
#define SPMV_UTIL_H

#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "spmv_hip.h"

struct SpMat {
    int nRow, nCol, nNnz;
    int *row_idx;
    int *col_idx;
    double *val;
};

struct Vec {
    int size;
    double *val;
};

/* LoadSparseMatrix semantics (src/util.cpp:30-66); exits like the reference
 * when the file cannot be read. */
inline void LoadSparseMatrix(SpMat &A, const std::string &path) {
    int32_t m, n, nnz;
    int32_t *r, *c;
    double *v;
    const int st = spmv_load_mtx(path.c_str(), &m, &n, &nnz, &r, &c, &v);
    if (st != SPMV_SUCCESS) {
        std::fprintf(stderr, "%s\n", spmv_last_error());
        std::exit(1);
    }
    A.nRow = m;
    A.nCol = n;
    A.nNnz = nnz;
    A.row_idx = r;
    A.col_idx = c;
    A.val = v;
}

/* rand()/RAND_MAX per entry, the caller seeds with srand (src/util.cpp:92-102) */
inline Vec CreateRandomVector(int size) {
    Vec x;
    x.size = size;
    x.val = static_cast<double *>(std::aligned_alloc(64, sizeof(double) * (size_t)(size > 0 ? (size + 7) / 8 * 8 : 8)));
    spmv_rand_vector(size, x.val);
    return x;
}

/* VerifyResult (src/util.cpp:67-83) */
inline bool VerifyResult(const SpMat &A, const Vec &x, const Vec &y) {
    const int64_t bad = spmv_verify_coo(A.nRow, A.nNnz, A.row_idx, A.col_idx, A.val, x.val, y.val);
    if (bad >= 0) std::fprintf(stderr, "Error: row %lld mismatches\n", (long long)bad);
    return bad < 0;
}

inline double GetTimeBySec() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_sec + tv.tv_usec * 1e-6;
}

inline std::string GetBasename(const std::string &path) {
    const size_t p = path.rfind('/');
    return p == std::string::npos ? path : path.substr(p + 1);
}

#endif /* SPMV_UTIL_H */

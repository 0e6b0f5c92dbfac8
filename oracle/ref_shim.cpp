// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin C entry point around the REFERENCE's own sources, compiled where
// they lie under /root/reference/src by oracle/Makefile (one shared library
// per format, because every reference plugin defines SpMatOpt/VecOpt/SpMV with
// the same names -- src/opt.h:1-28).  Nothing here restates the reference;
// it only calls its LoadSparseMatrix / CreateRandomVector / OptimizeProblem /
// SpMV / VerifyResult so tests can pin oracle/oracle.c against the real code.
//
// Outputs go to oracle/_ref/ (git-ignored).  Never shipped, never used by the
// product path.
#include <omp.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "opt.h"
#include "param.h"
#include "util.h"

extern std::vector<double> g_profile;

extern "C" {

// LoadSparseMatrix (src/util.cpp:30-66).  Arrays are new[]'d by the reference
// and copied into caller-provided buffers by ref_copy_coo; the handle is freed
// by ref_free_coo.
void *ref_load(const char *path, int *m, int *n, int *nnz) {
    SpMat *A = new SpMat;
    LoadSparseMatrix(*A, std::string(path));
    *m = A->nRow;
    *n = A->nCol;
    *nnz = A->nNnz;
    return A;
}

void ref_copy_coo(void *h, int *row_idx, int *col_idx, double *val) {
    SpMat *A = (SpMat *)h;
    std::memcpy(row_idx, A->row_idx, sizeof(int) * A->nNnz);
    std::memcpy(col_idx, A->col_idx, sizeof(int) * A->nNnz);
    std::memcpy(val, A->val, sizeof(double) * A->nNnz);
}

void ref_free_coo(void *h) {
    SpMat *A = (SpMat *)h;
    delete[] A->row_idx;
    delete[] A->col_idx;
    delete[] A->val;
    delete A;
}

// srand(3) + CreateRandomVector (src/main.cpp:18,31-32; src/util.cpp:92-102)
void ref_srand(unsigned s) { srand(s); }
void ref_random_vector(int n, double *out) {
    Vec v = CreateRandomVector(n);
    std::memcpy(out, v.val, sizeof(double) * n);
    free(v.val);  // _mm_free == free for the glibc _mm_malloc
}

// OptimizeProblem once, then SpMV `calls` times (each call overwrites y), the
// way src/main.cpp:36-55 drives a plugin.  y must hold m doubles; it is
// pre-filled with garbage (the driver's random y) by the caller.
int ref_run(int m, int n, int nnz, const int *row_idx, const int *col_idx,
            const double *val, const double *x, double *y, int calls) {
    SpMat A;
    A.nRow = m;
    A.nCol = n;
    A.nNnz = nnz;
    A.row_idx = const_cast<int *>(row_idx);
    A.col_idx = const_cast<int *>(col_idx);
    A.val = const_cast<double *>(val);
    Vec xv;
    xv.size = n;
    xv.val = const_cast<double *>(x);
    Vec yv;
    yv.size = m;
    yv.val = y;
    SpMatOpt A_opt;
    VecOpt x_opt;
    g_profile = std::vector<double>(10);
    OptimizeProblem(A, xv, A_opt, x_opt);
    for (int i = 0; i < calls; i++) SpMV(A_opt, x_opt, yv);
    // VerifyResult on the last call (src/util.cpp:67-83): 1 = pass
    return VerifyResult(A, xv, yv) ? 1 : 0;
}

// thread count of the reference's OpenMP regions (0 = runtime default)
void ref_set_threads(int n) {
    static const int dflt = omp_get_max_threads();
    omp_set_num_threads(n > 0 ? n : dflt);
}

// The reference driver's timing of a plugin (src/main.cpp:36, 58-102):
// OptimizeProblem once; warm-up doubling `loop` until the cumulative time
// reaches min_seconds (1.0 in the reference); then ntry batches of `loop`
// calls (10 in the reference), min mean seconds per call.  y gets the last
// result.
double ref_time(int m, int n, int nnz, const int *row_idx, const int *col_idx, const double *val,
                const double *x, double *y, double min_seconds, int ntry, int *loop_out) {
    SpMat A;
    A.nRow = m;
    A.nCol = n;
    A.nNnz = nnz;
    A.row_idx = const_cast<int *>(row_idx);
    A.col_idx = const_cast<int *>(col_idx);
    A.val = const_cast<double *>(val);
    Vec xv;
    xv.size = n;
    xv.val = const_cast<double *>(x);
    Vec yv;
    yv.size = m;
    yv.val = y;
    SpMatOpt A_opt;
    VecOpt x_opt;
    g_profile = std::vector<double>(10);
    OptimizeProblem(A, xv, A_opt, x_opt);
    int loop = 1;
    const double t0 = GetTimeBySec();
    do {
        for (int i = 0; i < loop; i++) SpMV(A_opt, x_opt, yv);
        loop *= 2;
    } while (GetTimeBySec() - t0 < min_seconds);
    double best = 0;
    for (int t = 0; t < ntry; t++) {
        const double a = GetTimeBySec();
        for (int i = 0; i < loop; i++) SpMV(A_opt, x_opt, yv);
        const double e = (GetTimeBySec() - a) / loop;
        best = t == 0 ? e : (e < best ? e : best);
    }
    *loop_out = loop;
    return best;
}

}  // extern "C"

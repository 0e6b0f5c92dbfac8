/*
 * oracle.h -- CPU restatement of the reference singleSpMV hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in singlespmv_amd/ links, imports or
 * calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker / the timed CPU
 * baseline -- never as the product path.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the upstream repository hir0shim/singleSpMV).  Arithmetic is compiled with
 * -ffp-contract=off so each `a += v*x` is one rounded multiply followed by one
 * rounded add -- the IEEE semantics of the reference source as written.
 *
 * Parity pinning: tests/test_oracle.py checks these functions against
 *   (1) golden vectors in tests/golden/ produced by the reference sources
 *       themselves (oracle/_ref, built by oracle/Makefile from the reference
 *       src/ files where they lie), and
 *   (2) the known-answer properties of the reference fixtures
 *       (matrix/test/{3x3,5x5,10x10,random}.mtx).
 */
#ifndef SPMV_ORACLE_H
#define SPMV_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- IO / vectors (src/util.cpp) -------------------------------------- */

/* LoadSparseMatrix (src/util.cpp:30-66): skip leading lines whose first char
 * is '%', read "M N L", read exactly L whitespace-separated triplets, convert
 * 1-based -> 0-based, sort row-major by (row, col) keeping duplicates.
 * Arrays are malloc'd; free with orc_free.  Returns 0 on success, -1 when the
 * file cannot be opened, -2 when the header or a triplet cannot be parsed. */
int orc_load_mtx(const char *path, int *m, int *n, int *nnz,
                 int **row_idx, int **col_idx, double **val);
void orc_free(void *p);

/* srand / CreateRandomVector (src/main.cpp:18, src/util.cpp:92-102):
 * out[i] = double(rand()) / RAND_MAX with glibc rand(). */
void orc_srand(unsigned seed);
void orc_rand_fill(int n, double *out);

/* VerifyResult (src/util.cpp:67-83): serial COO product, a row fails iff
 * abs_err > 1e-6 AND rel_err > 1e-6.  Returns -1 when every row passes, else
 * the first failing row.  ref_out (optional, may be NULL) receives the serial
 * COO product `res`. */
int64_t orc_verify(int m, int64_t nnz, const int *row_idx, const int *col_idx,
                   const double *val, const double *x, const double *y,
                   double *ref_out);
/* Same criterion for CSR input (row_ptr int64) -- used at sizes where a COO
 * copy is too large; the per-row order equals the COO order for sorted COO. */
int64_t orc_verify_csr(int64_t m, const int64_t *row_ptr, const int *col_idx,
                       const double *val, const double *x, const double *y);

/* ---- opt_crs (src/opt_crs.cpp) ---------------------------------------- */

/* OptimizeProblem (src/opt_crs.cpp:10-42): COO -> CSR by a linear scan. */
void orc_coo_to_csr(int m, int64_t nnz, const int *row_idx, const int *col_idx,
                    const double *val, int64_t *ptr, int *idx, double *csr_val);
/* SpMV (src/opt_crs.cpp:44-70): row-parallel OpenMP static schedule,
 * sequential per-row sum.  nthreads <= 0 -> OpenMP default. */
void orc_csr_spmv(int64_t m, const int64_t *ptr, const int *idx,
                  const double *val, const double *x, double *y, int nthreads);
/* Reference-method timing of orc_csr_spmv (src/main.cpp:58-102): double the
 * loop count until >= min_seconds elapsed, then ntry trials of `loop` calls,
 * return the minimum mean seconds per call; *loop_out gets the loop count. */
double orc_csr_time(int64_t m, const int64_t *ptr, const int *idx,
                    const double *val, const double *x, double *y,
                    int nthreads, double min_seconds, int ntry, int *loop_out);
int orc_max_threads(void);

/* ---- opt_ell (src/opt_ell.cpp) ---------------------------------------- */

/* OptimizeProblem (src/opt_ell.cpp:26-52): K = max row length, row-major
 * slots [m][K]; padding slot s of a row has col = s and val = 0. */
int orc_ell_width(int m, int64_t nnz, const int *row_idx);
void orc_ell_build(int m, int64_t nnz, const int *row_idx, const int *col_idx,
                   const double *val, int K, int *ell_col, double *ell_val);
/* SpMV (src/opt_ell.cpp:62-90): zero y, then y[r] += x[col] * val over all
 * K slots (padding included). */
void orc_ell_spmv(int m, int K, const int *ell_col, const double *ell_val,
                  const double *x, double *y);

/* ---- opt_dia (src/opt_dia.cpp) ---------------------------------------- */

/* OptimizeProblem (src/opt_dia.cpp:21-62): diagonal d = col - row + (m-1);
 * ioff[] = occupied d in ascending order; diag[p][col] indexed by COLUMN,
 * zero filled; duplicates of one (row, col) keep the LAST value (reference
 * behaviour: plain store at :55).  Returns nDiag; ioff may be NULL to count. */
int orc_dia_count(int m, int n, int64_t nnz, const int *row_idx,
                  const int *col_idx, int *ioff);
void orc_dia_build(int m, int n, int64_t nnz, const int *row_idx,
                   const int *col_idx, const double *val, int nDiag,
                   const int *ioff, double *diag /* [nDiag][n] */);
/* SpMV (src/opt_dia.cpp:65-97): serial over diagonals then columns,
 * y[col + (m-1) - ioff[i]] += diag[i][col] * x[col]. */
void orc_dia_spmv(int m, int n, int nDiag, const int *ioff, const double *diag,
                  const double *x, double *y);

/* ---- opt_ss (src/opt_ss.cpp) ------------------------------------------ */

/* SpMV SIMPLE (src/opt_ss.cpp:188-221): products into val_buf, then
 * sequential per-row sums.  W must be a power of two. */
void orc_ss_simple_spmv(int m, int64_t nnz, const int64_t *row_ptr,
                        const int *col_idx, const double *val, int W,
                        const double *x, double *y);
/* SpMV OPTIMIZED without PADDING (src/opt_ss.cpp:91-142 segment index and
 * step lists, :222-303 Mul / Sum1 tree fold / Sum2 head-tail-center). */
void orc_ss_optimized_spmv(int m, int64_t nnz, const int64_t *row_ptr,
                           const int *col_idx, const double *val, int W,
                           const double *x, double *y);

#ifdef __cplusplus
}
#endif
#endif

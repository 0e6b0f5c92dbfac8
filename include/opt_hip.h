/*
 * opt_hip.h -- drop-in format plugin for the reference's opt_* dispatch
 * surface (reference src/opt.h:1-28): the same OptimizeProblem / SpMV pair
 * every plugin exports (e.g. src/opt_crs.h:15-18, src/opt_cusparse.h:33-37),
 * backed by libspmv_hip.so on an MI355X.
 *
 *   void OptimizeProblem(const SpMat&, const Vec&, SpMatOpt&, VecOpt&);
 *       mangled _Z15OptimizeProblemRK5SpMatRK3VecR8SpMatOptR6VecOpt
 *   extern "C" void SpMV(const SpMatOpt&, const VecOpt&, Vec&);
 *
 * Format: the first of -DOPT_HIP_{CRS,ELL,SS,DIA,HYB,CSS,COO,JDS,BIN} that is defined
 * (default AUTO); the environment variable SPMV_HIP_FORMAT
 * (crs|csr|ell|ss|dia|hyb|css|coo|jds|bin|auto, case-insensitive; anything
 * else means auto) overrides it at run time.
 *
 * CRS keeps opt_crs's semantics, not its storage: every row is the
 * sequential column-order sum bit for bit (src/opt_crs.cpp:57-69) on the
 * fastest layout that sums so for the matrix (spmv_options_t.crs_exact: DIA
 * for a band, BIN for a wide random x -- 3.6x the CSR kernels at config 2 --,
 * sliced ELL for near-uniform short rows, else one-lane CSR).  The layout is
 * in SpMatOpt.format (spmv_plan_info).  SPMV_HIP_CRS_EXACT=0 selects the CSR
 * kernels themselves (row groups of lanes with butterfly sums: within 1e-12,
 * not bit-exact).
 *
 * x handling follows the reference: x_opt.val aliases the caller's x
 * (src/opt_crs.cpp:11-12) and SpMV uploads it on every call the way
 * opt_cusparse does (src/opt_cusparse.cpp:72).  SPMV_HIP_X_RESIDENT=1 uploads
 * x only on the first call (the reference driver never changes x,
 * src/main.cpp:36-102).  y is downloaded on every call (opt_cusparse.cpp:82)
 * unless SPMV_HIP_Y_RESIDENT=1: y then stays on the device (SPMV_Y_STAGED)
 * and the caller fetches it with SpMVFetch before reading it -- a driver
 * change (tools/spmv_main.cpp --device-y), since the reference main.cpp
 * reads y after SpMV; at config 2 the 80 MB download per call is 1.5 ms of
 * PCIe against a 0.8 ms kernel.
 *
 * Multi-GPU: SPMV_HIP_GPUS=N (set, N >= 1) makes OptimizeProblem build a dist plan
 * over devices 0..N-1 (spmv_dist_create_csr: nnz-balanced row ranges, one
 * plan per device, x broadcast and y all-gathered by RCCL over xGMI) and SpMV
 * run it -- the unchanged reference driver then spans the node (BASELINE
 * config 5).  SPMV_HIP_X_RESIDENT applies to the broadcast x the same way.
 *
 * Errors: the signatures are void, so a failure prints spmv_last_error() and
 * exits, as CUDA_SAFE_CALL does in the reference (src/util.h:48-55).
 */
#ifndef OPT_HIP_H
#define OPT_HIP_H

#ifndef OPT_HIP_USE_REFERENCE_TYPES
#include "spmv_util.h"
#endif
#include "spmv_hip.h"

struct SpMatOpt {
    int nRow;
    int nCol;
    int nNnz;
    spmv_plan_t plan;
    int format;       /* resolved spmv_format_t */
    double *d_x;      /* device copy of x (owned by the plan's allocator) */
    int x_uploaded;
    spmv_dist_t dist; /* SPMV_HIP_GPUS > 1: the multi-GPU plan (plan is NULL) */
    int n_gpus;
};

struct VecOpt {
    int size;
    double *val;
};

void OptimizeProblem(const SpMat &A, const Vec &x, SpMatOpt &A_opt, VecOpt &x_opt);
extern "C" {
void SpMV(const SpMatOpt &A, const VecOpt &x, Vec &y);
/* (new) release the plan -- the reference never frees its SpMatOpt */
void SpMVRelease(SpMatOpt &A);
/* (new) SPMV_HIP_Y_RESIDENT=1: copy the y of the last SpMV to the host */
void SpMVFetch(const SpMatOpt &A, Vec &y);
}

#endif /* OPT_HIP_H */

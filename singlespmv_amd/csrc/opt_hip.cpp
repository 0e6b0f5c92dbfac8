// opt_hip.cpp -- the drop-in OptimizeProblem / SpMV of include/opt_hip.h.
//
// Compile this file into the driver (as the reference's opt.cpp #includes its
// plugin, src/opt.cpp:1-33) so -DOPT_HIP_<FMT> selects the format; it is
// also built as libopt_hip.so (format from SPMV_HIP_FORMAT, default AUTO) for
// the ABI tests.
#include "opt_hip.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>

#include <vector>

static int opt_hip_format() {
    int f = SPMV_FORMAT_AUTO;
#if defined(OPT_HIP_CRS)
    f = SPMV_FORMAT_CSR;
#elif defined(OPT_HIP_ELL)
    f = SPMV_FORMAT_ELL;
#elif defined(OPT_HIP_SS)
    f = SPMV_FORMAT_SS;
#elif defined(OPT_HIP_DIA)
    f = SPMV_FORMAT_DIA;
#elif defined(OPT_HIP_HYB)
    f = SPMV_FORMAT_HYB;
#elif defined(OPT_HIP_CSS)
    f = SPMV_FORMAT_CSS;
#elif defined(OPT_HIP_COO)
    f = SPMV_FORMAT_COO;
#elif defined(OPT_HIP_JDS)
    f = SPMV_FORMAT_JDS;
#elif defined(OPT_HIP_BIN)
    f = SPMV_FORMAT_BIN;
#endif
    const char *e = std::getenv("SPMV_HIP_FORMAT");
    if (e && *e) {
        if (!strcasecmp(e, "crs") || !strcasecmp(e, "csr")) f = SPMV_FORMAT_CSR;
        else if (!strcasecmp(e, "ell")) f = SPMV_FORMAT_ELL;
        else if (!strcasecmp(e, "ss")) f = SPMV_FORMAT_SS;
        else if (!strcasecmp(e, "dia")) f = SPMV_FORMAT_DIA;
        else if (!strcasecmp(e, "hyb")) f = SPMV_FORMAT_HYB;
        else if (!strcasecmp(e, "css")) f = SPMV_FORMAT_CSS;
        else if (!strcasecmp(e, "coo")) f = SPMV_FORMAT_COO;
        else if (!strcasecmp(e, "jds")) f = SPMV_FORMAT_JDS;
        else if (!strcasecmp(e, "bin")) f = SPMV_FORMAT_BIN;
        else f = SPMV_FORMAT_AUTO;
    }
    return f;
}

static void opt_hip_die(const char *what, int st) {
    std::fprintf(stderr, "[Error] %s: %s (%s)\n", what, spmv_status_string(st), spmv_last_error());
    std::exit(st ? st : 1);
}

void OptimizeProblem(const SpMat &A, const Vec &x, SpMatOpt &A_opt, VecOpt &x_opt) {
    // x_opt aliases the caller's x, as every reference plugin does
    // (src/opt_crs.cpp:11-12)
    x_opt.size = x.size;
    x_opt.val = x.val;
    spmv_options_t o;
    spmv_options_default(&o);
    o.format = opt_hip_format();
    // SPMV_HIP_EXACT=1: every row the sequential opt_crs sum bit for bit --
    // BIN keeps long power-law rows off its run path (spmv_hip.h bin_long_len)
    if (const char *ex = std::getenv("SPMV_HIP_EXACT"))
        if (std::atoi(ex) != 0) o.bin_long_len = -1;
    // CRS is the opt_crs plugin: its semantics (each row's sequential sum,
    // src/opt_crs.cpp:57-69) on the fastest layout that keeps them
    // (spmv_options_t.crs_exact); SPMV_HIP_CRS_EXACT=0 asks for the CSR
    // kernels themselves (row groups of lanes, butterfly sums)
    if (o.format == SPMV_FORMAT_CSR) {
        const char *ce = std::getenv("SPMV_HIP_CRS_EXACT");
        o.crs_exact = (ce && *ce && std::atoi(ce) == 0) ? 0 : 1;
    }
    A_opt.nRow = A.nRow;
    A_opt.nCol = A.nCol;
    A_opt.nNnz = A.nNnz;
    A_opt.plan = nullptr;
    A_opt.dist = nullptr;
    A_opt.d_x = nullptr;
    A_opt.x_uploaded = 0;
    A_opt.n_gpus = 1;
    const char *gpus = std::getenv("SPMV_HIP_GPUS");
    if (gpus && *gpus) A_opt.n_gpus = std::atoi(gpus) > 1 ? std::atoi(gpus) : 1;
    if (gpus && *gpus) {  // set (even to 1): the multi-GPU plan
        // the rows over n_gpus devices: COO -> CSR row pointers, one dist plan
        std::vector<int64_t> rp((size_t)A.nRow + 1);
        int st = spmv_coo_to_csr(A.nRow, A.nNnz, A.row_idx, rp.data());
        if (st != SPMV_SUCCESS) opt_hip_die("OptimizeProblem", st);
        st = spmv_dist_create_csr(A_opt.n_gpus, nullptr, A.nRow, A.nCol, A.nNnz, rp.data(), A.col_idx, A.val, &o,
                                  &A_opt.dist);
        if (st != SPMV_SUCCESS) opt_hip_die("OptimizeProblem (SPMV_HIP_GPUS)", st);
        spmv_plan_t p0 = nullptr;
        int32_t nd = 0;
        spmv_dist_info(A_opt.dist, &nd, nullptr, nullptr);
        std::vector<spmv_plan_t> plans((size_t)nd);
        spmv_dist_info(A_opt.dist, &nd, nullptr, plans.data());
        p0 = plans[0];
        spmv_plan_info_t info;
        spmv_plan_info(p0, &info);
        A_opt.format = info.format;
        return;
    }
    spmv_plan_t plan = nullptr;
    const int st = spmv_plan_create_coo(A.nRow, A.nCol, A.nNnz, A.row_idx, A.col_idx, A.val, &o, &plan);
    if (st != SPMV_SUCCESS) opt_hip_die("OptimizeProblem", st);
    spmv_plan_info_t info;
    spmv_plan_info(plan, &info);
    A_opt.plan = plan;
    A_opt.format = info.format;
}

extern "C" {

static bool env_flag(const char *name) {
    const char *e = std::getenv(name);
    return e && *e == '1';
}

void SpMV(const SpMatOpt &A, const VecOpt &x, Vec &y) {
    // read per call (a getenv is ~0.1 us against a >= 2 us launch), so a
    // process may switch modes between plans
    const bool resident = env_flag("SPMV_HIP_X_RESIDENT"), y_resident = env_flag("SPMV_HIP_Y_RESIDENT");
    SpMatOpt &a = const_cast<SpMatOpt &>(A);  // the reference passes const& too
    const bool staged_x = resident && a.x_uploaded;
    int st;
    if (a.dist) {  // SPMV_HIP_GPUS: H2D x, RCCL broadcast, local SpMVs, RCCL all-gather, D2H y
        st = spmv_dist_execute(a.dist, staged_x ? nullptr : x.val, y_resident ? nullptr : y.val,
                               staged_x ? SPMV_X_STAGED : 0u);
    } else {
        // H2D x (or the staged copy), kernels, D2H y (or y left staged)
        st = spmv_execute(a.plan, staged_x ? nullptr : x.val, y_resident ? nullptr : y.val,
                          (staged_x ? SPMV_X_STAGED : 0u) | (y_resident ? SPMV_Y_STAGED : 0u));
    }
    a.x_uploaded = 1;
    if (st != SPMV_SUCCESS) opt_hip_die("SpMV", st);
}

void SpMVFetch(const SpMatOpt &A, Vec &y) {
    const int st = A.dist ? spmv_dist_fetch_y(A.dist, y.val) : spmv_fetch_y(A.plan, y.val);
    if (st != SPMV_SUCCESS) opt_hip_die("SpMVFetch", st);
}

void SpMVRelease(SpMatOpt &A) {
    spmv_plan_destroy(A.plan);
    spmv_dist_destroy(A.dist);
    A.plan = nullptr;
    A.dist = nullptr;
}

}  // extern "C"

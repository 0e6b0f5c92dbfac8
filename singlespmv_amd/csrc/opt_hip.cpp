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
    spmv_plan_t plan = nullptr;
    const int st = spmv_plan_create_coo(A.nRow, A.nCol, A.nNnz, A.row_idx, A.col_idx, A.val, &o, &plan);
    if (st != SPMV_SUCCESS) opt_hip_die("OptimizeProblem", st);
    spmv_plan_info_t info;
    spmv_plan_info(plan, &info);
    A_opt.nRow = A.nRow;
    A_opt.nCol = A.nCol;
    A_opt.nNnz = A.nNnz;
    A_opt.plan = plan;
    A_opt.format = info.format;
    A_opt.d_x = nullptr;
    A_opt.x_uploaded = 0;
}

extern "C" {

void SpMV(const SpMatOpt &A, const VecOpt &x, Vec &y) {
    static int resident = -1;
    if (resident < 0) {
        const char *e = std::getenv("SPMV_HIP_X_RESIDENT");
        resident = (e && *e == '1') ? 1 : 0;
    }
    SpMatOpt &a = const_cast<SpMatOpt &>(A);  // the reference passes const& too
    int st;
    if (!resident) {
        st = spmv_execute(a.plan, x.val, y.val, 0u);  // H2D x, kernels, D2H y
    } else {
        if (!a.x_uploaded) {
            st = spmv_execute(a.plan, x.val, y.val, 0u);
            a.x_uploaded = 1;
        } else {
            st = spmv_execute(a.plan, nullptr, y.val, SPMV_X_STAGED);
        }
    }
    if (st != SPMV_SUCCESS) opt_hip_die("SpMV", st);
}

void SpMVRelease(SpMatOpt &A) {
    spmv_plan_destroy(A.plan);
    A.plan = nullptr;
}

}  // extern "C"

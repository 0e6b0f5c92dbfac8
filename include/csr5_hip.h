/* csr5_hip.h -- drop-in for the CSR5 benchmark's handle API vendored in the
 * reference (opt/Benchmark_SpMV_using_CSR5/CSR5_cuda/anonymouslib_cuda.h:11-53,
 * return codes detail/common.h:13-22), on top of libspmv_hip's C-ABI: the
 * benchmark's driver (CSR5_cuda/main.cu: call_anonymouslib) keeps its calls
 *
 *     anonymouslibHandle<int, unsigned int, double> A(m, n);
 *     A.inputCSR(nnz, d_row_ptr, d_col_idx, d_val);   // device arrays
 *     A.setX(d_x);
 *     A.setSigma(ANONYMOUSLIB_AUTO_TUNED_SIGMA);
 *     A.warmup();
 *     A.asCSR5();                                      // format conversion
 *     A.spmv(alpha, d_y);                              // y = alpha * A * x
 *     A.destroy();
 *
 * Differences, all in the caller's favour:
 *  - asCSR5 converts on the device into the plan's own storage (the SS tile
 *    layout: 64 lanes x sigma, not CSR5's 32 x sigma); the caller's CSR arrays
 *    are only read -- CSR5 transposes them in place and restores them in
 *    asCSR/destroy (anonymouslib_cuda.h:203-204, 286-291);
 *  - spmv overwrites y (beta = 0) and repeated calls are identical
 *    (CSR5 is not);
 *  - sigma is rounded to the SS kernel's supported set {4,8,...,24,32,48,64}
 *    (the benchmark's auto rule picks at most 32; 48 / 64 by setSigma).
 * Only <int, unsigned int, double> is instantiable (fp64 engine). */
#ifndef CSR5_HIP_H
#define CSR5_HIP_H

#include <type_traits>

#include "spmv_hip.h"

#ifndef ANONYMOUSLIB_SUCCESS
#define ANONYMOUSLIB_SUCCESS 0
#define ANONYMOUSLIB_UNKOWN_FORMAT -1
#define ANONYMOUSLIB_UNSUPPORTED_CSR5_OMEGA -2
#define ANONYMOUSLIB_CSR_TO_CSR5_FAILED -3
#define ANONYMOUSLIB_UNSUPPORTED_CSR_SPMV -4
#define ANONYMOUSLIB_UNSUPPORTED_VALUE_TYPE -5
#define ANONYMOUSLIB_FORMAT_CSR 0
#define ANONYMOUSLIB_FORMAT_CSR5 1
#define ANONYMOUSLIB_FORMAT_HYB5 2
#endif
#ifndef ANONYMOUSLIB_AUTO_TUNED_SIGMA
#define ANONYMOUSLIB_AUTO_TUNED_SIGMA -1
#endif
#define ANONYMOUSLIB_CSR5_OMEGA_HIP 64 /* lanes per tile (wave64) */

template <class ANONYMOUSLIB_IT, class ANONYMOUSLIB_UIT, class ANONYMOUSLIB_VT>
class anonymouslibHandle {
    static_assert(std::is_same<ANONYMOUSLIB_IT, int>::value && std::is_same<ANONYMOUSLIB_VT, double>::value,
                  "libspmv_hip is an fp64 engine with int32 indices: anonymouslibHandle<int, unsigned, double>");

public:
    anonymouslibHandle(ANONYMOUSLIB_IT m, ANONYMOUSLIB_IT n) : _m(m), _n(n) {}
    ~anonymouslibHandle() { drop(); }
    anonymouslibHandle(const anonymouslibHandle &) = delete;
    anonymouslibHandle &operator=(const anonymouslibHandle &) = delete;

    int warmup() { return ANONYMOUSLIB_SUCCESS; }

    int inputCSR(ANONYMOUSLIB_IT nnz, ANONYMOUSLIB_IT *csr_row_pointer, ANONYMOUSLIB_IT *csr_column_index,
                 ANONYMOUSLIB_VT *csr_value) {
        drop();
        _format = ANONYMOUSLIB_FORMAT_CSR;
        _nnz = nnz;
        _rp = csr_row_pointer;
        _col = csr_column_index;
        _val = csr_value;
        return ANONYMOUSLIB_SUCCESS;
    }

    /* CSR5 -> CSR: the plan is released (the caller's arrays never changed) */
    int asCSR() {
        drop();
        _format = ANONYMOUSLIB_FORMAT_CSR;
        return ANONYMOUSLIB_SUCCESS;
    }

    int asCSR5() {
        if (_format == ANONYMOUSLIB_FORMAT_CSR5) return ANONYMOUSLIB_SUCCESS;
        spmv_options_t o;
        spmv_options_default(&o);
        o.format = SPMV_FORMAT_SS;
        if (_sigma == ANONYMOUSLIB_AUTO_TUNED_SIGMA) setSigma(ANONYMOUSLIB_AUTO_TUNED_SIGMA);
        o.ss_sigma = supported_sigma(_sigma);
        if (spmv_plan_create_csr32_device(_m, _n, _nnz, _rp, _col, _val, &o, &_plan) != SPMV_SUCCESS) {
            _plan = nullptr;
            return ANONYMOUSLIB_CSR_TO_CSR5_FAILED;
        }
        _format = ANONYMOUSLIB_FORMAT_CSR5;
        return ANONYMOUSLIB_SUCCESS;
    }

    int setX(ANONYMOUSLIB_VT *x) {
        _x = x;
        return ANONYMOUSLIB_SUCCESS;
    }

    /* y = alpha * A * x, device x and y (anonymouslib_cuda.h:262-284) */
    int spmv(const ANONYMOUSLIB_VT alpha, ANONYMOUSLIB_VT *y) {
        if (_format == ANONYMOUSLIB_FORMAT_CSR) return ANONYMOUSLIB_UNSUPPORTED_CSR_SPMV;
        if (spmv_execute_alpha(_plan, alpha, _x, y, SPMV_X_DEVICE | SPMV_Y_DEVICE) != SPMV_SUCCESS)
            return ANONYMOUSLIB_UNKOWN_FORMAT;
        return ANONYMOUSLIB_SUCCESS;
    }

    int destroy() { return asCSR(); }

    /* the benchmark's auto rule (anonymouslib_cuda.h:294-317), on nnz/m */
    void setSigma(int sigma) {
        if (sigma == ANONYMOUSLIB_AUTO_TUNED_SIGMA) {
            const int nnz_per_row = _m ? _nnz / _m : 0;
            if (nnz_per_row <= 4) _sigma = 4;
            else if (nnz_per_row <= 32) _sigma = nnz_per_row;
            else if (nnz_per_row <= 256) _sigma = 32;
            else _sigma = 6;
        } else {
            _sigma = sigma;
        }
    }

    /* the engine's own plan (e.g. for spmv_plan_info / spmv_profile) */
    spmv_plan_t plan() const { return _plan; }

private:
    /* the SS kernel's sigma set {4,8,...,24,32,48,64}: the nearest member
     * (ties upward); an explicit setSigma beyond 64 takes 64 */
    static int supported_sigma(int s) {
        static const int kSet[] = {4, 8, 12, 16, 20, 24, 32, 48, 64};
        int best = kSet[0];
        for (int c : kSet)
            if ((c > s ? c - s : s - c) <= (best > s ? best - s : s - best)) best = c;
        return best;
    }
    void drop() {
        if (_plan) spmv_plan_destroy(_plan);
        _plan = nullptr;
    }

    int _format = ANONYMOUSLIB_FORMAT_CSR;
    ANONYMOUSLIB_IT _m, _n, _nnz = 0;
    ANONYMOUSLIB_IT *_rp = nullptr, *_col = nullptr;
    ANONYMOUSLIB_VT *_val = nullptr, *_x = nullptr;
    int _sigma = ANONYMOUSLIB_AUTO_TUNED_SIGMA;
    spmv_plan_t _plan = nullptr;
};

#endif /* CSR5_HIP_H */

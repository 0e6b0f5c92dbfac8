// capi.cpp -- the C-ABI of include/spmv_hip.h: plan life cycle, execute,
// timing, info.  Every entry point returns an int status; nothing exit()s.
#include <omp.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "internal.hpp"

namespace spmv {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
const char *last_error() { return g_err.c_str(); }

// Placement of the streamed arrays of the row-parallel formats (CSR, ELL,
// HYB, JDS, SS, COO, CSS; BIN and DIA place their large buffer themselves):
// AUTO maps every array of >= kStreamVmmMinBytes into 2-MB VMM handles
// (config 4, same launches on both placements, interleaved in one process:
// CSR 2.95 -> 2.81 ms, ELL 2.57 -> 2.40; profiles/round4/probe/
// c4_csr_vec4_slab_caps_vmm_plain.jsonl, c4_ell_caps_unroll_vmm_plain.jsonl), VMM does so from 32 MB, PLAIN never.
static void stream_placement(spmv_plan_s *p, int fmt, const spmv_options_t &o) {
    if (fmt == SPMV_FORMAT_BIN || fmt == SPMV_FORMAT_DIA) return;
    if (o.placement == SPMV_PLACEMENT_AUTO) p->arena.vmm_min = kStreamVmmMinBytes;
    else if (o.placement == SPMV_PLACEMENT_VMM) p->arena.vmm_min = kBinVmmMinBytes;
    if (const char *e = probe_env("SPMV_ARENA_VMM_MB")) p->arena.vmm_min = (size_t)std::max(0, std::atoi(e)) << 20;
}

static int check_device(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible (libspmv_hip needs an MI355X / gfx950)");
        return SPMV_ERROR_NO_DEVICE;
    }
    if (device >= count) {
        set_error("device ordinal out of range");
        return SPMV_ERROR_INVALID_VALUE;
    }
    hipDeviceProp_t prop;
    SPMV_HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error(std::string("device is ") + prop.gcnArchName + "; kernels are built for gfx950 only");
        return SPMV_ERROR_NO_DEVICE;
    }
    return SPMV_SUCCESS;
}

// Validate a host CSR before anything touches the GPU: an out-of-range
// column would become an out-of-bounds gather on the device.
static int validate_csr(const HostCsr &A) {
    SPMV_CHECK_ARG(A.m >= 0 && A.n >= 0 && A.nnz >= 0, "negative dimension");
    SPMV_CHECK_ARG(A.m < (int64_t)INT32_MAX && A.n < (int64_t)INT32_MAX,
                   "m and n must be < 2^31 (int32 column indices)");
    SPMV_CHECK_ARG(A.row_ptr != nullptr, "row_ptr is NULL");
    SPMV_CHECK_ARG(A.nnz == 0 || (A.col != nullptr && A.val != nullptr), "col/val is NULL");
    SPMV_CHECK_ARG(A.row_ptr[0] == 0, "row_ptr[0] != 0");
    SPMV_CHECK_ARG(A.row_ptr[A.m] == A.nnz, "row_ptr[m] != nnz");
    int64_t bad_rp = 0, bad_col = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad_rp)
    for (int64_t r = 0; r < A.m; ++r) bad_rp += A.row_ptr[r + 1] < A.row_ptr[r];
    SPMV_CHECK_ARG(bad_rp == 0, "row_ptr is not non-decreasing");
    const int64_t n = A.n;
#pragma omp parallel for schedule(static) reduction(+ : bad_col)
    for (int64_t j = 0; j < A.nnz; ++j) bad_col += (A.col[j] < 0) | (A.col[j] >= n);
    SPMV_CHECK_ARG(bad_col == 0, "column index outside [0, n)");
    return SPMV_SUCCESS;
}

// spmv_options_t::build AUTO: host CSRs from this many entries up are built
// by the device builders (config 4's DIA plan: 10.3 s through the host
// builders; below this size a host build takes well under a second)
constexpr int64_t kDeviceBuildMinNnz = (int64_t)1 << 24;

static int create_from_csr(const HostCsr &A, const spmv_options_t *opt_in, spmv_plan_t *out);

// spmv_plan_create_csr_device's body.  A plan the device builders do not
// make (BIN rows out of strip order when the device has no room for their
// sorted copy) is built by the host builders: from a D2H copy of the CSR, or --
// when need_host_fmt is given (create_via_device, whose caller still holds the
// host CSR) -- by returning kNeedHostBuild with the resolved options there
// (format chosen, crs_exact's rewrites applied, build = HOST).
constexpr int kNeedHostBuild = -2000;
static int create_device_impl(int64_t m, int64_t n, int64_t nnz, const int64_t *d_row_ptr,
                              const int32_t *d_col_idx, const double *d_val, const spmv_options_t *opt_in,
                              spmv_plan_t *out, spmv_options_t *need_host) {
    SPMV_CHECK_ARG(out != nullptr, "plan out-pointer is NULL");
    *out = nullptr;
    spmv_options_t o;
    if (opt_in) o = *opt_in;
    else spmv_options_default(&o);
    SPMV_CHECK_ARG(m >= 0 && n >= 0 && nnz >= 0, "negative dimension");
    SPMV_CHECK_ARG(m < (int64_t)INT32_MAX && n < (int64_t)INT32_MAX, "m and n must be < 2^31 (int32 column indices)");
    SPMV_CHECK_ARG(d_row_ptr != nullptr, "row_ptr is NULL");
    SPMV_CHECK_ARG(nnz == 0 || (d_col_idx != nullptr && d_val != nullptr), "col/val is NULL");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible (libspmv_hip needs an MI355X / gfx950)");
        return SPMV_ERROR_NO_DEVICE;
    }
    int dev = o.device;
    if (dev < 0) SPMV_HIP_TRY(hipGetDevice(&dev));
    SPMV_RETURN_IF(check_device(dev));
    SPMV_HIP_TRY(hipSetDevice(dev));
    const void *ptrs[3] = {d_row_ptr, d_col_idx, d_val};
    for (int k = 0; k < (nnz ? 3 : 1); ++k) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, ptrs[k]) != hipSuccess || a.type != hipMemoryTypeDevice || a.device != dev) {
            (void)hipGetLastError();
            set_error("spmv_plan_create_csr_device: arrays must be device memory on the plan's device");
            return SPMV_ERROR_INVALID_VALUE;
        }
    }
    SPMV_RETURN_IF(validate_csr_device(d_row_ptr, m, d_col_idx, nnz, n));
    spmv_plan_s *p = new (std::nothrow) spmv_plan_s;
    if (!p) {
        set_error("host allocation of the plan failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    p->device = dev;
    p->arena.device = dev;
    if (const char *e = probe_env("SPMV_ARENA_VMM_MB")) p->arena.vmm_min = (size_t)std::max(0, std::atoi(e)) << 20;
    p->m = m;
    p->n = n;
    p->nnz = nnz;
    // the row pointers are the only part of the matrix the host sees: row
    // lengths drive AUTO and every slice / bin / overflow decision
    std::vector<int64_t> hrp;
    const bool need_rp = o.format == SPMV_FORMAT_AUTO || o.format == SPMV_FORMAT_ELL || o.format == SPMV_FORMAT_HYB ||
                         o.format == SPMV_FORMAT_JDS || o.format == SPMV_FORMAT_CSS ||
                         (o.format == SPMV_FORMAT_CSR && o.crs_exact);
    if (need_rp) {
        hrp.resize((size_t)m + 1);
        const hipError_t e = hipMemcpy(hrp.data(), d_row_ptr, 8 * (size_t)(m + 1), hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            delete p;
            set_error(std::string("row_ptr to host: ") + hipGetErrorString(e));
            (void)hipGetLastError();
            return SPMV_ERROR_HIP;
        }
    }
    const DevCsr A{m, n, nnz, hrp.data(), d_row_ptr, d_col_idx, d_val};
    int fmt = o.format, st = SPMV_SUCCESS;
    if (fmt == SPMV_FORMAT_AUTO) {
        int census = SPMV_SUCCESS;
        fmt = choose_format_rp(m, n, nnz, hrp.data(), o, [&]() {
            std::vector<int32_t> offs;
            census = dia_offsets_device(p, A, 256, 1.25, offs);
            return census == SPMV_SUCCESS;
        });
        if (census != SPMV_SUCCESS && census != kDiaRefused) st = census;
    }
    if (st == SPMV_SUCCESS && fmt == SPMV_FORMAT_CSR && o.crs_exact) {
        int census = SPMV_SUCCESS;
        fmt = choose_crs_exact(
            m, n, nnz, hrp.data(), o,
            [&]() {
                std::vector<int32_t> offs;
                census = dia_offsets_device(p, A, 256, 1.25, offs);
                return census == SPMV_SUCCESS;
            },
            [&]() {
                int order = kRowsUnsorted;
                const int s2 = rows_order_device(p, A, &order);
                if (s2 != SPMV_SUCCESS) census = s2;
                return order;
            });
        if (census != SPMV_SUCCESS && census != kDiaRefused) st = census;
    }
    const double mean = m ? (double)nnz / (double)m : 0.0;
    bool host_build = false;
    if (st == SPMV_SUCCESS) {
        stream_placement(p, fmt, o);
        switch (fmt) {
            case SPMV_FORMAT_CSR: st = build_csr_device(p, d_row_ptr, d_col_idx, d_val, o, mean); break;
            case SPMV_FORMAT_SS: st = build_ss_device(p, d_row_ptr, d_col_idx, d_val, o, mean); break;
            case SPMV_FORMAT_DIA: st = build_dia_device(p, A, o); break;
            case SPMV_FORMAT_ELL: st = build_ell_device(p, A, o); break;
            case SPMV_FORMAT_HYB: st = build_hyb_device(p, A, o); break;
            case SPMV_FORMAT_JDS: st = build_jds_device(p, A, o); break;
            case SPMV_FORMAT_COO: st = build_coo_device(p, A, o); break;
            case SPMV_FORMAT_BIN:
                if (probe_env("SPMV_BIN_HOST_BUILD")) host_build = true;
                else st = build_bin_device(p, d_row_ptr, d_col_idx, d_val, o);
                // (kBinNeedHostBuild: rows out of strip order and no room
                // for their sorted copy -- the host builder below)
                if (st == kBinNeedHostBuild) host_build = true;
                break;
            case SPMV_FORMAT_CSS: st = build_css_device(p, A, o); break;
            default:
                set_error("unknown format");
                st = SPMV_ERROR_INVALID_VALUE;
        }
    }
    if (st == SPMV_SUCCESS && !host_build) {
        p->format = fmt;
        p->built_on_device = 1;
        *out = p;
        return SPMV_SUCCESS;
    }
    p->arena.release();
    delete p;
    if (!host_build) return st;
    if (need_host) {
        *need_host = o;
        need_host->device = dev;
        need_host->format = fmt;  // AUTO resolved above
        need_host->build = SPMV_BUILD_HOST;
        return kNeedHostBuild;
    }
    {
        // host builders: stage the CSR through host memory
        std::vector<int64_t> rp((size_t)m + 1);
        std::vector<int32_t> col((size_t)nnz);
        std::vector<double> val((size_t)nnz);
        SPMV_HIP_TRY(hipMemcpy(rp.data(), d_row_ptr, 8 * (size_t)(m + 1), hipMemcpyDeviceToHost));
        if (nnz) {
            SPMV_HIP_TRY(hipMemcpy(col.data(), d_col_idx, 4 * (size_t)nnz, hipMemcpyDeviceToHost));
            SPMV_HIP_TRY(hipMemcpy(val.data(), d_val, 8 * (size_t)nnz, hipMemcpyDeviceToHost));
        }
        o.device = dev;
        o.format = fmt;  // AUTO resolved above
        o.build = SPMV_BUILD_HOST;
        HostCsr H{m, n, nnz, rp.data(), col.data(), val.data()};
        return create_from_csr(H, &o, out);
    }
}

// Stage a (validated) host CSR into HBM and build the plan there
// (create_device_impl: the same layouts byte for byte, AUTO resolved by the
// same chooser).  A format the device builders do not make comes back as
// kNeedHostBuild with the resolved options in *host_opts;
// SPMV_ERROR_OUT_OF_MEMORY when the staging copy does not fit.  Either way
// the caller then takes the host builders.
static int create_via_device(const HostCsr &A, spmv_options_t o, int dev, spmv_plan_t *out,
                             spmv_options_t *host_opts) {
    void *d[3] = {nullptr, nullptr, nullptr};
    const size_t bytes[3] = {8 * (size_t)(A.m + 1), 4 * (size_t)std::max<int64_t>(A.nnz, 1),
                             8 * (size_t)std::max<int64_t>(A.nnz, 1)};
    auto release = [&]() {
        (void)hipDeviceSynchronize();  // the builders' kernels have read the staging copy
        for (void *q : d)
            if (q) (void)hipFree(q);
    };
    for (int k = 0; k < 3; ++k)
        if (hipMalloc(&d[k], bytes[k]) != hipSuccess) {
            (void)hipGetLastError();
            release();
            set_error("device staging of the CSR: out of device memory");
            return SPMV_ERROR_OUT_OF_MEMORY;
        }
    hipError_t e = hipMemcpy(d[0], A.row_ptr, bytes[0], hipMemcpyHostToDevice);
    if (e == hipSuccess && A.nnz) e = hipMemcpy(d[1], A.col, 4 * (size_t)A.nnz, hipMemcpyHostToDevice);
    if (e == hipSuccess && A.nnz) e = hipMemcpy(d[2], A.val, 8 * (size_t)A.nnz, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        release();
        set_error(std::string("device staging of the CSR: ") + hipGetErrorString(e));
        return SPMV_ERROR_HIP;
    }
    o.device = dev;
    const int st = create_device_impl(A.m, A.n, A.nnz, (const int64_t *)d[0], (const int32_t *)d[1],
                                      (const double *)d[2], &o, out, host_opts);
    release();
    return st;
}

static int create_from_csr(const HostCsr &A, const spmv_options_t *opt_in, spmv_plan_t *out) {
    SPMV_CHECK_ARG(out != nullptr, "plan out-pointer is NULL");
    *out = nullptr;
    spmv_options_t o;
    if (opt_in) o = *opt_in;
    else spmv_options_default(&o);
    SPMV_CHECK_ARG(o.build >= SPMV_BUILD_AUTO && o.build <= SPMV_BUILD_DEVICE, "build must be SPMV_BUILD_*");
    SPMV_RETURN_IF(validate_csr(A));
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible (libspmv_hip needs an MI355X / gfx950)");
        return SPMV_ERROR_NO_DEVICE;
    }
    int dev = o.device;
    if (dev < 0) SPMV_HIP_TRY(hipGetDevice(&dev));
    SPMV_RETURN_IF(check_device(dev));
    SPMV_HIP_TRY(hipSetDevice(dev));
    // the device builders make every format; what they cannot (BIN rows out
    // of strip order without room for their sorted copy) and a staging copy
    // that does not fit take the host builders below -- with the format AUTO
    // resolved on the device
    if (o.build == SPMV_BUILD_DEVICE || (o.build == SPMV_BUILD_AUTO && A.nnz >= kDeviceBuildMinNnz)) {
        spmv_options_t ho = o;
        const int st = create_via_device(A, o, dev, out, &ho);
        if (st != SPMV_ERROR_OUT_OF_MEMORY && st != kNeedHostBuild) return st;
        if (st == kNeedHostBuild) o = ho;
        SPMV_HIP_TRY(hipSetDevice(dev));
    }
    spmv_plan_s *p = new (std::nothrow) spmv_plan_s;
    if (!p) {
        set_error("host allocation of the plan failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    p->device = dev;
    p->arena.device = dev;
    if (const char *e = probe_env("SPMV_ARENA_VMM_MB")) p->arena.vmm_min = (size_t)std::max(0, std::atoi(e)) << 20;
    p->m = A.m;
    p->n = A.n;
    p->nnz = A.nnz;
    int fmt = o.format == SPMV_FORMAT_AUTO ? choose_format(A, o) : o.format;
    if (fmt == SPMV_FORMAT_CSR && o.crs_exact) fmt = choose_crs_exact(A, o);
    stream_placement(p, fmt, o);
    int st;
    switch (fmt) {
        case SPMV_FORMAT_CSR: st = build_csr(p, A, o); break;
        case SPMV_FORMAT_ELL: st = build_ell(p, A, o, INT32_MAX); break;
        case SPMV_FORMAT_HYB: st = build_hyb(p, A, o); break;
        case SPMV_FORMAT_SS: st = build_ss(p, A, o); break;
        case SPMV_FORMAT_DIA: st = build_dia(p, A, o); break;
        case SPMV_FORMAT_CSS: st = build_css(p, A, o); break;
        case SPMV_FORMAT_COO: st = build_coo(p, A, o); break;
        case SPMV_FORMAT_JDS: st = build_jds(p, A, o); break;
        case SPMV_FORMAT_BIN: st = build_bin(p, A, o); break;
        default:
            set_error("unknown format");
            st = SPMV_ERROR_INVALID_VALUE;
    }
    if (st != SPMV_SUCCESS) {
        p->arena.release();
        delete p;
        return st;
    }
    p->format = fmt;
    *out = p;
    return SPMV_SUCCESS;
}

static int dispatch(const spmv_plan_s *p, const double *x, double *y) {
    switch (p->format) {
        case SPMV_FORMAT_CSR: return launch_csr(p, x, y);
        case SPMV_FORMAT_ELL: return launch_ell(p, x, y);
        case SPMV_FORMAT_HYB:
            SPMV_RETURN_IF(launch_ell(p, x, y));
            phase_mark(p);  // ell | overflow
            return launch_hyb_overflow(p, x, y);
        case SPMV_FORMAT_SS: return launch_ss(p, x, y);
        case SPMV_FORMAT_DIA: return launch_dia(p, x, y);
        case SPMV_FORMAT_CSS: return launch_css(p, x, y);
        case SPMV_FORMAT_COO: return launch_coo(p, x, y);
        case SPMV_FORMAT_JDS:
            SPMV_RETURN_IF(launch_ell(p, x, y));
            phase_mark(p);  // ell | overflow
            return launch_hyb_overflow(p, x, y);
        case SPMV_FORMAT_BIN: return launch_bin(p, x, y);
    }
    set_error("plan has an unknown format");
    return SPMV_ERROR_INVALID_VALUE;
}

static int bind_device(const spmv_plan_s *p) {
    int cur = -1;
    SPMV_HIP_TRY(hipGetDevice(&cur));
    if (cur != p->device) SPMV_HIP_TRY(hipSetDevice(p->device));
    return SPMV_SUCCESS;
}

}  // namespace spmv

using namespace spmv;

extern "C" {

int spmv_api_version(void) { return SPMV_HIP_API_VERSION; }

void spmv_options_default(spmv_options_t *o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->format = SPMV_FORMAT_AUTO;
    o->device = -1;
}

int spmv_plan_create_csr(int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr,
                         const int32_t *col_idx, const double *val, const spmv_options_t *opt,
                         spmv_plan_t *plan) {
    HostCsr A{m, n, nnz, row_ptr, col_idx, val};
    return create_from_csr(A, opt, plan);
}

int spmv_plan_create_csr32(int32_t m, int32_t n, int32_t nnz, const int32_t *row_ptr,
                           const int32_t *col_idx, const double *val, const spmv_options_t *opt,
                           spmv_plan_t *plan) {
    SPMV_CHECK_ARG(m >= 0 && row_ptr != nullptr, "bad m or NULL row_ptr");
    std::vector<int64_t> rp((size_t)m + 1);
    for (int32_t i = 0; i <= m; ++i) rp[i] = row_ptr[i];
    HostCsr A{m, n, nnz, rp.data(), col_idx, val};
    return create_from_csr(A, opt, plan);
}

int spmv_plan_create_csr_device(int64_t m, int64_t n, int64_t nnz, const int64_t *d_row_ptr,
                                const int32_t *d_col_idx, const double *d_val, const spmv_options_t *opt_in,
                                spmv_plan_t *out) {
    return create_device_impl(m, n, nnz, d_row_ptr, d_col_idx, d_val, opt_in, out, nullptr);
}

int spmv_plan_create_csr32_device(int32_t m, int32_t n, int32_t nnz, const int32_t *d_row_ptr,
                                  const int32_t *d_col_idx, const double *d_val, const spmv_options_t *opt,
                                  spmv_plan_t *out) {
    SPMV_CHECK_ARG(out != nullptr, "plan out-pointer is NULL");
    *out = nullptr;
    SPMV_CHECK_ARG(m >= 0 && n >= 0 && nnz >= 0 && d_row_ptr != nullptr, "bad dimensions or NULL row_ptr");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible (libspmv_hip needs an MI355X / gfx950)");
        return SPMV_ERROR_NO_DEVICE;
    }
    int dev = opt && opt->device >= 0 ? opt->device : -1;
    if (dev < 0) SPMV_HIP_TRY(hipGetDevice(&dev));
    SPMV_RETURN_IF(check_device(dev));
    SPMV_HIP_TRY(hipSetDevice(dev));
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, d_row_ptr) != hipSuccess || a.type != hipMemoryTypeDevice || a.device != dev) {
        (void)hipGetLastError();
        set_error("spmv_plan_create_csr32_device: arrays must be device memory on the plan's device");
        return SPMV_ERROR_INVALID_VALUE;
    }
    int64_t *rp64 = nullptr;
    SPMV_RETURN_IF(widen_row_ptr_device(d_row_ptr, m, &rp64));
    const int st = spmv_plan_create_csr_device(m, n, nnz, rp64, d_col_idx, d_val, opt, out);
    (void)hipFree(rp64);
    return st;
}

int spmv_coo_to_csr(int32_t m, int64_t nnz, const int32_t *row_idx, int64_t *row_ptr) {
    SPMV_CHECK_ARG(m >= 0 && nnz >= 0 && row_ptr != nullptr, "bad arguments");
    SPMV_CHECK_ARG(nnz == 0 || row_idx != nullptr, "row_idx is NULL");
    // the linear scan of src/opt_crs.cpp:26-33
    int64_t p = 0;
    for (int64_t i = 0; i < nnz; ++i) {
        const int32_t r = row_idx[i];
        SPMV_CHECK_ARG(r >= 0 && r < m, "row index outside [0, m)");
        SPMV_CHECK_ARG(r + 1 >= p, "COO rows are not sorted");
        while (p <= r) row_ptr[p++] = i;
    }
    while (p <= m) row_ptr[p++] = nnz;
    return SPMV_SUCCESS;
}

int spmv_plan_create_coo(int32_t m, int32_t n, int32_t nnz, const int32_t *row_idx,
                         const int32_t *col_idx, const double *val, const spmv_options_t *opt,
                         spmv_plan_t *plan) {
    SPMV_CHECK_ARG(m >= 0 && nnz >= 0, "negative dimension");
    std::vector<int64_t> rp((size_t)m + 1);
    SPMV_RETURN_IF(spmv_coo_to_csr(m, nnz, row_idx, rp.data()));
    HostCsr A{m, n, nnz, rp.data(), col_idx, val};
    return create_from_csr(A, opt, plan);
}

int spmv_plan_destroy(spmv_plan_t p) {
    if (!p) return SPMV_SUCCESS;
    (void)bind_device(p);
    p->arena.release();
    delete p;
    return SPMV_SUCCESS;
}

int spmv_set_stream(spmv_plan_t p, void *stream) {
    SPMV_CHECK_ARG(p != nullptr, "plan is NULL");
    p->stream = (hipStream_t)stream;
    return SPMV_SUCCESS;
}

static int execute_impl(spmv_plan_t p, double alpha, const double *x, double *y, uint32_t flags);

int spmv_execute(spmv_plan_t p, const double *x, double *y, uint32_t flags) {
    return execute_impl(p, 1.0, x, y, flags);
}

int spmv_execute_alpha(spmv_plan_t p, double alpha, const double *x, double *y, uint32_t flags) {
    return execute_impl(p, alpha, x, y, flags);
}

static int execute_impl(spmv_plan_t p, double alpha, const double *x, double *y, uint32_t flags) {
    SPMV_CHECK_ARG(p != nullptr, "plan is NULL");
    const bool staged = (flags & SPMV_X_STAGED) != 0;
    const bool y_staged = (flags & SPMV_Y_STAGED) != 0;
    SPMV_CHECK_ARG((x != nullptr || p->n == 0 || staged) && (y != nullptr || p->m == 0 || y_staged),
                   "x or y is NULL");
    SPMV_CHECK_ARG(!(y_staged && (flags & SPMV_Y_DEVICE)), "SPMV_Y_STAGED with SPMV_Y_DEVICE");
    SPMV_CHECK_ARG(!staged || p->x_stage != nullptr, "SPMV_X_STAGED without a previously staged x");
    SPMV_RETURN_IF(bind_device(p));
    // spmv_fetch_y serves the y of the latest execute only when that execute
    // was SPMV_Y_STAGED: any other execute (device y, host y) clears the mark
    p->y_staged = false;
    const double *dx = x;
    double *dy = y;
    if (staged) {
        dx = p->x_stage;
        flags |= SPMV_X_DEVICE;
    } else if (!(flags & SPMV_X_DEVICE)) {
        // opt_cusparse.cpp:72 -- H2D copy of x on every call
        if (!p->x_stage) {
            void *q;
            SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(double) * (size_t)std::max<int64_t>(p->n, 1)));
            p->x_stage = (double *)q;
        }
        if (p->n) SPMV_HIP_TRY(hipMemcpyAsync(p->x_stage, x, sizeof(double) * p->n, hipMemcpyHostToDevice, p->stream));
        dx = p->x_stage;
    }
    if (!(flags & SPMV_Y_DEVICE)) {
        if (!p->y_stage) {
            void *q;
            SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(double) * (size_t)std::max<int64_t>(p->m, 1)));
            p->y_stage = (double *)q;
        }
        dy = p->y_stage;
    }
    SPMV_RETURN_IF(dispatch(p, dx, dy));
    SPMV_RETURN_IF(launch_scale(p, dy, alpha));
    if (y_staged) {
        p->y_staged = true;
        if (!(flags & SPMV_ASYNC) || !(flags & SPMV_X_DEVICE)) SPMV_HIP_TRY(hipStreamSynchronize(p->stream));
    } else if (!(flags & SPMV_Y_DEVICE)) {
        // opt_cusparse.cpp:82 -- D2H copy of y on every call
        if (p->m) SPMV_HIP_TRY(hipMemcpyAsync(y, dy, sizeof(double) * p->m, hipMemcpyDeviceToHost, p->stream));
        SPMV_HIP_TRY(hipStreamSynchronize(p->stream));
    } else if (!(flags & SPMV_ASYNC) || !(flags & SPMV_X_DEVICE)) {
        SPMV_HIP_TRY(hipStreamSynchronize(p->stream));
    }
    return SPMV_SUCCESS;
}

int spmv_fetch_y(spmv_plan_t p, double *y) {
    SPMV_CHECK_ARG(p != nullptr && (y != nullptr || p->m == 0), "plan or y is NULL");
    SPMV_CHECK_ARG(p->y_staged && p->y_stage, "spmv_fetch_y without a previous SPMV_Y_STAGED execute");
    SPMV_RETURN_IF(bind_device(p));
    if (p->m) SPMV_HIP_TRY(hipMemcpyAsync(y, p->y_stage, sizeof(double) * p->m, hipMemcpyDeviceToHost, p->stream));
    SPMV_HIP_TRY(hipStreamSynchronize(p->stream));
    return SPMV_SUCCESS;
}

int spmv_time(spmv_plan_t p, const double *x_dev, double *y_dev, int32_t iters, double *ms) {
    SPMV_CHECK_ARG(p != nullptr && ms != nullptr && iters > 0, "bad arguments");
    SPMV_RETURN_IF(bind_device(p));
    hipEvent_t a, b;
    SPMV_HIP_TRY(hipEventCreate(&a));
    SPMV_HIP_TRY(hipEventCreate(&b));
    SPMV_HIP_TRY(hipEventRecord(a, p->stream));
    int st = SPMV_SUCCESS;
    for (int i = 0; i < iters && st == SPMV_SUCCESS; ++i) st = dispatch(p, x_dev, y_dev);
    SPMV_HIP_TRY(hipEventRecord(b, p->stream));
    SPMV_HIP_TRY(hipEventSynchronize(b));
    float f = 0;
    SPMV_HIP_TRY(hipEventElapsedTime(&f, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *ms = f;
    return st;
}

}  // extern "C"

struct spmv_graph_s {
    spmv_plan_t plan = nullptr;  // launches use the plan's stream; destroy does not touch it
    int device = 0;              // the plan's device, for destroy
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    int32_t reps = 0;
};

namespace spmv {

// Capture `reps` dispatches on a private stream (the plan's stream may be the
// null stream, which cannot be captured); the plan's stream is restored
// whatever happens.
static int graph_capture(spmv_plan_s *p, const double *x, double *y, int32_t reps, hipGraph_t *out) {
    hipStream_t cs = nullptr;
    SPMV_HIP_TRY(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    const hipStream_t saved = p->stream;
    const int saved_prof = p->prof_k;
    p->stream = cs;
    p->prof_k = -1;  // no profile events inside the graph
    int st = SPMV_SUCCESS;
    hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
        for (int32_t r = 0; r < reps && st == SPMV_SUCCESS; ++r) st = dispatch(p, x, y);
        hipGraph_t g = nullptr;
        const hipError_t e2 = hipStreamEndCapture(cs, &g);
        if (st == SPMV_SUCCESS && e2 != hipSuccess) e = e2;
        if (st == SPMV_SUCCESS && e == hipSuccess) *out = g;
        else if (g) (void)hipGraphDestroy(g);
    }
    p->stream = saved;
    p->prof_k = saved_prof;
    (void)hipStreamDestroy(cs);
    if (st != SPMV_SUCCESS) return st;
    if (e != hipSuccess) {
        set_error(std::string("graph capture: ") + hipGetErrorString(e));
        (void)hipGetLastError();
        return SPMV_ERROR_HIP;
    }
    return SPMV_SUCCESS;
}

}  // namespace spmv

extern "C" {

int spmv_graph_create(spmv_plan_t p, const double *x_dev, double *y_dev, int32_t reps, spmv_graph_t *out) {
    SPMV_CHECK_ARG(out != nullptr, "graph out-pointer is NULL");
    *out = nullptr;
    SPMV_CHECK_ARG(p != nullptr && reps > 0, "bad arguments");
    SPMV_CHECK_ARG((x_dev != nullptr || p->n == 0) && (y_dev != nullptr || p->m == 0), "x or y is NULL");
    if (p->format == SPMV_FORMAT_CSS) {
        // the sweep's progress flags are tagged with a per-launch sequence
        // number passed as a kernel argument: a replayed graph would repeat it
        set_error("spmv_graph_create: CSS plans cannot be replayed from a graph");
        return SPMV_ERROR_NOT_SUPPORTED;
    }
    SPMV_RETURN_IF(bind_device(p));
    hipGraph_t g = nullptr;
    SPMV_RETURN_IF(graph_capture(p, x_dev, y_dev, reps, &g));
    hipGraphExec_t ex = nullptr;
    const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        (void)hipGraphDestroy(g);
        set_error(std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
        (void)hipGetLastError();
        return SPMV_ERROR_HIP;
    }
    spmv_graph_s *G = new (std::nothrow) spmv_graph_s;
    if (!G) {
        (void)hipGraphExecDestroy(ex);
        (void)hipGraphDestroy(g);
        set_error("host allocation of the graph failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    G->plan = p;
    G->device = p->device;
    G->graph = g;
    G->exec = ex;
    G->reps = reps;
    *out = G;
    return SPMV_SUCCESS;
}

int spmv_graph_launch(spmv_graph_t G, uint32_t flags) {
    SPMV_CHECK_ARG(G != nullptr && G->exec != nullptr, "graph is NULL");
    SPMV_RETURN_IF(bind_device(G->plan));
    SPMV_HIP_TRY(hipGraphLaunch(G->exec, G->plan->stream));
    if (!(flags & SPMV_ASYNC)) SPMV_HIP_TRY(hipStreamSynchronize(G->plan->stream));
    return SPMV_SUCCESS;
}

int spmv_graph_time(spmv_graph_t G, int32_t launches, double *ms) {
    SPMV_CHECK_ARG(G != nullptr && G->exec != nullptr && ms != nullptr && launches > 0, "bad arguments");
    SPMV_RETURN_IF(bind_device(G->plan));
    const hipStream_t s = G->plan->stream;
    hipEvent_t a, b;
    SPMV_HIP_TRY(hipEventCreate(&a));
    SPMV_HIP_TRY(hipEventCreate(&b));
    hipError_t e = hipEventRecord(a, s);
    for (int32_t i = 0; i < launches && e == hipSuccess; ++i) e = hipGraphLaunch(G->exec, s);
    if (e == hipSuccess) e = hipEventRecord(b, s);
    if (e == hipSuccess) e = hipEventSynchronize(b);
    float f = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&f, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    SPMV_HIP_TRY(e);
    *ms = f;
    return SPMV_SUCCESS;
}

int spmv_graph_destroy(spmv_graph_t G) {
    if (!G) return SPMV_SUCCESS;
    // the plan may already be gone (the header asks for graphs first, but a
    // destroy must not read it): bind the recorded device only
    (void)hipSetDevice(G->device);
    if (G->exec) (void)hipGraphExecDestroy(G->exec);
    if (G->graph) (void)hipGraphDestroy(G->graph);
    delete G;
    return SPMV_SUCCESS;
}

static const char *const kPhases[][3] = {
    {"", "", ""},           {"csr", "", ""},   {"ell", "", ""},     {"tile", "fixup", ""},
    {"dia", "", ""},        {"ell", "overflow", ""}, {"sweep", "", ""}, {"zero_y", "segment", ""},
    {"ell", "overflow", ""}};

const char *spmv_phase_name(spmv_plan_t p, int32_t k) {
    static const char *const kBinPhases[8] = {"mul", "sum", "mul.1", "sum.1", "mul.2", "sum.2", "mul.3", "sum.3"};
    if (p && p->format == SPMV_FORMAT_BIN) {
        if (!p->bin.reuse) return k == 0 ? "mul" : k == 1 ? "sum" : "";  // groups' Mul launches: one phase
        return k >= 0 && k < 8 && k < 2 * p->bin.G ? kBinPhases[k] : "";
    }
    if (!p || k < 0 || k > 2 || p->format < 0 || p->format > SPMV_FORMAT_JDS) return "";
    return kPhases[p->format][k];
}

int spmv_profile(spmv_plan_t p, const double *x_dev, double *y_dev, int32_t iters, double *phase_ms,
                 int32_t max_phases, int32_t *n_phases) {
    SPMV_CHECK_ARG(p != nullptr && iters > 0 && phase_ms != nullptr && n_phases != nullptr && max_phases > 0,
                   "bad arguments");
    SPMV_RETURN_IF(bind_device(p));
    for (auto &e : p->prof_ev) SPMV_HIP_TRY(hipEventCreate(&e));
    std::vector<double> acc(8, 0.0);
    int nph = 1, st = SPMV_SUCCESS;
    for (int i = 0; i < iters && st == SPMV_SUCCESS; ++i) {
        p->prof_k = 0;
        (void)hipEventRecord(p->prof_ev[0], p->stream);
        st = dispatch(p, x_dev, y_dev);
        const int k = p->prof_k;
        p->prof_k = -1;
        (void)hipEventRecord(p->prof_ev[k + 1], p->stream);
        if (hipEventSynchronize(p->prof_ev[k + 1]) != hipSuccess) {
            st = SPMV_ERROR_HIP;
            set_error("spmv_profile: event synchronisation failed");
            break;
        }
        nph = k + 1;
        for (int j = 0; j <= k; ++j) {
            float f = 0;
            (void)hipEventElapsedTime(&f, p->prof_ev[j], p->prof_ev[j + 1]);
            acc[j] += f;
        }
    }
    p->prof_k = -1;
    for (auto &e : p->prof_ev) (void)hipEventDestroy(e);
    *n_phases = nph;
    for (int j = 0; j < std::min(nph, max_phases); ++j) phase_ms[j] = acc[j] / iters;
    return st;
}

// internal (not in the public header): the CSS per-wave timestamps of the
// last launch when the plan was built with SPMV_CSS_DEBUG & 32
int64_t spmv_css_timestamps(spmv_plan_t p, uint64_t *out, int64_t cap) {
    if (!p || p->format != SPMV_FORMAT_CSS || !p->css.tstamp) return -1;
    const int64_t n = (int64_t)p->css.P * p->css.nwg * (kCssWorkers + 2);
    if (out && cap >= n && hipMemcpy(out, p->css.tstamp, 8 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return n;
}

// internal: the CSS block/list layout (bstart [P*nwg+1], woff [P*nwg*15+1])
int spmv_css_layout(spmv_plan_t p, int64_t *bstart, int64_t *woff) {
    if (!p || p->format != SPMV_FORMAT_CSS) return -1;
    const int64_t nb = (int64_t)p->css.P * p->css.nwg;
    if (hipMemcpy(bstart, p->css.bstart, 8 * (size_t)(nb + 1), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (hipMemcpy(woff, p->css.woff, 8 * (size_t)(nb * kCssWorkers + 1), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return 0;
}

// internal (experiment): give the BIN product buffer a fresh allocation (the
// old one is kept until the plan is destroyed, so the new one lands elsewhere)
int spmv_bin_realloc_prod(spmv_plan_t p) {
    if (!p || p->format != SPMV_FORMAT_BIN || !p->bin.prod) return -1;
    void *q = nullptr;
    if (p->arena.alloc(&q, sizeof(double) * (size_t)(std::max<int64_t>(p->bin.prod_cap, 1) + kBinProdSlack)) !=
        SPMV_SUCCESS)
        return -1;
    p->bin.prod = (double *)q;
    return 0;
}

// internal (placement experiments): the BIN product buffer
int spmv_bin_prod(spmv_plan_t p, void **buf, int64_t *bytes) {
    if (!p || p->format != SPMV_FORMAT_BIN || !p->bin.prod || !buf || !bytes) return -1;
    *buf = p->bin.prod;
    *bytes = 8 * std::max<int64_t>(p->bin.prod_cap, 1);
    return 0;
}

int spmv_plan_built_on_device(spmv_plan_t p, int32_t *on_device) {
    SPMV_CHECK_ARG(p != nullptr && on_device != nullptr, "NULL plan or out-pointer");
    *on_device = p->built_on_device;
    return SPMV_SUCCESS;
}

int spmv_plan_info(spmv_plan_t p, spmv_plan_info_t *info) {
    SPMV_CHECK_ARG(p != nullptr && info != nullptr, "NULL argument");
    std::memset(info, 0, sizeof(*info));
    info->format = p->format;
    info->device = p->device;
    info->m = p->m;
    info->n = p->n;
    info->nnz = p->nnz;
    info->stored_slots = p->stored_slots;
    info->device_bytes = p->arena.bytes;
    info->algo_bytes = p->algo_bytes;
    info->row_ptr_bytes = p->csr.rp64 ? 8 : 4;
    info->csr_lanes = p->format == SPMV_FORMAT_HYB ? p->hyb.lanes : p->csr.lanes;
    info->ell_width = p->ell.max_width;
    info->ss_sigma = p->ss.sigma;
    info->n_diags = p->dia.n_diags;
    info->css_passes = p->css.P;
    info->css_slabs = p->css.S;
    info->n_kernels = p->n_kernels;
    info->overflow_nnz = p->hyb.nnz;
    info->empty_rows = p->empty_rows;
    info->css_split_rows = p->css.split_rows;
    std::strncpy(info->kernel, p->kernel_name.c_str(), sizeof(info->kernel) - 1);
    if (p->format == SPMV_FORMAT_BIN) {
        info->bin_bins = p->bin.n_bins;
        info->bin_strips = p->bin.n_strips;
        info->bin_strip_cols = p->bin.strip;
        info->bin_pad = 1 << p->bin.pad_log;
        info->bin_sum_waves = p->bin.sum_waves;
        info->bin_groups = p->bin.G;
        info->bin_long_len = (int32_t)p->bin.long_len;
        info->bin_product_order = p->bin.mo ? SPMV_BIN_ORDER_MUL : SPMV_BIN_ORDER_SUM;
        info->bin_long_rows = p->bin.long_rows;
        info->bin_long_pieces = p->bin.long_pieces;
        info->bin_products = p->bin.prod_cap;
        info->bin_long_entries = p->bin.long_entries;
        info->bin_sum_entries = p->bin.n_entries;
    }
    const std::vector<float> *pm = nullptr;
    if (p->format == SPMV_FORMAT_BIN) {
        info->placement = p->bin.placement;
        pm = &p->bin.placement_ms;
    } else if (p->format == SPMV_FORMAT_DIA) {
        info->placement = p->dia.placement;
        pm = &p->dia.placement_ms;
    } else {
        info->placement = p->arena.maps.empty() ? SPMV_PLACEMENT_PLAIN : SPMV_PLACEMENT_VMM;
    }
    if (pm && !pm->empty()) {
        info->placement_candidates = (int32_t)pm->size();
        info->placement_best_ms = *std::min_element(pm->begin(), pm->end());
        info->placement_worst_ms = *std::max_element(pm->begin(), pm->end());
    }
    return SPMV_SUCCESS;
}

const char *spmv_status_string(int s) {
    switch (s) {
        case SPMV_SUCCESS: return "success";
        case SPMV_ERROR_INVALID_VALUE: return "invalid value";
        case SPMV_ERROR_NOT_SUPPORTED: return "not supported by this format";
        case SPMV_ERROR_OUT_OF_MEMORY: return "out of memory";
        case SPMV_ERROR_HIP: return "HIP runtime error";
        case SPMV_ERROR_IO: return "I/O error";
        case SPMV_ERROR_NO_DEVICE: return "no usable gfx950 device";
    }
    return "unknown status";
}

const char *spmv_last_error(void) { return spmv::last_error(); }

int spmv_partition_rows(const int64_t *row_ptr, int64_t m, int32_t parts, int64_t *cuts) {
    SPMV_CHECK_ARG(row_ptr && cuts && parts > 0 && m >= 0, "bad arguments");
    const int64_t nnz = row_ptr[m];
    cuts[0] = 0;
    for (int k = 1; k < parts; ++k) {
        const int64_t target = (int64_t)((__int128)nnz * k / parts);
        cuts[k] = std::lower_bound(row_ptr, row_ptr + m, target) - row_ptr;
        if (cuts[k] < cuts[k - 1]) cuts[k] = cuts[k - 1];
    }
    cuts[parts] = m;
    return SPMV_SUCCESS;
}

}  // extern "C"

// dist.cpp -- multi-GPU SpMV in one process over N local devices (SURVEY
// §8(e)): the C-ABI counterpart of the per-rank torch.distributed flow
// (singlespmv_amd/dist.py, bench.py) for C/C++ callers of the drop-in -- the
// reference's driver calls OptimizeProblem / SpMV from C++ (src/main.cpp:36,
// 87) and its GPU backend owns its device arrays (src/opt_cusparse.cpp:36-45,
// 72-82).
//
//   rows   nnz-balanced row ranges (spmv_partition_rows); one plan per device
//          over its rows with GLOBAL column indices (n columns each)
//   x      host -> device 0, then ncclBroadcast from device 0 to every
//          device (RCCL over xGMI); SPMV_X_STAGED re-uses it
//   y      every device writes its slice of `slice` rows (padded to the
//          longest range), ncclAllGather assembles the full y on every device
//          (the iterative y -> next x shape), device 0's copy goes to the host
//
// Communicators come from ncclCommInitAll (one per device, this process);
// every device has its own non-blocking stream.  No collective sits inside a
// device's SpMV: the kernels are the single-GPU plans unchanged.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "internal.hpp"

struct spmv_dist_s {
    int nd = 0;
    int64_t m = 0, n = 0, nnz = 0, slice = 0;
    std::vector<int> devs;
    std::vector<int64_t> cuts;
    std::vector<spmv_plan_t> plans;
    std::vector<hipStream_t> streams;
    std::vector<ncclComm_t> comms;
    std::vector<double *> d_x, d_yloc, d_yfull;
    bool x_staged = false;
};

namespace spmv {

#define SPMV_NCCL_TRY(call)                                                               \
    do {                                                                                  \
        ncclResult_t r_ = (call);                                                         \
        if (r_ != ncclSuccess) {                                                          \
            ::spmv::set_error(std::string(#call) + ": " + ncclGetErrorString(r_));        \
            return SPMV_ERROR_HIP;                                                        \
        }                                                                                 \
    } while (0)

static void dist_free(spmv_dist_s *d) {
    for (int k = 0; k < (int)d->devs.size(); ++k) {
        (void)hipSetDevice(d->devs[k]);
        if (k < (int)d->streams.size() && d->streams[k]) (void)hipStreamSynchronize(d->streams[k]);
        if (k < (int)d->plans.size()) spmv_plan_destroy(d->plans[k]);
        if (k < (int)d->d_x.size()) (void)hipFree(d->d_x[k]);
        if (k < (int)d->d_yloc.size()) (void)hipFree(d->d_yloc[k]);
        if (k < (int)d->d_yfull.size()) (void)hipFree(d->d_yfull[k]);
    }
    for (ncclComm_t c : d->comms)
        if (c) (void)ncclCommDestroy(c);
    for (int k = 0; k < (int)d->streams.size(); ++k) {
        (void)hipSetDevice(d->devs[k]);
        if (d->streams[k]) (void)hipStreamDestroy(d->streams[k]);
    }
    delete d;
}

// broadcast d_x[0] to every device, on each device's stream
static int dist_bcast_x(spmv_dist_s *d) {
    if (d->n == 0) return SPMV_SUCCESS;  // (N = 1 too: an in-place RCCL broadcast on one rank)
    SPMV_NCCL_TRY(ncclGroupStart());
    for (int k = 0; k < d->nd; ++k) {
        const ncclResult_t r = ncclBroadcast(d->d_x[0], d->d_x[k], (size_t)d->n, ncclDouble, 0, d->comms[k],
                                             d->streams[k]);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            set_error(std::string("ncclBroadcast: ") + ncclGetErrorString(r));
            return SPMV_ERROR_HIP;
        }
    }
    SPMV_NCCL_TRY(ncclGroupEnd());
    return SPMV_SUCCESS;
}

static int dist_local_spmv(spmv_dist_s *d) {
    for (int k = 0; k < d->nd; ++k)
        SPMV_RETURN_IF(spmv_execute(d->plans[k], d->d_x[k], d->d_yloc[k], SPMV_X_DEVICE | SPMV_Y_DEVICE | SPMV_ASYNC));
    return SPMV_SUCCESS;
}

static int dist_gather_y(spmv_dist_s *d) {
    SPMV_NCCL_TRY(ncclGroupStart());
    for (int k = 0; k < d->nd; ++k) {
        const ncclResult_t r = ncclAllGather(d->d_yloc[k], d->d_yfull[k], (size_t)d->slice, ncclDouble, d->comms[k],
                                             d->streams[k]);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            set_error(std::string("ncclAllGather: ") + ncclGetErrorString(r));
            return SPMV_ERROR_HIP;
        }
    }
    SPMV_NCCL_TRY(ncclGroupEnd());
    return SPMV_SUCCESS;
}

// The y reassembly of a dist plan: part k's rows [cuts[k], cuts[k+1]) sit at
// the start of its slice in the all-gathered buffer (k * slice); one copy per
// non-empty part.  Shared by spmv_dist_execute (device -> host copies) and
// spmv_dist_assemble (host, testable without a second GPU).
struct SliceCopy {
    int64_t src, dst, rows;
};
static std::vector<SliceCopy> dist_copies(const int64_t *cuts, int32_t parts, int64_t slice) {
    std::vector<SliceCopy> c;
    for (int k = 0; k < parts; ++k) {
        const int64_t rows = cuts[k + 1] - cuts[k];
        if (rows > 0) c.push_back(SliceCopy{(int64_t)k * slice, cuts[k], rows});
    }
    return c;
}

// Part k's CSR: rows [cuts[k], cuts[k+1]) with row pointers rebased to its
// first entry (global column indices kept); *entry0 = that entry's index.
static void dist_shard_rows(const int64_t *row_ptr, const int64_t *cuts, int32_t k, int64_t *rp, int64_t *entry0) {
    const int64_t r0 = cuts[k], r1 = cuts[k + 1], b = row_ptr[r0];
    for (int64_t r = r0; r <= r1; ++r) rp[r - r0] = row_ptr[r] - b;
    *entry0 = b;
}

static int dist_sync(spmv_dist_s *d) {
    for (int k = 0; k < d->nd; ++k) {
        SPMV_HIP_TRY(hipSetDevice(d->devs[k]));
        SPMV_HIP_TRY(hipStreamSynchronize(d->streams[k]));
    }
    return SPMV_SUCCESS;
}

}  // namespace spmv

using namespace spmv;

extern "C" {

int spmv_dist_layout(const int64_t *row_ptr, int64_t m, int32_t parts, int64_t *cuts, int64_t *slice_rows) {
    SPMV_CHECK_ARG(row_ptr && cuts && slice_rows && parts > 0 && m >= 0, "bad arguments");
    SPMV_RETURN_IF(spmv_partition_rows(row_ptr, m, parts, cuts));
    int64_t s = 1;
    for (int k = 0; k < parts; ++k) s = std::max<int64_t>(s, cuts[k + 1] - cuts[k]);
    *slice_rows = s;
    return SPMV_SUCCESS;
}

int spmv_dist_shard(const int64_t *row_ptr, const int64_t *cuts, int32_t parts, int32_t k, int64_t *rp,
                    int64_t *entry0) {
    SPMV_CHECK_ARG(row_ptr && cuts && rp && entry0 && parts > 0 && k >= 0 && k < parts, "bad arguments");
    SPMV_CHECK_ARG(cuts[k] <= cuts[k + 1], "cuts are not non-decreasing");
    dist_shard_rows(row_ptr, cuts, k, rp, entry0);
    return SPMV_SUCCESS;
}

int spmv_dist_assemble(const double *gathered, const int64_t *cuts, int32_t parts, int64_t slice, double *y) {
    SPMV_CHECK_ARG(gathered && cuts && y && parts > 0 && slice >= 1, "bad arguments");
    for (int k = 0; k < parts; ++k)
        SPMV_CHECK_ARG(cuts[k] <= cuts[k + 1] && cuts[k + 1] - cuts[k] <= slice, "a part is longer than the slice");
    for (const SliceCopy &c : dist_copies(cuts, parts, slice))
        std::memcpy(y + c.dst, gathered + c.src, 8 * (size_t)c.rows);
    return SPMV_SUCCESS;
}

int spmv_dist_create_csr(int32_t n_devices, const int32_t *devices, int64_t m, int64_t n, int64_t nnz,
                         const int64_t *row_ptr, const int32_t *col_idx, const double *val,
                         const spmv_options_t *opt, spmv_dist_t *out) {
    SPMV_CHECK_ARG(out != nullptr, "dist out-pointer is NULL");
    *out = nullptr;
    SPMV_CHECK_ARG(n_devices >= 1 && n_devices <= 64, "n_devices must be in [1, 64]");
    SPMV_CHECK_ARG(m >= 0 && n >= 0 && nnz >= 0 && row_ptr != nullptr, "bad dimensions or NULL row_ptr");
    SPMV_CHECK_ARG(row_ptr[0] == 0 && row_ptr[m] == nnz, "row_ptr[0] != 0 or row_ptr[m] != nnz");
    SPMV_CHECK_ARG(nnz == 0 || (col_idx != nullptr && val != nullptr), "col/val is NULL");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible (libspmv_hip needs an MI355X / gfx950)");
        return SPMV_ERROR_NO_DEVICE;
    }
    spmv_dist_s *d = new (std::nothrow) spmv_dist_s;
    if (!d) {
        set_error("host allocation of the dist plan failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    d->nd = n_devices;
    d->m = m;
    d->n = n;
    d->nnz = nnz;
    for (int k = 0; k < n_devices; ++k) {
        const int dev = devices ? devices[k] : k;
        if (dev < 0 || dev >= count || std::count(d->devs.begin(), d->devs.end(), dev)) {
            delete d;
            set_error("device list: ordinals must be distinct and < " + std::to_string(count));
            return SPMV_ERROR_INVALID_VALUE;
        }
        d->devs.push_back(dev);
    }
    d->cuts.assign((size_t)n_devices + 1, 0);
    int st = spmv_dist_layout(row_ptr, m, n_devices, d->cuts.data(), &d->slice);
    spmv_options_t o;
    if (opt) o = *opt;
    else spmv_options_default(&o);
    std::vector<int64_t> rp;
    for (int k = 0; k < n_devices && st == SPMV_SUCCESS; ++k) {
        const int dev = d->devs[k];
        if (hipSetDevice(dev) != hipSuccess) {
            st = SPMV_ERROR_HIP;
            set_error("hipSetDevice failed");
            break;
        }
        hipStream_t s = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
            st = SPMV_ERROR_HIP;
            set_error("hipStreamCreate failed");
            break;
        }
        d->streams.push_back(s);
        // this device's rows: rebased row pointers, global columns
        const int64_t r0 = d->cuts[k], r1 = d->cuts[k + 1];
        int64_t b = 0;
        rp.resize((size_t)(r1 - r0 + 1));
        dist_shard_rows(row_ptr, d->cuts.data(), k, rp.data(), &b);
        o.device = dev;
        spmv_plan_t p = nullptr;
        st = spmv_plan_create_csr(r1 - r0, n, row_ptr[r1] - b, rp.data(), col_idx ? col_idx + b : nullptr,
                                  val ? val + b : nullptr, &o, &p);
        if (st != SPMV_SUCCESS) break;
        d->plans.push_back(p);
        spmv_set_stream(p, s);
        double *q = nullptr;
        if (hipMalloc(&q, 8 * (size_t)std::max<int64_t>(n, 1)) != hipSuccess) st = SPMV_ERROR_OUT_OF_MEMORY;
        d->d_x.push_back(q);
        q = nullptr;
        if (st == SPMV_SUCCESS && hipMalloc(&q, 8 * (size_t)d->slice) != hipSuccess) st = SPMV_ERROR_OUT_OF_MEMORY;
        if (q) (void)hipMemset(q, 0, 8 * (size_t)d->slice);
        d->d_yloc.push_back(q);
        double *f = nullptr;
        if (st == SPMV_SUCCESS && hipMalloc(&f, 8 * (size_t)d->slice * n_devices) != hipSuccess)
            st = SPMV_ERROR_OUT_OF_MEMORY;
        d->d_yfull.push_back(f);
        if (st != SPMV_SUCCESS) {
            (void)hipGetLastError();
            set_error("spmv_dist_create_csr: device allocation failed on device " + std::to_string(dev));
        }
    }
    // RCCL communicators at every N, N = 1 included, so the single-GPU box
    // runs the same broadcast / all-gather path as an 8-GPU node
    if (st == SPMV_SUCCESS) {
        d->comms.assign((size_t)n_devices, nullptr);
        const ncclResult_t r = ncclCommInitAll(d->comms.data(), n_devices, d->devs.data());
        if (r != ncclSuccess) {
            d->comms.clear();
            set_error(std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
            st = SPMV_ERROR_HIP;
        }
    }
    if (st != SPMV_SUCCESS) {
        dist_free(d);
        return st;
    }
    *out = d;
    return SPMV_SUCCESS;
}

int spmv_dist_execute(spmv_dist_t d, const double *x, double *y, uint32_t flags) {
    SPMV_CHECK_ARG(d != nullptr, "dist plan is NULL");
    // host x / host y only (x is uploaded to the first device and broadcast,
    // y comes back from the all-gathered copy there); the device-pointer and
    // asynchronous flags of spmv_execute are not implemented here
    SPMV_CHECK_ARG((flags & ~(uint32_t)SPMV_X_STAGED) == 0,
                   "spmv_dist_execute takes host x / y: flags other than SPMV_X_STAGED are not supported");
    const bool staged = (flags & SPMV_X_STAGED) != 0;
    SPMV_CHECK_ARG(staged || x != nullptr || d->n == 0, "x is NULL");
    SPMV_CHECK_ARG(!staged || d->x_staged, "SPMV_X_STAGED without a previously broadcast x");
    if (!staged) {
        SPMV_HIP_TRY(hipSetDevice(d->devs[0]));
        if (d->n)
            SPMV_HIP_TRY(hipMemcpyAsync(d->d_x[0], x, 8 * (size_t)d->n, hipMemcpyHostToDevice, d->streams[0]));
        SPMV_RETURN_IF(dist_bcast_x(d));
        d->x_staged = true;
    }
    SPMV_RETURN_IF(dist_local_spmv(d));
    SPMV_RETURN_IF(dist_gather_y(d));
    if (y) {
        SPMV_HIP_TRY(hipSetDevice(d->devs[0]));
        const double *full = d->d_yfull[0];
        for (const SliceCopy &c : dist_copies(d->cuts.data(), d->nd, d->slice))
            SPMV_HIP_TRY(hipMemcpyAsync(y + c.dst, full + c.src, 8 * (size_t)c.rows, hipMemcpyDeviceToHost,
                                        d->streams[0]));
    }
    return dist_sync(d);
}

int spmv_dist_fetch_y(spmv_dist_t d, double *y) {
    SPMV_CHECK_ARG(d != nullptr && (y != nullptr || d->m == 0), "dist plan or y is NULL");
    SPMV_CHECK_ARG(d->x_staged, "spmv_dist_fetch_y before any spmv_dist_execute");
    SPMV_HIP_TRY(hipSetDevice(d->devs[0]));
    const double *full = d->d_yfull[0];
    for (const SliceCopy &c : dist_copies(d->cuts.data(), d->nd, d->slice))
        SPMV_HIP_TRY(hipMemcpyAsync(y + c.dst, full + c.src, 8 * (size_t)c.rows, hipMemcpyDeviceToHost, d->streams[0]));
    SPMV_HIP_TRY(hipStreamSynchronize(d->streams[0]));
    return SPMV_SUCCESS;
}

int spmv_dist_time(spmv_dist_t d, int32_t iters, double *spmv_ms, double *gather_ms) {
    SPMV_CHECK_ARG(d != nullptr && iters > 0 && spmv_ms && gather_ms, "bad arguments");
    SPMV_CHECK_ARG(d->x_staged, "spmv_dist_time needs an x broadcast by spmv_dist_execute first");
    // one exit path: the first error is kept, every event created is
    // destroyed, and nothing is recorded or read after an error
    std::vector<hipEvent_t> ev((size_t)d->nd * 3, nullptr);
    int st = SPMV_SUCCESS;
    auto hip = [&](hipError_t e, const char *what) {
        if (st == SPMV_SUCCESS && e != hipSuccess) {
            set_error(std::string(what) + ": " + hipGetErrorString(e));
            (void)hipGetLastError();
            st = SPMV_ERROR_HIP;
        }
    };
    for (int k = 0; k < d->nd && st == SPMV_SUCCESS; ++k) {
        hip(hipSetDevice(d->devs[k]), "hipSetDevice");
        for (int j = 0; j < 3 && st == SPMV_SUCCESS; ++j) hip(hipEventCreate(&ev[(size_t)k * 3 + j]), "hipEventCreate");
    }
    if (st == SPMV_SUCCESS) st = dist_sync(d);
    auto mark = [&](int j) {
        for (int k = 0; k < d->nd && st == SPMV_SUCCESS; ++k) {
            hip(hipSetDevice(d->devs[k]), "hipSetDevice");
            if (st == SPMV_SUCCESS) hip(hipEventRecord(ev[(size_t)k * 3 + j], d->streams[k]), "hipEventRecord");
        }
    };
    mark(0);
    for (int i = 0; i < iters && st == SPMV_SUCCESS; ++i) st = dist_local_spmv(d);
    mark(1);
    for (int i = 0; i < iters && st == SPMV_SUCCESS; ++i) st = dist_gather_y(d);
    mark(2);
    if (st == SPMV_SUCCESS) st = dist_sync(d);
    double a = 0, g = 0;
    for (int k = 0; k < d->nd && st == SPMV_SUCCESS; ++k) {
        float f1 = 0, f2 = 0;
        hip(hipEventElapsedTime(&f1, ev[(size_t)k * 3], ev[(size_t)k * 3 + 1]), "hipEventElapsedTime");
        hip(hipEventElapsedTime(&f2, ev[(size_t)k * 3 + 1], ev[(size_t)k * 3 + 2]), "hipEventElapsedTime");
        a = std::max(a, (double)f1);
        g = std::max(g, (double)f2);
    }
    for (int k = 0; k < d->nd; ++k) {
        (void)hipSetDevice(d->devs[k]);
        for (int j = 0; j < 3; ++j)
            if (ev[(size_t)k * 3 + j]) (void)hipEventDestroy(ev[(size_t)k * 3 + j]);
    }
    if (st != SPMV_SUCCESS) return st;
    *spmv_ms = a / iters;
    *gather_ms = g / iters;
    return SPMV_SUCCESS;
}

int spmv_dist_info(spmv_dist_t d, int32_t *n_devices, int64_t *cuts, spmv_plan_t *plans) {
    SPMV_CHECK_ARG(d != nullptr && n_devices != nullptr, "NULL argument");
    *n_devices = d->nd;
    if (cuts) std::copy(d->cuts.begin(), d->cuts.end(), cuts);
    if (plans) std::copy(d->plans.begin(), d->plans.end(), plans);
    return SPMV_SUCCESS;
}

int spmv_dist_destroy(spmv_dist_t d) {
    if (d) dist_free(d);
    return SPMV_SUCCESS;
}

}  // extern "C"

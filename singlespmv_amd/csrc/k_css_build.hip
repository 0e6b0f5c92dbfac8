// k_css_build.hip -- the CSS plan built from a CSR in HBM (css_fill_host's
// counterpart in formats.cpp).  css_layout decides everything from the row
// pointers -- row blocks, long-row pieces, the LPT dealing of pieces to the
// 15 worker waves, list offsets -- and the entries never visit the host:
// each worker-wave list's entries are expanded in list order (pieces in
// dealing order, a piece in CSR order) with the key (list, column), stably
// radix-sorted (hipCUB, the key's significant bits only: within a list by
// column, a row's entries of one column keeping their CSR order, as
// std::stable_sort does on the host), and scattered into the list's
// 256-entry chunks.  Byte-identical to the host fill (spmv_plan_digest); no
// 32-bit entry limit.
#include <hipcub/hipcub.hpp>

#include "device.hpp"
#include "internal.hpp"

namespace spmv {

namespace {

// one wave per list: its pieces' entries in list order; key = list <<
// cbits | column, value = entry index << 16 | LDS slot
__global__ __launch_bounds__(256) void css_expand_kernel(int64_t nlists, const int64_t *__restrict__ poff,
                                                         const int64_t *__restrict__ pb,
                                                         const int64_t *__restrict__ pe,
                                                         const int32_t *__restrict__ ps,
                                                         const int64_t *__restrict__ eoff, int cbits,
                                                         const int32_t *__restrict__ col, uint64_t *__restrict__ keys,
                                                         uint64_t *__restrict__ vals) {
    const int64_t L = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (L >= nlists) return;
    int64_t k = eoff[L];
    for (int64_t q = poff[L]; q < poff[L + 1]; ++q) {
        const int64_t b = pb[q], len = pe[q] - b;
        const uint64_t slot = (uint32_t)ps[q];
        for (int64_t i = lane; i < len; i += 64) {
            keys[k + i] = ((uint64_t)L << cbits) | (uint32_t)col[b + i];
            vals[k + i] = ((uint64_t)(b + i) << 16) | slot;
        }
        k += len;
    }
}

// one wave per list: sorted entry i to chunk i / 256, lane i % 256
__global__ __launch_bounds__(256) void css_scatter_kernel(int64_t nlists, const int64_t *__restrict__ eoff,
                                                          const int64_t *__restrict__ woff, int64_t chunk_stride,
                                                          const uint64_t *__restrict__ keys, int cbits,
                                                          const uint64_t *__restrict__ vals,
                                                          const double *__restrict__ val, int32_t *__restrict__ ocol,
                                                          uint16_t *__restrict__ orow, double *__restrict__ oval) {
    const int64_t L = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (L >= nlists) return;
    const int64_t e0 = eoff[L], len = eoff[L + 1] - e0, base = woff[L];
    for (int64_t i = lane; i < len; i += 64) {
        const int64_t out = base + (i >> 8) * chunk_stride + (i & 255);
        const uint64_t v = vals[e0 + i];
        ocol[out] = (int32_t)(keys[e0 + i] & (((uint64_t)1 << cbits) - 1));
        orow[out] = (uint16_t)(v & 0xFFFFu);
        oval[out] = val[v >> 16];
    }
}

__global__ void css_fill_u16(uint16_t *__restrict__ a, int64_t n, uint16_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = v;
}

unsigned waves_grid(int64_t waves) { return (unsigned)std::max<int64_t>(1, (waves + 3) / 4); }

struct Scratch {
    hipStream_t st;
    std::vector<void *> v;
    ~Scratch() {
        (void)hipStreamSynchronize(st);
        for (void *t : v) (void)hipFree(t);
    }
    template <typename T>
    int alloc(T **q, size_t count) {
        void *t = nullptr;
        if (hipMalloc(&t, sizeof(T) * std::max<size_t>(count, 1)) != hipSuccess) {
            (void)hipGetLastError();
            set_error("device CSS build: out of device memory for scratch");
            return SPMV_ERROR_OUT_OF_MEMORY;
        }
        v.push_back(t);
        *q = (T *)t;
        return SPMV_SUCCESS;
    }
    template <typename T>
    int upload(T **q, const std::vector<T> &h) {
        SPMV_RETURN_IF(alloc(q, h.size()));
        if (!h.empty()) SPMV_HIP_TRY(hipMemcpyAsync(*q, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice, st));
        return SPMV_SUCCESS;
    }
};

template <typename T>
int plan_alloc(spmv_plan_s *p, T **dst, int64_t count) {
    void *q = nullptr;
    SPMV_RETURN_IF(p->arena.alloc(&q, sizeof(T) * (size_t)std::max<int64_t>(count, 1)));
    *dst = (T *)q;
    return SPMV_SUCCESS;
}

}  // namespace

int build_css_device(spmv_plan_s *p, const DevCsr &A, const spmv_options_t &o) {
    CssLayout CL;
    SPMV_RETURN_IF(css_layout(p, A.h_rp, A.m, A.n, A.nnz, o, CL));
    CssDev &c = p->css;
    const hipStream_t st = p->stream;
    const int64_t nl = CL.nlists, total = CL.total;
    // the pieces, flattened in list order, and each list's entry offset
    std::vector<int64_t> poff((size_t)nl + 1, 0), pb, pe;
    std::vector<int32_t> ps;
    std::vector<int64_t> eoff((size_t)nl + 1, 0);
    for (int64_t L = 0; L < nl; ++L) {
        int64_t len = 0;
        for (const CssPiece &pc : CL.wave_pieces[(size_t)L]) {
            pb.push_back(pc.begin);
            pe.push_back(pc.end);
            ps.push_back(pc.slot);
            len += pc.end - pc.begin;
        }
        std::vector<CssPiece>().swap(CL.wave_pieces[(size_t)L]);
        poff[(size_t)L + 1] = (int64_t)pb.size();
        eoff[(size_t)L + 1] = eoff[(size_t)L] + len;
    }
    if (eoff[(size_t)nl] != A.nnz) {
        set_error("device CSS build: the lists do not cover the entries");
        return SPMV_ERROR_INVALID_VALUE;
    }
    // the plan's entry arrays, as the host fill leaves them: padding entries
    // (col 0, slot kCssMaxRows, val 0) and 256 zeroed entries past the end
    SPMV_RETURN_IF(plan_alloc(p, &c.col, total + 256));
    SPMV_RETURN_IF(plan_alloc(p, &c.row, total + 256));
    SPMV_RETURN_IF(plan_alloc(p, &c.val, total + 256));
    SPMV_HIP_TRY(hipMemsetAsync(c.col, 0, sizeof(int32_t) * (size_t)(total + 256), st));
    SPMV_HIP_TRY(hipMemsetAsync(c.val, 0, sizeof(double) * (size_t)(total + 256), st));
    SPMV_HIP_TRY(hipMemsetAsync(c.row + total, 0, sizeof(uint16_t) * 256, st));
    if (total > 0)
        hipLaunchKernelGGL(css_fill_u16, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 65536)), dim3(256), 0,
                           st, c.row, total, (uint16_t)kCssMaxRows);
    if (A.nnz > 0) {
        Scratch sc{st, {}};
        int64_t *d_poff, *d_pb, *d_pe, *d_woff, *d_eoff;
        int32_t *d_ps;
        uint64_t *k_in, *k_out, *v_in, *v_out;
        SPMV_RETURN_IF(sc.upload(&d_poff, poff));
        SPMV_RETURN_IF(sc.upload(&d_pb, pb));
        SPMV_RETURN_IF(sc.upload(&d_pe, pe));
        SPMV_RETURN_IF(sc.upload(&d_ps, ps));
        SPMV_RETURN_IF(sc.upload(&d_eoff, eoff));
        SPMV_RETURN_IF(sc.upload(&d_woff, CL.woff));
        SPMV_RETURN_IF(sc.alloc(&k_in, (size_t)A.nnz));
        SPMV_RETURN_IF(sc.alloc(&k_out, (size_t)A.nnz));
        SPMV_RETURN_IF(sc.alloc(&v_in, (size_t)A.nnz));
        SPMV_RETURN_IF(sc.alloc(&v_out, (size_t)A.nnz));
        // key bits: the column's, then the list's above them
        int cbits = 1, lbits = 1;
        while (cbits < 31 && ((int64_t)1 << cbits) < A.n) ++cbits;
        while (lbits < 32 && ((int64_t)1 << lbits) < nl) ++lbits;
        hipLaunchKernelGGL(css_expand_kernel, dim3(waves_grid(nl)), dim3(256), 0, st, nl, d_poff, d_pb, d_pe, d_ps,
                           d_eoff, cbits, A.d_col, k_in, v_in);
        hipcub::DoubleBuffer<uint64_t> dk(k_in, k_out), dv(v_in, v_out);
        size_t tb = 0;
        SPMV_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dv, A.nnz, 0, cbits + lbits, st));
        void *tmp = nullptr;
        SPMV_RETURN_IF(sc.alloc((char **)&tmp, tb));
        SPMV_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dv, A.nnz, 0, cbits + lbits, st));
        hipLaunchKernelGGL(css_scatter_kernel, dim3(waves_grid(nl)), dim3(256), 0, st, nl, d_eoff, d_woff,
                           c.chunk_stride, (const uint64_t *)dk.Current(), cbits, (const uint64_t *)dv.Current(), A.d_val,
                           c.col, c.row, c.val);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            set_error(std::string("device CSS build: ") + hipGetErrorString(e));
            (void)hipGetLastError();
            return SPMV_ERROR_HIP;
        }
    }
    SPMV_RETURN_IF(css_finish(p, CL, A.m, A.n, A.nnz));
    SPMV_HIP_TRY(hipStreamSynchronize(st));
    return SPMV_SUCCESS;
}

}  // namespace spmv

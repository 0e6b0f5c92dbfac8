// mmio.cpp -- Matrix Market ingest, parallel, plus an
// mmap-able binary CSR cache so 1 G-nnz inputs are parsed once.
//
// spmv_load_mtx keeps the reference's LoadSparseMatrix semantics exactly
// (src/util.cpp:30-66): leading lines whose first character is '%' are
// skipped (:37-39); the next line gives "M N L" (:41-42); then exactly L
// whitespace-separated triplets are read token by token, whatever the line
// structure (:44-50) -- extra trailing entries are ignored (matrix/test/10x10
// declares 27 of its 28 triplets); indices become 0-based; entries are sorted
// row-major by (row, col) with duplicates kept.  Equal keys come out in the
// order the reference's own std::sort (:51, not stable) leaves them: runs of
// duplicates are re-sorted with std::sort on the reference's comparator
// (below), pinned by the golden mtx_dups fixture.
// Values are parsed with strtod (correctly rounded, as the stream extraction
// of the reference).  Unlike the reference, a truncated file or an index
// outside the declared shape is an error, not undefined behaviour.
//
// spmv_load_mtx_csr keeps the banner-aware loader of the CSR5 benchmark
// (opt/Benchmark_SpMV_using_CSR5/CSR5_cuda/main.cu:157-306) for real
// SuiteSparse inputs: pattern -> 1.0, integer values, complex refused,
// symmetric/hermitian off-diagonals mirrored; rows keep file order (the
// counter scatter of :262-300), optionally column-sorted.
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "internal.hpp"

using namespace spmv;

namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

struct Mapped {
    const char *base = nullptr;
    size_t size = 0;
    ~Mapped() {
        if (base && size) munmap((void *)base, size);
    }
};

// Parse one token [p, q) as a double / integer.  Tokens near the end of the
// mapping are copied so strtod never reads past it.
bool tok_double(const char *p, const char *q, double &v) {
    char buf[128];
    const size_t n = (size_t)(q - p);
    if (n == 0 || n >= sizeof(buf)) return false;
    std::memcpy(buf, p, n);
    buf[n] = 0;
    char *e;
    v = std::strtod(buf, &e);
    return e == buf + n;
}
bool tok_long(const char *p, const char *q, long long &v) {
    bool neg = false;
    if (p < q && (*p == '+' || *p == '-')) neg = *p++ == '-';
    if (p == q) return false;
    long long r = 0;
    for (; p < q; ++p) {
        if (*p < '0' || *p > '9') return false;
        r = r * 10 + (*p - '0');
        if (r > (1ll << 40)) return false;
    }
    v = neg ? -r : r;
    return true;
}

int map_file(const char *path, Mapped &mp) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
        set_error(std::string("File not Found: ") + path);  // util.cpp:32-35
        return SPMV_ERROR_IO;
    }
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        set_error("fstat failed");
        return SPMV_ERROR_IO;
    }
    if (st.st_size) {
        void *q = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (q == MAP_FAILED) {
            close(fd);
            set_error("mmap failed");
            return SPMV_ERROR_IO;
        }
        mp.base = (const char *)q;
        mp.size = (size_t)st.st_size;
        madvise(q, mp.size, MADV_SEQUENTIAL);
    }
    close(fd);
    return SPMV_SUCCESS;
}

const char *next_line(const char *p, const char *end) {
    const char *nl = (const char *)std::memchr(p, '\n', (size_t)(end - p));
    return nl ? nl + 1 : end;
}

// "M N L" on the line starting at p; returns the start of the next line
const char *read_size_line(const char *p, const char *end, long long hdr[3]) {
    const char *hl_end = (const char *)std::memchr(p, '\n', (size_t)(end - p));
    if (!hl_end) hl_end = end;
    const char *t = p;
    for (int k = 0; k < 3; ++k) {
        while (t < hl_end && is_ws(*t)) ++t;
        const char *u = t;
        while (u < hl_end && !is_ws(*u)) ++u;
        if (!tok_long(t, u, hdr[k])) return nullptr;
        t = u;
    }
    return hl_end < end ? hl_end + 1 : end;
}

enum { VAL_REAL = 0, VAL_INTEGER = 1, VAL_PATTERN = 2 };

// Parse the first L entries of [body, end) -- `per` tokens each (2: row col,
// 3: row col value) -- in parallel chunks cut at whitespace, into file-order
// arrays.  Pass 1 counts tokens per chunk, pass 2 parses each chunk at its
// global token offset, so no token is split and the order is the file's.
int parse_entries(const char *body, const char *end, long long L, long long M, long long N, int per, int kind,
                  std::vector<int32_t> &tr, std::vector<int32_t> &tc, std::vector<double> &tv) {
    const int64_t bytes = end - body;
    const int T = std::max(1, std::min<int>(omp_get_max_threads(), (int)(bytes / (1 << 20)) + 1));
    std::vector<const char *> cut((size_t)T + 1);
    cut[0] = body;
    cut[T] = end;
    for (int t = 1; t < T; ++t) {
        const char *c = body + bytes * t / T;
        while (c < end && !is_ws(*c)) ++c;
        cut[t] = std::max(c, cut[t - 1]);
    }
    std::vector<int64_t> ntok((size_t)T + 1, 0);
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; ++t) {
        int64_t k = 0;
        bool in = false;
        for (const char *c = cut[t]; c < cut[t + 1]; ++c) {
            const bool w = is_ws(*c);
            if (!w && !in) ++k;
            in = !w;
        }
        ntok[t + 1] = k;
    }
    for (int t = 0; t < T; ++t) ntok[t + 1] += ntok[t];
    const int64_t need = (int64_t)per * L;
    if (ntok[T] < need) {
        set_error("truncated triplet list (fewer than L entries)");
        return SPMV_ERROR_IO;
    }
    tr.assign((size_t)L, 0);
    tc.assign((size_t)L, 0);
    tv.assign((size_t)L, 1.0);  // pattern entries stay 1.0 (main.cu:232-236)
    int bad = 0;
#pragma omp parallel for num_threads(T) schedule(static, 1) reduction(| : bad)
    for (int t = 0; t < T; ++t) {
        int64_t k = ntok[t];
        if (k >= need) continue;
        const char *c = cut[t], *ce = cut[t + 1];
        while (c < ce && k < need) {
            while (c < ce && is_ws(*c)) ++c;
            if (c >= ce) break;
            const char *u = c;
            while (u < ce && !is_ws(*u)) ++u;
            const int64_t e = k / per;
            const int f = (int)(k % per);
            if (f == 2) {
                if (kind == VAL_INTEGER) {
                    long long v = 0;
                    if (!tok_long(c, u, v)) bad = 1;
                    tv[(size_t)e] = (double)v;
                } else {
                    double v = 0;
                    if (!tok_double(c, u, v)) bad = 1;
                    tv[(size_t)e] = v;
                }
            } else {
                long long v;
                if (!tok_long(c, u, v) || v < 1 || v > (f == 0 ? M : N)) bad = 1;
                else if (f == 0) tr[(size_t)e] = (int32_t)(v - 1);
                else tc[(size_t)e] = (int32_t)(v - 1);
            }
            ++k;
            c = u;
        }
    }
    if (bad) {
        set_error("unparsable token or entry outside the declared shape");
        return SPMV_ERROR_IO;
    }
    return SPMV_SUCCESS;
}

// stable (by input order) sort of each row's entries by column
void sort_rows(const int64_t *rp, int64_t M, int32_t *ci, double *vv) {
#pragma omp parallel
    {
        std::vector<std::pair<int32_t, double>> buf;
#pragma omp for schedule(dynamic, 4096)
        for (int64_t r = 0; r < M; ++r) {
            const int64_t b = rp[r], e = rp[r + 1];
            bool sorted = true;
            for (int64_t j = b + 1; j < e && sorted; ++j) sorted = ci[j - 1] <= ci[j];
            if (sorted) continue;
            buf.clear();
            for (int64_t j = b; j < e; ++j) buf.push_back({ci[j], vv[j]});
            std::stable_sort(buf.begin(), buf.end(),
                             [](const std::pair<int32_t, double> &a, const std::pair<int32_t, double> &c2) {
                                 return a.first < c2.first;
                             });
            for (int64_t j = b; j < e; ++j) {
                ci[j] = buf[(size_t)(j - b)].first;
                vv[j] = buf[(size_t)(j - b)].second;
            }
        }
    }
}

std::string lower_word(const char *&t, const char *e) {
    while (t < e && is_ws(*t)) ++t;
    std::string w;
    while (t < e && !is_ws(*t)) w += (char)std::tolower((unsigned char)*t++);
    return w;
}

}  // namespace

extern "C" {

void spmv_free_host(void *p) { std::free(p); }

int spmv_load_mtx(const char *path, int32_t *m, int32_t *n, int32_t *nnz, int32_t **row_idx,
                  int32_t **col_idx, double **val) {
    SPMV_CHECK_ARG(path && m && n && nnz && row_idx && col_idx && val, "NULL argument");
    Mapped mp;
    SPMV_RETURN_IF(map_file(path, mp));
    const char *p = mp.base, *end = mp.base + mp.size;
    while (p < end && *p == '%') p = next_line(p, end);  // util.cpp:37-39
    long long hdr[3];
    const char *body = read_size_line(p, end, hdr);  // util.cpp:41-42
    if (!body) {
        set_error("bad Matrix Market header");
        return SPMV_ERROR_IO;
    }
    const long long M = hdr[0], N = hdr[1], L = hdr[2];
    if (M < 0 || N < 0 || L < 0 || M >= INT32_MAX || N >= INT32_MAX || L >= INT32_MAX) {
        set_error("bad Matrix Market header");
        return SPMV_ERROR_IO;
    }
    std::vector<int32_t> tr, tc;
    std::vector<double> tv;
    SPMV_RETURN_IF(parse_entries(body, end, L, M, N, 3, VAL_REAL, tr, tc, tv));
    // stable counting sort by row, then each row by column (stable)
    std::vector<int64_t> rp((size_t)M + 1, 0);
    for (long long i = 0; i < L; ++i) ++rp[(size_t)tr[(size_t)i] + 1];
    for (long long r = 0; r < M; ++r) rp[(size_t)r + 1] += rp[(size_t)r];
    const size_t k = L ? (size_t)L : 1;
    int32_t *ri = (int32_t *)std::malloc(sizeof(int32_t) * k);
    int32_t *ci = (int32_t *)std::malloc(sizeof(int32_t) * k);
    double *vv = (double *)std::malloc(sizeof(double) * k);
    if (!ri || !ci || !vv) {
        std::free(ri);
        std::free(ci);
        std::free(vv);
        set_error("host allocation failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    {
        std::vector<int64_t> pos(rp.begin(), rp.end() - 1);
        for (long long i = 0; i < L; ++i) {
            const int64_t d = pos[(size_t)tr[(size_t)i]]++;
            ri[d] = tr[(size_t)i];
            ci[d] = tc[(size_t)i];
            vv[d] = tv[(size_t)i];
        }
    }
    sort_rows(rp.data(), M, ci, vv);
    // Equal (row, col) keys: the reference's std::sort (src/util.cpp:51) is
    // not stable, so duplicates leave it in an order of its own.  The file
    // order and the comparator (src/util.h:35-38) fix that order for a given
    // libstdc++; when duplicates exist, the whole list is re-sorted exactly as
    // the reference does (one thread), so their summation order matches too.
    bool dups = false;
#pragma omp parallel for schedule(static) reduction(|| : dups)
    for (long long r = 0; r < M; ++r)
        for (int64_t j = rp[(size_t)r] + 1; j < rp[(size_t)r + 1]; ++j) dups = dups || ci[j] == ci[j - 1];
    if (dups) {
        struct Element {  // the reference's triplet and operator< (src/util.h:30-39)
            int row, col;
            double val;
            bool operator<(const Element &e) const {
                if (row == e.row) return col < e.col;
                return row < e.row;
            }
        };
        std::vector<Element> el((size_t)L);
        for (long long i = 0; i < L; ++i) el[(size_t)i] = Element{tr[(size_t)i], tc[(size_t)i], tv[(size_t)i]};
        std::sort(el.begin(), el.end());
        for (long long i = 0; i < L; ++i) {
            ri[i] = el[(size_t)i].row;
            ci[i] = el[(size_t)i].col;
            vv[i] = el[(size_t)i].val;
        }
    }
    *m = (int32_t)M;
    *n = (int32_t)N;
    *nnz = (int32_t)L;
    *row_idx = ri;
    *col_idx = ci;
    *val = vv;
    return SPMV_SUCCESS;
}

int spmv_load_mtx_csr(const char *path, uint32_t flags, int64_t *m, int64_t *n, int64_t *nnz, int64_t **row_ptr,
                      int32_t **col_idx, double **val, uint32_t *info) {
    SPMV_CHECK_ARG(path && m && n && nnz && row_ptr && col_idx && val, "NULL argument");
    Mapped mp;
    SPMV_RETURN_IF(map_file(path, mp));
    const char *p = mp.base, *end = mp.base + mp.size;
    // banner (mm_read_banner): %%MatrixMarket matrix coordinate <field> <symmetry>
    const char *le = (const char *)std::memchr(p, '\n', (size_t)(end - p));
    if (!le) le = end;
    const char *t = p;
    const std::string w0 = lower_word(t, le), w1 = lower_word(t, le), w2 = lower_word(t, le),
                      field = lower_word(t, le), sym = lower_word(t, le);
    if (w0 != "%%matrixmarket" || w1 != "matrix" || w2 != "coordinate") {
        set_error("Could not process Matrix Market banner (need '%%MatrixMarket matrix coordinate ...')");
        return SPMV_ERROR_IO;
    }
    if (field == "complex") {  // main.cu:176-180
        set_error("data type 'complex' is not supported");
        return SPMV_ERROR_NOT_SUPPORTED;
    }
    int kind;
    if (field == "real" || field == "double") kind = VAL_REAL;
    else if (field == "integer") kind = VAL_INTEGER;
    else if (field == "pattern") kind = VAL_PATTERN;
    else {
        set_error("unknown Matrix Market field '" + field + "'");
        return SPMV_ERROR_IO;
    }
    if (sym != "general" && sym != "symmetric" && sym != "hermitian" && sym != "skew-symmetric") {
        set_error("unknown Matrix Market symmetry '" + sym + "'");
        return SPMV_ERROR_IO;
    }
    // mm_is_symmetric || mm_is_hermitian (main.cu:190-193); skew-symmetric is
    // not expanded by the reference, and is not here
    const bool mirror = (sym == "symmetric" || sym == "hermitian") && !(flags & SPMV_MTX_NO_EXPAND);
    p = le < end ? le + 1 : end;
    while (p < end && *p == '%') p = next_line(p, end);  // mm_read_mtx_crd_size skips comments
    while (p < end && (*p == '\n' || *p == '\r')) ++p;
    long long hdr[3];
    const char *body = read_size_line(p, end, hdr);
    if (!body || hdr[0] < 0 || hdr[1] < 0 || hdr[2] < 0 || hdr[0] >= INT32_MAX || hdr[1] >= INT32_MAX) {
        set_error("bad Matrix Market size line");
        return SPMV_ERROR_IO;
    }
    const long long M = hdr[0], N = hdr[1], L = hdr[2];
    if (mirror && M != N) {
        set_error("symmetric Matrix Market file with m != n");
        return SPMV_ERROR_IO;
    }
    std::vector<int32_t> tr, tc;
    std::vector<double> tv;
    SPMV_RETURN_IF(parse_entries(body, end, L, M, N, kind == VAL_PATTERN ? 2 : 3, kind, tr, tc, tv));
    // counts (main.cu:228-247), exclusive scan (:249-258)
    std::vector<int64_t> rp((size_t)M + 1, 0);
    for (long long i = 0; i < L; ++i) {
        ++rp[(size_t)tr[(size_t)i] + 1];
        if (mirror && tr[(size_t)i] != tc[(size_t)i]) ++rp[(size_t)tc[(size_t)i] + 1];
    }
    for (long long r = 0; r < M; ++r) rp[(size_t)r + 1] += rp[(size_t)r];
    const int64_t NNZ = rp[(size_t)M];
    int64_t *rpo = (int64_t *)std::malloc(8 * ((size_t)M + 1));
    int32_t *ci = (int32_t *)std::malloc(4 * (size_t)std::max<int64_t>(NNZ, 1));
    double *vv = (double *)std::malloc(8 * (size_t)std::max<int64_t>(NNZ, 1));
    if (!rpo || !ci || !vv) {
        std::free(rpo);
        std::free(ci);
        std::free(vv);
        set_error("host allocation failed");
        return SPMV_ERROR_OUT_OF_MEMORY;
    }
    std::memcpy(rpo, rp.data(), 8 * ((size_t)M + 1));
    // scatter in file order; a mirrored entry right after its original
    // (main.cu:266-300)
    std::vector<int64_t> pos(rp.begin(), rp.end() - 1);
    for (long long i = 0; i < L; ++i) {
        const int32_t r = tr[(size_t)i], c = tc[(size_t)i];
        int64_t d = pos[(size_t)r]++;
        ci[d] = c;
        vv[d] = tv[(size_t)i];
        if (mirror && r != c) {
            d = pos[(size_t)c]++;
            ci[d] = r;
            vv[d] = tv[(size_t)i];
        }
    }
    if (flags & SPMV_MTX_SORT_COLUMNS) sort_rows(rpo, M, ci, vv);
    *m = M;
    *n = N;
    *nnz = NNZ;
    *row_ptr = rpo;
    *col_idx = ci;
    *val = vv;
    if (info) *info = (uint32_t)kind | (mirror ? 4u : 0u) | (sym == "skew-symmetric" ? 8u : 0u);
    return SPMV_SUCCESS;
}

// ---- binary CSR cache ------------------------------------------------------
// Layout: "SPMVCSR1" | int64 m | int64 n | int64 nnz | int64 row_ptr[m+1] |
//         int32 col[nnz] | pad to 8 | double val[nnz]   (little endian)
static const char kMagic[8] = {'S', 'P', 'M', 'V', 'C', 'S', 'R', '1'};

int spmv_save_csr_bin(const char *path, int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr,
                      const int32_t *col_idx, const double *val) {
    SPMV_CHECK_ARG(path && row_ptr && m >= 0 && n >= 0 && nnz >= 0, "bad arguments");
    SPMV_CHECK_ARG(nnz == 0 || (col_idx && val), "col/val is NULL");
    FILE *f = std::fopen(path, "wb");
    if (!f) {
        set_error(std::string("cannot create ") + path);
        return SPMV_ERROR_IO;
    }
    const int64_t hdr[3] = {m, n, nnz};
    const int64_t pad = (4 * nnz) % 8 ? 8 - (4 * nnz) % 8 : 0;
    const char zeros[8] = {0};
    bool ok = std::fwrite(kMagic, 1, 8, f) == 8 && std::fwrite(hdr, 8, 3, f) == 3 &&
              std::fwrite(row_ptr, 8, (size_t)m + 1, f) == (size_t)m + 1 &&
              std::fwrite(col_idx, 4, (size_t)nnz, f) == (size_t)nnz &&
              std::fwrite(zeros, 1, (size_t)pad, f) == (size_t)pad &&
              std::fwrite(val, 8, (size_t)nnz, f) == (size_t)nnz;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        set_error(std::string("write failed: ") + path);
        return SPMV_ERROR_IO;
    }
    return SPMV_SUCCESS;
}

int spmv_load_csr_bin(const char *path, int64_t *m, int64_t *n, int64_t *nnz, int64_t **row_ptr,
                      int32_t **col_idx, double **val) {
    SPMV_CHECK_ARG(path && m && n && nnz && row_ptr && col_idx && val, "NULL argument");
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        set_error(std::string("File not Found: ") + path);
        return SPMV_ERROR_IO;
    }
    char magic[8];
    int64_t hdr[3];
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, kMagic, 8) != 0 ||
        std::fread(hdr, 8, 3, f) != 3 || hdr[0] < 0 || hdr[1] < 0 || hdr[2] < 0) {
        std::fclose(f);
        set_error("not a SPMVCSR1 file");
        return SPMV_ERROR_IO;
    }
    const int64_t M = hdr[0], NN = hdr[2];
    int64_t *rp = (int64_t *)std::malloc(8 * (size_t)(M + 1));
    int32_t *ci = (int32_t *)std::malloc(4 * (size_t)(NN ? NN : 1));
    double *vv = (double *)std::malloc(8 * (size_t)(NN ? NN : 1));
    const int64_t pad = (4 * NN) % 8 ? 8 - (4 * NN) % 8 : 0;
    char zeros[8];
    bool ok = rp && ci && vv && std::fread(rp, 8, (size_t)M + 1, f) == (size_t)M + 1 &&
              std::fread(ci, 4, (size_t)NN, f) == (size_t)NN &&
              std::fread(zeros, 1, (size_t)pad, f) == (size_t)pad &&
              std::fread(vv, 8, (size_t)NN, f) == (size_t)NN;
    std::fclose(f);
    ok = ok && rp[0] == 0 && rp[M] == NN;
    if (!ok) {
        std::free(rp);
        std::free(ci);
        std::free(vv);
        set_error("truncated or inconsistent SPMVCSR1 file");
        return SPMV_ERROR_IO;
    }
    *m = M;
    *n = hdr[1];
    *nnz = NN;
    *row_ptr = rp;
    *col_idx = ci;
    *val = vv;
    return SPMV_SUCCESS;
}

}  // extern "C"

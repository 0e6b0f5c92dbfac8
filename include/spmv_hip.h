/*
 * spmv_hip.h -- C-ABI of the MI355X-native fp64 SpMV engine (libspmv_hip.so).
 *
 * This is the drop-in boundary for the reference's `opt_*` format-dispatch
 * surface (hir0shim/singleSpMV).  Plain C types only: pointers, sizes, int
 * status codes.  No exit(), no torch types, no C++ in the signatures.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repository):
 *
 *   spmv_plan_create_coo   OptimizeProblem(const SpMat&, const Vec&, SpMatOpt&,
 *                          VecOpt&) of every plugin, e.g. src/opt_crs.h:15,
 *                          src/opt_ell.h:16, src/opt_ss.h:35, src/opt_dia.h:16,
 *                          src/opt_cusparse.h:33; SpMat is src/util.h:7-19.
 *   spmv_plan_create_csr*  opt_crs SpMatOpt {ptr, idx, val} (src/opt_crs.h:3-9)
 *                          and the device CSR of src/opt_cusparse.cpp:36-42.
 *   spmv_execute           extern "C" SpMV(const SpMatOpt&, const VecOpt&,
 *                          Vec&) (e.g. src/opt_crs.h:16-18); with host x / host
 *                          y it reproduces src/opt_cusparse.cpp:72-82 (H2D x,
 *                          y = 1*A*x + 0*y, D2H y).
 *   spmv_plan_destroy      (the reference never frees; no counterpart)
 *   spmv_load_mtx          LoadSparseMatrix (src/util.cpp:30-66), parallel
 *   spmv_load_mtx_csr      the CSR5 benchmark's banner-aware loader
 *                          (CSR5_cuda/main.cu:157-306): pattern/integer,
 *                          symmetric expansion, straight to CSR
 *   spmv_{save,load}_csr_bin (new) binary CSR cache
 *   spmv_rand_vector       srand + CreateRandomVector (src/main.cpp:18,
 *                          src/util.cpp:92-102)
 *   spmv_verify_coo        VerifyResult (src/util.cpp:67-83)
 *   spmv_gen_*             (new) seeded synthetic matrices for the BASELINE
 *                          configs, generated in memory instead of .mtx text
 *   spmv_partition_rows    (new) nnz-balanced row ranges for multi-GPU
 *
 * Semantics shared by every format (β = 0): spmv_execute overwrites every
 * entry of y (src/opt_crs.cpp:68; src/opt_ell.cpp:78; src/opt_dia.cpp:82) and
 * is idempotent -- repeated calls give identical y (the two-call verification
 * of src/main.cpp:41-55).  Host input arrays are borrowed read-only during
 * plan creation and never mutated (unlike the CSR5 handle, which transposes
 * the caller's arrays in place, CSR5_cuda/anonymouslib_cuda.h:203-204).
 *
 * Threading: thread-compatible.  One plan per thread; a plan may be used from
 * any thread but not concurrently.
 */
#ifndef SPMV_HIP_H
#define SPMV_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version 2 changed the layout of spmv_options_t (the bin_* / placement
 * fields, round 2) and spmv_plan_info_t: a caller built against a version-1
 * header passes structs of the wrong size and must be rebuilt.  Version 3
 * (round 3) took bin_product_order from spmv_options_t's reserved words (same
 * size) and appended bin_sum_entries to spmv_plan_info_t.  crs_exact and build
 * (round 5) took the last reserved words: same size, and 0
 * (spmv_options_default) keeps the version-3 results (build = AUTO moves only
 * where the layout is made, not what it is).  Callers may
 * check spmv_api_version() == SPMV_HIP_API_VERSION once at startup; the
 * structs are only ever filled by spmv_options_default / spmv_plan_info of a
 * library with the same version. */
#define SPMV_HIP_API_VERSION 3
int spmv_api_version(void);

/* ---- status codes -------------------------------------------------------- */
typedef enum spmv_status {
    SPMV_SUCCESS = 0,
    SPMV_ERROR_INVALID_VALUE = 1,  /* bad argument / inconsistent arrays    */
    SPMV_ERROR_NOT_SUPPORTED = 2,  /* format cannot hold this matrix        */
    SPMV_ERROR_OUT_OF_MEMORY = 3,  /* host or device allocation failed      */
    SPMV_ERROR_HIP = 4,            /* a HIP runtime call failed             */
    SPMV_ERROR_IO = 5,             /* file missing / unparsable             */
    SPMV_ERROR_NO_DEVICE = 6       /* no usable gfx950 device               */
} spmv_status_t;

/* ---- storage formats (the reference's -DOPT_<FMT> plugins) --------------- */
typedef enum spmv_format {
    SPMV_FORMAT_AUTO = 0, /* chosen from the row-length histogram             */
    SPMV_FORMAT_CSR = 1,  /* opt_crs   (src/opt_crs.cpp)                        */
    SPMV_FORMAT_ELL = 2,  /* opt_ell   (src/opt_ell.cpp), device: sliced ELL    */
    SPMV_FORMAT_SS = 3,   /* opt_ss / CSR5: segmented sum over 64 x sigma tiles */
    SPMV_FORMAT_DIA = 4,  /* opt_dia   (src/opt_dia.cpp), device: row-indexed   */
    SPMV_FORMAT_HYB = 5,  /* ELL(K) + CSR overflow (BASELINE config 3)          */
    SPMV_FORMAT_CSS = 6,  /* opt_css lineage: column-slab sweep, y in LDS, x    */
                          /* slab L2-resident per XCD (large random matrices)  */
    SPMV_FORMAT_COO = 7,  /* opt_coo   (src/opt_coo.cpp): f64 atomics per row segment */
    SPMV_FORMAT_JDS = 8,  /* opt_jds   (src/opt_jds.cpp): rows sorted by length,  */
                          /* jagged 64-row slices, y permuted back             */
    SPMV_FORMAT_BIN = 9   /* opt_ss Mul/Sum x opt_css column blocks: Mul with   */
                          /* the x strip in LDS, products binned by row block,  */
                          /* Sum per bin with y in LDS (large random matrices)  */
} spmv_format_t;

typedef struct spmv_plan_s *spmv_plan_t;

typedef struct spmv_options {
    int32_t format;     /* spmv_format_t                                      */
    int32_t device;     /* HIP device ordinal; -1 = the calling thread's current */
    int32_t csr_lanes;  /* CSR: lanes per row 1..64 (power of two), 0 = auto   */
    int32_t ell_width;  /* HYB: ELL width K, 0 = auto (row-length histogram)   */
    int32_t ss_sigma;   /* SS: nnz per lane per tile, 0 = auto                 */
    int32_t dia_max_diags; /* DIA: refuse beyond this many diagonals (0 = 1024) */
    double dia_max_fill;   /* DIA: refuse when stored/nnz exceeds this (0 = 3) */
    int32_t css_slab_shift; /* CSS: slab = 2^shift columns (0 = 18, 2 MiB of x) */
    int32_t css_lag;        /* CSS: pacing slack in slabs (0 = 4, -1 = no pacing) */
    int32_t css_pace;       /* CSS: 0/1 pace against every XCD, 2 own XCD only */
    int32_t bin_strip_cols;  /* BIN: x strip width, 64..20480 columns (0 = 20480) */
    int32_t bin_groups;      /* BIN: row groups sharing one product buffer (0 = 1) */
    int32_t bin_sum_waves;   /* BIN: Sum waves per workgroup 2 | 4 | 8 (0 = auto) */
    int32_t bin_pad;         /* BIN: segment padding 8 | 16 | 32 entries (0 = auto) */
    int32_t csr_row_ptr64;   /* CSR: 1 = 64-bit row pointers below 2^31 nnz too */
    int32_t placement;       /* BIN product buffer / DIA values, see SPMV_PLACEMENT_* */
    int32_t bin_long_len;    /* BIN: rows with >= this many entries are reduced per
                                strip run in the Mul (partial sums, <= 1e-12 from
                                the sequential sum); 0 = auto (max(128, strips)
                                when such rows hold >= 5 % of nnz), -1 = never
                                (every row bit-exact)                         */
    int32_t bin_product_order; /* BIN: where the Mul writes its products
                                (SPMV_BIN_ORDER_*; 0 = auto)                   */
    int32_t crs_exact;       /* CSR requests: 1 = opt_crs semantics -- every row
                                the sequential column-order sum bit for bit
                                (src/opt_crs.cpp:57-69) on the fastest layout
                                that sums so for this matrix: DIA (AUTO's banded
                                rule, rows strictly ascending: no duplicates),
                                BIN with no run path (AUTO's wide-x rule, rows
                                strictly ascending: strip order = CSR order),
                                ELL (near-uniform rows, none > 64), else CSR with
                                one lane per row; spmv_plan_info reports the
                                layout.  Bit for bit for finite x: DIA and ELL
                                padding adds 0 * x[c], which is NaN where x[c]
                                is Inf or NaN (opt_crs skips no entry but has
                                no padding).  0 = the CSR kernels as configured
                                (row groups of L lanes: butterfly sums)       */
    int32_t build;           /* plan builders (SPMV_BUILD_*): AUTO = a host CSR of
                                >= 2^24 entries is staged into HBM and built by
                                the device builders (every format;
                                byte-identical layouts, spmv_plan_digest), when
                                the staging copy fits in device memory
                                (else the host builders, with the format
                                resolved there); smaller ones take the host
                                builders */
} spmv_options_t;

/* Where spmv_plan_create_csr / _csr32 / _coo build the layout. */
typedef enum spmv_build {
    SPMV_BUILD_AUTO = 0,
    SPMV_BUILD_HOST = 1,    /* host builders (formats.cpp, build_bin.cpp)       */
    SPMV_BUILD_DEVICE = 2   /* stage the CSR into HBM and build there whatever
                               the size (same exceptions as AUTO)              */
} spmv_build_t;

/* Placement of the large buffers of a plan (the BIN product buffer, the DIA
 * values, the streamed col / val arrays of CSR, ELL, HYB, JDS, SS, COO, CSS).  The BIN Mul ran ~15 % slower with one
 * plain hipMalloc on most plans than with the same buffer built from 2-MB
 * physical handles (profiles/round1/README.md §4a "Placement, round 3").
 *
 * Known limitation: placement is not fully under the library's control.
 * Measured residual spread of AUTO over 8 same-size plans kept alive in one
 * process (profiles/round5/placement/): config-4 DIA 1.472-1.562 ms (6.1 %,
 * every later plan within 1 % of the first or faster), config-2 BIN
 * 0.797-0.897 ms (12.6 %, worst 7.6 % above the first).  SEARCH narrowed
 * that to 1.2 % (DIA 1.478-1.495) and 4.2 % (BIN 0.801-0.835) at 0.6-7.3 s
 * of build per plan and transient candidate buffers over the free HBM, so it
 * stays an explicit opt-in; a caller who needs the best time builds its hot
 * plan first or with SEARCH (spmv_plan_info reports the mode, the candidates
 * and their best / worst launch). */
#define SPMV_PLACEMENT_AUTO 0   /* BIN products >= 32 MB, DIA values >= 256 MB and
                                   the streamed arrays (col / val / slots) of the
                                   other formats >= 256 MB: VMM; the rest PLAIN  */
#define SPMV_PLACEMENT_PLAIN 1  /* one hipMalloc                                     */
#define SPMV_PLACEMENT_SEARCH 2 /* BIN product buffer (>= 32 MB) / DIA values
                                   (>= 256 MB): up to 8 plain candidates spread
                                   over all free HBM, each timed with one launch
                                   over a zero x, the fastest kept (build-time
                                   cost and transient memory: see above); other
                                   formats: as AUTO                               */
#define SPMV_PLACEMENT_VMM 3    /* hipMemCreate handles of 2 MB mapped back to back
                                   into one VA range aligned to 1 GB (no transient
                                   device memory)                                 */

/* Product order of a BIN plan (spmv_options_t.bin_product_order).  Either
 * way each row is summed in column order (bit-identical y). */
#define SPMV_BIN_ORDER_AUTO 0  /* MUL for short segments (< 112 entries per
                                  row bin x column strip: the wide multi-GPU
                                  rank shapes) where the layout allows it (no
                                  long rows, one row group, < 2^31 entries),
                                  else SUM                                    */
#define SPMV_BIN_ORDER_SUM 1   /* the Mul scatters each product into its (bin,
                                  strip) segment of the Sum's order; the Sum
                                  streams each bin as one contiguous run       */
#define SPMV_BIN_ORDER_MUL 2   /* the Mul writes its products contiguously in
                                  its own order (no segment padding, no
                                  destination array); the Sum gathers each
                                  bin's segments in 8-entry chunks through a
                                  chunk table                                  */

/* Fill `opt` with defaults (AUTO format, current device, auto tuning). */
void spmv_options_default(spmv_options_t *opt);

/* Plan builds are untimed setup (OptimizeProblem, src/main.cpp:36).  They
 * allocate the plan's device arrays and nothing else.
 *
 * Plan from a host sorted COO (the reference SpMat, src/util.h:7-19).
 * Rows must be sorted ascending (LoadSparseMatrix guarantees it); columns
 * within a row may be in any order, duplicates are summed. */
int spmv_plan_create_coo(int32_t m, int32_t n, int32_t nnz, const int32_t *row_idx,
                         const int32_t *col_idx, const double *val,
                         const spmv_options_t *opt, spmv_plan_t *plan);

/* Plan from a host CSR with 64-bit row pointers (nnz may exceed 2^31). */
int spmv_plan_create_csr(int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr,
                         const int32_t *col_idx, const double *val,
                         const spmv_options_t *opt, spmv_plan_t *plan);

/* Plan from a host CSR with 32-bit row pointers (opt_crs SpMatOpt layout). */
int spmv_plan_create_csr32(int32_t m, int32_t n, int32_t nnz, const int32_t *row_ptr,
                           const int32_t *col_idx, const double *val,
                           const spmv_options_t *opt, spmv_plan_t *plan);

/* Plan from a CSR that already lives in device memory (64-bit row pointers;
 * all three arrays on the plan's device, only read).  Every format is built
 * on the device (the CSR5 conversion pipeline's role,
 * CSR5_cuda/detail/cuda/format_cuda.h:21-718): only the row pointers (and,
 * for BIN, the (bin, strip) counts and the long rows' run descriptors) visit
 * the host, for the layout decisions that depend on row lengths alone; AUTO
 * is resolved there too, its diagonal census run on the device; CSS's
 * per-wave column sorts are one stable radix sort.  The layouts are
 * byte-identical to the host builders' (spmv_plan_digest); BIN sorts rows
 * whose columns are not ascending by 20480-column strip on the device first
 * (when the device has no room for that copy, the CSR is copied to the host
 * and the host builder runs).  The input is validated on the device like
 * spmv_plan_create_csr's host check. */
int spmv_plan_create_csr_device(int64_t m, int64_t n, int64_t nnz, const int64_t *d_row_ptr,
                                const int32_t *d_col_idx, const double *d_val,
                                const spmv_options_t *opt, spmv_plan_t *plan);

/* The same from 32-bit device row pointers (the CSR5 handle's inputCSR,
 * CSR5_cuda/anonymouslib_cuda.h:60-73, takes int arrays on the device). */
int spmv_plan_create_csr32_device(int32_t m, int32_t n, int32_t nnz, const int32_t *d_row_ptr,
                                  const int32_t *d_col_idx, const double *d_val,
                                  const spmv_options_t *opt, spmv_plan_t *plan);

int spmv_plan_destroy(spmv_plan_t plan);

/* ---- per-phase profile (replaces the g_profile / PROF_BEGIN instrumentation
 * of src/util.cpp:16-18, src/util.h:59-65 and the Mul/Sum split printed by
 * src/main.cpp:172-175).  Runs `iters` synchronised calls on device x/y and
 * returns the mean ms of each phase of the plan's launch sequence:
 *   CSR "csr" | ELL, JDS "ell" | HYB "ell","overflow" | SS "tile","fixup" |
 *   DIA "dia" | CSS "sweep" | COO "zero_y","segment" | BIN "mul","sum"
 *   (repeated per row group). */
int spmv_profile(spmv_plan_t plan, const double *x_dev, double *y_dev, int32_t iters,
                 double *phase_ms, int32_t max_phases, int32_t *n_phases);
const char *spmv_phase_name(spmv_plan_t plan, int32_t k);

/* Measured STREAM-read ceiling of `device` (GB/s): nontemporal 16-byte reads
 * of a `bytes` buffer (use >> 256 MB), `iters` launches timed with events. */
int spmv_stream_probe(int32_t device, int64_t bytes, int32_t iters, double *read_gbs);

/* Measured STREAM-write ceiling of `device` (GB/s): nontemporal 16-byte
 * stores over a `bytes` buffer, `iters` launches timed with events. */
int spmv_stream_write_probe(int32_t device, int64_t bytes, int32_t iters, double *write_gbs);

/* Measured mixed read + write ceiling of `device` (GB/s of reads + writes): a
 * grid-stride stream reading `bytes` (16-byte loads) and writing
 * write_quarters/4 of them back (nontemporal 16-byte stores), the fastest of
 * `iters` launches; BIN's Mul moves about 3 quarters. */
int spmv_mixed_probe(int32_t device, int64_t bytes, int32_t write_quarters, int32_t iters, double *gbs);

/* Measured ceiling of random 8-byte gathers (gathers/s): n streamed int32
 * indices into a `table_bytes` table (1 MB: L2-resident, the best case of a
 * gather-bound SpMV), 8 gathers in flight per lane, best of 5 launches. */
int spmv_gather_probe(int32_t device, int64_t n, int64_t table_bytes, double *g_per_s);

/* Exactness guard of the BIN and CSS formats: `rounds` wave-wide atomic adds
 * of f64 into 64 LDS slots (one ds_add_f64 instruction each; lane l of round
 * r adds val[r*64+l] to slot[r*64+l]); out[64] = the slots afterwards.  BIN
 * and CSS are bit-identical to the sequential opt_crs sum only if lanes of
 * one instruction that hit the same slot are applied in lane order. */
int spmv_lds_order_probe(int32_t device, int32_t rounds, const int32_t *slot, const double *val,
                         double *out);

/* ---- execution ----------------------------------------------------------- */
#define SPMV_X_DEVICE 0x1u /* x is a device pointer (else host: H2D per call) */
#define SPMV_Y_DEVICE 0x2u /* y is a device pointer (else host: D2H per call).
                              COO plans add into y with device f64 atomics
                              (-munsafe-fp-atomics): a device y must be
                              ordinary (coarse-grained) device memory, as
                              hipMalloc returns -- not fine-grained or host-
                              mapped memory, where those atomics are not
                              performed atomically                            */
#define SPMV_ASYNC 0x4u    /* device x and y: return without synchronising    */
#define SPMV_X_STAGED 0x8u /* re-use the host x uploaded by the previous call
                              (x may be NULL); error if none was staged       */
#define SPMV_Y_STAGED 0x10u /* leave y in the plan's device staging buffer (y
                              may be NULL; no D2H copy): spmv_fetch_y copies it
                              to the host when the caller reads it -- the
                              per-call 8m-byte download of opt_cusparse
                              (src/opt_cusparse.cpp:82) leaves the timed loop */

/* y = A * x.  x holds n doubles, y holds m doubles. */
int spmv_execute(spmv_plan_t plan, const double *x, double *y, uint32_t flags);

/* Copy the y of the latest execute to host memory (m doubles); that execute
 * must have been SPMV_Y_STAGED (any other execute since then makes this
 * SPMV_ERROR_INVALID_VALUE instead of returning an older y). */
int spmv_fetch_y(spmv_plan_t plan, double *y_host);

/* y = alpha * A * x (the CSR5 handle's spmv(alpha, y),
 * CSR5_cuda/anonymouslib_cuda.h:262-284); alpha is applied to the finished
 * row sums (one rounded multiply), beta = 0 as everywhere. */
int spmv_execute_alpha(spmv_plan_t plan, double alpha, const double *x, double *y, uint32_t flags);

/* Kernels are launched on this stream (a hipStream_t; NULL = null stream). */
int spmv_set_stream(spmv_plan_t plan, void *hip_stream);

/* Bench helper: `iters` back-to-back executes (device x, device y) between two
 * hipEvents recorded on the plan's stream; *ms = elapsed milliseconds total. */
int spmv_time(spmv_plan_t plan, const double *x_dev, double *y_dev, int32_t iters,
              double *ms);

/* ---- HIP graph of the device-resident execute -----------------------------
 * The plan's launch sequence for (x_dev -> y_dev), captured `reps` times in a
 * row into one hipGraph (stream capture on a private stream) and
 * instantiated.  spmv_graph_launch enqueues all reps x n_kernels kernels on
 * the plan's current stream with one submission -- the per-call launch cost
 * that dominates small matrices, whose kernels are shorter than their
 * launches (the reference driver repeats SpMV until >= 1 s,
 * src/main.cpp:58-102).  Each rep computes exactly what spmv_execute does
 * (y bit-identical); x_dev and y_dev are fixed in the graph, so the caller
 * keeps them allocated until spmv_graph_destroy.  A graph replays the plan's
 * kernels on the plan's device arrays: destroy every graph of a plan before
 * the plan (launching a graph whose plan is gone is undefined; destroying it
 * is safe).  CSS plans (whose sweep
 * tags its progress flags with a per-launch sequence number) return
 * SPMV_ERROR_NOT_SUPPORTED. */
typedef struct spmv_graph_s *spmv_graph_t;
int spmv_graph_create(spmv_plan_t plan, const double *x_dev, double *y_dev, int32_t reps,
                      spmv_graph_t *graph);
/* flags: SPMV_ASYNC = return without synchronising the stream */
int spmv_graph_launch(spmv_graph_t graph, uint32_t flags);
/* `launches` back-to-back graph launches between two hipEvents on the plan's
 * stream; *ms = elapsed milliseconds total (launches x reps executes). */
int spmv_graph_time(spmv_graph_t graph, int32_t launches, double *ms);
int spmv_graph_destroy(spmv_graph_t graph);

typedef struct spmv_plan_info {
    int32_t format;          /* resolved spmv_format_t                         */
    int32_t device;
    int64_t m, n, nnz;
    int64_t stored_slots;    /* ELL/HYB/DIA slots incl. padding; CSR/SS = nnz   */
    int64_t device_bytes;    /* device memory held by the plan                 */
    int64_t algo_bytes;      /* compulsory bytes per execute (roofline model)  */
    int32_t row_ptr_bytes;   /* 4 or 8                                         */
    int32_t csr_lanes;       /* CSR / HYB overflow                             */
    int32_t ell_width;       /* ELL: max slice width; HYB: K                   */
    int32_t ss_sigma;
    int32_t n_diags;         /* DIA                                            */
    int32_t css_passes;      /* CSS: row passes, slabs per pass                */
    int32_t css_slabs;
    int32_t n_kernels;       /* launches per execute                           */
    int64_t overflow_nnz;    /* HYB: entries outside the ELL part              */
    int64_t empty_rows;
    int64_t css_split_rows;  /* CSS: rows split into pieces (long rows)       */
    char kernel[64];         /* name of the dominant kernel                    */
    int64_t bin_bins;        /* BIN: row bins (one Sum wave each), strips      */
    int64_t bin_strips;
    int32_t bin_strip_cols;  /* BIN: x strip width in columns                  */
    int32_t bin_pad;         /* BIN: segment padding (entries)                 */
    int32_t bin_sum_waves;   /* BIN: Sum waves per workgroup                   */
    int32_t bin_groups;      /* BIN: row groups (Mul launches)                 */
    int32_t placement;       /* BIN/DIA: the SPMV_PLACEMENT_* the build used   */
    int32_t placement_candidates; /* SEARCH: candidates timed                  */
    float placement_best_ms;  /* SEARCH: fastest / slowest candidate launch    */
    float placement_worst_ms;
    int32_t bin_long_len;     /* BIN: long-row threshold in use (0 = none)      */
    int32_t bin_product_order; /* BIN: SPMV_BIN_ORDER_SUM or _MUL (resolved)   */
    int64_t bin_long_rows;    /* BIN: rows on the run path, their run pieces    */
    int64_t bin_long_pieces;
    int64_t bin_products;     /* BIN: products + partials the Sum reads         */
    int64_t bin_long_entries; /* BIN: Mul entries in long blocks (with padding) */
    int64_t bin_sum_entries;  /* BIN: Sum-order positions (segments padded)     */
} spmv_plan_info_t;

int spmv_plan_info(spmv_plan_t plan, spmv_plan_info_t *info);

/* Layout digest (new; a check, not a compute path): one 64-bit hash per
 * device array of the plan (its logical bytes, position-keyed), so two plans
 * of one matrix -- e.g. a host build and a device build -- can be compared
 * array by array without copying them out.  *n_arrays = the plan's array
 * count (digests beyond `cap` are not written); spmv_plan_digest_name(plan,
 * k) names array k.  Every format (BIN: its entry, slot, destination and
 * run-path arrays and the small tables; not the product scratch). */
int spmv_plan_digest(spmv_plan_t plan, uint64_t *digests, int32_t cap, int32_t *n_arrays);
const char *spmv_plan_digest_name(spmv_plan_t plan, int32_t k);

/* *on_device = 1 when the plan's layout was built in HBM (by
 * spmv_plan_create_csr_device, or from a host CSR under
 * spmv_options_t::build), 0 when by the host builders. */
int spmv_plan_built_on_device(spmv_plan_t plan, int32_t *on_device);

const char *spmv_status_string(int status);
/* Detail of the last failure on the calling thread ("" if none). */
const char *spmv_last_error(void);

/* ---- multi-GPU in one process (new -- the reference is
 * single-device) -------------------------------------------------------------
 * The matrix is cut into nnz-balanced row ranges (spmv_partition_rows), one
 * plan per device over its rows with global column indices (n columns each).
 * x is copied to the first device and replicated by an RCCL broadcast over
 * xGMI; every device computes its rows; the y slices (padded to the longest
 * range) are all-gathered by RCCL into a full y on every device, and the
 * first device's copy is returned.  A C/C++ caller of the drop-in (the
 * reference driver, src/main.cpp:36,87) reaches config 5 through it; see
 * opt_hip.h SPMV_HIP_GPUS. */
typedef struct spmv_dist_s *spmv_dist_t;

/* The row cut a dist plan uses: cuts[parts+1] (spmv_partition_rows) and the
 * padded slice length (the longest range, >= 1).  Host only. */
int spmv_dist_layout(const int64_t *row_ptr, int64_t m, int32_t parts, int64_t *cuts, int64_t *slice_rows);

/* Host halves of a dist plan's data movement, exported so the reassembly can
 * be checked without a second GPU (the same code runs inside
 * spmv_dist_create_csr / spmv_dist_execute):
 *   spmv_dist_shard     part k's rows [cuts[k], cuts[k+1]): rp (rows + 1
 *                       entries) = row_ptr rebased to the part's first entry,
 *                       *entry0 = that entry (its col / val start there)
 *   spmv_dist_assemble  y (m doubles) from the all-gathered buffer of `parts`
 *                       slices of `slice` rows each (part k's rows at the
 *                       start of slice k, padding after them) */
int spmv_dist_shard(const int64_t *row_ptr, const int64_t *cuts, int32_t parts, int32_t k, int64_t *rp,
                    int64_t *entry0);
int spmv_dist_assemble(const double *gathered, const int64_t *cuts, int32_t parts, int64_t slice, double *y);

/* devices: n_devices distinct ordinals, or NULL for 0..n_devices-1.  opt
 * applies to every per-device plan (opt->device is ignored). */
int spmv_dist_create_csr(int32_t n_devices, const int32_t *devices, int64_t m, int64_t n, int64_t nnz,
                         const int64_t *row_ptr, const int32_t *col_idx, const double *val,
                         const spmv_options_t *opt, spmv_dist_t *dist);

/* y = A x with host x (n doubles) and host y (m doubles; NULL: the result
 * stays on the devices).  SPMV_X_STAGED: re-use the x broadcast by the
 * previous call (x may be NULL).  Returns after every device is done.  Any
 * other flag bit (SPMV_X_DEVICE, SPMV_Y_DEVICE, SPMV_ASYNC) is refused with
 * SPMV_ERROR_INVALID_VALUE. */
int spmv_dist_execute(spmv_dist_t dist, const double *x, double *y, uint32_t flags);

/* The full y of the last spmv_dist_execute (as assembled on the first
 * device) to host memory (m doubles) -- after a call made with y = NULL. */
int spmv_dist_fetch_y(spmv_dist_t dist, double *y_host);

/* Per-step times over `iters` steps with the staged x: the local SpMV (max
 * over devices of the event time on each device's stream) and, separately,
 * the all-gather of the y slices. */
int spmv_dist_time(spmv_dist_t dist, int32_t iters, double *spmv_ms, double *gather_ms);

/* n_devices, the row cuts (n_devices + 1, optional) and the per-device plans
 * (optional; owned by the dist plan). */
int spmv_dist_info(spmv_dist_t dist, int32_t *n_devices, int64_t *cuts, spmv_plan_t *plans);
int spmv_dist_destroy(spmv_dist_t dist);

/* ---- host utilities ------------------------------------------------------ */

/* LoadSparseMatrix semantics (src/util.cpp:30-66): skip leading '%' lines,
 * header "M N L", exactly L triplets, 1->0 based, stable row-major sort,
 * duplicates kept.  Arrays are malloc'd; release with spmv_free_host. */
int spmv_load_mtx(const char *path, int32_t *m, int32_t *n, int32_t *nnz,
                  int32_t **row_idx, int32_t **col_idx, double **val);
void spmv_free_host(void *p);

/* Banner-aware Matrix Market -> CSR with the CSR5 benchmark's semantics
 * (opt/Benchmark_SpMV_using_CSR5/CSR5_cuda/main.cu:157-306): needs a
 * "%%MatrixMarket matrix coordinate <field> <symmetry>" banner; field real |
 * integer | pattern (values 1.0); complex -> SPMV_ERROR_NOT_SUPPORTED;
 * symmetric/hermitian off-diagonal entries are mirrored (skew-symmetric is
 * not, as in the reference).  Rows keep file order (a mirrored entry right
 * after its original) unless SPMV_MTX_SORT_COLUMNS.  *info (optional) =
 * field (0 real, 1 integer, 2 pattern) | 4 if mirrored | 8 if skew. */
#define SPMV_MTX_SORT_COLUMNS 0x1u
#define SPMV_MTX_NO_EXPAND 0x2u
int spmv_load_mtx_csr(const char *path, uint32_t flags, int64_t *m, int64_t *n, int64_t *nnz,
                      int64_t **row_ptr, int32_t **col_idx, double **val, uint32_t *info);

/* Binary CSR cache ("SPMVCSR1": header, int64 row_ptr, int32 col, f64 val) so
 * a large Matrix Market file is parsed once.  Arrays from the loader are
 * malloc'd; release with spmv_free_host. */
int spmv_save_csr_bin(const char *path, int64_t m, int64_t n, int64_t nnz, const int64_t *row_ptr,
                      const int32_t *col_idx, const double *val);
int spmv_load_csr_bin(const char *path, int64_t *m, int64_t *n, int64_t *nnz, int64_t **row_ptr,
                      int32_t **col_idx, double **val);

/* glibc srand(seed) then out[i] = rand()/RAND_MAX -- CreateRandomVector
 * (src/util.cpp:92-102).  Consecutive calls continue the rand() stream. */
void spmv_srand(uint32_t seed);
void spmv_rand_vector(int32_t n, double *out);

/* VerifyResult (src/util.cpp:67-83): returns -1 if every row passes, else the
 * first failing row (abs_err > 1e-6 AND rel_err > 1e-6). */
int64_t spmv_verify_coo(int32_t m, int32_t nnz, const int32_t *row_idx,
                        const int32_t *col_idx, const double *val,
                        const double *x, const double *y);

/* COO (sorted rows) -> CSR, the linear scan of src/opt_crs.cpp:26-33. */
int spmv_coo_to_csr(int32_t m, int64_t nnz, const int32_t *row_idx, int64_t *row_ptr);

/* ---- synthetic matrices (BASELINE configs 2-5) ---------------------------- */
typedef enum spmv_gen_kind {
    SPMV_GEN_UNIFORM = 1,  /* `per_row` nnz per row, columns uniform on [0,n)   */
    SPMV_GEN_POWERLAW = 2, /* row length ~ P(k) ∝ k^-alpha on [1, max_len]      */
    SPMV_GEN_BANDED = 3    /* diagonals band_lo..band_hi (col - row), all present */
} spmv_gen_kind_t;

typedef struct spmv_gen_spec {
    int32_t kind;        /* spmv_gen_kind_t                                  */
    int32_t per_row;     /* UNIFORM                                          */
    int64_t m, n;        /* global shape                                     */
    int32_t max_len;     /* POWERLAW upper bound (10000 for config 3)        */
    double alpha;        /* POWERLAW exponent (2.0)                          */
    int32_t band_lo;     /* BANDED lowest offset  (-32 for config 4)         */
    int32_t band_hi;     /* BANDED highest offset (+31 for config 4)         */
    int32_t integer_values; /* 1: values in {0..9} (bitwise-exact sums)      */
    uint64_t seed;
} spmv_gen_spec_t;

/* Number of nonzeros of global rows [row_begin, row_end). */
int spmv_gen_count(const spmv_gen_spec_t *spec, int64_t row_begin, int64_t row_end,
                   int64_t *nnz);
/* Fill the CSR of rows [row_begin, row_end): row_ptr has (rows+1) entries and
 * starts at 0; columns are global, sorted within each row.  With col_idx and
 * val both NULL only row_ptr is filled (the row lengths are a function of
 * (seed, row) alone -- what an nnz-balanced shard cut needs). */
int spmv_gen_fill(const spmv_gen_spec_t *spec, int64_t row_begin, int64_t row_end,
                  int64_t *row_ptr, int32_t *col_idx, double *val);
/* x[i] for global indices [begin, begin+count): U[0,1) (or {0..9}). */
int spmv_gen_vector(uint64_t seed, int32_t integer_values, int64_t begin,
                    int64_t count, double *out);

/* nnz-balanced cut rows: cuts[k] = first row r with row_ptr[r] >= k*nnz/parts
 * (cuts[0] = 0, cuts[parts] = m). */
int spmv_partition_rows(const int64_t *row_ptr, int64_t m, int32_t parts, int64_t *cuts);

#ifdef __cplusplus
}
#endif
#endif /* SPMV_HIP_H */

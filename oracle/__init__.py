"""oracle -- CPU restatement of the reference singleSpMV hot path.

TEST INFRASTRUCTURE ONLY.  ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` are the only callers.  The product
package ``singlespmv_amd`` never imports this module.

Two backends, both loaded with ctypes:

* ``liboracle.so`` -- oracle.c, our own restatement (each C function cites the
  reference file:line it follows).
* ``_ref/libref_<fmt>.so`` -- the REFERENCE's own src/ files compiled where
  they lie by oracle/Makefile (``make ref``); used to pin oracle.c and to
  generate tests/golden/.  Absent on machines without /root/reference unless
  the prebuilt files travelled with the snapshot.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_I32P = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_I64P = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_F64P = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")

_lib = None


def build() -> None:
    """Compile liboracle.so (and _ref/ when the reference tree is present)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])
    subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def lib():
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.join(HERE, "liboracle.so")
    if not os.path.exists(path):
        build()
    L = C.CDLL(path)
    i64, i32, f64 = C.c_int64, C.c_int, C.c_double
    L.orc_load_mtx.argtypes = [C.c_char_p, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32),
                               C.POINTER(C.POINTER(i32)), C.POINTER(C.POINTER(i32)),
                               C.POINTER(C.POINTER(f64))]
    L.orc_load_mtx.restype = i32
    L.orc_free.argtypes = [C.c_void_p]
    L.orc_srand.argtypes = [C.c_uint]
    L.orc_rand_fill.argtypes = [i32, _F64P]
    L.orc_verify.argtypes = [i32, i64, _I32P, _I32P, _F64P, _F64P, _F64P, C.c_void_p]
    L.orc_verify.restype = i64
    L.orc_verify_csr.argtypes = [i64, _I64P, _I32P, _F64P, _F64P, _F64P]
    L.orc_verify_csr.restype = i64
    L.orc_coo_to_csr.argtypes = [i32, i64, _I32P, _I32P, _F64P, _I64P, _I32P, _F64P]
    L.orc_csr_spmv.argtypes = [i64, _I64P, _I32P, _F64P, _F64P, _F64P, i32]
    L.orc_csr_time.argtypes = [i64, _I64P, _I32P, _F64P, _F64P, _F64P, i32, f64, i32,
                               C.POINTER(i32)]
    L.orc_csr_time.restype = f64
    L.orc_max_threads.restype = i32
    L.orc_ell_width.argtypes = [i32, i64, _I32P]
    L.orc_ell_width.restype = i32
    L.orc_ell_build.argtypes = [i32, i64, _I32P, _I32P, _F64P, i32, _I32P, _F64P]
    L.orc_ell_spmv.argtypes = [i32, i32, _I32P, _F64P, _F64P, _F64P]
    L.orc_dia_count.argtypes = [i32, i32, i64, _I32P, _I32P, C.c_void_p]
    L.orc_dia_count.restype = i32
    L.orc_dia_build.argtypes = [i32, i32, i64, _I32P, _I32P, _F64P, i32, _I32P, _F64P]
    L.orc_dia_spmv.argtypes = [i32, i32, i32, _I32P, _F64P, _F64P, _F64P]
    L.orc_ss_simple_spmv.argtypes = [i32, i64, _I64P, _I32P, _F64P, i32, _F64P, _F64P]
    L.orc_ss_optimized_spmv.argtypes = [i32, i64, _I64P, _I32P, _F64P, i32, _F64P, _F64P]
    _lib = L
    return L


# ---------------------------------------------------------------- IO / vectors
def load_mtx(path: str):
    """LoadSparseMatrix (src/util.cpp:30-66) -> (m, n, row, col, val) COO."""
    L = lib()
    m, n, nnz = C.c_int(), C.c_int(), C.c_int()
    r, c, v = C.POINTER(C.c_int)(), C.POINTER(C.c_int)(), C.POINTER(C.c_double)()
    st = L.orc_load_mtx(path.encode(), C.byref(m), C.byref(n), C.byref(nnz),
                        C.byref(r), C.byref(c), C.byref(v))
    if st != 0:
        raise IOError(f"orc_load_mtx({path}) failed: {st}")
    k = nnz.value
    row = np.ctypeslib.as_array(r, shape=(max(k, 1),))[:k].copy()
    col = np.ctypeslib.as_array(c, shape=(max(k, 1),))[:k].copy()
    val = np.ctypeslib.as_array(v, shape=(max(k, 1),))[:k].copy()
    for p in (r, c, v):
        L.orc_free(C.cast(p, C.c_void_p))
    return m.value, n.value, row, col, val


def rand_vectors(n: int, m: int, seed: int = 3):
    """srand(seed); x = CreateRandomVector(n); y = CreateRandomVector(m)
    (src/main.cpp:18,31-32)."""
    L = lib()
    L.orc_srand(seed)
    x = np.empty(max(n, 1), np.float64)
    y = np.empty(max(m, 1), np.float64)
    L.orc_rand_fill(n, x)
    L.orc_rand_fill(m, y)
    return x[:n], y[:m]


def verify(m, row, col, val, x, y) -> int:
    """VerifyResult (src/util.cpp:67-83): -1 = pass, else first failing row."""
    return int(lib().orc_verify(m, len(val), row, col, val, x, np.ascontiguousarray(y), None))


def coo_reference_product(m, row, col, val, x) -> np.ndarray:
    """The serial COO product VerifyResult compares against."""
    res = np.empty(max(m, 1), np.float64)
    lib().orc_verify(m, len(val), row, col, val, x, np.zeros(max(m, 1)), res.ctypes.data)
    return res[:m]


def verify_csr(row_ptr, col, val, x, y) -> int:
    return int(lib().orc_verify_csr(len(row_ptr) - 1, row_ptr, col, val, x, y))


# ---------------------------------------------------------------- formats
def coo_to_csr(m, row, col, val):
    """opt_crs OptimizeProblem (src/opt_crs.cpp:10-42)."""
    nnz = len(val)
    ptr = np.empty(m + 1, np.int64)
    idx = np.empty(max(nnz, 1), np.int32)
    cv = np.empty(max(nnz, 1), np.float64)
    lib().orc_coo_to_csr(m, nnz, row, col, val, ptr, idx, cv)
    return ptr, idx[:nnz], cv[:nnz]


def csr_spmv(row_ptr, col, val, x, nthreads: int = 0) -> np.ndarray:
    """opt_crs SpMV (src/opt_crs.cpp:44-70)."""
    m = len(row_ptr) - 1
    y = np.empty(max(m, 1), np.float64)
    lib().orc_csr_spmv(m, row_ptr, col, val, x, y, nthreads)
    return y[:m]


def csr_time(row_ptr, col, val, x, nthreads=0, min_seconds=1.0, ntry=10):
    """src/main.cpp:58-102 timing of the restated opt_crs SpMV."""
    m = len(row_ptr) - 1
    y = np.empty(max(m, 1), np.float64)
    loop = C.c_int()
    t = lib().orc_csr_time(m, row_ptr, col, val, x, y, nthreads, min_seconds, ntry,
                           C.byref(loop))
    return t, loop.value, y[:m]


def max_threads() -> int:
    return int(lib().orc_max_threads())


def ell_spmv(m, row, col, val, x):
    """opt_ell OptimizeProblem + SpMV (src/opt_ell.cpp:26-90); returns (K, y)."""
    L = lib()
    K = L.orc_ell_width(m, len(val), row)
    ec = np.empty(max(m * K, 1), np.int32)
    ev = np.empty(max(m * K, 1), np.float64)
    L.orc_ell_build(m, len(val), row, col, val, K, ec, ev)
    y = np.empty(max(m, 1), np.float64)
    L.orc_ell_spmv(m, K, ec, ev, x, y)
    return K, y[:m]


def dia_spmv(m, n, row, col, val, x):
    """opt_dia OptimizeProblem + SpMV (src/opt_dia.cpp:21-97); returns
    (ioff, y) with ioff the occupied diagonals d = col - row + (m - 1)."""
    L = lib()
    nd = L.orc_dia_count(m, n, len(val), row, col, None)
    ioff = np.empty(max(nd, 1), np.int32)
    L.orc_dia_count(m, n, len(val), row, col, ioff.ctypes.data)
    diag = np.empty(max(nd * n, 1), np.float64)
    L.orc_dia_build(m, n, len(val), row, col, val, nd, ioff, diag)
    y = np.empty(max(m, 1), np.float64)
    L.orc_dia_spmv(m, n, nd, ioff, diag, x, y)
    return ioff[:nd], y[:m]


def ss_spmv(row_ptr, col, val, x, W: int, optimized: bool = True):
    """opt_ss SpMV, SIMPLE (src/opt_ss.cpp:188-221) or OPTIMIZED (:222-303)."""
    m = len(row_ptr) - 1
    y = np.empty(max(m, 1), np.float64)
    f = lib().orc_ss_optimized_spmv if optimized else lib().orc_ss_simple_spmv
    f(m, len(val), row_ptr, col, val, W, x, y)
    return y[:m]


# ---------------------------------------------------------------- reference
REF_FORMATS = ("crs", "ell", "dia", "ss_simple", "ss_opt")
_ref_libs = {}


def ref_available(fmt: str = "crs") -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", f"libref_{fmt}.so"))


def ref_lib(fmt: str):
    if fmt in _ref_libs:
        return _ref_libs[fmt]
    path = os.path.join(HERE, "_ref", f"libref_{fmt}.so")
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    L = C.CDLL(path, mode=C.RTLD_LOCAL)
    L.ref_load.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                           C.POINTER(C.c_int)]
    L.ref_load.restype = C.c_void_p
    L.ref_copy_coo.argtypes = [C.c_void_p, _I32P, _I32P, _F64P]
    L.ref_free_coo.argtypes = [C.c_void_p]
    L.ref_srand.argtypes = [C.c_uint]
    L.ref_random_vector.argtypes = [C.c_int, _F64P]
    L.ref_run.argtypes = [C.c_int, C.c_int, C.c_int, _I32P, _I32P, _F64P, _F64P, _F64P,
                          C.c_int]
    L.ref_run.restype = C.c_int
    L.ref_time.argtypes = [C.c_int, C.c_int, C.c_int, _I32P, _I32P, _F64P, _F64P, _F64P,
                           C.c_double, C.c_int, C.POINTER(C.c_int)]
    L.ref_time.restype = C.c_double
    L.ref_set_threads.argtypes = [C.c_int]
    _ref_libs[fmt] = L
    return L


def ref_load_mtx(path: str, fmt: str = "crs"):
    L = ref_lib(fmt)
    m, n, nnz = C.c_int(), C.c_int(), C.c_int()
    h = L.ref_load(path.encode(), C.byref(m), C.byref(n), C.byref(nnz))
    k = nnz.value
    row = np.empty(max(k, 1), np.int32)
    col = np.empty(max(k, 1), np.int32)
    val = np.empty(max(k, 1), np.float64)
    L.ref_copy_coo(h, row, col, val)
    L.ref_free_coo(h)
    return m.value, n.value, row[:k], col[:k], val[:k]


def ref_rand_vectors(n: int, m: int, seed: int = 3, fmt: str = "crs"):
    L = ref_lib(fmt)
    L.ref_srand(seed)
    x = np.empty(max(n, 1), np.float64)
    y = np.empty(max(m, 1), np.float64)
    L.ref_random_vector(n, x)
    L.ref_random_vector(m, y)
    return x[:n], y[:m]


def ref_spmv(fmt: str, m, n, row, col, val, x, y_init=None, calls: int = 2
             ) -> Tuple[np.ndarray, bool]:
    """Run the reference plugin `fmt`: OptimizeProblem once, SpMV `calls`
    times over a garbage-initialised y; returns (y, VerifyResult passed)."""
    L = ref_lib(fmt)
    y = (np.full(max(m, 1), 12345.678) if y_init is None
         else np.ascontiguousarray(y_init, np.float64).copy())
    ok = L.ref_run(m, n, len(val), np.ascontiguousarray(row, np.int32),
                   np.ascontiguousarray(col, np.int32),
                   np.ascontiguousarray(val, np.float64),
                   np.ascontiguousarray(x, np.float64), y, calls)
    return y[:m], bool(ok)


def ref_time(fmt: str, m, n, row, col, val, x, min_seconds: float = 1.0, ntry: int = 10,
             nthreads: int = 0):
    """The reference driver's timing (src/main.cpp:58-102) of the REFERENCE's
    own plugin `fmt` (compiled from its sources): (seconds per call, loop, y).
    nthreads > 0 sets the OpenMP thread count for the call (0 = default)."""
    L = ref_lib(fmt)
    L.ref_set_threads(int(nthreads))
    y = np.empty(max(m, 1))
    loop = C.c_int()
    t = L.ref_time(m, n, len(val), np.ascontiguousarray(row, np.int32), np.ascontiguousarray(col, np.int32),
                   np.ascontiguousarray(val, np.float64), np.ascontiguousarray(x, np.float64), y,
                   float(min_seconds), int(ntry), C.byref(loop))
    L.ref_set_threads(0)
    return t, loop.value, y[:m]


def load_mtx_csr5(path: str):
    """Pure-Python restatement of the CSR5 benchmark's loader
    (opt/Benchmark_SpMV_using_CSR5/CSR5_cuda/main.cu:157-306) for small files:
    banner field/symmetry (:169-193), fscanf triplets (:208-239), counters +
    mirrored counts (:241-247), exclusive scan (:249-258), file-order scatter
    with the mirrored copy right after its original (:266-300).
    Returns (m, n, row_ptr, col, val) or raises ValueError."""
    with open(path) as f:
        banner = f.readline().split()
        if len(banner) < 5 or banner[0].lower() != "%%matrixmarket":
            raise ValueError("banner")
        field, sym = banner[3].lower(), banner[4].lower()
        if field == "complex":
            raise ValueError("complex")
        lines = f.read().split("\n")
    i = 0
    while lines[i].startswith("%") or not lines[i].strip():
        i += 1
    m, n, nnz_rep = (int(t) for t in lines[i].split()[:3])
    toks = " ".join(lines[i + 1:]).split()
    per = 2 if field == "pattern" else 3
    rows, cols, vals = [], [], []
    for e in range(nnz_rep):
        r, c = int(toks[per * e]) - 1, int(toks[per * e + 1]) - 1
        if field == "pattern":
            v = 1.0
        elif field == "integer":
            v = float(int(toks[per * e + 2]))
        else:
            v = float(toks[per * e + 2])
        rows.append(r)
        cols.append(c)
        vals.append(v)
    symmetric = sym in ("symmetric", "hermitian")
    counter = [0] * (m + 1)
    for r in rows:
        counter[r] += 1
    if symmetric:
        for r, c in zip(rows, cols):
            if r != c:
                counter[c] += 1
    ptr = [0] * (m + 1)
    for r in range(1, m + 1):
        ptr[r] = ptr[r - 1] + counter[r - 1]
    nnz = ptr[m]
    col = [0] * nnz
    val = [0.0] * nnz
    fill = [0] * m
    for r, c, v in zip(rows, cols, vals):
        off = ptr[r] + fill[r]
        col[off], val[off] = c, v
        fill[r] += 1
        if symmetric and r != c:
            off = ptr[c] + fill[c]
            col[off], val[off] = r, v
            fill[c] += 1
    return m, n, np.array(ptr, np.int64), np.array(col, np.int32), np.array(val, np.float64)

"""singlespmv_amd -- MI355X-native fp64 SpMV engine (Python host mirror).

Thin ctypes layer over ``libspmv_hip.so`` (include/spmv_hip.h).  It mirrors
the reference driver's vocabulary (hir0shim/singleSpMV src/util.h:40-45,
src/opt_crs.h:15-18):

    A = load_sparse_matrix(path)            # LoadSparseMatrix
    x = create_random_vector(n)             # srand(3) + CreateRandomVector
    A_opt = optimize_problem(A, fmt="auto") # OptimizeProblem -> device plan
    spmv(A_opt, x, y)                       # SpMV (y overwritten, beta = 0)
    verify_result(A, x, y)                  # VerifyResult

plus the plan object for device-resident x/y (torch tensors or raw device
pointers), the seeded synthetic generators of the BASELINE configs, and the
nnz-balanced row partition used by the multi-GPU bench.

PyTorch is plumbing only (device memory, streams, torch.distributed).  There
is no CPU fallback: if the HIP library is missing every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

try:  # load torch's HIP runtime first so the engine shares it (one runtime)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# SPMV_HIP_LIBRARY selects another build of the same C-ABI (the tools/
# experiments load probes_build/libspmv_hip.so, `make probes`)
LIB_PATH = os.environ.get("SPMV_HIP_LIBRARY") or os.path.join(HERE, "libspmv_hip.so")
OPT_LIB_PATH = os.path.join(HERE, "libopt_hip.so")

FORMATS = {"auto": 0, "csr": 1, "crs": 1, "ell": 2, "ss": 3, "dia": 4, "hyb": 5, "css": 6, "coo": 7, "jds": 8, "bin": 9}
FORMAT_NAMES = {0: "auto", 1: "csr", 2: "ell", 3: "ss", 4: "dia", 5: "hyb", 6: "css", 7: "coo", 8: "jds", 9: "bin"}
X_DEVICE, Y_DEVICE, ASYNC, X_STAGED, Y_STAGED = 0x1, 0x2, 0x4, 0x8, 0x10
GEN_UNIFORM, GEN_POWERLAW, GEN_BANDED = 1, 2, 3
API_VERSION = 3  # SPMV_HIP_API_VERSION of the structs mirrored here

_I32P = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_I64P = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_F64P = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


class SpmvError(RuntimeError):
    pass


class Options(C.Structure):
    _fields_ = [("format", C.c_int32), ("device", C.c_int32), ("csr_lanes", C.c_int32),
                ("ell_width", C.c_int32), ("ss_sigma", C.c_int32), ("dia_max_diags", C.c_int32),
                ("dia_max_fill", C.c_double), ("css_slab_shift", C.c_int32), ("css_lag", C.c_int32),
                ("css_pace", C.c_int32), ("bin_strip_cols", C.c_int32), ("bin_groups", C.c_int32),
                ("bin_sum_waves", C.c_int32), ("bin_pad", C.c_int32), ("csr_row_ptr64", C.c_int32),
                ("placement", C.c_int32), ("bin_long_len", C.c_int32), ("bin_product_order", C.c_int32),
                ("crs_exact", C.c_int32), ("build", C.c_int32)]


PLACEMENTS = {"auto": 0, "plain": 1, "search": 2, "vmm": 3}
BUILDS = {"auto": 0, "host": 1, "device": 2}


class PlanInfo(C.Structure):
    _fields_ = [("format", C.c_int32), ("device", C.c_int32), ("m", C.c_int64), ("n", C.c_int64),
                ("nnz", C.c_int64), ("stored_slots", C.c_int64), ("device_bytes", C.c_int64),
                ("algo_bytes", C.c_int64), ("row_ptr_bytes", C.c_int32), ("csr_lanes", C.c_int32),
                ("ell_width", C.c_int32), ("ss_sigma", C.c_int32), ("n_diags", C.c_int32),
                ("css_passes", C.c_int32), ("css_slabs", C.c_int32), ("n_kernels", C.c_int32), ("overflow_nnz", C.c_int64), ("empty_rows", C.c_int64),
                ("css_split_rows", C.c_int64), ("kernel", C.c_char * 64),
                ("bin_bins", C.c_int64), ("bin_strips", C.c_int64), ("bin_strip_cols", C.c_int32),
                ("bin_pad", C.c_int32), ("bin_sum_waves", C.c_int32), ("bin_groups", C.c_int32),
                ("placement", C.c_int32), ("placement_candidates", C.c_int32),
                ("placement_best_ms", C.c_float), ("placement_worst_ms", C.c_float),
                ("bin_long_len", C.c_int32), ("bin_product_order", C.c_int32), ("bin_long_rows", C.c_int64),
                ("bin_long_pieces", C.c_int64), ("bin_products", C.c_int64),
                ("bin_long_entries", C.c_int64), ("bin_sum_entries", C.c_int64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["kernel"] = self.kernel.decode()
        d["format"] = FORMAT_NAMES.get(self.format, str(self.format))
        d["placement"] = {v: k for k, v in PLACEMENTS.items()}.get(self.placement, str(self.placement))
        return d


class GenSpec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("per_row", C.c_int32), ("m", C.c_int64), ("n", C.c_int64),
                ("max_len", C.c_int32), ("alpha", C.c_double), ("band_lo", C.c_int32),
                ("band_hi", C.c_int32), ("integer_values", C.c_int32), ("seed", C.c_uint64)]


# Exported symbols of include/spmv_hip.h (checked by tests/test_abi.py).
EXPORTS = [
    "spmv_options_default", "spmv_plan_create_coo", "spmv_plan_create_csr",
    "spmv_plan_create_csr32", "spmv_plan_create_csr_device", "spmv_plan_create_csr32_device",
    "spmv_plan_destroy", "spmv_execute", "spmv_execute_alpha", "spmv_set_stream", "spmv_time",
    "spmv_profile", "spmv_phase_name", "spmv_stream_probe", "spmv_gather_probe", "spmv_plan_info",
    "spmv_api_version", "spmv_status_string", "spmv_last_error", "spmv_load_mtx", "spmv_load_mtx_csr", "spmv_free_host",
    "spmv_srand", "spmv_rand_vector", "spmv_verify_coo", "spmv_coo_to_csr", "spmv_gen_count",
    "spmv_gen_fill", "spmv_gen_vector", "spmv_partition_rows", "spmv_save_csr_bin",
    "spmv_load_csr_bin", "spmv_lds_order_probe", "spmv_dist_layout", "spmv_dist_create_csr",
    "spmv_dist_execute", "spmv_dist_time", "spmv_dist_info", "spmv_dist_destroy", "spmv_stream_write_probe",
    "spmv_mixed_probe", "spmv_graph_create", "spmv_graph_launch", "spmv_graph_time", "spmv_graph_destroy",
    "spmv_plan_digest", "spmv_plan_digest_name", "spmv_dist_shard", "spmv_dist_assemble",
    "spmv_fetch_y", "spmv_dist_fetch_y", "spmv_plan_built_on_device",
]

_lib = None


def lib():
    """The loaded libspmv_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SpmvError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build()) first; "
                        "there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    # the ctypes structs below mirror version API_VERSION of include/spmv_hip.h
    ver_fn = getattr(L, "spmv_api_version", None)
    if ver_fn is None:
        raise SpmvError(f"{LIB_PATH} exports no spmv_api_version (built before C-ABI version {API_VERSION}): "
                        "rebuild it with `make`")
    ver_fn.argtypes = []
    ver_fn.restype = C.c_int32
    if ver_fn() != API_VERSION:
        raise SpmvError(f"{LIB_PATH} implements C-ABI version {ver_fn()}, this mirror {API_VERSION}")
    vp, i32, i64, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    L.spmv_options_default.argtypes = [C.POINTER(Options)]
    L.spmv_plan_create_coo.argtypes = [i32, i32, i32, vp, vp, vp, C.POINTER(Options), C.POINTER(vp)]
    L.spmv_plan_create_csr.argtypes = [i64, i64, i64, vp, vp, vp, C.POINTER(Options), C.POINTER(vp)]
    L.spmv_plan_create_csr32.argtypes = [i32, i32, i32, vp, vp, vp, C.POINTER(Options), C.POINTER(vp)]
    L.spmv_plan_create_csr_device.argtypes = [i64, i64, i64, vp, vp, vp, C.POINTER(Options),
                                              C.POINTER(vp)]
    L.spmv_plan_destroy.argtypes = [vp]
    L.spmv_execute.argtypes = [vp, vp, vp, C.c_uint32]
    L.spmv_execute_alpha.argtypes = [vp, f64, vp, vp, C.c_uint32]
    L.spmv_fetch_y.argtypes = [vp, vp]
    L.spmv_dist_fetch_y.argtypes = [vp, vp]
    L.spmv_plan_create_csr32_device.argtypes = [i32, i32, i32, vp, vp, vp, C.POINTER(Options), C.POINTER(vp)]
    L.spmv_set_stream.argtypes = [vp, vp]
    L.spmv_time.argtypes = [vp, vp, vp, i32, C.POINTER(f64)]
    L.spmv_graph_create.argtypes = [vp, vp, vp, i32, C.POINTER(vp)]
    L.spmv_graph_launch.argtypes = [vp, C.c_uint32]
    L.spmv_graph_time.argtypes = [vp, i32, C.POINTER(f64)]
    L.spmv_graph_destroy.argtypes = [vp]
    L.spmv_profile.argtypes = [vp, vp, vp, i32, C.POINTER(f64), i32, C.POINTER(i32)]
    L.spmv_stream_probe.argtypes = [i32, i64, i32, C.POINTER(f64)]
    L.spmv_stream_write_probe.argtypes = [i32, i64, i32, C.POINTER(f64)]
    L.spmv_mixed_probe.argtypes = [i32, i64, i32, i32, C.POINTER(f64)]
    L.spmv_gather_probe.argtypes = [i32, i64, i64, C.POINTER(f64)]
    L.spmv_lds_order_probe.argtypes = [i32, i32, _I32P, _F64P, _F64P]
    L.spmv_dist_layout.argtypes = [_I64P, i64, i32, _I64P, C.POINTER(i64)]
    L.spmv_dist_shard.argtypes = [_I64P, _I64P, i32, i32, _I64P, C.POINTER(i64)]
    L.spmv_dist_assemble.argtypes = [_F64P, _I64P, i32, i64, _F64P]
    L.spmv_dist_create_csr.argtypes = [i32, vp, i64, i64, i64, vp, vp, vp, C.POINTER(Options), C.POINTER(vp)]
    L.spmv_dist_execute.argtypes = [vp, vp, vp, C.c_uint32]
    L.spmv_dist_time.argtypes = [vp, i32, C.POINTER(f64), C.POINTER(f64)]
    L.spmv_dist_info.argtypes = [vp, C.POINTER(i32), vp, vp]
    L.spmv_dist_destroy.argtypes = [vp]
    L.spmv_phase_name.argtypes = [vp, i32]
    L.spmv_phase_name.restype = C.c_char_p
    L.spmv_plan_info.argtypes = [vp, C.POINTER(PlanInfo)]
    L.spmv_plan_digest.argtypes = [vp, C.POINTER(C.c_uint64), i32, C.POINTER(i32)]
    L.spmv_plan_built_on_device.argtypes = [vp, C.POINTER(i32)]
    L.spmv_plan_digest_name.argtypes = [vp, i32]
    L.spmv_plan_digest_name.restype = C.c_char_p
    L.spmv_status_string.argtypes = [C.c_int]
    L.spmv_status_string.restype = C.c_char_p
    L.spmv_last_error.restype = C.c_char_p
    L.spmv_load_mtx.argtypes = [C.c_char_p, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32),
                                C.POINTER(C.POINTER(i32)), C.POINTER(C.POINTER(i32)),
                                C.POINTER(C.POINTER(f64))]
    L.spmv_load_mtx_csr.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(i64), C.POINTER(i64),
                                    C.POINTER(i64), C.POINTER(C.POINTER(i64)),
                                    C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.POINTER(f64)),
                                    C.POINTER(C.c_uint32)]
    L.spmv_free_host.argtypes = [vp]
    L.spmv_srand.argtypes = [C.c_uint32]
    L.spmv_rand_vector.argtypes = [i32, _F64P]
    L.spmv_verify_coo.argtypes = [i32, i32, _I32P, _I32P, _F64P, _F64P, _F64P]
    L.spmv_verify_coo.restype = i64
    L.spmv_coo_to_csr.argtypes = [i32, i64, _I32P, _I64P]
    L.spmv_gen_count.argtypes = [C.POINTER(GenSpec), i64, i64, C.POINTER(i64)]
    L.spmv_gen_fill.argtypes = [C.POINTER(GenSpec), i64, i64, _I64P, vp, vp]
    L.spmv_gen_vector.argtypes = [C.c_uint64, i32, i64, i64, _F64P]
    L.spmv_partition_rows.argtypes = [_I64P, i64, i32, _I64P]
    L.spmv_save_csr_bin.argtypes = [C.c_char_p, i64, i64, i64, _I64P, vp, vp]
    L.spmv_load_csr_bin.argtypes = [C.c_char_p, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64),
                                    C.POINTER(C.POINTER(i64)), C.POINTER(C.POINTER(i32)),
                                    C.POINTER(C.POINTER(f64))]
    _lib = L
    return L


def _check(st: int, what: str):
    if st != 0:
        L = lib()
        raise SpmvError(f"{what}: {L.spmv_status_string(st).decode()} "
                        f"({L.spmv_last_error().decode()})")


def _ptr(a) -> int:
    """Device or host address of a numpy array / torch tensor / int."""
    if a is None:
        return 0
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())  # torch tensor


def _is_device(a) -> bool:
    return (a is not None and not isinstance(a, (np.ndarray, int))
            and getattr(a, "is_cuda", False))


# ---------------------------------------------------------------- host types
@dataclass
class SpMat:
    """Sorted COO (reference src/util.h:7-19)."""
    nRow: int
    nCol: int
    row_idx: np.ndarray
    col_idx: np.ndarray
    val: np.ndarray

    @property
    def nNnz(self) -> int:
        return int(self.val.shape[0])

    def to_csr(self):
        return coo_to_csr(self.nRow, self.row_idx), self.col_idx, self.val


def load_sparse_matrix(path: str) -> SpMat:
    """LoadSparseMatrix (src/util.cpp:30-66)."""
    L = lib()
    m, n, nnz = C.c_int32(), C.c_int32(), C.c_int32()
    r, c, v = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_double)()
    _check(L.spmv_load_mtx(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), C.byref(r),
                           C.byref(c), C.byref(v)), f"load_sparse_matrix({path})")
    k = nnz.value
    out = SpMat(m.value, n.value,
                np.ctypeslib.as_array(r, shape=(max(k, 1),))[:k].copy(),
                np.ctypeslib.as_array(c, shape=(max(k, 1),))[:k].copy(),
                np.ctypeslib.as_array(v, shape=(max(k, 1),))[:k].copy())
    for p in (r, c, v):
        L.spmv_free_host(C.cast(p, C.c_void_p))
    return out


def load_mtx_csr(path: str, sort_columns: bool = False, expand: bool = True):
    """(m, n, row_ptr, col, val, info) with the CSR5 benchmark's loader
    semantics (CSR5_cuda/main.cu:157-306); info = {"field", "mirrored", "skew"}."""
    L = lib()
    m, n, nnz, inf = C.c_int64(), C.c_int64(), C.c_int64(), C.c_uint32()
    rp, c, v = C.POINTER(C.c_int64)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_double)()
    flags = (1 if sort_columns else 0) | (0 if expand else 2)
    _check(L.spmv_load_mtx_csr(path.encode(), flags, C.byref(m), C.byref(n), C.byref(nnz), C.byref(rp),
                               C.byref(c), C.byref(v), C.byref(inf)), f"load_mtx_csr({path})")
    k = nnz.value
    out = (m.value, n.value, np.ctypeslib.as_array(rp, shape=(m.value + 1,)).copy(),
           np.ctypeslib.as_array(c, shape=(max(k, 1),))[:k].copy(),
           np.ctypeslib.as_array(v, shape=(max(k, 1),))[:k].copy(),
           {"field": ["real", "integer", "pattern"][inf.value & 3], "mirrored": bool(inf.value & 4),
            "skew": bool(inf.value & 8)})
    for q in (rp, c, v):
        L.spmv_free_host(C.cast(q, C.c_void_p))
    return out


def save_csr_bin(path: str, m: int, n: int, row_ptr, col, val) -> None:
    """Write the SPMVCSR1 binary cache (parse a .mtx once, mmap-load later)."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float64)
    _check(lib().spmv_save_csr_bin(path.encode(), m, n, len(val), rp, col.ctypes.data, val.ctypes.data),
           f"save_csr_bin({path})")


def load_csr_bin(path: str):
    """(m, n, row_ptr, col, val) from a SPMVCSR1 file."""
    L = lib()
    m, n, nnz = C.c_int64(), C.c_int64(), C.c_int64()
    rp, c, v = C.POINTER(C.c_int64)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_double)()
    _check(L.spmv_load_csr_bin(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), C.byref(rp),
                               C.byref(c), C.byref(v)), f"load_csr_bin({path})")
    k = nnz.value
    out = (m.value, n.value, np.ctypeslib.as_array(rp, shape=(m.value + 1,)).copy(),
           np.ctypeslib.as_array(c, shape=(max(k, 1),))[:k].copy(),
           np.ctypeslib.as_array(v, shape=(max(k, 1),))[:k].copy())
    for q in (rp, c, v):
        L.spmv_free_host(C.cast(q, C.c_void_p))
    return out


def srand(seed: int) -> None:
    lib().spmv_srand(seed)


def create_random_vector(n: int) -> np.ndarray:
    """CreateRandomVector (src/util.cpp:92-102); seed first with srand()."""
    x = np.empty(max(n, 1), np.float64)
    lib().spmv_rand_vector(n, x)
    return x[:n]


def verify_result(A: SpMat, x: np.ndarray, y: np.ndarray) -> bool:
    """VerifyResult (src/util.cpp:67-83)."""
    bad = lib().spmv_verify_coo(A.nRow, A.nNnz, A.row_idx, A.col_idx, A.val,
                                np.ascontiguousarray(x, np.float64),
                                np.ascontiguousarray(y, np.float64))
    return bad < 0


def stream_probe(device: int = 0, bytes_: int = 2 << 30, iters: int = 10) -> float:
    """Measured STREAM-read GB/s of the device (the practical HBM ceiling)."""
    g = C.c_double()
    _check(lib().spmv_stream_probe(device, bytes_, iters, C.byref(g)), "spmv_stream_probe")
    return g.value


def stream_write_probe(device: int = 0, bytes_: int = 2 << 30, iters: int = 10) -> float:
    """Measured STREAM-write GB/s of the device (nontemporal 16-B stores)."""
    g = C.c_double()
    _check(lib().spmv_stream_write_probe(device, bytes_, iters, C.byref(g)), "spmv_stream_write_probe")
    return g.value


def mixed_probe(device: int = 0, bytes_: int = 1792 << 20, write_quarters: int = 3, iters: int = 10) -> float:
    """Measured GB/s of reads + writes when a stream writes back
    write_quarters/4 of what it reads (BIN's Mul: about 3/4)."""
    g = C.c_double()
    _check(lib().spmv_mixed_probe(device, bytes_, write_quarters, iters, C.byref(g)), "spmv_mixed_probe")
    return g.value


def gather_probe(device: int = 0, n: int = 64 << 20, table_bytes: int = 1 << 20) -> float:
    """Measured random 8-byte gathers/s from an L2-resident table."""
    g = C.c_double()
    _check(lib().spmv_gather_probe(device, n, table_bytes, C.byref(g)), "spmv_gather_probe")
    return g.value


def lds_order_probe(slots, vals, device: int = 0) -> np.ndarray:
    """64 LDS slots after len(slots)//64 wave-wide ds_add_f64 rounds (lane l
    of round r adds vals[r*64+l] to slots[r*64+l]): the lane-order guarantee
    BIN and CSS exactness rests on (spmv_lds_order_probe)."""
    s = np.ascontiguousarray(slots, np.int32)
    v = np.ascontiguousarray(vals, np.float64)
    if s.shape != v.shape or s.size == 0 or s.size % 64:
        raise ValueError("slots and vals: equal length, a positive multiple of 64")
    out = np.empty(64, np.float64)
    _check(lib().spmv_lds_order_probe(device, s.size // 64, s, v, out), "spmv_lds_order_probe")
    return out


def coo_to_csr(m: int, row_idx: np.ndarray) -> np.ndarray:
    rp = np.empty(m + 1, np.int64)
    _check(lib().spmv_coo_to_csr(m, len(row_idx), np.ascontiguousarray(row_idx, np.int32), rp),
           "coo_to_csr")
    return rp


# ---------------------------------------------------------------- plans
def make_options(fmt="auto", device: int = -1, csr_lanes: int = 0, ell_width: int = 0,
                 ss_sigma: int = 0, dia_max_diags: int = 0, dia_max_fill: float = 0.0,
                 css_slab_shift: int = 0, css_lag: int = 0, css_pace: int = 0,
                 bin_strip_cols: int = 0, bin_groups: int = 0, bin_sum_waves: int = 0,
                 bin_pad: int = 0, csr_row_ptr64: bool = False, placement="auto",
                 bin_long_len: int = 0, bin_product_order: int = 0, crs_exact: bool = False,
                 build="auto") -> Options:
    o = Options()
    lib().spmv_options_default(C.byref(o))
    o.format = FORMATS[fmt] if isinstance(fmt, str) else int(fmt)
    o.device, o.csr_lanes, o.ell_width, o.ss_sigma = device, csr_lanes, ell_width, ss_sigma
    o.dia_max_diags, o.dia_max_fill = dia_max_diags, dia_max_fill
    o.css_slab_shift, o.css_lag, o.css_pace = css_slab_shift, css_lag, css_pace
    o.bin_strip_cols, o.bin_groups = bin_strip_cols, bin_groups
    o.bin_sum_waves, o.bin_pad, o.csr_row_ptr64 = bin_sum_waves, bin_pad, 1 if csr_row_ptr64 else 0
    o.placement = PLACEMENTS[placement] if isinstance(placement, str) else int(placement)
    o.bin_long_len = bin_long_len
    o.bin_product_order = bin_product_order
    o.crs_exact = 1 if crs_exact else 0
    o.build = BUILDS[build] if isinstance(build, str) else int(build)
    return o


def _check_vec(a, length: int, name: str, device: int, writable: bool) -> None:
    """A vector handed to the C-ABI: float64, C-contiguous, at least `length`
    elements, and -- for a device tensor -- on the plan's device.  Raises
    ValueError instead of letting the kernels or the D2H copy run past it."""
    if isinstance(a, np.ndarray):
        if a.dtype != np.float64:
            raise ValueError(f"{name} must be float64, got {a.dtype}")
        if not a.flags.c_contiguous:
            raise ValueError(f"{name} must be C-contiguous")
        if writable and not a.flags.writeable:
            raise ValueError(f"{name} is read-only")
        if a.size < length:
            raise ValueError(f"{name} holds {a.size} values, the plan needs {length}")
        return
    if torch is not None and isinstance(a, torch.Tensor):
        if a.dtype != torch.float64:
            raise ValueError(f"{name} must be torch.float64, got {a.dtype}")
        if not a.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        if a.numel() < length:
            raise ValueError(f"{name} holds {a.numel()} values, the plan needs {length}")
        if a.is_cuda and a.device.index != device:
            raise ValueError(f"{name} is on cuda:{a.device.index}, the plan on cuda:{device}")
        if not a.is_cuda:
            raise ValueError(f"{name}: pass CPU data as a numpy array (host buffer)")
        return
    if a is None and length == 0:
        return
    raise ValueError(f"{name} must be a numpy array or a torch tensor (raw addresses: use the C-ABI)")


class Graph:
    """An instantiated HIP graph of `reps` executes of one plan (spmv_graph_*)."""

    def __init__(self, handle: int, plan, keep, reps: int):
        self._h = C.c_void_p(handle)
        self._plan, self._keep, self.reps = plan, keep, reps

    def launch(self, async_: bool = False) -> None:
        _check(lib().spmv_graph_launch(self._h, ASYNC if async_ else 0), "spmv_graph_launch")

    def time(self, launches: int) -> float:
        """Milliseconds for `launches` back-to-back graph launches (launches x
        reps executes), HIP events on the plan's stream."""
        ms = C.c_double()
        _check(lib().spmv_graph_time(self._h, launches, C.byref(ms)), "spmv_graph_time")
        return ms.value

    def destroy(self) -> None:
        if self._h is not None and self._h.value:
            lib().spmv_graph_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class Plan:
    """A device-resident matrix in one format (the SpMatOpt of a plugin)."""

    def __init__(self, handle: int, keep=None):
        self._h = C.c_void_p(handle)
        self._keep = keep
        i = self.info()
        self.m, self.n, self.device = i["m"], i["n"], i["device"]

    def _check_xy(self, x, y) -> None:
        _check_vec(x, self.n, "x", self.device, writable=False)
        _check_vec(y, self.m, "y", self.device, writable=True)

    # construction -------------------------------------------------------
    @classmethod
    def from_csr(cls, m: int, n: int, row_ptr, col, val, fmt="auto", **opts) -> "Plan":
        rp = np.ascontiguousarray(row_ptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        val = np.ascontiguousarray(val, np.float64)
        o = make_options(fmt, **opts)
        h = C.c_void_p()
        _check(lib().spmv_plan_create_csr(m, n, len(val), rp.ctypes.data, col.ctypes.data,
                                          val.ctypes.data, C.byref(o), C.byref(h)),
               "spmv_plan_create_csr")
        return cls(h.value)

    @classmethod
    def from_device_csr(cls, m: int, n: int, row_ptr, col, val, fmt="auto", **opts) -> "Plan":
        """Plan from torch CUDA tensors (int64 row_ptr, int32 col, float64
        val): every format is built on the device, AUTO resolved there
        (spmv_plan_create_csr_device).  The one exception: BIN rows out of
        strip order when the device has no room for their sorted copy are
        copied to the host and built by the host builders (same layout)."""
        for name, t, dt in (("row_ptr", row_ptr, torch.int64), ("col", col, torch.int32),
                            ("val", val, torch.float64)):
            if not _is_device(t) or t.dtype != dt or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous {dt} CUDA tensor")
        if "device" not in opts:
            opts["device"] = row_ptr.device.index or 0
        o = make_options(fmt, **opts)
        h = C.c_void_p()
        _check(lib().spmv_plan_create_csr_device(m, n, val.numel(), _ptr(row_ptr), _ptr(col), _ptr(val),
                                                 C.byref(o), C.byref(h)),
               "spmv_plan_create_csr_device")
        return cls(h.value)

    @classmethod
    def from_coo(cls, A: SpMat, fmt="auto", **opts) -> "Plan":
        o = make_options(fmt, **opts)
        h = C.c_void_p()
        r = np.ascontiguousarray(A.row_idx, np.int32)
        c = np.ascontiguousarray(A.col_idx, np.int32)
        v = np.ascontiguousarray(A.val, np.float64)
        _check(lib().spmv_plan_create_coo(A.nRow, A.nCol, A.nNnz, r.ctypes.data, c.ctypes.data,
                                          v.ctypes.data, C.byref(o), C.byref(h)),
               "spmv_plan_create_coo")
        return cls(h.value)

    # execution ------------------------------------------------------------
    def execute(self, x, y, async_: bool = False, alpha: float = 1.0) -> None:
        """y = alpha * A x (alpha = 1: y = A x).  numpy arrays are host buffers
        (H2D x / D2H y per call, as src/opt_cusparse.cpp:72,82); torch CUDA
        tensors are device buffers."""
        self._check_xy(x, y)
        flags = (X_DEVICE if _is_device(x) else 0) | (Y_DEVICE if _is_device(y) else 0)
        if async_:
            flags |= ASYNC
        if alpha == 1.0:
            _check(lib().spmv_execute(self._h, _ptr(x), _ptr(y), flags), "spmv_execute")
        else:
            _check(lib().spmv_execute_alpha(self._h, float(alpha), _ptr(x), _ptr(y), flags),
                   "spmv_execute_alpha")

    def __call__(self, x, y=None):
        if y is None:
            info = self.info()
            if _is_device(x):
                y = torch.empty(info["m"], dtype=torch.float64, device=x.device)
            else:
                y = np.empty(info["m"], np.float64)
        self.execute(x, y)
        return y

    def set_stream(self, stream) -> None:
        s = stream if isinstance(stream, int) else (0 if stream is None else stream.cuda_stream)
        _check(lib().spmv_set_stream(self._h, C.c_void_p(s)), "spmv_set_stream")

    def time(self, x_dev, y_dev, iters: int) -> float:
        """Milliseconds for `iters` back-to-back executes (HIP events on the
        plan's stream)."""
        self._check_xy(x_dev, y_dev)
        if not (_is_device(x_dev) or self.n == 0) or not (_is_device(y_dev) or self.m == 0):
            raise ValueError("time() needs device tensors for x and y")
        ms = C.c_double()
        _check(lib().spmv_time(self._h, _ptr(x_dev), _ptr(y_dev), iters, C.byref(ms)), "spmv_time")
        return ms.value

    def graph(self, x_dev, y_dev, reps: int = 1) -> "Graph":
        """The device-resident execute x_dev -> y_dev captured `reps` times
        into one HIP graph (spmv_graph_create); keep x_dev / y_dev alive."""
        self._check_xy(x_dev, y_dev)
        if not (_is_device(x_dev) or self.n == 0) or not (_is_device(y_dev) or self.m == 0):
            raise ValueError("graph() needs device tensors for x and y")
        h = C.c_void_p()
        _check(lib().spmv_graph_create(self._h, _ptr(x_dev), _ptr(y_dev), reps, C.byref(h)),
               "spmv_graph_create")
        return Graph(h.value, self, (x_dev, y_dev), reps)

    def profile(self, x_dev, y_dev, iters: int = 10) -> dict:
        """Mean ms per phase of one execute ({"tile": .., "fixup": ..} for SS),
        the counterpart of the reference's g_profile Mul/Sum split."""
        self._check_xy(x_dev, y_dev)
        if not (_is_device(x_dev) or self.n == 0) or not (_is_device(y_dev) or self.m == 0):
            raise ValueError("profile() needs device tensors for x and y")
        ms = (C.c_double * 8)()
        n = C.c_int32()
        _check(lib().spmv_profile(self._h, _ptr(x_dev), _ptr(y_dev), iters, ms, 8, C.byref(n)),
               "spmv_profile")
        L = lib()
        return {L.spmv_phase_name(self._h, k).decode() or f"phase{k}": ms[k] for k in range(n.value)}

    def info(self) -> dict:
        i = PlanInfo()
        _check(lib().spmv_plan_info(self._h, C.byref(i)), "spmv_plan_info")
        return i.as_dict()

    def built_on_device(self) -> bool:
        """True when the layout was built in HBM (spmv_plan_built_on_device)."""
        v = C.c_int32()
        _check(lib().spmv_plan_built_on_device(self._h, C.byref(v)), "spmv_plan_built_on_device")
        return bool(v.value)

    def digest(self) -> dict:
        """{array name: 64-bit layout digest} (spmv_plan_digest): equal dicts
        = byte-identical device layouts."""
        n = C.c_int32(0)
        _check(lib().spmv_plan_digest(self._h, None, 0, C.byref(n)), "spmv_plan_digest")
        buf = (C.c_uint64 * max(1, n.value))()
        _check(lib().spmv_plan_digest(self._h, buf, n.value, C.byref(n)), "spmv_plan_digest")
        return {lib().spmv_plan_digest_name(self._h, k).decode(): int(buf[k]) for k in range(n.value)}

    def destroy(self) -> None:
        if self._h is not None and self._h.value:
            lib().spmv_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def dist_shard(row_ptr, cuts, k: int):
    """(rebased row pointers, first entry) of part k of a dist plan
    (spmv_dist_shard, host only)."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    c = np.ascontiguousarray(cuts, np.int64)
    out = np.empty(int(c[k + 1] - c[k]) + 1, np.int64)
    e0 = C.c_int64(0)
    _check(lib().spmv_dist_shard(rp, c, len(c) - 1, k, out, C.byref(e0)), "spmv_dist_shard")
    return out, e0.value


def dist_assemble(gathered, cuts, slice_rows: int) -> np.ndarray:
    """y from the all-gathered padded slices (spmv_dist_assemble, host only)."""
    g = np.ascontiguousarray(gathered, np.float64)
    c = np.ascontiguousarray(cuts, np.int64)
    y = np.empty(int(c[-1]), np.float64)
    _check(lib().spmv_dist_assemble(g, c, len(c) - 1, slice_rows, y), "spmv_dist_assemble")
    return y


def dist_layout(row_ptr, parts: int):
    """(cuts, slice_rows) of a multi-GPU plan over `parts` devices
    (spmv_dist_layout: nnz-balanced cuts, slices padded to the longest)."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cuts = np.empty(parts + 1, np.int64)
    sl = C.c_int64()
    _check(lib().spmv_dist_layout(rp, len(rp) - 1, parts, cuts, C.byref(sl)), "spmv_dist_layout")
    return cuts, sl.value


class DistPlan:
    """One process over N local GPUs (spmv_dist_*): row ranges per device,
    x broadcast and y all-gather by RCCL -- the C-ABI multi-GPU path."""

    def __init__(self, m: int, n: int, row_ptr, col, val, devices, fmt="auto", **opts):
        rp = np.ascontiguousarray(row_ptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        val = np.ascontiguousarray(val, np.float64)
        devs = np.ascontiguousarray(devices, np.int32)
        o = make_options(fmt, **opts)
        h = C.c_void_p()
        _check(lib().spmv_dist_create_csr(len(devs), devs.ctypes.data, m, n, len(val), rp.ctypes.data,
                                          col.ctypes.data, val.ctypes.data, C.byref(o), C.byref(h)),
               "spmv_dist_create_csr")
        self._h, self.m, self.n, self.n_devices = h, m, n, len(devs)

    def execute(self, x, y=None, staged: bool = False) -> None:
        """y = A x on host arrays (y None: result left on the devices)."""
        if not staged:
            _check_vec(x, self.n, "x", -1, writable=False)
        if y is not None:
            _check_vec(y, self.m, "y", -1, writable=True)
        _check(lib().spmv_dist_execute(self._h, None if staged else _ptr(x), _ptr(y), X_STAGED if staged else 0),
               "spmv_dist_execute")

    def time(self, iters: int):
        """(local SpMV ms, y all-gather ms) per step, staged x."""
        a, g = C.c_double(), C.c_double()
        _check(lib().spmv_dist_time(self._h, iters, C.byref(a), C.byref(g)), "spmv_dist_time")
        return a.value, g.value

    def cuts(self) -> np.ndarray:
        nd = C.c_int32()
        cuts = np.empty(self.n_devices + 1, np.int64)
        _check(lib().spmv_dist_info(self._h, C.byref(nd), cuts.ctypes.data, None), "spmv_dist_info")
        return cuts

    def destroy(self) -> None:
        if self._h is not None and self._h.value:
            lib().spmv_dist_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def optimize_problem(A: SpMat, fmt="auto", **opts) -> Plan:
    """OptimizeProblem (e.g. src/opt_crs.cpp:10-42): build the device format."""
    return Plan.from_coo(A, fmt, **opts)


def spmv(A_opt: Plan, x, y) -> None:
    """SpMV (e.g. src/opt_crs.cpp:44-70): y = A x, y overwritten."""
    A_opt.execute(x, y)


# ---------------------------------------------------------------- generators
def gen_spec(kind: str, m: int, n: Optional[int] = None, per_row: int = 16, max_len: int = 10000,
             alpha: float = 2.0, band_lo: int = -32, band_hi: int = 31, integer_values=False,
             seed: int = 42) -> GenSpec:
    k = {"uniform": GEN_UNIFORM, "powerlaw": GEN_POWERLAW, "banded": GEN_BANDED}[kind]
    return GenSpec(k, per_row, m, m if n is None else n, max_len, alpha, band_lo, band_hi,
                   1 if integer_values else 0, seed)


def generate_csr(spec: GenSpec, row_begin: int = 0, row_end: Optional[int] = None):
    """CSR (row_ptr int64, col int32, val f64) of global rows [row_begin, row_end)."""
    L = lib()
    re = spec.m if row_end is None else row_end
    nnz = C.c_int64()
    _check(L.spmv_gen_count(C.byref(spec), row_begin, re, C.byref(nnz)), "spmv_gen_count")
    rp = np.empty(re - row_begin + 1, np.int64)
    col = np.empty(max(nnz.value, 1), np.int32)
    val = np.empty(max(nnz.value, 1), np.float64)
    _check(L.spmv_gen_fill(C.byref(spec), row_begin, re, rp, col.ctypes.data, val.ctypes.data),
           "spmv_gen_fill")
    return rp, col[:nnz.value], val[:nnz.value]


def generate_row_ptr(spec: GenSpec, row_begin: int = 0, row_end: Optional[int] = None) -> np.ndarray:
    """row_ptr (int64, from 0) of global rows [row_begin, row_end) without
    the entries: spmv_gen_fill with col_idx = val = NULL."""
    re = spec.m if row_end is None else row_end
    rp = np.empty(re - row_begin + 1, np.int64)
    _check(lib().spmv_gen_fill(C.byref(spec), row_begin, re, rp, None, None), "spmv_gen_fill")
    return rp


def generate_vector(n: int, seed: int = 43, begin: int = 0, integer_values=False) -> np.ndarray:
    out = np.empty(max(n, 1), np.float64)
    _check(lib().spmv_gen_vector(seed, 1 if integer_values else 0, begin, n, out), "spmv_gen_vector")
    return out[:n]


def partition_rows(row_ptr: np.ndarray, parts: int) -> np.ndarray:
    """nnz-balanced cut rows: cuts[k] = first row with
    row_ptr[r] >= k*nnz/parts."""
    cuts = np.empty(parts + 1, np.int64)
    rp = np.ascontiguousarray(row_ptr, np.int64)
    _check(lib().spmv_partition_rows(rp, len(rp) - 1, parts, cuts), "spmv_partition_rows")
    return cuts


def algorithmic_bytes_csr(m: int, n: int, nnz: int, rp_bytes: int = 4) -> int:
    """12*nnz + rp*(m+1) + 8*n + 8*m."""
    return 12 * nnz + rp_bytes * (m + 1) + 8 * n + 8 * m

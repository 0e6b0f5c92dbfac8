"""The C-ABI boundary: libspmv_hip.so loads, exports every symbol the public
headers declare, and fails loudly (status codes, no exit) without a GPU."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import singlespmv_amd as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(spmv_\w+)\s*\(", src, flags=re.M)))


def dynsyms(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_exports_every_declared_symbol():
    declared = header_functions(os.path.join(ROOT, "include", "spmv_hip.h"))
    assert len(declared) >= 20
    syms = dynsyms(sp.LIB_PATH)
    missing = [f for f in declared if f not in syms]
    assert not missing, f"declared but not exported: {missing}"
    assert set(sp.EXPORTS) <= set(declared)
    sp.lib()  # ctypes load with argtypes


def test_dropin_exports_reference_symbols():
    """OptimizeProblem keeps the reference's C++ mangled name and SpMV is
    extern "C" (src/opt_crs.h:15-18)."""
    for path in (sp.OPT_LIB_PATH, os.path.join(ROOT, "bin", "spmv")):
        syms = dynsyms(path) if path.endswith(".so") else set(
            l.split()[-1] for l in subprocess.check_output(["nm", path], text=True).splitlines()
            if " T " in l)
        assert "_Z15OptimizeProblemRK5SpMatRK3VecR8SpMatOptR6VecOpt" in syms
        assert "SpMV" in syms


def test_status_strings_and_errors_without_device():
    L = sp.lib()
    assert L.spmv_status_string(0) == b"success"
    assert L.spmv_status_string(2).startswith(b"not supported")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    rp = np.array([0, 1], np.int64)
    with pytest.raises(sp.SpmvError, match="no usable gfx950 device|no HIP device"):
        sp.Plan.from_csr(1, 1, rp, np.array([0], np.int32), np.array([1.0]))


def test_invalid_inputs_rejected_before_device():
    rp = np.array([0, 2, 1], np.int64)  # decreasing
    with pytest.raises(sp.SpmvError, match="row_ptr"):
        sp.Plan.from_csr(2, 2, rp, np.array([0], np.int32), np.array([1.0]))
    rp = np.array([0, 1], np.int64)
    with pytest.raises(sp.SpmvError, match="column index"):
        sp.Plan.from_csr(1, 1, rp, np.array([5], np.int32), np.array([1.0]))
    with pytest.raises(sp.SpmvError, match="row_ptr\\[m\\]"):
        sp.Plan.from_csr(1, 1, np.array([0, 3], np.int64), np.array([0], np.int32), np.array([1.0]))


def test_graph_entry_points_reject_bad_arguments():
    """spmv_graph_*: NULL plan / graph and non-positive counts come back as
    SPMV_ERROR_INVALID_VALUE (no device needed); destroy(NULL) is a no-op."""
    L = sp.lib()
    g = C.c_void_p()
    assert L.spmv_graph_create(None, None, None, 1, C.byref(g)) == 1
    assert g.value is None
    assert L.spmv_graph_launch(None, 0) == 1
    ms = C.c_double()
    assert L.spmv_graph_time(None, 1, C.byref(ms)) == 1
    assert L.spmv_graph_destroy(None) == 0


def test_options_struct_layout_matches_header(tmp_path):
    """The ctypes mirrors of spmv_options_t / spmv_plan_info_t match the C
    header field for field (sizeof and every offsetof, compiled with gcc)."""
    import subprocess
    fields = {"spmv_options_t": sp.Options, "spmv_plan_info_t": sp.PlanInfo}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "spmv_hip.h"', "int main(void) {"]
    for cname, py in fields.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    got = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        cname, f, v = line.split()
        got[(cname, f)] = int(v)
    for cname, py in fields.items():
        assert got[(cname, "sizeof")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)

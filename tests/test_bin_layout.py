"""BIN layout invariants on the host (no GPU): tests/bin_layout_check.cpp
includes the builder (singlespmv_amd/csrc/build_bin.cpp) and checks the row
bins, both segment orders and the Sum's grouped slot layout against the
kernel's load formula for 60 random CSRs x strip widths x Sum wave counts x
paddings."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bin_layout_invariants(tmp_path):
    lib = os.path.join(ROOT, "singlespmv_amd", "libspmv_hip.so")
    if not os.path.exists(lib):
        pytest.skip("libspmv_hip.so not built")
    exe = tmp_path / "bin_layout_check"
    subprocess.check_call(
        ["/opt/rocm/bin/hipcc", "-x", "c++", "-D__HIP_PLATFORM_AMD__", "-O1", "-std=c++17", "-fopenmp",
         "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "singlespmv_amd", "csrc"), "-I", "/opt/rocm/include",
         os.path.join(ROOT, "tests", "bin_layout_check.cpp"), "-o", str(exe),
         "-L", os.path.join(ROOT, "singlespmv_amd"), "-lspmv_hip",
         "-Wl,-rpath," + os.path.join(ROOT, "singlespmv_amd")])
    out = subprocess.check_output([str(exe)], text=True, timeout=300)
    assert out.startswith("ok"), out

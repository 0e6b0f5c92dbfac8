"""Beyond 2^31 entries (opt-in: SPMV_HUGE_TESTS=1, ~2 min and ~130 GB of
HBM): every format that takes a 2.16 G-entry CSR (135 M x 135 M, 16 per row)
is built on the device from the CSR in HBM, and y is checked against the
oracle's opt_crs restatement (src/opt_crs.cpp:44-70) -- bit for bit where
the format sums each row in column order, to 1e-12 elsewhere.  Results of a
run: profiles/round5/device_build/beyond_2_31.jsonl."""
import json
import os
import time

import numpy as np
import pytest

import oracle
import singlespmv_amd as sp

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("SPMV_HUGE_TESTS") != "1", reason="opt-in: SPMV_HUGE_TESTS=1")]

M = 135_000_000
EXACT = {"ss", "ell", "hyb", "jds", "css", "bin"}  # column-order sums on this matrix (uniform, 16 per row)


@pytest.fixture(scope="module")
def huge():
    import torch
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", M, per_row=16, seed=42))
    assert int(rp[-1]) >= 2 ** 31
    x = sp.generate_vector(M, seed=43)
    yo = oracle.csr_spmv(rp, col, val, x)
    d = tuple(torch.from_numpy(a).cuda() for a in (rp, col, val))
    del col, val
    return d, torch.from_numpy(x).cuda(), yo


@pytest.mark.parametrize("fmt", ["csr", "ss", "ell", "hyb", "jds", "coo", "css", "bin"])
def test_device_build_beyond_2_31(huge, fmt):
    import torch
    (drp, dcol, dval), xd, yo = huge
    t0 = time.perf_counter()
    p = sp.Plan.from_device_csr(M, M, drp, dcol, dval, fmt)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    y = torch.full((M,), float("nan"), dtype=torch.float64, device="cuda")
    p.execute(xd, y)
    yh = y.cpu().numpy()
    rel = float(np.max(np.abs(yh - yo) / np.abs(yo)))
    print(json.dumps({"format": fmt, "built_on_device": p.built_on_device(), "build_s": round(build_s, 2),
                      "bit_exact": bool(np.array_equal(yh, yo)), "max_rel": rel,
                      "device_gb": p.info()["device_bytes"] / 1e9}), flush=True)
    assert p.built_on_device()
    assert rel <= 1e-12, (fmt, rel)
    if fmt in EXACT:
        assert np.array_equal(yh, yo), fmt
    p.destroy()
    torch.cuda.empty_cache()

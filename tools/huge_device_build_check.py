#!/usr/bin/env python3
"""Beyond 2^31 entries: plans built on the device from a 2.16 G-entry CSR
already in HBM (135 M x 135 M, 16 per row), y against the oracle's opt_crs
restatement (to 1e-12; bit_exact reported).  One JSON line per format.
  python tools/huge_device_build_check.py [m] [fmt,fmt,...]   (default css,bin)
A one-off check (too heavy for the suite)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import singlespmv_amd as sp  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 135_000_000
fmts = sys.argv[2].split(",") if len(sys.argv) > 2 else ["css", "bin"]
t0 = time.time()
rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=16, seed=42))
nnz = int(rp[-1])
x = sp.generate_vector(m, seed=43)
yo = oracle.csr_spmv(rp, col, val, x)
print(json.dumps({"m": m, "nnz": nnz, "over_2_31": nnz >= 2**31, "gen_and_oracle_s": round(time.time() - t0, 1)}),
      flush=True)
drp, dcol, dval = (torch.from_numpy(a).cuda() for a in (rp, col, val))
del col, val
xd = torch.from_numpy(x).cuda()
y = torch.empty(m, dtype=torch.float64, device="cuda")
for fmt in fmts:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p = sp.Plan.from_device_csr(m, m, drp, dcol, dval, fmt)
    torch.cuda.synchronize()
    tb = time.perf_counter() - t0
    y.fill_(float("nan"))
    p.execute(xd, y)
    yh = y.cpu().numpy()
    rel = float(np.max(np.abs(yh - yo) / np.abs(yo)))
    info = p.info()
    print(json.dumps({"format": fmt, "built_on_device": p.built_on_device(), "build_s": round(tb, 2),
                      "ms": round(p.time(xd, y, 5) / 5, 3), "bit_exact": bool(np.array_equal(yh, yo)),
                      "max_rel": rel, "device_gb": info["device_bytes"] / 1e9}), flush=True)
    assert rel <= 1e-12, (fmt, rel)
    p.destroy()
    torch.cuda.empty_cache()
print(json.dumps({"done": True}), flush=True)

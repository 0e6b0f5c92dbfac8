#!/usr/bin/env python3
"""Config-2 CSS plan: host builder vs device builder (build time, digest and
y equality, ms per execute).  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import singlespmv_amd as sp  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=16, seed=42))
x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
out = {"m": m, "nnz": int(rp[-1])}
ys = {}
digests = {}
for name in ("host", "device"):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if name == "host":
        p = sp.Plan.from_csr(m, m, rp, col, val, "css", build="host")
    else:
        drp, dcol, dval = (torch.from_numpy(a).cuda() for a in (rp, col, val))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = sp.Plan.from_device_csr(m, m, drp, dcol, dval, "css")
    torch.cuda.synchronize()
    out[f"{name}_build_s"] = round(time.perf_counter() - t0, 3)
    out[f"{name}_on_device"] = p.built_on_device()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    p.execute(x, y)
    ys[name] = y.cpu().numpy()
    out[f"{name}_ms"] = round(p.time(x, y, 20) / 20, 4)
    digests[name] = p.digest()
    p.destroy()
out["digest_equal"] = digests["host"] == digests["device"]
out["y_equal"] = bool(np.array_equal(ys["host"], ys["device"]))
print(json.dumps(out), flush=True)

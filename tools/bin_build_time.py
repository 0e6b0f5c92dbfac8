"""Plan build time of BIN from a host CSR (host builder + upload) vs from a
device CSR (k_bin_build.hip), at a BASELINE config, plus a bit-equality check
of the two plans' y.  One JSON line.

    python tools/bin_build_time.py [--config c2|c3] [--repeat 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import singlespmv_amd as sp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    import torch
    if a.config == "c2":
        spec = sp.gen_spec("uniform", 10_000_000, per_row=16, seed=42)
    else:
        spec = sp.gen_spec("powerlaw", 5_000_000, max_len=10000, alpha=2.0, seed=42)
    rp, col, val = sp.generate_csr(spec)
    m = len(rp) - 1
    drp, dcol, dval = (torch.from_numpy(t).cuda() for t in (rp, col, val))
    x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
    out = {"config": a.config, "m": m, "nnz": int(len(val)), "host_s": [], "device_s": []}
    ys = {}
    for r in range(a.repeat):
        for kind in ("host", "device"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if kind == "host":
                p = sp.Plan.from_csr(m, m, rp, col, val, "bin")
            else:
                p = sp.Plan.from_device_csr(m, m, drp, dcol, dval, "bin")
            torch.cuda.synchronize()
            out[kind + "_s"].append(round(time.perf_counter() - t0, 3))
            y = torch.empty(m, dtype=torch.float64, device="cuda")
            p.execute(x, y)
            ys[kind] = y.cpu().numpy()
            info = p.info()
            out[kind + "_slots"] = info["stored_slots"]
            p.destroy()
    out["y_equal"] = bool(np.array_equal(ys["host"], ys["device"]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

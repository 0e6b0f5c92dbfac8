#!/usr/bin/env python3
"""CSS timeline: per-wave finish times of one launch (SPMV_CSS_DEBUG=32),
to separate tail imbalance from throughput.  Development tool."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SPMV_CSS_DEBUG"] = str(int(os.environ.get("SPMV_CSS_DEBUG", "0")) | 32)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--max-len", type=int, default=10000)
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    m = a.rows
    spec = sp.gen_spec(a.kind, m, m, per_row=16, max_len=a.max_len, seed=42)
    rp, col, val = sp.generate_csr(spec)
    x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    plan = sp.Plan.from_csr(m, m, rp, col, val, "css")
    info = plan.info()
    for _ in range(5):
        plan.time(x, y, 3)
    ms = plan.time(x, y, 1)
    L = sp.lib()
    L.spmv_css_timestamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    L.spmv_css_timestamps.restype = C.c_int64
    n = L.spmv_css_timestamps(plan._h, None, 0)
    buf = np.zeros(n, np.uint64)
    L.spmv_css_timestamps(plan._h, buf.ctypes.data, n)
    P, nwg = info["css_passes"], n // (info["css_passes"] * 17)
    t = buf.reshape(P, nwg, 17).astype(np.float64) * 10e-3  # 100 MHz -> us
    t0 = t[0, :, 0].min()
    t -= t0
    out = {"launch_ms": ms, "P": P, "nwg": nwg, "slabs": info["css_slabs"]}
    for p in range(P):
        start = t[p, :, 0]
        wave_end = t[p, :, 1:16]
        end = t[p, :, 16]
        busy = wave_end - start[:, None]
        out[f"pass{p}"] = {
            "start_us": [round(float(start.min()), 1), round(float(start.max()), 1)],
            "wave_end_us": [round(float(np.percentile(wave_end, q)), 1) for q in (0, 10, 50, 90, 100)],
            "wg_end_us": [round(float(np.percentile(end, q)), 1) for q in (0, 10, 50, 90, 100)],
            "wave_spread_in_wg_us_median": round(float(np.median(wave_end.max(1) - wave_end.min(1))), 1),
            "by_label_end_us": [round(float(end[l::8].mean()), 1) for l in range(8)],
            "busy_mean_us": round(float(busy.mean()), 1),
        }
    L.spmv_css_layout.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    bst = np.zeros(P * nwg + 1, np.int64)
    wof = np.zeros(P * nwg * 15 + 1, np.int64)
    L.spmv_css_layout(plan._h, bst.ctypes.data, wof.ctypes.data)
    ent = np.diff(wof).reshape(P, nwg, 15)
    nrows = np.diff(bst).reshape(P, nwg)
    lens = np.diff(rp)
    for p in range(P):
        end = t[p, :, 16] - t[p, :, 0]
        slow = np.argsort(-end)[:6]
        fast = np.argsort(end)[:3]
        rows_info = []
        for b in list(slow) + list(fast):
            r0, r1 = bst[p * nwg + b], bst[p * nwg + b + 1]
            rows_info.append({"wg": int(b), "us": round(float(end[b]), 1), "rows": int(nrows[p, b]),
                              "nnz": int(rp[r1] - rp[r0]), "maxlen": int(lens[r0:r1].max()) if r1 > r0 else 0,
                              "wave_ent": [int(ent[p, b].min()), int(ent[p, b].max())],
                              "wave_end": [round(float(v), 1) for v in np.sort(t[p, b, 1:16] - t[p, b, 0])[[0, 7, 14]]]})
        out[f"pass{p}_extremes"] = rows_info
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Parameter sweep of one format on one workload, interleaved rounds in ONE
process (cdna_hip_programming.md rule 24).  Prints one JSON line per config.

  python tools/tune.py --fmt css --grid 'css_slab_shift=15,16,17,18,19;css_lag=-1,2'
"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("TUNE_PKG_ROOT"):  # A/B against another build of the package
    sys.path.insert(0, os.environ["TUNE_PKG_ROOT"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fmt", default="css")
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--ncols", type=int, default=0, help="columns (default: rows)")
    ap.add_argument("--max-len", type=int, default=10000)
    ap.add_argument("--grid", default="")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--placement", default="", help="plan placement (e.g. search); default: the library's")
    ap.add_argument("--check", action="store_true", help="max rel err (and bit-equality) vs the oracle")
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    m = a.rows
    n = a.ncols or m
    spec = sp.gen_spec(a.kind, n, n, per_row=a.per_row, max_len=a.max_len, seed=42)
    rp, col, val = sp.generate_csr(spec, 0, m)
    x = torch.from_numpy(sp.generate_vector(n, seed=43)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    keys, vals = [], []
    for part in filter(None, a.grid.split(";")):
        k, v = part.split("=")
        keys.append(k)
        vals.append([int(t) for t in v.split(",")])
    plans = []
    for combo in itertools.product(*vals) if vals else [()]:
        kw = dict(zip(keys, combo))
        if a.placement:
            kw["placement"] = a.placement
        t0 = time.time()
        p = sp.Plan.from_csr(m, n, rp, col, val, a.fmt, **kw)
        plans.append((kw, p, time.time() - t0))
    nnz = int(rp[-1])
    res = {i: [] for i in range(len(plans))}
    for _ in range(a.rounds):
        for i, (kw, p, _) in enumerate(plans):
            p.time(x, y, 3)
            res[i].append(p.time(x, y, a.iters) / a.iters)
    yref = None
    if a.check:
        import numpy as np
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import oracle
        yref = oracle.csr_spmv(rp, col, val, x.cpu().numpy())
    for i, (kw, p, tb) in enumerate(plans):
        ms = min(res[i])
        if yref is not None:
            y.fill_(float("nan"))
            p.execute(x, y)
            yg = y.cpu().numpy()
            kw = dict(kw, max_rel=float(np.max(np.abs(yg - yref) / np.maximum(np.abs(yref), 1e-300))),
                      bit_exact=bool(np.array_equal(yg, yref)))
        print(json.dumps({"fmt": a.fmt, **kw, "ms": round(ms, 4), "median_ms": round(sorted(res[i])[len(res[i]) // 2], 4),
                          "gflops": round(2 * nnz / ms / 1e6, 1), "build_s": round(tb, 2),
                          "info": {k: v for k, v in p.info().items() if k in ("css_passes", "css_slabs", "kernel")}}),
              flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Late-plan placement (include/spmv_hip.h, SPMV_PLACEMENT_*): N successive
same-size plans of one matrix in ONE process, per placement mode, each timed
over interleaved rounds -- the spread a long-lived caller sees from plan to
plan, and whether the placement search removes the slow draws.

Plans are built from the CSR in HBM (spmv_plan_create_csr_device: the DIA /
BIN fills run on the device, so eight config-4 plans cost seconds, not
minutes).  --keep holds every plan of a mode (a process with several plans
alive); without it each plan is destroyed before the next (a caller that
rebuilds).  SEARCH exists only in the probe build:

  SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so python tools/placement_series.py \
      --config c4 --fmt dia --modes auto,search --plans 8 --keep

One JSON line per (mode, plan, round) and a summary line per mode.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"c2": dict(kind="uniform", per_row=16, rows=10_000_000),
          "c4": dict(kind="banded", band_lo=-32, band_hi=31, rows=20_000_000)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4", choices=sorted(SHAPES))
    ap.add_argument("--fmt", default="auto")
    ap.add_argument("--modes", default="auto,search")
    ap.add_argument("--plans", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--keep", action="store_true", help="keep every plan of a mode alive")
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    sh = dict(SHAPES[a.config])
    m = sh.pop("rows")
    spec = sp.gen_spec(sh.pop("kind"), m, m, seed=42, **sh)
    rp, col, val = sp.generate_csr(spec)
    drp, dcol, dval = (torch.from_numpy(v).cuda() for v in (rp, col, val))
    del col, val
    x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    for mode in a.modes.split(","):
        plans, times = [], {}
        for i in range(a.plans):
            t0 = time.time()
            p = sp.Plan.from_device_csr(m, m, drp, dcol, dval, a.fmt, placement=mode)
            tb = time.time() - t0
            info = p.info()
            plans.append((i, p, info, tb))
            if not a.keep:  # time it now, then drop it before the next build
                for r in range(a.rounds):
                    p.time(x, y, 3)
                    ms = p.time(x, y, a.iters) / a.iters
                    times.setdefault(i, []).append(ms)
                    print(json.dumps({"mode": mode, "plan": i, "round": r, "ms": round(ms, 4), "build_s": round(tb, 3),
                                      "placement": info["placement"], "candidates": info["placement_candidates"],
                                      "best_ms": round(info["placement_best_ms"], 4),
                                      "worst_ms": round(info["placement_worst_ms"], 4)}), flush=True)
                p.destroy()
                plans[-1] = (i, None, info, tb)
        if a.keep:  # every plan alive: interleaved rounds over all of them
            for r in range(a.rounds):
                for i, p, info, tb in plans:
                    p.time(x, y, 3)
                    ms = p.time(x, y, a.iters) / a.iters
                    times.setdefault(i, []).append(ms)
                    print(json.dumps({"mode": mode, "plan": i, "round": r, "ms": round(ms, 4), "build_s": round(tb, 3),
                                      "placement": info["placement"], "candidates": info["placement_candidates"],
                                      "best_ms": round(info["placement_best_ms"], 4),
                                      "worst_ms": round(info["placement_worst_ms"], 4)}), flush=True)
            for i, p, info, tb in plans:
                p.destroy()
        best = [min(v) for _, v in sorted(times.items())]
        print(json.dumps({"summary": mode, "config": a.config, "fmt": plans[0][2]["format"], "keep": a.keep,
                          "plan_ms": [round(b, 4) for b in best], "first_ms": round(best[0], 4),
                          "max_over_first": round(max(best) / best[0], 4),
                          "spread": round(max(best) / min(best), 4),
                          "build_s": [round(t[3], 3) for t in plans]}), flush=True)
        del plans
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

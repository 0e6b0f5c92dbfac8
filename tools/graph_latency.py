"""Per-execute time of stream launches vs a HIP graph replay (spmv_graph_*).

For each size and format: `spmv_time` (one hipLaunchKernelGGL per kernel per
execute), a graph of 1 execute launched K times, and a graph of R executes
launched K/R times.  One JSON line per (m, format) on stdout.

  python tools/graph_latency.py [--sizes 1000,10000,...] [--formats csr,bin,ss]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import singlespmv_amd as sp  # noqa: E402


def best(fn, trials=5):
    return min(fn() for _ in range(trials))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000,10000,100000,1000000,10000000")
    ap.add_argument("--formats", default="csr,ss,bin")
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    for m in [int(s) for s in args.sizes.split(",")]:
        rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=args.per_row, seed=42))
        xd = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
        yd = torch.empty(m, dtype=torch.float64, device="cuda")
        iters = max(args.reps, min(2000, int(2e8 // max(1, len(val)))) // args.reps * args.reps)
        for fmt in args.formats.split(","):
            plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
            plan.time(xd, yd, 10)
            t_stream = best(lambda: plan.time(xd, yd, iters)) / iters
            g1 = plan.graph(xd, yd, reps=1)
            g1.time(10)
            t_g1 = best(lambda: g1.time(iters)) / iters
            gr = plan.graph(xd, yd, reps=args.reps)
            gr.time(2)
            t_gr = best(lambda: gr.time(iters // args.reps)) / iters
            info = plan.info()
            print(json.dumps({"m": m, "nnz": len(val), "format": info["format"], "kernels": info.get("n_kernels"),
                              "iters": iters, "stream_us": round(t_stream * 1e3, 3),
                              "graph1_us": round(t_g1 * 1e3, 3), f"graph{args.reps}_us": round(t_gr * 1e3, 3),
                              "gain_graph_reps": round(t_stream / t_gr, 3)}), flush=True)
            g1.destroy()
            gr.destroy()
            plan.destroy()


if __name__ == "__main__":
    main()

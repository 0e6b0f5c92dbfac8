"""AUTO crossover between CSS, BIN and CSR: ms per execute (HIP events, best
of 3 trials) for uniform and power-law matrices of growing size, with the
format AUTO picks.  One JSON line per (kind, m, format).

  python tools/auto_cross.py [--sizes 500000,1000000,...] [--formats css,bin,csr,auto]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import singlespmv_amd as sp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="500000,1000000,2000000,3000000,5000000")
    ap.add_argument("--kinds", default="uniform,powerlaw")
    ap.add_argument("--formats", default="css,bin,csr,auto")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--max-len", type=int, default=2000)
    args = ap.parse_args()
    for kind in args.kinds.split(","):
        for m in [int(s) for s in args.sizes.split(",")]:
            spec = sp.gen_spec(kind, m, per_row=args.per_row, max_len=args.max_len, seed=42)
            rp, col, val = sp.generate_csr(spec)
            xd = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
            yd = torch.empty(m, dtype=torch.float64, device="cuda")
            for fmt in args.formats.split(","):
                plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
                plan.time(xd, yd, 3)
                ms = min(plan.time(xd, yd, args.iters) for _ in range(3)) / args.iters
                print(json.dumps({"kind": kind, "m": m, "per_row": args.per_row, "max_len": args.max_len, "nnz": len(val), "format": fmt,
                                  "chosen": plan.info()["format"], "ms": round(ms, 5),
                                  "gflops": round(2 * len(val) / ms / 1e6, 1)}), flush=True)
                plan.destroy()


if __name__ == "__main__":
    main()

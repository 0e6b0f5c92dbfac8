#!/usr/bin/env python3
"""Which hardware counter separates a slow-mode BIN Mul from a fast one?

Builds K BIN plans of the same matrix in one process (library default
placement, so some land in the slow mode, profiles/round1/README.md §4a) and runs each plan's
execute `reps` times, plan after plan, so the k-th block of `reps`
bin_mul_kernel dispatches belongs to plan k.  Run it under
`rocprofv3 --kernel-trace --pmc <counters>`: within ONE pass the kernel trace
gives each dispatch's duration and the counter file its counters, so slow
and fast Mul dispatches of the same process can be compared
(tools/placement_pmc_summary.py).  Prints one JSON line per plan (its Mul /
Sum phase times measured with HIP events before the profiled executes).

  rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum ... -d out -o run -- \\
      python3 tools/placement_pmc.py --plans 8 --rows 10000000
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plans", type=int, default=8)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--ncols", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--placement", default="auto")
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    m = a.rows
    n = a.ncols or m
    spec = sp.gen_spec("uniform", n, n, per_row=16, seed=42)
    rp, col, val = sp.generate_csr(spec, 0, m)
    x = torch.from_numpy(sp.generate_vector(n, seed=43)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    plans = [sp.Plan.from_csr(m, n, rp, col, val, "bin", placement=a.placement) for _ in range(a.plans)]
    for k, p in enumerate(plans):
        ph = p.profile(x, y, 10)
        print(json.dumps({"plan": k, "placement": p.info()["placement"], **{q: round(v, 4) for q, v in ph.items()}}),
              flush=True)
    torch.cuda.synchronize()
    for p in plans:  # the profiled block: reps executes per plan, in plan order
        p.time(x, y, a.reps)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-phase times (Mul / Sum) of BIN plans on one workload, with the
streamed bytes of each phase -> effective GB/s.  One process, interleaved.

  python tools/bin_probe.py --rows 10000000 --grid 'bin_groups=1,2;bin_strip_cols=16384' [--dbg 0,1,2]
"""
import argparse
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--ncols", type=int, default=0)
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--max-len", type=int, default=10000)
    ap.add_argument("--grid", default="bin_groups=1")
    ap.add_argument("--dbg", default="0", help="SPMV_BIN_DEBUG values (comma list)")
    ap.add_argument("--env", default="", help="grid of builder env knobs, e.g. 'SPMV_BIN_PADLOG=3,4'")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--repeat", type=int, default=1, help="identical plans per variant (placement effects)")
    ap.add_argument("--prealloc-gb", type=float, default=0, help="allocate and free this much device memory first")
    ap.add_argument("--hold-gb", type=float, default=0, help="allocate this much device memory first and keep it")
    ap.add_argument("--throwaway", action="store_true", help="build and destroy one plan before the measured ones")
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    m = a.rows
    n = a.ncols or m
    spec = sp.gen_spec(a.kind, n, n, per_row=a.per_row, max_len=a.max_len, seed=42)
    rp, col, val = sp.generate_csr(spec, 0, m)
    nnz = int(rp[-1])
    x = torch.from_numpy(sp.generate_vector(n, seed=43)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    if a.prealloc_gb:
        t = torch.empty(int(a.prealloc_gb * (1 << 30)), dtype=torch.uint8, device="cuda")
        t.fill_(1)
        torch.cuda.synchronize()
        del t
        torch.cuda.empty_cache()
    if a.hold_gb:
        hold = torch.empty(int(a.hold_gb * (1 << 30)), dtype=torch.uint8, device="cuda")  # noqa: F841
        hold.fill_(1)
    if a.throwaway:
        sp.Plan.from_csr(m, n, rp, col, val, "bin").destroy()
    keys, vals = [], []
    for part in filter(None, a.grid.split(";")):
        k, v = part.split("=")
        keys.append(k)
        vals.append([int(t) for t in v.split(",")])
    ekeys, evals = [], []
    for part in filter(None, a.env.split(";")):
        k, v = part.split("=")
        ekeys.append(k)
        evals.append(v.split(","))
    plans = []
    for dbg in a.dbg.split(","):
        os.environ["SPMV_BIN_DEBUG"] = dbg
        for ecombo in itertools.product(*evals):
            env = dict(zip(ekeys, ecombo))
            os.environ.update(env)
            for combo in itertools.product(*vals):
                kw = dict(zip(keys, combo))
                for rep in range(a.repeat):
                    plans.append((dict(kw, dbg=int(dbg), rep=rep, **env),
                                  sp.Plan.from_csr(m, n, rp, col, val, "bin", **kw)))
    for rnd in range(2):
        for kw, p in plans:
            p.time(x, y, 3)
            tot = p.time(x, y, a.iters) / a.iters
            ph = p.profile(x, y, a.iters)
            info = p.info()
            E = info["stored_slots"]
            mul = sum(v for k, v in ph.items() if k.startswith("mul"))
            sm = sum(v for k, v in ph.items() if k.startswith("sum"))
            # streamed bytes: Mul 8+2+0.5 read + 8 write per entry (+ x), Sum 8+2 read (+ y)
            out = {**kw, "round": rnd, "ms": round(tot, 4), "gflops": round(2 * nnz / tot / 1e6, 1),
                   "mul_ms": round(mul, 4), "sum_ms": round(sm, 4),
                   "mul_gbs": round((18.5 * E + 8 * n) / mul / 1e6, 0) if mul else None,
                   "sum_gbs": round((10 * E + 8 * m) / sm / 1e6, 0) if sm else None,
                   "pad_frac": round(E / nnz - 1, 4), "phases": {k: round(v, 4) for k, v in ph.items()}}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

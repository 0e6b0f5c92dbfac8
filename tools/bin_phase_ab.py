#!/usr/bin/env python3
"""In-process A/B of BIN plan variants, Mul and Sum timed separately.

Each variant is a set of probe-build environment switches read at plan build
(SPMV_BIN_*; run with SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so); every
plan of the process is built from the same CSR, then the plans are profiled
in interleaved rounds (cdna_hip_programming.md rule 24).  One JSON line per
(round, variant).

  SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so python tools/bin_phase_ab.py \
      --variants 'base:;ld16:SPMV_BIN_DEBUG=1024' --rows 10000000
"""
import argparse
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True,
                    help="name:VAR=v,opt=v;name:... (UPPER-case keys: probe environment; lower-case: plan options)")
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--fmt", default="bin")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--ncols", type=int, default=0)
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--max-len", type=int, default=10000)
    ap.add_argument("--band", default="-32,31", help="banded: lowest,highest diagonal offset")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--placement", default="plain", help="default placement (a variant's placement=K overrides)")
    ap.add_argument("--check", action="store_true", help="bit-equality of each variant's y vs the first")
    ap.add_argument("--launch-variants", default="",
                    help="name:VAR=v,...;... environment set around each timing (probe build: "
                         "SPMV_LAUNCH_DEBUG, SPMV_LAUNCH_DIA_LDS_KB are read at every launch): "
                         "every plan is timed under every launch variant, so they share placements")
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    m = a.rows
    n = a.ncols or m
    blo, bhi = (int(v) for v in a.band.split(","))
    spec = sp.gen_spec(a.kind, n, n, per_row=a.per_row, max_len=a.max_len, band_lo=blo, band_hi=bhi, seed=42)
    rp, col, val = sp.generate_csr(spec, 0, m)
    x = torch.from_numpy(sp.generate_vector(n, seed=43)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    plans = []
    for part in filter(None, a.variants.split(";")):
        name, _, envs = part.partition(":")
        saved, opts, fmt = {}, {}, a.fmt
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=")
            if k == "fmt":  # this variant's format (the others: --fmt)
                fmt = v
                continue
            if k.islower():
                opts[k] = int(v)
                continue
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        kw = dict(placement=a.placement)
        kw.update(opts)
        p = sp.Plan.from_csr(m, n, rp, col, val, fmt, **kw)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        info = p.info()
        plans.append((name, p, info))
    lvars = []
    for part in filter(None, a.launch_variants.split(";")):
        lname, _, envs = part.partition(":")
        lvars.append((lname, dict(kv.split("=") for kv in filter(None, envs.split(",")))))
    yref = None
    if a.check:  # every plan under every launch variant against the first
        for (name, p, _), (lname, lenv) in itertools.product(plans, lvars or [("", {})]):
            os.environ.update(lenv)
            y.fill_(float("nan"))
            p.execute(x, y)
            torch.cuda.synchronize()
            for k in lenv:
                os.environ.pop(k, None)
            if yref is None:
                yref = y.clone()
            print(json.dumps({"variant": name, "launch": lname,
                              "bit_equal_to_first": bool(torch.equal(y, yref))}), flush=True)
    for r in range(a.rounds):
        for (name, p, info), (lname, lenv) in itertools.product(plans, lvars or [("", {})]):
            for k, v in lenv.items():
                os.environ[k] = v
            ph = p.profile(x, y, a.iters)
            tot = p.time(x, y, a.iters) / a.iters
            for k in lenv:
                os.environ.pop(k, None)
            print(json.dumps({"round": r, "variant": name, "launch": lname, "ms": round(tot, 4),
                              "long_rows": info.get("bin_long_rows"), "pieces": info.get("bin_long_pieces"),
                              "products": info.get("bin_products"), "stored": info.get("stored_slots"),
                              **{k: round(v, 4) for k, v in ph.items()},
                              "placement_ms": [round(info.get("placement_best_ms", 0), 4),
                                               round(info.get("placement_worst_ms", 0), 4)],
                              "m": m, "n": n}), flush=True)

if __name__ == "__main__":
    main()

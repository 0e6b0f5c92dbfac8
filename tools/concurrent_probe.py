#!/usr/bin/env python3
"""Feasibility probe: BIN (HBM-stream bound) and CSS (L2-gather-rate bound)
on disjoint CU sets at the same time (hipExtStreamCreateWithCUMask).  Each
plan runs the FULL config-2 matrix; the probe reports each alone on its CU
half, each on the whole chip, and both concurrently, so a row split between
them can be priced.  One JSON line per measurement.

  python tools/concurrent_probe.py [--rows 10000000] [--iters 20] [--masks alt8,half]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cu_mask(kind, part, ncu=256):
    bits = []
    for i in range(ncu):
        if kind == "half":
            on = (i < ncu // 2)
        elif kind == "even":
            on = (i % 2 == 0)
        elif kind == "alt8":
            on = ((i // 8) % 2 == 0)
        elif kind.startswith("frac"):  # fracK: K/32 of each 32-CU group on side 0
            k = int(kind[4:])
            on = (i % 32) < k
        else:
            raise ValueError(kind)
        bits.append(on if part == 0 else not on)
    words = [0] * ((ncu + 31) // 32)
    for i, b in enumerate(bits):
        if b:
            words[i // 32] |= 1 << (i % 32)
    return words


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--masks", default="alt8,half")
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    hip = C.CDLL("libamdhip64.so")
    m = a.rows
    spec = sp.gen_spec("uniform", m, m, per_row=16, seed=42)
    rp, col, val = sp.generate_csr(spec)
    nnz = int(rp[-1])
    x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
    yb = torch.empty(m, dtype=torch.float64, device="cuda")
    yc = torch.empty(m, dtype=torch.float64, device="cuda")
    drp, dcol, dval = (torch.from_numpy(t).cuda() for t in (rp, col, val))

    def mk_stream(words):
        s = C.c_void_p()
        arr = (C.c_uint32 * len(words))(*words)
        st = hip.hipExtStreamCreateWithCUMask(C.byref(s), len(words), arr)
        assert st == 0, st
        return s.value

    def wall(pairs, iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            for plan, y in pairs:
                plan.execute(x, y, async_=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / iters

    out = lambda d: print(json.dumps(d), flush=True)
    full_bin = sp.Plan.from_device_csr(m, m, drp, dcol, dval, "bin")
    full_css = sp.Plan.from_device_csr(m, m, drp, dcol, dval, "css")
    s0 = torch.cuda.Stream()
    full_bin.set_stream(s0.cuda_stream)
    full_css.set_stream(s0.cuda_stream)
    for p in (full_bin, full_css):
        wall([(p, yb)], 3)
    ref = None
    out({"what": "full", "bin_ms": wall([(full_bin, yb)], a.iters), "css_ms": wall([(full_css, yc)], a.iters),
         "nnz": nnz})
    yref = yb.clone()
    full_bin.destroy()
    full_css.destroy()
    os.environ["SPMV_BIN_CUS"] = "128"
    os.environ["SPMV_CSS_WGS"] = "128"
    pb = sp.Plan.from_device_csr(m, m, drp, dcol, dval, "bin")
    pc = sp.Plan.from_device_csr(m, m, drp, dcol, dval, "css")
    for mk in a.masks.split(","):
        sa, sb = mk_stream(cu_mask(mk, 0)), mk_stream(cu_mask(mk, 1))
        for order in ((sa, sb), (sb, sa)):
            pb.set_stream(order[0])
            pc.set_stream(order[1])
            wall([(pb, yb), (pc, yc)], 3)
            tb = wall([(pb, yb)], a.iters)
            tc = wall([(pc, yc)], a.iters)
            tboth = wall([(pb, yb), (pc, yc)], a.iters)
            ok = bool(torch.equal(yb, yref)) and bool(torch.allclose(yc, yref, rtol=1e-12, atol=0))
            out({"what": "masked", "mask": mk, "bin_side": 0 if order[0] == sa else 1, "bin_ms": round(tb, 4),
                 "css_ms": round(tc, 4), "both_ms": round(tboth, 4), "y_ok": ok})


if __name__ == "__main__":
    main()

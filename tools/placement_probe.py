"""Placement experiment: the BIN Mul's speed against how the product buffer
was allocated.  In ONE process, build the config-2 BIN plan `--plans` times
per placement mode (each plan destroyed before the next, as a caller that
rebuilds plans would), and time Mul / Sum with spmv_profile.

  SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so python tools/placement_probe.py \
      --modes plain,vmm:2,vmm:0,search --plans 6

vmm:<MB> sets SPMV_VMM_CHUNK_MB (0 = one handle for the whole buffer; probe
build only).  One JSON line per plan.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="plain,vmm:2,search")
    ap.add_argument("--plans", type=int, default=6)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--window-mb", type=int, default=64)
    ap.add_argument("--hold-gb", type=float, default=0.0,
                    help="allocate (and keep) this much device memory before the plans")
    ap.add_argument("--churn-gb", type=float, default=0.0,
                    help="allocate and free this much torch memory between plans")
    a = ap.parse_args()
    import torch
    import singlespmv_amd as sp
    L = sp.lib()
    L.spmv_bin_prod.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
    L.spmv_line_write_probe.argtypes = [C.c_int32, C.c_void_p, C.c_int64, C.c_int64, C.c_int32,
                                        C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_int32)]
    hold = None
    if a.hold_gb > 0:
        hold = torch.empty(int(a.hold_gb * 2**30) // 8, dtype=torch.float64, device="cuda")
    m = a.rows
    n = a.cols or m
    spec = sp.gen_spec("uniform", n, n, per_row=16, seed=42)
    rp, col, val = sp.generate_csr(spec, 0, m)
    x = torch.from_numpy(sp.generate_vector(n, seed=43)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    yref = None
    for mode in a.modes.split(","):
        mode, _, envs = mode.partition("@")  # mode@VAR=V[@VAR=V]: probe-build variables for this mode
        env = dict(kv.split("=", 1) for kv in envs.split("@") if kv)
        os.environ.update(env)
        name, _, chunk = mode.partition(":")
        if name == "vmm":
            os.environ["SPMV_VMM_CHUNK_MB"] = chunk or "2"
            if chunk == "0":
                os.environ["SPMV_VMM_CHUNK_MB"] = str(1 << 20)  # larger than any buffer: one handle
        for i in range(a.plans):
            free0 = torch.cuda.mem_get_info()[0]
            t0 = time.time()
            plan = sp.Plan.from_csr(m, n, rp, col, val, "bin", placement=name)
            tb = time.time() - t0
            free1 = torch.cuda.mem_get_info()[0]
            plan.time(x, y, 3)
            ph = plan.profile(x, y, a.iters)
            if yref is None:
                yref = y.clone()
            same = bool(torch.equal(y, yref))
            info = plan.info()
            # the scattered-line write probe over 64 MB windows of the product buffer
            L = sp.lib()
            buf, nb = C.c_void_p(), C.c_int64()
            win = []
            if L.spmv_bin_prod(plan._h, C.byref(buf), C.byref(nb)) == 0:
                gbs = (C.c_double * 256)()
                nw = C.c_int32()
                L.spmv_line_write_probe(0, buf, nb.value, a.window_mb << 20, 3, gbs, 256, C.byref(nw))
                win = [round(gbs[k]) for k in range(nw.value)]
                plan.time(x, y, 3)
                ph2 = plan.profile(x, y, a.iters)
            print(json.dumps({"mode": mode, "env": env, "plan": i, "hold_gb": a.hold_gb, "mul_ms": round(ph["mul"], 4), "sum_ms": round(ph["sum"], 4),
                              "mul_ms_after": round(ph2["mul"], 4) if win else None,
                              "build_s": round(tb, 2), "plan_gb": round(info["device_bytes"] / 2**30, 3),
                              "free_drop_gb": round((free0 - free1) / 2**30, 3), "y_same": same,
                              "prod_va": hex(buf.value or 0),
                              "win_gbs_min": min(win) if win else None, "win_gbs_max": max(win) if win else None,
                              "win_gbs": win}), flush=True)
            plan.destroy()
            del plan
            if a.churn_gb > 0:
                t = torch.empty(int(a.churn_gb * 2**30) // 8, dtype=torch.float64, device="cuda")
                t.fill_(1.0)
                del t
                torch.cuda.empty_cache()
        os.environ.pop("SPMV_VMM_CHUNK_MB", None)
        for k in env:
            os.environ.pop(k, None)


if __name__ == "__main__":
    main()

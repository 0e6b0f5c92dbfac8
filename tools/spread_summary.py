#!/usr/bin/env python3
"""Per-plan, per-channel summary of tools/spread_pmc.sh passes (config 2 BIN
placement spread, VERDICT r5 "next" #2).

Each pass dir holds rocprofv3's JSON (`--output-format json`): counter
records per dispatch with one value per counter instance (TCC: 16 channels x
8 XCDs).  For every plan (the k-th block of `reps` dispatches of a kernel,
tools/placement_pmc.py's profiled order) and kernel (bin_mul_kernel, the Sum)
it prints the mean duration, each counter's per-dispatch total, and how the
counter spreads over its instances (max / mean, the coefficient of
variation, the hottest instances) -- so a slow plan whose stalls sit on a
subset of channels shows it.

  python3 tools/spread_summary.py <pass dir> [...] --plans 8 --reps 5
"""
import argparse
import collections
import glob
import json
import os
import statistics


def load(d):
    f = glob.glob(os.path.join(d, "**", "*results.json"), recursive=True)
    if not f:
        return None
    return json.load(open(f[0]))["rocprofiler-sdk-tool"][0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--plans", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kernels", default="bin_mul_kernel,bin_sum")
    a = ap.parse_args()
    kernels = a.kernels.split(",")
    for d in a.dirs:
        t = load(d)
        if t is None:
            print(json.dumps({"dir": d, "error": "no results.json"}))
            continue
        names = {}
        for ks in t.get("kernel_symbols", []):
            names[ks["kernel_id"]] = ks.get("formatted_kernel_name") or ks.get("kernel_name", "")
        cname, cinst = {}, {}
        for c in t["counters"]:
            cid = c["id"]["handle"]
            cname[cid] = c["name"]
            cinst[cid] = ["/".join(f"{x['dimension_name'].replace('DIMENSION_', '')[0]}{x['index']}"
                                   for x in i["dimensions"]) for i in c.get("instances", [])]
        disp = []
        for r in t["callback_records"]["counter_collection"]:
            di = r["dispatch_data"]["dispatch_info"]
            name = names.get(di["kernel_id"], "")
            vals = collections.defaultdict(list)
            for rec in r["records"]:
                vals[rec["counter_id"]["handle"]].append(rec["value"])
            disp.append((r["dispatch_data"]["start_timestamp"], name,
                         (r["dispatch_data"]["end_timestamp"] - r["dispatch_data"]["start_timestamp"]) / 1e3, vals))
        disp.sort(key=lambda v: v[0])
        for kn in kernels:
            ks = [v for v in disp if kn in v[1]][-a.plans * a.reps:]
            for k in range(a.plans):
                blk = ks[k * a.reps:(k + 1) * a.reps]
                if not blk:
                    continue
                out = {"dir": os.path.basename(d.rstrip("/")), "kernel": kn, "plan": k,
                       "us": round(statistics.mean(b[2] for b in blk), 1)}
                for cid in blk[0][3]:
                    per_inst = [statistics.mean(b[3][cid][i] for b in blk) for i in range(len(blk[0][3][cid]))]
                    tot = sum(per_inst)
                    mean = tot / max(1, len(per_inst))
                    out[cname.get(cid, str(cid))] = {
                        "total": tot, "max_over_mean": round(max(per_inst) / mean, 3) if mean else None,
                        "cv": round(statistics.pstdev(per_inst) / mean, 3) if mean else None,
                        "hot": [cinst.get(cid, [])[i] if i < len(cinst.get(cid, [])) else i
                                for i in sorted(range(len(per_inst)), key=lambda i: -per_inst[i])[:4]]}
                print(json.dumps(out))


if __name__ == "__main__":
    main()

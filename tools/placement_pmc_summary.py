#!/usr/bin/env python3
"""Summarise tools/placement_pmc.py passes: per plan, the mean duration and
mean counters of its last `reps` bin_mul_kernel dispatches.

  python3 tools/placement_pmc_summary.py <pass dir> [<pass dir> ...] --plans 8 --reps 5

Each pass dir holds rocprofv3 `run_kernel_trace.csv` and
`run_counter_collection.csv` (one --pmc pass with --kernel-trace).  Prints
one JSON line per (pass, plan): Mul µs and each counter's per-dispatch mean.
"""
import argparse
import collections
import csv
import glob
import json
import os


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--plans", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kernel", default="bin_mul_kernel")
    a = ap.parse_args()
    need = a.plans * a.reps
    for d in a.dirs:
        tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not tr or not cc:
            print(json.dumps({"dir": d, "error": "missing csv"}))
            continue
        disp = [r for r in rows(tr[0]) if a.kernel in r["Kernel_Name"]]
        disp.sort(key=lambda r: int(r["Start_Timestamp"]))
        dur = {int(r["Dispatch_Id"]): (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in disp}
        ids = [int(r["Dispatch_Id"]) for r in disp][-need:]
        ctr = collections.defaultdict(dict)
        for r in rows(cc[0]):
            if a.kernel in r["Kernel_Name"]:
                ctr[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        for k in range(a.plans):
            blk = ids[k * a.reps:(k + 1) * a.reps]
            if not blk:
                continue
            out = {"dir": os.path.basename(d.rstrip("/")), "plan": k,
                   "mul_us": round(sum(dur[i] for i in blk) / len(blk), 1)}
            names = sorted({n for i in blk for n in ctr.get(i, {})})
            for n in names:
                vals = [ctr[i][n] for i in blk if n in ctr.get(i, {})]
                out[n] = sum(vals) / len(vals)
            print(json.dumps(out))


if __name__ == "__main__":
    main()

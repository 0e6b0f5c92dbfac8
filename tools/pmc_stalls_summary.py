#!/usr/bin/env python3
"""Summarise tools/pmc_stalls.sh passes: per kernel (name up to its first
'(' ), the mean duration and the per-dispatch mean of every counter, plus the
derived ratios that tell an issue-bound kernel from a memory-bound one.

  python3 tools/pmc_stalls_summary.py gpurun_out/stalls_<tag>  > summary.json

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles on gfx950
(MI355X_MICROARCH.md, cycle constants); WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~= WAVE_CYCLES, so their shares of WAVE_CYCLES are reported.
Only the kernels of the last `--last` dispatches per name are averaged (the
bench's timed launches, not its warm-up).
"""
import collections
import csv
import glob
import json
import os
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def short(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("void ", "").replace("spmv::", "").strip()


def main(root: str) -> None:
    kern = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(glob.glob(os.path.join(root, "pass*"))):
        if not os.path.isdir(d):
            continue
        cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if tr:
            for r in rows(tr[0]):
                k = short(r["Kernel_Name"])
                kern[k]["duration_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if cc:
            for r in rows(cc[0]):
                kern[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, ctrs in kern.items():
        if len(ctrs.get("duration_us", [])) < 3:
            continue
        m = {c: sum(v) / len(v) for c, v in ctrs.items() if v}
        m["dispatches"] = len(ctrs["duration_us"])
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in m:
                    m[c + "_share"] = m[c] / wc
        if m.get("SQ_WAVES"):
            m["wave_cycles_per_wave"] = wc / m["SQ_WAVES"] if wc else None
        if m.get("SQ_LEVEL_WAVES") and m.get("GRBM_GUI_ACTIVE"):
            m["mean_waves_resident_per_xcd_cycle"] = m["SQ_LEVEL_WAVES"] / m["GRBM_GUI_ACTIVE"]
        if m.get("GRBM_GUI_ACTIVE") and m.get("duration_us"):
            m["clock_ghz_est"] = m["GRBM_GUI_ACTIVE"] / 8 / (m["duration_us"] * 1e3)
        if m.get("TCP_TCC_READ_REQ_sum"):
            m["l2_read_latency_cycles"] = m.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / m["TCP_TCC_READ_REQ_sum"]
        if m.get("TCC_EA0_RDREQ_sum"):
            m["dram_credit_stall_per_rdreq"] = m.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", 0.0) / m["TCC_EA0_RDREQ_sum"]
        if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
            tot = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            m["l2_hit_rate"] = m["TCC_HIT_sum"] / tot if tot else None
        out[k] = m
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])

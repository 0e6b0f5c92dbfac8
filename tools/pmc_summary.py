#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/<tag>/.

Writes
  profiles/<tag>/kernel_stats.csv      (rocprofv3 --kernel-trace --stats)
  profiles/<tag>/pmc_summary.json      per-kernel mean FETCH_SIZE / WRITE_SIZE
                                       (KB, as rocprofv3 reports them) and the
                                       per-launch HBM-side bytes
  profiles/<tag>/bench_*.json          the bench lines of each pass
and merges {"<config>:<m>x<n>:<kernel>": bytes} into profiles/pmc_traffic.json
(raw FETCH+WRITE) and profiles/pmc_traffic_calibrated.json (2*FETCH+WRITE,
the gfx950 correction below), read by bench.py to fill roofline.traffic for
exactly that rank shape (bench.traffic_key).

gfx950 note (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per
TCC_EA0_RDREQ and reads exactly half of a wide (16 B/lane) coalesced stream;
other access widths are uncalibrated.  `traffic_raw` is (FETCH+WRITE)*1024;
`traffic_stream_corrected` adds back the half of the streamed matrix bytes
(the kernel's algorithmic stream, 12 B/nnz) that FETCH_SIZE does not see.
"""
import csv
import collections
import json
import os
import shutil
import sys


def main(src, tag, config_key_prefix):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for f in os.listdir(src):
        if f.startswith("bench_") and f.endswith(".json"):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    bench = json.load(open(os.path.join(src, "bench_trace.json")))
    stream_bytes = {}
    for fmt, r in bench.get("formats", {}).items():
        if "kernel" in r:
            stream_bytes[r["kernel"]] = r["algo_bytes"]
    summary = {}
    for k, d in agg.items():
        fetch = sum(d.get("FETCH_SIZE", [0])) / max(1, len(d.get("FETCH_SIZE", [1])))
        write = sum(d.get("WRITE_SIZE", [0])) / max(1, len(d.get("WRITE_SIZE", [1])))
        summary[k] = {"FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write,
                      "launches": len(d.get("FETCH_SIZE", [])),
                      "traffic_raw": (fetch + write) * 1024,
                      "traffic_calibrated": (2 * fetch + write) * 1024}
    json.dump({"source": src, "kernels": summary}, open(os.path.join(dst, "pmc_summary.json"), "w"),
              indent=1)
    for fname, field in (("pmc_traffic.json", "traffic_raw"), ("pmc_traffic_calibrated.json", "traffic_calibrated")):
        tfile = os.path.join(root, "profiles", fname)
        traffic = json.load(open(tfile)) if os.path.exists(tfile) else {}
        for k, s in summary.items():
            short = k.split("(")[0].replace("void ", "").replace("spmv::", "")
            for kern, algo in stream_bytes.items():
                if "+" not in kern and kern.split("<")[0] in short:
                    traffic[f"{config_key_prefix}:{kern}"] = (
                        s[field] if field == "traffic_raw" else {"bytes": s[field], "source": f"profiles/{tag}/pmc_summary.json"})
        # multi-kernel formats ("a+b", e.g. BIN's Mul + Sum): bytes of one
        # execute = the sum of each kernel's mean bytes per launch
        for kern in stream_bytes:
            if "+" in kern:
                parts = kern.split("+")
                tot, found = 0.0, 0
                for part in parts:
                    # the instantiation the timed loop ran: most launches
                    # (template arguments stripped: "ell_slice_kernel<perm>" is
                    # the instance "ell_slice_kernel<2, false, true>"; profile one
                    # format per run so a part names one instantiation)
                    cands = [s for k, s in summary.items() if part.split("<")[0] in k.split("(")[0]]
                    if cands:
                        tot += max(cands, key=lambda s: s["launches"])[field]
                        found += 1
                if found == len(parts):
                    traffic[f"{config_key_prefix}:{kern}"] = (
                        tot if field == "traffic_raw" else
                        {"bytes": tot, "source": f"profiles/{tag}/pmc_summary.json: 2*FETCH_SIZE + WRITE_SIZE "
                                                 "summed over the kernels of one execute"})
        json.dump(traffic, open(tfile, "w"), indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "c2:10000000x10000000")

#!/usr/bin/env python3
"""One-off wide run of tests/test_gpu_parity.py::test_device_build_fuzz over
many more seeds (host build vs device build: digests and y; y against the
oracle).  Prints one JSON line per failing (seed, format) and a summary line.
  python tests/fuzz_device_build.py 40 640
"""
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import test_gpu_parity as T  # noqa: E402

lo, hi = int(sys.argv[1]), int(sys.argv[2])
bad = 0
for seed in range(lo, hi):
    try:
        T.test_device_build_fuzz(seed)
    except Exception as e:  # report and go on
        bad += 1
        print(json.dumps({"seed": seed, "error": str(e)[:400], "tb": traceback.format_exc()[-600:]}), flush=True)
print(json.dumps({"seeds": [lo, hi], "failed": bad}), flush=True)

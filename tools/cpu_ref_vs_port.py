"""Cross-check of the CPU baseline (build container only: the reference never
ships to the GPU box).  Times the REFERENCE's own opt_crs SpMV (compiled from
/root/reference/src into oracle/_ref by `make ref`) and the oracle's
restatement that bench.py times on the box, on the same matrix, same threads,
same method (src/main.cpp:58-102: doubling warm-up, min over trials), and
checks they produce the same y.  Writes one JSON object to stdout."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# host cores of this process, read before an OpenMP runtime pins the main thread
THREADS = len(os.sched_getaffinity(0))
import oracle  # noqa: E402
import singlespmv_amd as sp  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    threads = THREADS
    spec = sp.gen_spec("uniform", rows, per_row=16, seed=42)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(rows, seed=43)
    row_idx = np.repeat(np.arange(rows, dtype=np.int32), np.diff(rp))
    t_ref, loop_ref, y_ref = oracle.ref_time("crs", rows, rows, row_idx, col, val, x, min_seconds=2.0, ntry=3,
                                             nthreads=threads)
    t_port, loop_port, y_port = oracle.csr_time(rp, col, val, x, nthreads=threads, min_seconds=2.0, ntry=3)
    nnz = int(rp[-1])
    print(json.dumps({
        "matrix": f"uniform {rows} x {rows}, 16 nnz/row (config 2 generator, seed 42)",
        "threads": threads, "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": "),
        "reference_opt_crs": {"ms_per_call": t_ref * 1e3, "gflops": 2 * nnz / t_ref / 1e9, "calls": loop_ref},
        "port_oracle_crs": {"ms_per_call": t_port * 1e3, "gflops": 2 * nnz / t_port / 1e9, "calls": loop_port},
        "port_over_reference": t_ref / t_port,
        "y_identical": bool(np.array_equal(y_ref, y_port)),
    }, indent=1))


if __name__ == "__main__":
    main()

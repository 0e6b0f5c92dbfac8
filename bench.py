#!/usr/bin/env python3
"""bench.py -- SpMV GFLOP/s + achieved HBM GB/s (fp64) on 1..8 MI355X.

Workload (BASELINE.json configs[1], weak-scaled): every rank owns a block of
10M rows x 16 nnz/row of a uniform random CSR whose column space is the
whole matrix (N*10M columns): N=1 is the 10M x 10M config, N=8 is the
80M x 80M row-partitioned config (configs[4]).  x is generated on rank 0 and
replicated with an RCCL broadcast over xGMI (setup, untimed -- x is fixed
across calls as in the reference driver, src/main.cpp:36-102); y slices are
gathered with RCCL all_gather, timed separately ("collective_ms").

A step = one y = A x over the rank's rows (device-resident x and y).  W
untimed warm-up steps, then T trials of exactly K steps, each bracketed by
barrier + torch.cuda.synchronize(); a trial's time is the max over ranks and
`value` comes from the fastest trial -- the reference driver's "min over
trials of the mean per call" (src/main.cpp:58-102).  The same K steps are
timed with HIP events on the plan's stream (spmv_time): that per-launch
duration feeds `roofline.achieved`.

`--gpus N` with no torchrun environment starts `torch.distributed.run` with N
ranks (one per GPU) as a child process before anything touches the GPU, and
exits with the child's return code.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--trials T]
                  [--config c2|c3|c4] [--formats auto,auto@plain,csr,ell,ss,css] [--no-cpu]

The headline plan asks for the build-time placement search (--placement
search: the bench owns the GPU); `formats["auto@plain"]` is the same plan with
the library's default single allocation, reported beside it.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

CONFIGS = {
    # name: (generator kwargs per rank, description)
    "c2": (dict(kind="uniform", per_row=16), "uniform 10M x 10M, 16 nnz/row (per GPU)", 10_000_000),
    "c3": (dict(kind="powerlaw", max_len=10000, alpha=2.0), "power-law 5M rows, 1-10k nnz/row", 5_000_000),
    "c4": (dict(kind="banded", band_lo=-32, band_hi=31), "banded 20M rows, 64 diagonals", 20_000_000),
}


def streamed_bytes(info) -> dict:
    """BIN's own HBM byte model per execute (the format's streams, not the
    algorithmic 12 B/nnz): Mul reads val 8 + column-in-strip 2 B per stored
    entry, one int32 destination per padded group, the x strips (each strip
    once, plus one re-load per workgroup range boundary) and writes 8 B
    products; Sum reads products 8 + row slot 2 B and writes y."""
    E = info["stored_slots"]  # Mul entries (segments, voids, long blocks)
    EL = info.get("bin_long_entries", 0)  # long blocks: 4 B lcode instead of a destination per group
    P = info.get("bin_products") or E  # products + run partials (+ the trash line)
    mul_read = E * (8 + 2) + (E - EL) // max(1, info["bin_pad"]) * 4 + 4 * EL + 8 * info["n"]
    mul_write = 8 * P
    sum_read = P * (8 + 2)
    sum_write = 8 * info["m"]
    return {"mul": mul_read + mul_write, "sum": sum_read + sum_write,
            "total": mul_read + mul_write + sum_read + sum_write,
            "mul_read": mul_read, "mul_write": mul_write, "sum_read": sum_read, "sum_write": sum_write}


def bin_ceiling(model: dict, read_gbs: float, write_gbs: float, mixed_gbs: float, nnz: int) -> dict:
    """BIN's own floor: its streamed bytes (not the 12 B/nnz roofline) moved at
    the measured ceilings of this GPU, Mul then Sum -- everything at the
    STREAM-read rate (`implied_ms`), and the Mul's reads + writes at the
    measured mixed read/write rate with the Sum at the read rate
    (`implied_ms_mixed`, the tighter one: HBM turns writes around slower)."""
    ms = model["total"] / read_gbs / 1e6
    ms_rw = ((model["mul_read"] + model["sum_read"]) / read_gbs + (model["mul_write"] + model["sum_write"]) / write_gbs) / 1e6
    ms_mixed = (model["mul"] / mixed_gbs + model["sum"] / read_gbs) / 1e6
    return {"model": "BIN streamed bytes (Mul 8+2+0.25 B read + 8 B write, Sum 8+2 B read per stored entry, "
                     "x strips, y), all moved at the measured STREAM-read ceiling; _mixed: the Mul at the "
                     "measured mixed read+write ceiling (3/4 written back), the Sum at the read ceiling",
            "bytes": model["total"], "read_gbs": read_gbs, "write_gbs": write_gbs, "mixed_gbs": mixed_gbs,
            "implied_ms": ms, "implied_gflops": 2.0 * nnz / (ms * 1e-3) / 1e9,
            "implied_ms_separate_write": ms_rw, "implied_ms_mixed": ms_mixed}


def _bin_ceiling_line(model, read_gbs, write_gbs, mixed_gbs, nnz, launch_ms) -> dict:
    c = bin_ceiling(model, read_gbs, write_gbs, mixed_gbs, nnz)
    c["frac_of_ceiling"] = c["implied_ms"] / launch_ms
    c["frac_of_ceiling_mixed"] = c["implied_ms_mixed"] / launch_ms
    return c


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--trials", type=int, default=5,
                    help="timed trials of K steps; value = the fastest (src/main.cpp:58-102)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (default: the config's)")
    ap.add_argument("--formats", default="auto,auto@plain,csr,ell,ss,css",
                    help="first entry is the headline plan; the rest are reported alongside; "
                         "fmt@placement overrides --placement for that plan (auto@plain: the "
                         "library's default placement, reported beside the searched one)")
    ap.add_argument("--placement", default="search", choices=["search", "plain", "vmm", "auto"],
                    help="plan-build placement of the BIN product buffer / DIA values (spmv_hip.h "
                         "SPMV_PLACEMENT_*): the bench owns the GPU, so it asks for the build-time search")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=2.0)
    ap.add_argument("--verify", action="store_true",
                    help="gather y to rank 0 and compare with the oracle over the full matrix "
                         "(tests; small sizes only)")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="development: run rank 0's share of a K-GPU job on one GPU "
                         "(n = K * rows); the JSON marks it as emulated")
    return ap.parse_args()


def self_launch(args):
    """--gpus N outside torchrun: run this script under torch.distributed.run
    with N ranks (rendezvous on 127.0.0.1) and return its exit code.  Called
    before any GPU call in this process (device_count() does not initialise
    the GPU); None = run in-process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus <= 1 or world == args.gpus or args.sim_world:
        return None
    if "WORLD_SIZE" in os.environ:
        print(json.dumps({"error": f"--gpus {args.gpus} inside a launcher with WORLD_SIZE={world}"}))
        return 2
    if os.environ.get("BENCH_DIST_BACKEND", "nccl") == "nccl":
        import torch
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print(json.dumps({"error": f"--gpus {args.gpus} but {ndev} GPUs visible "
                                       "(BENCH_DIST_BACKEND=gloo shares one GPU between ranks)"}))
            return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def traffic_key(config: str, m: int, n: int, kernel: str) -> str:
    """profiles/pmc_traffic*.json key: the PMC bytes of one launch of
    `kernel` on an m x n rank shape of `config` (none for other shapes)."""
    return f"{config}:{m}x{n}:{kernel}"


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        return rc
    # host cores of this process, read before any OpenMP runtime pins the
    # main thread to one place
    host_cores = len(os.sched_getaffinity(0))
    if int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # CPU baseline on all cores of the affinity, pinned (SURVEY §8(d):
        # binding moved the reference CRS from 4.5 to 7.0 GFLOP/s); set before
        # any OpenMP runtime is loaded.  Not for N>1: ranks share the host.
        os.environ.setdefault("OMP_PROC_BIND", "close")
        os.environ.setdefault("OMP_PLACES", "cores")
    elif os.environ.get("OMP_NUM_THREADS", "1") == "1":
        # torchrun's default of one OpenMP thread per rank would serialise the
        # host generator and format builders (untimed, but minutes at the
        # 8-GPU shape): share the host cores between the node's ranks instead
        # (read by the library's OpenMP runtime when it loads, below)
        local_world = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
        os.environ["OMP_NUM_THREADS"] = str(max(1, host_cores // local_world))
    import torch
    import torch.distributed as dist

    import singlespmv_amd as sp
    from singlespmv_amd import dist as sdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo lets several ranks share one GPU (development
    # rehearsal of the multi-GPU flow); the driver's runs use nccl = RCCL.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if backend == "gloo" else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    local = local_dev
    distributed = world > 1
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    sdist.set_cpu_collectives(backend == "gloo")

    gen_kw, desc, rows_default = CONFIGS[args.config]
    rows = args.rows or rows_default
    shape_world = args.sim_world if (args.sim_world and world == 1) else world
    m_glob = rows * shape_world
    n_glob = m_glob
    t0 = time.time()
    kind = gen_kw["kind"]
    spec = sp.gen_spec(kind, m_glob, n_glob, per_row=gen_kw.get("per_row", 16),
                       max_len=gen_kw.get("max_len", 10000), alpha=gen_kw.get("alpha", 2.0),
                       band_lo=gen_kw.get("band_lo", -32), band_hi=gen_kw.get("band_hi", 31),
                       seed=42)
    (row0, row1), rp, col, val = sdist.shard_generated(spec, rank, shape_world)
    nnz_local = int(rp[-1])
    # total flops of the job: every rank's own nnz (power-law rows make the
    # equal row blocks unequal in nnz)
    nnz_total = int(round(sdist.sum_over_ranks([float(nnz_local)], dev)[0]))
    t_gen = time.time() - t0

    # x: generated once on rank 0, replicated by RCCL broadcast over xGMI
    x = torch.empty(n_glob, dtype=torch.float64, device=dev)
    if rank == 0:
        x.copy_(torch.from_numpy(sp.generate_vector(n_glob, seed=43)))
    t_bcast = 0.0
    if distributed:
        torch.cuda.synchronize()
        dist.barrier()
        tb = time.perf_counter()
        sdist.replicate_x(x, src=0)
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - tb
    y = torch.empty(rows, dtype=torch.float64, device=dev)

    fmts = [f for f in args.formats.split(",") if f]
    results = {}
    headline = None
    for fi, spec_f in enumerate(fmts):
        fmt, _, placement = spec_f.partition("@")
        placement = placement or args.placement
        tp = time.time()
        try:
            plan = sp.Plan.from_csr(rows, n_glob, rp, col, val, fmt=fmt, device=local, placement=placement)
        except sp.SpmvError as e:
            results[spec_f] = {"error": str(e)}
            continue
        t_plan = time.time() - tp
        info = plan.info()
        stream = torch.cuda.Stream(device=dev)
        plan.set_stream(stream)
        torch.cuda.synchronize()
        # warm-up
        if args.warmup:
            plan.time(x, y, args.warmup)
        trials = []  # (max-over-ranks wall s, this rank's event ms)
        for _ in range(args.trials if fi == 0 else min(args.trials, 2)):
            torch.cuda.synchronize()
            if distributed:
                dist.barrier()
            torch.cuda.synchronize()
            tw = time.perf_counter()
            ev_ms = plan.time(x, y, args.steps)  # K launches between HIP events
            torch.cuda.synchronize()
            if distributed:
                dist.barrier()
            wall = time.perf_counter() - tw
            wall_max, _ = sdist.max_over_ranks([wall, ev_ms], dev)
            trials.append((wall_max, ev_ms))
        wall_max, ev_ms = min(trials)
        launch_s = ev_ms / 1e3 / args.steps
        flops_total = 2.0 * nnz_total * args.steps
        r = {
            "format": info["format"], "kernel": info["kernel"],
            "gflops": flops_total / wall_max / 1e9,
            "ms_per_step": wall_max / args.steps * 1e3,
            "trials_ms_per_step": [round(t[0] / args.steps * 1e3, 5) for t in trials],
            "event_ms_per_launch": launch_s * 1e3,
            "achieved_gbs": info["algo_bytes"] / launch_s / 1e9,
            "algo_bytes": info["algo_bytes"], "stored_slots": info["stored_slots"],
            "device_bytes": info["device_bytes"], "plan_build_s": round(t_plan, 3),
            "n_kernels": info["n_kernels"],
            "placement": info["placement"],
        }
        if info["placement_candidates"]:
            r["placement_candidates_ms"] = [round(info["placement_best_ms"], 4), round(info["placement_worst_ms"], 4),
                                            info["placement_candidates"]]
        relevant = {"csr": ("csr_lanes",), "ss": ("ss_sigma",), "ell": ("ell_width",),
                    "hyb": ("ell_width",), "dia": ("n_diags",), "css": ("css_passes", "css_slabs"),
                    "bin": ("bin_bins", "bin_strips", "bin_strip_cols", "bin_pad", "bin_sum_waves",
                            "bin_long_len", "bin_long_rows", "bin_long_pieces", "bin_products")}
        if info["format"] == "bin" and fi != 0:
            r["phases_ms"] = plan.profile(x, y, 10)  # Mul / Sum split (opt_ss MulPerf / SumPerf)
        for k in relevant.get(info["format"], ()):
            r[k] = info[k]
        results[spec_f if spec_f not in results else f"{spec_f}_{fi}"] = r
        if fi == 0:
            r["phases_ms"] = plan.profile(x, y, 10)
            headline = (plan, info, r)
            y_head = y.clone()
        else:
            del plan
        torch.cuda.synchronize()

    if headline is None:
        if rank == 0:
            print(json.dumps({"error": "no plan could be built", "details": results}))
        return 1
    plan, info, r = headline

    # y gather (RCCL all_gather over xGMI), timed separately from the kernel
    coll_ms = None
    if distributed:
        for _ in range(3):
            sdist.gather_y(y_head, rows)
        torch.cuda.synchronize()
        dist.barrier()
        tc = time.perf_counter()
        reps = 10
        for _ in range(reps):
            sdist.gather_y(y_head, rows)
        torch.cuda.synchronize()
        coll_ms = (time.perf_counter() - tc) / reps * 1e3

    # iterative use (power-iteration shape): every step is the
    # local SpMV followed by ONE all_gather of the y slices into the next x
    # (RCCL over xGMI), both on the current stream; reported beside `value`,
    # never as it.  Runs on a copy of x.
    iterative = None
    if distributed and n_glob == rows * world:
        x_it = x.clone()
        cur = torch.cuda.current_stream(dev)
        plan.set_stream(cur)
        for _ in range(2):
            plan.execute(x_it, y_head, async_=True)
            sdist.allgather_into(x_it, y_head)
        torch.cuda.synchronize()
        dist.barrier()
        ti = time.perf_counter()
        for _ in range(args.steps):
            plan.execute(x_it, y_head, async_=True)
            sdist.allgather_into(x_it, y_head)
        torch.cuda.synchronize()
        dist.barrier()
        t_it = sdist.max_over_ranks([time.perf_counter() - ti], dev)[0] / args.steps
        iterative = {"ms_per_iter": t_it * 1e3, "gflops": 2.0 * nnz_total / t_it / 1e9,
                     "step": "local SpMV + all_gather(y slices -> next x)"}
        del x_it
        plan.set_stream(stream)
        plan.execute(x, y_head)  # y_head back to A x for the checks below

    # the drop-in's host-buffer mode (opt_cusparse's per-call H2D x / D2H y,
    # src/opt_cusparse.cpp:72,82): PCIe-inclusive, reported beside `value`
    host_mode = None
    if rank == 0 and world == 1:
        xh = np.ascontiguousarray(x.cpu().numpy())
        yh = np.empty(rows, np.float64)
        reps = 5
        plan.execute(xh, yh)
        th = time.perf_counter()
        for _ in range(reps):
            plan.execute(xh, yh)
        t_h = (time.perf_counter() - th) / reps
        host_mode = {"ms_per_call": t_h * 1e3, "gflops": 2.0 * nnz_local / t_h / 1e9,
                     "pcie_bytes": 8 * (n_glob + rows),
                     "note": "host x and y (numpy): H2D x + SpMV + D2H y per call, like opt_cusparse"}
        del xh, yh

    verify_rel = None
    if args.verify:
        # the whole y (all ranks' slices, RCCL/gloo all_gather) vs the oracle's
        # opt_crs restatement of the full global matrix
        import oracle
        y_full = sdist.gather_y(y_head, rows)[:m_glob].cpu().numpy() if distributed else y_head.cpu().numpy()
        if rank == 0:
            grp, gcol, gval = sp.generate_csr(spec)
            yref = oracle.csr_spmv(grp, gcol, gval, x.cpu().numpy())
            verify_rel = float(np.max(np.abs(y_full - yref) / np.maximum(np.abs(yref), 1e-300)))

    # CPU baseline: the oracle's restatement of opt_crs SpMV (src/opt_crs.cpp:
    # 44-70; OpenMP static over rows, every host core of this process's
    # affinity, pinned), timed with the reference driver's method
    # (src/main.cpp:58-102: doubling warm-up to --cpu-seconds, min over 3
    # trials of the mean per call) on rank 0 at N = 1.  The reference's own
    # compiled opt_crs never ships to the GPU box; it was
    # timed beside the port in the build container (profiles/round2/cpu_ref_vs_port.json).
    cpu = None
    max_rel = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle
        nthreads = min(host_cores, int(os.environ.get("OMP_NUM_THREADS", host_cores)))
        x_host = x.cpu().numpy()
        t_cpu, loop, y_cpu = oracle.csr_time(rp, col, val, x_host, nthreads=nthreads,
                                             min_seconds=args.cpu_seconds, ntry=3)
        # the 1-thread figure BASELINE.md §4 asks for (short doubling warm-up,
        # one trial: a bounded sample of the same matrix)
        t_cpu1, _, _ = oracle.csr_time(rp, col, val, x_host, nthreads=1, min_seconds=0.5, ntry=1)
        ygpu = y_head.cpu().numpy()
        max_rel = float(np.max(np.abs(ygpu - y_cpu) / np.maximum(np.abs(y_cpu), 1e-300)))
        cpu = {"value": 2.0 * nnz_local / t_cpu / 1e9, "unit": "GFLOP/s", "cores": nthreads,
               "kind": "port", "nproc": os.cpu_count(),
               "omp_proc_bind": os.environ.get("OMP_PROC_BIND"),
               "omp_places": os.environ.get("OMP_PLACES"),
               "sample": f"full {rows}-row matrix ({nnz_local} nnz), oracle opt_crs restatement "
                         f"(oracle/oracle.c, src/opt_crs.cpp:44-70), {loop} calls x 3 trials after a "
                         f"{args.cpu_seconds:.0f} s doubling warm-up, min mean per call, "
                         f"{nthreads} threads = the host cores of this process's affinity",
               "ms_per_call": t_cpu * 1e3,
               "gbs": (12 * nnz_local + 4 * (rows + 1) + 16 * rows) / t_cpu / 1e9,
               "value_1thread": 2.0 * nnz_local / t_cpu1 / 1e9,
               "cpu_model": cpu_model()}

    achieved = r["achieved_gbs"]
    # measured STREAM-read ceiling of this GPU (reported beside the spec peak)
    stream_gbs = sp.stream_probe(local, 2 << 30, 10)
    stream_write_gbs = sp.stream_write_probe(local, 2 << 30, 10)
    mixed_gbs = sp.mixed_probe(local, 1792 << 20, 3, 20)
    # and the measured ceiling of random 8-byte x gathers that hit L2: every
    # format here issues one x gather per nnz, so this bounds the gather side
    gather_gps = sp.gather_probe(local, 64 << 20, 1 << 20)
    # ... and from a table of x's own size (beyond L2 once x > 4 MB): the
    # ceiling of the row-parallel formats, whose gathers go wherever x is
    gather_x_gps = sp.gather_probe(local, 64 << 20, min(max(8 * n_glob, 1 << 20), 2 << 30))
    gathers_gps = nnz_local / (r["event_ms_per_launch"] * 1e-3)
    gather_fields = {}
    if r["format"] not in ("dia", "bin"):  # DIA and BIN read x from LDS, not by gathers
        gather_fields = {"x_gathers_per_s": gathers_gps, "gather_ceiling_per_s": gather_gps,
                         "frac_of_gather_ceiling": gathers_gps / gather_gps}
    # per format: x gathers/s against the ceiling of where its gathers land
    # (CSS: an L2-resident slab; CSR/ELL/SS/COO/JDS/HYB: an x-sized table of
    # random gathers -- > 1 when the gathers are not random, as on a banded
    # matrix, whose bound is then the stream)
    for fr in results.values():
        if "event_ms_per_launch" not in fr:
            continue
        # and its algorithmic bytes against the measured STREAM-read ceiling
        fr["frac_of_stream"] = fr["achieved_gbs"] / stream_gbs
        if fr["format"] in ("dia", "bin"):
            continue
        g = nnz_local / (fr["event_ms_per_launch"] * 1e-3)
        ceil = gather_gps if fr["format"] == "css" else gather_x_gps
        fr["x_gathers_per_s"] = g
        fr["gather_ceiling_per_s"] = ceil
        fr["gather_ceiling_table"] = "1 MB (L2)" if fr["format"] == "css" else f"{8 * n_glob >> 20} MB (x)"
        fr["frac_of_gather_ceiling"] = g / ceil
    # the reference's CSR5 byte model (CSR5_cuda/detail/utils.h:10-14), which
    # charges x per nnz -- for comparability with published CSR5 numbers only
    csr5_bytes = (rows + 1 + nnz_local) * 4 + (2 * nnz_local + rows) * 8
    out = {
        "metric": "SpMV GFLOP/s (fp64) + achieved HBM GB/s",
        "value": r["gflops"],
        "unit": "GFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "trials": args.trials,
        "placement": args.placement,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded generator, seed 42; x seed 43)",
        "config": {"workload": f"{args.config}: {desc}", "rows_per_gpu": rows,
                   "m": m_glob, "n": n_glob, "nnz_per_gpu": nnz_local, "nnz_total": nnz_total,
                   "format": r["format"], "kernel": r["kernel"],
                   "parallelism": f"row-partition x{world}, x replicated (RCCL broadcast)"},
        "achieved_gbs": achieved,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": r["kernel"], "algo_bytes_per_launch": r["algo_bytes"],
                     "launch_ms": r["event_ms_per_launch"],
                     "stream_ceiling_gbs": stream_gbs, "frac_of_stream": achieved / stream_gbs,
                     "stream_write_gbs": stream_write_gbs, "mixed_rw_gbs": mixed_gbs,
                     **gather_fields,
                     "csr5_model_gbs": csr5_bytes / (r["event_ms_per_launch"] * 1e-3) / 1e9},
        "cpu_baseline": cpu,
        "streamed_bytes_model": streamed_bytes(info) if info["format"] == "bin" else None,
        # BIN's own byte floor: what this format could do on this GPU at best;
        # the headline's launch time over it is how close the kernels are
        "ceiling": (_bin_ceiling_line(streamed_bytes(info), stream_gbs, stream_write_gbs, mixed_gbs, nnz_local,
                                      r["event_ms_per_launch"])
                    if info["format"] == "bin" else None),
        "formats": results,
        "gen_s": round(t_gen, 2),
        "x_broadcast_ms": round(t_bcast * 1e3, 3) if distributed else None,
        "collective_ms": coll_ms,
        "iterative": iterative,
        "host_buffers": host_mode,
        "max_rel_err_vs_cpu": max_rel,
        "verify_max_rel": verify_rel,
    }
    if shape_world != world:
        out["emulated_world"] = shape_world
        out["config"]["parallelism"] = f"EMULATED rank 0 of {shape_world} (development only)"
    # roofline.traffic: PMC bytes per launch of this kernel/config -- the
    # calibrated figure where one exists (FETCH_SIZE calibrated on a known
    # byte count of the same access pattern), else raw FETCH+WRITE
    key = traffic_key(args.config, rows, n_glob, r["kernel"])
    for fname, kind in (("pmc_traffic_calibrated.json", "pmc_calibrated"), ("pmc_traffic.json", "pmc_raw")):
        path = os.path.join(ROOT, "profiles", fname)
        try:
            t = json.load(open(path)) if os.path.exists(path) else {}
        except ValueError:
            t = {}
        if key in t:
            v = t[key]
            out["roofline"]["traffic"] = v["bytes"] if isinstance(v, dict) else v
            out["roofline"]["traffic_kind"] = kind
            # the HBM bandwidth the kernels actually sustain: the profiled
            # bytes of one launch over this run's launch time (BIN moves
            # ~2.4x the algorithmic bytes; frac above prices only those)
            tg = out["roofline"]["traffic"] / (r["event_ms_per_launch"] * 1e-3) / 1e9
            out["roofline"]["traffic_gbs"] = tg
            out["roofline"]["traffic_frac"] = tg / HBM_PEAK_GBS
            out["roofline"]["traffic_frac_of_stream"] = tg / stream_gbs
            break
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

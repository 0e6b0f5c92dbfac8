#!/usr/bin/env python3
"""bench.py -- SpMV GFLOP/s + achieved HBM GB/s (fp64) on 1..8 MI355X.

Headline workload (BASELINE.json configs[1], weak-scaled): every rank owns a
block of 10M rows x 16 nnz/row of a uniform random CSR whose column space is
the whole matrix (N*10M columns): N=1 is the 10M x 10M config, N=8 is the
80M x 80M row-partitioned config (configs[4]).  Rows are cut nnz-balanced
(equal blocks for the uniform matrix).  x is generated on rank 0
and replicated with an RCCL broadcast over xGMI (setup, untimed -- x is fixed
across calls as in the reference driver, src/main.cpp:36-102); y slices are
gathered with RCCL all_gather, timed separately ("collective_ms").

A step = one y = A x over the rank's rows (device-resident x and y).  W
untimed warm-up steps, then T trials of exactly K steps, each bracketed by
barrier + torch.cuda.synchronize(); a trial's time is the max over ranks and
`value` comes from the fastest trial -- the reference driver's "min over
trials of the mean per call" (src/main.cpp:58-102).  The same K steps are
timed with HIP events on the plan's stream (spmv_time): that per-launch
duration feeds `roofline.achieved`.  Every plan is built with the library's
default placement (what a caller of OptimizeProblem gets).

At N = 1 the same line also carries configs 3 and 4 (BASELINE.json
configs[2], configs[3]) under `configs`: the power-law matrix through AUTO
(BIN) and the banded matrix through DIA with CSR beside it ("report DIA
against CSR"), each with its own roofline, PMC traffic and
max_rel_err_vs_cpu against the CPU port on the same matrix (`--only-config`
skips them).  At N > 1 `per_rank` lists every rank's rows, nnz, Mul / Sum
phases and event time, so the max-over-ranks step can be read per rank.

Every timed format carries `max_rel_err_vs_cpu`, at every N: each rank
compares its y slice with the oracle's opt_crs restatement of its own shard
(computed once on the host, untimed), and the figure is the max over ranks
(`per_rank[*].max_rel_err_vs_cpu` holds each rank's).  The process group has
a bounded timeout (BENCH_PG_TIMEOUT_S, default 900 s), so a hung collective
ends the job with an error.

`--gpus N` with no torchrun environment starts `torch.distributed.run` with N
ranks (one per GPU) as a child process before anything in this process loads
HIP (the GPUs are counted from the KFD topology in sysfs), and exits with the
child's return code.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--trials T]
                  [--config c2|c3|c4] [--formats auto,csr,ell,ss,css] [--only-config] [--no-cpu]

Prints ONE JSON line on rank 0.
"""
import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

T_START = time.time()  # process start: the rank's setup time is measured from here
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

CONFIGS = {
    # name: (generator kwargs, description, rows per GPU)
    "c2": (dict(kind="uniform", per_row=16), "uniform 10M x 10M, 16 nnz/row (per GPU)", 10_000_000),
    "c3": (dict(kind="powerlaw", max_len=10000, alpha=2.0), "power-law 5M rows, 1-10k nnz/row", 5_000_000),
    "c4": (dict(kind="banded", band_lo=-32, band_hi=31), "banded 20M rows, 64 diagonals", 20_000_000),
}
# the configs the N = 1 line carries beside the headline: (config, formats)
EXTRA_CONFIGS = (("c3", ["auto", "hyb", "csr", "ss"]), ("c4", ["auto", "csr", "ell", "ss", "jds"]))
# plans built so far in this process: a late plan can land in slower memory
# (include/spmv_hip.h, placement), so every format result records its ordinal
PLAN_ORDINAL = [0]
KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def model_bytes(fmt: str, m: int, n: int, nnz: int, n_diags: int = 0) -> int:
    """SURVEY §8(d) algorithmic bytes of one y = A x over an m x n rank shape
    (x read once, y written once): DIA 8 nnz + 4 nDiag + 8 n + 8 m; every
    other format is priced as CSR, 12 nnz + 4 (m + 1) + 8 n + 8 m (BASELINE.md
    §3: 2.120 GB at config 2, 15.76 GB CSR / 10.56 GB DIA at config 4), so the
    formats of one matrix share one byte model (the format's own model, e.g.
    BIN's 12 nnz + 8 n + 8 m, is kept beside it as `format_bytes`)."""
    if fmt == "dia":
        return 8 * nnz + 4 * n_diags + 8 * n + 8 * m
    return 12 * nnz + 4 * (m + 1) + 8 * n + 8 * m


def streamed_bytes(info) -> dict:
    """BIN's own HBM byte model per execute (the format's streams, not the
    algorithmic 12 B/nnz): Mul reads val 8 + column-in-strip 2 B per stored
    entry, one int32 destination per padded group, the x strips (each strip
    once, plus one re-load per workgroup range boundary) and writes 8 B
    products; Sum reads products 8 + row slot 2 B and writes y."""
    E = info["stored_slots"]  # Mul entries (segments, voids, long blocks)
    EL = info.get("bin_long_entries", 0)  # long blocks: 4 B lcode instead of a destination per group
    P = info.get("bin_products") or E  # products + run partials (+ the trash line)
    if info.get("bin_product_order") == 2:
        # Mul-ordered products: the Mul streams its unpadded entries and writes
        # them in place; the Sum walks the padded Sum order (8 B product + 2 B
        # slot per position, a 4-B chunk base per 8 positions)
        V = info.get("bin_sum_entries") or E
        mul_read = E * (8 + 2) + 8 * info["n"]
        mul_write = 8 * P
        sum_read = V * (8 + 2) + V // 2
    else:
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


def progress(msg: str) -> None:
    """A progress line on stderr (every rank, tagged): long setups (the 8-rank
    rehearsal, 1.28 G-entry configs) stay visibly alive."""
    print(f"[bench r{os.environ.get('RANK', '0')} +{time.time() - T_START:.1f}s] {msg}", file=sys.stderr, flush=True)


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
    ap.add_argument("--trials", type=int, default=10,
                    help="timed trials of K steps of each config's headline plan; value = the fastest "
                         "(src/main.cpp:58-102: min of 10); the other formats get 3")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (default: the config's)")
    ap.add_argument("--formats", default=None,
                    help="first entry is the headline plan; the rest are reported alongside "
                         "(default: auto,csr,ell,ss,css at N = 1; auto,csr at N > 1, where every rank "
                         "builds each format of its shard)")
    ap.add_argument("--only-config", action="store_true",
                    help="time --config alone (no configs 3 / 4 beside the N = 1 headline)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=1.0,
                    help="CPU warm-up: double the calls until this long (src/main.cpp:58-71)")
    ap.add_argument("--verify", action="store_true",
                    help="gather y to rank 0 and compare with the oracle over the full matrix "
                         "(tests; small sizes only)")
    ap.add_argument("--build", default="auto", choices=["auto", "host", "device"],
                    help="plan builders (spmv_options_t.build; AUTO: host CSRs of >= 2^24 entries on the device)")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="development: run rank 0's share of a K-GPU job on one GPU "
                         "(n = K * rows); the JSON marks it as emulated")
    return ap.parse_args()


def visible_gpu_count(topology: str = None) -> int:
    """GPUs this process may use, counted WITHOUT loading HIP: KFD topology
    nodes with SIMDs (CPU nodes have none), capped by the length of a
    HIP/ROCR/CUDA_VISIBLE_DEVICES list.  (torch.cuda.device_count() needs
    amdsmi to stay off HIP; this does not depend on it.)"""
    root = topology or os.environ.get("BENCH_KFD_TOPOLOGY", KFD_TOPOLOGY)
    gpus = 0
    try:
        for node in os.listdir(root):
            try:
                for line in open(os.path.join(root, node, "properties")):
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        gpus += 1
                        break
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            gpus = min(gpus, len([t for t in v.split(",") if t.strip()]))
    return gpus


def self_launch(args, runner=None):
    """--gpus N outside torchrun: run this script under torch.distributed.run
    with N ranks (rendezvous on 127.0.0.1) and return its exit code.  Nothing
    here loads HIP (tests/test_guards.py checks the parent's memory map at
    the spawn); None = run in-process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus <= 1 or world == args.gpus or args.sim_world:
        return None
    if "WORLD_SIZE" in os.environ:
        print(json.dumps({"error": f"--gpus {args.gpus} inside a launcher with WORLD_SIZE={world}"}))
        return 2
    if os.environ.get("BENCH_DIST_BACKEND", "nccl") == "nccl":
        ndev = visible_gpu_count()
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
    return (runner or subprocess.call)(cmd, env=env)


def traffic_key(config: str, m: int, n: int, kernel: str) -> str:
    """profiles/pmc_traffic*.json key: the PMC bytes of one launch of
    `kernel` on an m x n rank shape of `config` (none for other shapes)."""
    return f"{config}:{m}x{n}:{kernel}"


def lookup_traffic(config: str, m: int, n: int, kernel: str):
    """(bytes, kind) of the profiled launch of `kernel` on this shape: the
    calibrated table (2*FETCH_SIZE + WRITE_SIZE, the gfx950 correction)
    first, else raw FETCH + WRITE; (None, None) for an unprofiled shape."""
    key = traffic_key(config, m, n, kernel)
    for fname, kind in (("pmc_traffic_calibrated.json", "pmc_calibrated"), ("pmc_traffic.json", "pmc_raw")):
        path = os.path.join(ROOT, "profiles", fname)
        try:
            t = json.load(open(path)) if os.path.exists(path) else {}
        except ValueError:
            t = {}
        if key in t:
            v = t[key]
            return (v["bytes"] if isinstance(v, dict) else v), kind
    return None, None


def cpu_time(oracle, rp, col, val, x, nthreads: int, min_seconds: float):
    """src/main.cpp:58-102 on the CPU port: double the calls until >=
    min_seconds, then the min over 10 trials of the mean per call."""
    return oracle.csr_time(rp, col, val, x, nthreads=nthreads, min_seconds=min_seconds, ntry=10)


class Ctx:
    """Process-wide state: ranks, device, distributed flags."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        from singlespmv_amd import dist as sdist
        self.torch, self.dist, self.sdist = torch, dist, sdist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # BENCH_DIST_BACKEND=gloo lets several ranks share one GPU (development
        # rehearsal of the multi-GPU flow); the driver's runs use nccl = RCCL.
        self.backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        self.local = local % ndev if self.backend == "gloo" else local
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        self.distributed = self.world > 1
        if self.distributed:
            # bounded: a rank that never reaches a collective (a hung peer, a
            # lost GPU) ends the job with an error instead of holding it until
            # the driver's kill.  Generous enough for the slowest untimed setup
            # step between two collectives (the 8-rank shard generation).
            timeout = datetime.timedelta(seconds=float(os.environ.get("BENCH_PG_TIMEOUT_S", "900")))
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev, timeout=timeout)
            else:
                dist.init_process_group(self.backend, timeout=timeout)
        sdist.set_cpu_collectives(self.backend == "gloo")
        self.shape_world = args.sim_world if (args.sim_world and self.world == 1) else self.world


def build_matrix(ctx, args, config: str, rows_override: int = 0):
    """This rank's shard of `config` (nnz-balanced rows) and the replicated x."""
    import singlespmv_amd as sp
    torch = ctx.torch
    gen_kw, desc, rows_default = CONFIGS[config]
    rows = rows_override or rows_default
    m_glob = rows * ctx.shape_world
    n_glob = m_glob
    t0 = time.time()
    spec = sp.gen_spec(gen_kw["kind"], m_glob, n_glob, per_row=gen_kw.get("per_row", 16),
                       max_len=gen_kw.get("max_len", 10000), alpha=gen_kw.get("alpha", 2.0),
                       band_lo=gen_kw.get("band_lo", -32), band_hi=gen_kw.get("band_hi", 31), seed=42)
    cuts = ctx.sdist.generated_cuts(spec, ctx.shape_world)
    rank = ctx.rank if ctx.world > 1 else 0
    (row0, row1), rp, col, val = ctx.sdist.shard_generated(spec, rank, ctx.shape_world, cuts)
    nnz_local = int(rp[-1])
    # total flops of the job: every rank's own nnz
    nnz_total = int(round(ctx.sdist.sum_over_ranks([float(nnz_local)], ctx.dev)[0]))
    t_gen = time.time() - t0
    progress(f"{config}: rows [{row0}, {row1}) generated, {nnz_local} nnz, {t_gen:.1f} s")
    # x: generated once on rank 0, replicated by RCCL broadcast over xGMI
    x = torch.empty(n_glob, dtype=torch.float64, device=ctx.dev)
    if ctx.rank == 0:
        x.copy_(torch.from_numpy(sp.generate_vector(n_glob, seed=43)))
    t_bcast = None
    if ctx.distributed:
        torch.cuda.synchronize()
        ctx.dist.barrier()
        tb = time.perf_counter()
        ctx.sdist.replicate_x(x, src=0)
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - tb
    return dict(config=config, desc=desc, spec=spec, cuts=cuts, rows=row1 - row0, row0=row0, row1=row1,
                rows_nominal=rows, m=m_glob, n=n_glob, rp=rp, col=col, val=val, nnz_local=nnz_local,
                nnz_total=nnz_total, x=x, gen_s=t_gen, bcast_s=t_bcast)


RELEVANT = {"csr": ("csr_lanes",), "ss": ("ss_sigma",), "ell": ("ell_width",),
            "hyb": ("ell_width",), "dia": ("n_diags",), "css": ("css_passes", "css_slabs"),
            "bin": ("bin_bins", "bin_strips", "bin_strip_cols", "bin_pad", "bin_sum_waves",
                    "bin_long_len", "bin_long_rows", "bin_long_pieces", "bin_products",
                    "bin_product_order", "bin_sum_entries")}


def host_rss_peak_gb() -> float:
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6  # KB -> GB


def time_formats(ctx, args, M, fmts, trials_head: int, y_check=None, setup_mark=False):
    """Build and time each format on M; the first is the headline (kept, with
    its y).  y_check(y) -> dict, if given, is applied to every format's y
    (its max_rel_err_vs_cpu).  Returns (results, headline (plan, info, r) or
    None, y_head)."""
    import singlespmv_amd as sp
    torch = ctx.torch
    y = torch.empty(M["rows"], dtype=torch.float64, device=ctx.dev)
    results, headline, y_head = {}, None, None
    for fi, fmt in enumerate(fmts):
        tp = time.time()
        plan, err = None, None
        try:
            plan = sp.Plan.from_csr(M["rows"], M["n"], M["rp"], M["col"], M["val"], fmt=fmt, device=ctx.local,
                                    build=args.build)
        except sp.SpmvError as e:
            err = str(e)
        # every rank skips a format that failed on any rank (the timed trials
        # below are collective: one rank skipping them alone would hang)
        if ctx.sdist.sum_over_ranks([0.0 if plan is None else 1.0], ctx.dev)[0] < ctx.world:
            results[fmt] = {"error": err or "failed on another rank"}
            if plan is not None:
                plan.destroy()
            continue
        t_plan = time.time() - tp
        PLAN_ORDINAL[0] += 1
        info = plan.info()
        progress(f"{M['config']}: {fmt} plan ({info['kernel']}) built in {t_plan:.1f} s")
        stream = torch.cuda.Stream(device=ctx.dev)
        plan.set_stream(stream)
        torch.cuda.synchronize()
        if args.warmup:
            plan.time(M["x"], y, args.warmup)
        if setup_mark and fi == 0:
            # the rank's setup (generation, x broadcast, headline plan build),
            # measured up to its first timed trial (multi-GPU rehearsals)
            free, total = torch.cuda.mem_get_info(ctx.dev)
            M["setup"] = {"setup_s": time.time() - T_START, "peak_rss_gb": host_rss_peak_gb(),
                          "device_used_gb": (total - free) / 1e9, "plan_device_gb": info["device_bytes"] / 1e9}
        trials = []  # (max-over-ranks wall s, this rank's event ms, this rank's wall s)
        for _ in range(trials_head if fi == 0 else min(trials_head, 3)):
            torch.cuda.synchronize()
            if ctx.distributed:
                ctx.dist.barrier()
            torch.cuda.synchronize()
            tw = time.perf_counter()
            ev_ms = plan.time(M["x"], y, args.steps)  # K launches between HIP events
            torch.cuda.synchronize()
            if ctx.distributed:
                ctx.dist.barrier()
            wall = time.perf_counter() - tw
            wall_max = ctx.sdist.max_over_ranks([wall], ctx.dev)[0]
            trials.append((wall_max, ev_ms, wall))
        wall_max, ev_ms, wall_own = min(trials)
        launch_s = ev_ms / 1e3 / args.steps
        algo = model_bytes(info["format"], M["rows"], M["n"], M["nnz_local"], info.get("n_diags", 0))
        r = {
            "format": info["format"], "kernel": info["kernel"],
            "gflops": 2.0 * M["nnz_total"] * args.steps / wall_max / 1e9,
            "ms_per_step": wall_max / args.steps * 1e3,
            "trials_ms_per_step": [round(t[0] / args.steps * 1e3, 5) for t in trials],
            "event_ms_per_launch": launch_s * 1e3,
            "own_wall_ms_per_step": wall_own / args.steps * 1e3,
            "achieved_gbs": algo / launch_s / 1e9,
            "algo_bytes": algo, "format_bytes": info["algo_bytes"], "stored_slots": info["stored_slots"],
            "device_bytes": info["device_bytes"], "plan_build_s": round(t_plan, 3),
            "built_on_device": plan.built_on_device(),
            "n_kernels": info["n_kernels"], "placement": info["placement"],
            "plan_ordinal": PLAN_ORDINAL[0],
            "placement_info": {"mode": info["placement"], "candidates": info["placement_candidates"],
                               "best_ms": round(info["placement_best_ms"], 5),
                               "worst_ms": round(info["placement_worst_ms"], 5)},
        }
        for k in RELEVANT.get(info["format"], ()):
            r[k] = info[k]
        if info["n_kernels"] > 1:
            r["phases_ms"] = plan.profile(M["x"], y, 10)  # e.g. BIN Mul / Sum (opt_ss MulPerf / SumPerf)
        tb, kind = lookup_traffic(M["config"], M["rows"], M["n"], info["kernel"])
        if tb is not None:
            r["traffic"], r["traffic_kind"] = tb, kind
            r["traffic_over_algo"] = tb / algo
        if y_check is not None:
            torch.cuda.synchronize()
            own = y_check(y)["max_rel_err_vs_cpu"]
            # every rank checks its own slice; the format's figure is the max
            r["max_rel_err_vs_cpu"] = ctx.sdist.max_over_ranks([own], ctx.dev)[0]
            r["own_max_rel_err_vs_cpu"] = own
        results[fmt if fmt not in results else f"{fmt}_{fi}"] = r
        if fi == 0:
            headline = (plan, info, r)
            y_head = y.clone()
        else:
            plan.destroy()
        torch.cuda.synchronize()
    return results, headline, y_head


def device_build_record(ctx, M, host_plan, y_host, host_build_s) -> dict:
    """The same AUTO plan built on the GPU from the CSR already in HBM
    (spmv_plan_create_csr_device): its build time (the CSR
    upload excluded), whether its layout is byte-identical to the host
    build's (spmv_plan_digest) and its y to the host plan's."""
    import singlespmv_amd as sp
    torch = ctx.torch
    drp = torch.from_numpy(M["rp"]).to(ctx.dev)
    dcol = torch.from_numpy(M["col"]).to(ctx.dev)
    dval = torch.from_numpy(M["val"]).to(ctx.dev)
    torch.cuda.synchronize()
    tp = time.time()
    pd = sp.Plan.from_device_csr(M["rows"], M["n"], drp, dcol, dval, "auto", device=ctx.local)
    t_dev = time.time() - tp
    PLAN_ORDINAL[0] += 1
    info = pd.info()
    rec = {"format": info["format"], "kernel": info["kernel"], "plan_build_s": round(t_dev, 4),
           "host_plan_build_s": host_build_s, "plan_ordinal": PLAN_ORDINAL[0]}
    try:
        rec["layout_identical_to_host_build"] = pd.digest() == host_plan.digest()
    except sp.SpmvError as e:
        rec["layout_identical_to_host_build"] = str(e)
    y = torch.empty(M["rows"], dtype=torch.float64, device=ctx.dev)
    pd.execute(M["x"], y)
    rec["y_identical_to_host_plan"] = bool(torch.equal(y, y_host))
    pd.destroy()
    del drp, dcol, dval, y
    torch.cuda.empty_cache()
    progress(f"{M['config']}: device-built {info['format']} plan in {t_dev:.3f} s")
    return rec


def roofline_of(config: str, M, r) -> dict:
    ach = r["achieved_gbs"]
    out = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
           "traffic": None, "kernel": r["kernel"], "algo_bytes_per_launch": r["algo_bytes"],
           "launch_ms": r["event_ms_per_launch"]}
    # roofline.traffic: PMC bytes per launch of this kernel on this rank shape
    tb, kind = lookup_traffic(config, M["rows"], M["n"], r["kernel"])
    if tb is not None:
        out["traffic"] = tb
        out["traffic_kind"] = kind
        # the HBM bandwidth the kernels actually sustain: the profiled bytes of
        # one launch over this run's launch time (frac above prices only the
        # algorithmic bytes)
        tg = tb / (r["event_ms_per_launch"] * 1e-3) / 1e9
        out["traffic_gbs"] = tg
        out["traffic_frac"] = tg / HBM_PEAK_GBS
    return out


def shard_check(M):
    """The correctness check every timed format carries (src/main.cpp:40-56
    verifies before timing): the oracle's opt_crs restatement (oracle/oracle.c,
    src/opt_crs.cpp:44-70) of THIS rank's shard -- its rows, global columns,
    the replicated x -- computed once on the host, untimed, outside every timed
    trial.  Returns (y_check, cpu ms of the one call); y_check(y) gives
    max_rel_err_vs_cpu of a format's y slice (relative to |y_cpu|, the
    north star's 1e-6 measure)."""
    import oracle
    x_host = M["x"].cpu().numpy()
    tc = time.perf_counter()
    y_cpu = oracle.csr_spmv(M["rp"], M["col"], M["val"], x_host)
    t_cpu = time.perf_counter() - tc
    den = np.maximum(np.abs(y_cpu), 1e-300)
    del x_host

    def y_check(y):
        return {"max_rel_err_vs_cpu": float(np.max(np.abs(y.cpu().numpy() - y_cpu) / den, initial=0.0))}

    return y_check, t_cpu * 1e3


def extra_config(ctx, args, config: str, fmts, stream_gbs: float) -> dict:
    """One of configs 3 / 4 beside the N = 1 headline: headline format, the
    others beside it, roofline + PMC traffic, y against the CPU port."""
    M = build_matrix(ctx, args, config)
    # the CPU port's y first (untimed for the GPU): every format's y is
    # checked against it right after that format's timed trials
    y_check, t_cpu_ms = shard_check(M)
    results, head, y_head = time_formats(ctx, args, M, fmts, trials_head=args.trials, y_check=y_check)
    if head is None:
        return {"error": "no plan could be built", "details": results}
    plan, info, r = head
    device_build = None
    if config == "c4":
        device_build = device_build_record(ctx, M, plan, y_head, results[fmts[0]].get("plan_build_s"))
    plan.destroy()
    max_rel = r["max_rel_err_vs_cpu"]
    for fr in results.values():
        if "achieved_gbs" in fr:
            fr["frac_of_stream"] = fr["achieved_gbs"] / stream_gbs
            fr["roofline_frac"] = fr["achieved_gbs"] / HBM_PEAK_GBS
    roof = roofline_of(config, M, r)
    roof["frac_of_stream"] = r["achieved_gbs"] / stream_gbs
    out = {"workload": f"{config}: {M['desc']}", "m": M["m"], "n": M["n"], "nnz": M["nnz_local"],
           "format": r["format"], "kernel": r["kernel"], "value": r["gflops"], "unit": "GFLOP/s",
           "ms_per_step": r["ms_per_step"], "event_ms_per_launch": r["event_ms_per_launch"],
           "roofline": roof, "max_rel_err_vs_cpu": max_rel,
           "cpu_check": {"kind": "port", "ms_one_call": t_cpu_ms,
                         "note": "oracle opt_crs restatement (src/opt_crs.cpp:44-70), all host threads, one call"},
           "gen_s": round(M["gen_s"], 2), "formats": results}
    if device_build is not None:
        out["device_build"] = device_build
    if "csr" in results and "event_ms_per_launch" in results["csr"] and r["format"] != "csr":
        out[f"{r['format']}_vs_csr"] = results["csr"]["event_ms_per_launch"] / r["event_ms_per_launch"]
    del M, y_head
    ctx.torch.cuda.empty_cache()
    return out


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
    import singlespmv_amd as sp

    ctx = Ctx(args)
    torch, dist, sdist = ctx.torch, ctx.dist, ctx.sdist
    world, rank, dev, distributed = ctx.world, ctx.rank, ctx.dev, ctx.distributed

    M = build_matrix(ctx, args, args.config, args.rows)
    rows, n_glob, m_glob = M["rows"], M["n"], M["m"]
    nnz_local, nnz_total, x = M["nnz_local"], M["nnz_total"], M["x"]

    fmts_arg = args.formats or ("auto,csr,ell,ss,css" if world == 1 else "auto,csr")
    fmts = [f for f in fmts_arg.split(",") if f]
    # every rank's oracle y of its own shard: each format's y is checked
    # against it after that format's timed trials, at every N
    y_check, t_check_ms = shard_check(M)
    progress(f"{args.config}: oracle y of this rank's shard in {t_check_ms:.0f} ms")
    results, headline, y_head = time_formats(ctx, args, M, fmts, args.trials, y_check=y_check, setup_mark=True)
    if headline is None:
        if rank == 0:
            print(json.dumps({"error": "no plan could be built", "details": results}))
        return 1
    plan, info, r = headline

    # per-rank view of the headline step (the value is the max over ranks)
    per_rank = None
    if distributed:
        ph = r.get("phases_ms", {})
        su = M.get("setup", {})
        rows_all = sdist.gather_floats([float(rank), float(M["row0"]), float(M["row1"]), float(nnz_local),
                                        r["own_wall_ms_per_step"], r["event_ms_per_launch"],
                                        float(ph.get("mul", -1.0)), float(ph.get("sum", -1.0)),
                                        su.get("setup_s", -1.0), su.get("peak_rss_gb", -1.0),
                                        su.get("device_used_gb", -1.0), su.get("plan_device_gb", -1.0),
                                        host_rss_peak_gb(), time.time() - T_START,
                                        r["own_max_rel_err_vs_cpu"]], dev)
        per_rank = [{"rank": int(v[0]), "rows": [int(v[1]), int(v[2])], "nnz": int(v[3]),
                     "wall_ms_per_step": v[4], "event_ms_per_launch": v[5],
                     "phases_ms": {"mul": v[6], "sum": v[7]} if v[6] >= 0 else None,
                     "placement": info["placement"],
                     "setup_s_to_first_trial": v[8], "peak_rss_gb_at_first_trial": v[9],
                     "device_used_gb_after_build": v[10], "headline_plan_device_gb": v[11],
                     "peak_rss_gb": v[12], "elapsed_s": v[13],
                     "max_rel_err_vs_cpu": v[14]} for v in rows_all]

    # y gather (RCCL all_gather over xGMI), timed separately from the kernel
    # (slices padded to the longest rank's rows)
    rows_max = int(np.max(np.diff(M["cuts"]))) if distributed else rows
    coll_ms = None
    if distributed:
        for _ in range(3):
            sdist.gather_y(y_head, rows_max)
        torch.cuda.synchronize()
        dist.barrier()
        tc = time.perf_counter()
        reps = 10
        for _ in range(reps):
            sdist.gather_y(y_head, rows_max)
        torch.cuda.synchronize()
        coll_ms = (time.perf_counter() - tc) / reps * 1e3

    # iterative use (power-iteration shape): every step is the
    # local SpMV followed by ONE all_gather of the y slices into the next x
    # (RCCL over xGMI), both on the current stream; reported beside `value`,
    # never as it.  Runs on a copy of x; needs equal slices (uniform rows).
    iterative = None
    equal_slices = bool(np.all(np.diff(M["cuts"]) == rows)) and n_glob == rows * world
    if distributed and equal_slices:
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
        if distributed:
            parts = sdist.gather_y(y_head, rows_max).cpu().numpy().reshape(world, rows_max)
            y_full = np.concatenate([parts[k, :int(M["cuts"][k + 1] - M["cuts"][k])] for k in range(world)])
        else:
            y_full = y_head.cpu().numpy()
        if rank == 0:
            grp, gcol, gval = sp.generate_csr(M["spec"])
            yref = oracle.csr_spmv(grp, gcol, gval, x.cpu().numpy())
            if ctx.shape_world != world:  # emulated rank 0: its rows only
                yref = yref[:rows]
            verify_rel = float(np.max(np.abs(y_full - yref) / np.maximum(np.abs(yref), 1e-300)))

    # CPU baseline: the oracle's restatement of opt_crs SpMV (src/opt_crs.cpp:
    # 44-70; OpenMP static over rows, every host core of this process's
    # affinity, pinned), timed with the reference driver's method
    # (src/main.cpp:58-102: double the calls until >= 1 s, then the min over
    # 10 trials of the mean per call) on rank 0 at N = 1; the 1-thread figure
    # the same way on a bounded sample (the matrix's first tenth of rows, all
    # of x).  The reference's own compiled opt_crs never ships to the GPU box
    # (SURVEY §8(c)); it was timed beside the port in the build container
    # (profiles/round2/cpu_ref_vs_port.json).
    cpu = None
    # the headline's y against the oracle, max over every rank's slice
    max_rel = r["max_rel_err_vs_cpu"]
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle
        nthreads = min(host_cores, int(os.environ.get("OMP_NUM_THREADS", host_cores)))
        x_host = x.cpu().numpy()
        t_cpu, loop, _ = cpu_time(oracle, M["rp"], M["col"], M["val"], x_host, nthreads, args.cpu_seconds)
        r1 = max(1, rows // 10)
        e1 = int(M["rp"][r1])
        t_cpu1, loop1, _ = cpu_time(oracle, M["rp"][:r1 + 1], M["col"][:e1], M["val"][:e1], x_host, 1,
                                    args.cpu_seconds)
        cpu = {"value": 2.0 * nnz_local / t_cpu / 1e9, "unit": "GFLOP/s", "cores": nthreads,
               "kind": "port", "nproc": os.cpu_count(),
               "omp_proc_bind": os.environ.get("OMP_PROC_BIND"),
               "omp_places": os.environ.get("OMP_PLACES"),
               "sample": f"full {rows}-row matrix ({nnz_local} nnz), oracle opt_crs restatement "
                         f"(oracle/oracle.c, src/opt_crs.cpp:44-70): calls doubled until >= "
                         f"{args.cpu_seconds:g} s ({loop} calls), then the min over 10 trials of the mean "
                         f"per call (src/main.cpp:58-102), {nthreads} threads = the host cores of this "
                         f"process's affinity",
               "ms_per_call": t_cpu * 1e3,
               "gbs": model_bytes("csr", rows, n_glob, nnz_local) / t_cpu / 1e9,
               "value_1thread": 2.0 * e1 / t_cpu1 / 1e9,
               "sample_1thread": f"first {r1} rows ({e1} nnz) of the same matrix, all of x, 1 thread, "
                                 f"same method ({loop1} calls per trial, min of 10)",
               "cpu_model": cpu_model()}

    # measured ceilings of this GPU (reported beside the spec peak)
    local = ctx.local
    stream_gbs = sp.stream_probe(local, 2 << 30, 10)
    stream_write_gbs = sp.stream_write_probe(local, 2 << 30, 10)
    mixed_gbs = sp.mixed_probe(local, 1792 << 20, 3, 20)
    # random 8-byte x gathers that hit L2 (CSS's slab), and from a table of
    # x's own size (the row-parallel formats' gathers)
    gather_gps = sp.gather_probe(local, 64 << 20, 1 << 20)
    gather_x_gps = sp.gather_probe(local, 64 << 20, min(max(8 * n_glob, 1 << 20), 2 << 30))
    for fr in results.values():
        if "event_ms_per_launch" not in fr:
            continue
        fr["frac_of_stream"] = fr["achieved_gbs"] / stream_gbs
        fr["roofline_frac"] = fr["achieved_gbs"] / HBM_PEAK_GBS
        if fr["format"] in ("dia", "bin"):  # DIA and BIN read x from LDS, not by gathers
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
    roof = roofline_of(args.config, M, r)
    roof.update({"stream_ceiling_gbs": stream_gbs, "frac_of_stream": r["achieved_gbs"] / stream_gbs,
                 "stream_write_gbs": stream_write_gbs, "mixed_rw_gbs": mixed_gbs,
                 "csr5_model_gbs": csr5_bytes / (r["event_ms_per_launch"] * 1e-3) / 1e9})
    if "traffic_gbs" in roof:
        roof["traffic_frac_of_stream"] = roof["traffic_gbs"] / stream_gbs
    out = {
        "metric": "SpMV GFLOP/s (fp64) + achieved HBM GB/s",
        "value": r["gflops"],
        "unit": "GFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "trials": args.trials,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded generator, seed 42; x seed 43)",
        "config": {"workload": f"{args.config}: {M['desc']}", "rows_per_gpu": M["rows_nominal"],
                   "m": m_glob, "n": n_glob, "nnz_per_gpu": nnz_local, "nnz_total": nnz_total,
                   "format": r["format"], "kernel": r["kernel"], "placement": info["placement"],
                   "parallelism": f"row-partition x{world} (nnz-balanced), x replicated (RCCL broadcast)"},
        "achieved_gbs": r["achieved_gbs"],
        "roofline": roof,
        "phases_ms": r.get("phases_ms"),
        "cpu_baseline": cpu,
        "streamed_bytes_model": streamed_bytes(info) if info["format"] == "bin" else None,
        # BIN's own byte floor: what this format could do on this GPU at best;
        # the headline's launch time over it is how close the kernels are
        "ceiling": (_bin_ceiling_line(streamed_bytes(info), stream_gbs, stream_write_gbs, mixed_gbs, nnz_local,
                                      r["event_ms_per_launch"])
                    if info["format"] == "bin" else None),
        "formats": results,
        "per_rank": per_rank,
        "gen_s": round(M["gen_s"], 2),
        "x_broadcast_ms": round(M["bcast_s"] * 1e3, 3) if M["bcast_s"] is not None else None,
        "collective_ms": coll_ms,
        "iterative": iterative,
        "host_buffers": host_mode,
        "max_rel_err_vs_cpu": max_rel,
        "check": "every format's y, on every rank, against the oracle's opt_crs restatement of that rank's "
                 "shard (oracle/oracle.c, src/opt_crs.cpp:44-70), after its timed trials; max over ranks",
        "verify_max_rel": verify_rel,
        "gather_ceilings_per_s": {"l2_table": gather_gps, "x_table": gather_x_gps},
    }
    if ctx.shape_world != world:
        out["emulated_world"] = ctx.shape_world
        out["config"]["parallelism"] = f"EMULATED rank 0 of {ctx.shape_world} (development only)"
    plan.destroy()
    del M, y_head
    torch.cuda.empty_cache()

    # configs 3 and 4 beside the N = 1 headline (BASELINE.json configs[2-3])
    if world == 1 and not args.only_config and not args.sim_world and not args.rows and args.config == "c2":
        out["configs"] = {c: extra_config(ctx, args, c, f, stream_gbs) for c, f in EXTRA_CONFIGS}

    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

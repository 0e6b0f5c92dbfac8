"""The multi-GPU flow of bench.py (row shards, x broadcast, y all_gather)
with two ranks sharing the box's GPU over gloo -- the same code the 8-GPU
RCCL runs take, checked end to end against the oracle (bench.py --verify)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("config,fmts,launch", [("c2", "css,csr", "torchrun"), ("c2", "bin,csr", "self"),
                                                ("c3", "auto,ss", "self")])
def test_two_rank_bench_flow(config, fmts, launch):
    """launch "self": `bench.py --gpus 2` starts torch.distributed.run itself
    (the driver's multi-GPU invocation without a launcher); "torchrun": the
    driver's documented torchrun command line."""
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    pre = [sys.executable]
    if launch == "torchrun":
        pre += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
    cmd = pre + [os.path.join(ROOT, "bench.py"),
                 "--gpus", "2", "--steps", "3", "--warmup", "1", "--trials", "2", "--rows", "150000",
                 "--config", config, "--formats", fmts, "--verify", "--no-cpu"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0 and d["trials"] == 2
    assert d["config"]["nnz_total"] >= d["config"]["nnz_per_gpu"]
    assert d["config"]["m"] == 300000 and d["collective_ms"] is not None
    assert d["verify_max_rel"] is not None and d["verify_max_rel"] <= 1e-12, d["verify_max_rel"]
    # the bench's own per-rank check (no --verify needed): every format, every rank
    assert d["max_rel_err_vs_cpu"] is not None and d["max_rel_err_vs_cpu"] <= 1e-12
    for f in d["formats"].values():
        assert f["max_rel_err_vs_cpu"] <= 1e-12, f
    if config == "c2":  # equal slices: the iterative all_gather(y -> next x) step
        assert d["iterative"] is not None and d["iterative"]["ms_per_iter"] > 0
    assert [p["rank"] for p in d["per_rank"]] == [0, 1]
    for p in d["per_rank"]:  # the multi-GPU rehearsal record: setup time and memory per rank
        assert p["setup_s_to_first_trial"] > 0 and p["peak_rss_gb"] > 0 and p["headline_plan_device_gb"] > 0
        assert p["device_used_gb_after_build"] >= p["headline_plan_device_gb"]


@pytest.mark.parametrize("ranks", [2, 4])
def test_power_law_shards_are_nnz_balanced(ranks):
    """bench.py --config c3 --gpus 2/4: the generated shards are cut
    nnz-balanced, every rank's nnz within 1 % of nnz / N, and --
    without --verify, as the driver runs it -- every rank's y slice matches
    the oracle on its own shard (per_rank max_rel_err_vs_cpu)."""
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--steps", "3", "--warmup", "1",
           "--trials", "1", "--rows", "500000", "--config", "c3", "--formats", "auto", "--no-cpu"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    nnz = [p["nnz"] for p in d["per_rank"]]
    assert len(nnz) == ranks and sum(nnz) == d["config"]["nnz_total"]
    mean = d["config"]["nnz_total"] / ranks
    assert max(abs(v - mean) for v in nnz) <= 0.01 * mean, nnz
    rows = [p["rows"] for p in d["per_rank"]]
    assert rows[0][0] == 0 and rows[-1][1] == d["config"]["m"]
    assert all(rows[k][1] == rows[k + 1][0] for k in range(ranks - 1))
    assert d["verify_max_rel"] is None  # not asked for
    errs = [p["max_rel_err_vs_cpu"] for p in d["per_rank"]]
    assert all(0 <= e <= 1e-12 for e in errs), errs
    assert d["max_rel_err_vs_cpu"] == max(errs)


def test_c_abi_dist_plan_one_device():
    """The C-ABI multi-GPU path (spmv_dist_*: per-device plans, RCCL
    broadcast of x, RCCL all-gather of y) through the same code at N = 1 on
    the box: y against the oracle, the staged-x re-use, the timing entry."""
    import numpy as np
    import oracle
    import singlespmv_amd as sp
    for kind, m in (("uniform", 300_000), ("powerlaw", 200_000)):
        spec = sp.gen_spec(kind, m, per_row=16, max_len=3000, seed=8)
        rp, col, val = sp.generate_csr(spec)
        x = sp.generate_vector(m, seed=9)
        yo = oracle.csr_spmv(rp, col, val, x)
        for fmt in ("auto", "bin", "csr"):
            d = sp.DistPlan(m, m, rp, col, val, [0], fmt=fmt)
            assert list(d.cuts()) == [0, m]
            y = np.full(m, np.nan)
            d.execute(x, y)
            if fmt == "bin" and kind == "uniform":  # BIN sums each row in column order: bit-exact
                assert np.array_equal(y, yo), (kind, fmt)
            else:
                assert np.all(np.abs(y - yo) <= 1e-12 * np.abs(yo) + 1e-300), (kind, fmt)
            y2 = np.full(m, np.nan)
            d.execute(None, y2, staged=True)
            assert np.array_equal(y, y2)
            t_spmv, t_gather = d.time(5)
            assert t_spmv > 0 and t_gather >= 0
            d.destroy()


RCCL_WORLD1 = r"""
import os, sys, datetime
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
import oracle
import singlespmv_amd as sp
from singlespmv_amd import dist as sdist

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=120))
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
sdist.set_cpu_collectives(False)
sdist.force_collectives(True)
m = 200_003
spec = sp.gen_spec("uniform", m, per_row=16, seed=5)
rp, col, val = sp.generate_csr(spec)
xh = sp.generate_vector(m, seed=6)
x = torch.from_numpy(xh).to(dev)
sdist.replicate_x(x, src=0)                      # RCCL broadcast, f64 device tensor
assert torch.equal(x.cpu(), torch.from_numpy(xh))
assert sdist.max_over_ranks([1.5, -2.0], dev) == [1.5, -2.0]
assert sdist.sum_over_ranks([3.0], dev) == [3.0]
assert sdist.gather_floats([7.0, 8.0], dev) == [[7.0, 8.0]]
plan = sp.Plan.from_csr(m, m, rp, col, val, "bin", device=0)
y = torch.empty(m, dtype=torch.float64, device=dev)
plan.execute(x, y)
yo = oracle.csr_spmv(rp, col, val, xh)
pad = 1000                                        # padded slice: all_gather_into_tensor output sizing
yf = sdist.gather_y(y, m + pad)
assert yf.is_cuda and yf.numel() == m + pad
assert np.array_equal(yf[:m].cpu().numpy(), yo) and not yf[m:].any()
xi = torch.empty(m, dtype=torch.float64, device=dev)
cur = torch.cuda.current_stream(dev)
plan.set_stream(cur)
plan.execute(x, y, async_=True)                   # iterative step: SpMV then all_gather(y -> next x)
sdist.allgather_into(xi, y)
torch.cuda.synchronize()
assert np.array_equal(xi.cpu().numpy(), yo)
plan.destroy()
dist.barrier()
dist.destroy_process_group()
print("RCCL_WORLD1_OK")
"""


def test_rccl_device_collectives_world_one():
    """The device-tensor RCCL branches of dist.py (broadcast of x,
    all_gather_into_tensor of padded y slices and of y into the next x, the
    float reductions) on the box's GPU: a world-1 `nccl` process group with
    the collectives forced on (dist.force_collectives), around a real plan,
    y against the oracle bit for bit (BIN sums rows in column order)."""
    env = dict(os.environ, REPO=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, "-c", RCCL_WORLD1], capture_output=True, text=True, timeout=300,
                         env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "RCCL_WORLD1_OK" in out.stdout

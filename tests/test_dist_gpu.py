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
    if config == "c2":  # equal slices: the iterative all_gather(y -> next x) step
        assert d["iterative"] is not None and d["iterative"]["ms_per_iter"] > 0
    assert [p["rank"] for p in d["per_rank"]] == [0, 1]
    for p in d["per_rank"]:  # the multi-GPU rehearsal record: setup time and memory per rank
        assert p["setup_s_to_first_trial"] > 0 and p["peak_rss_gb"] > 0 and p["headline_plan_device_gb"] > 0
        assert p["device_used_gb_after_build"] >= p["headline_plan_device_gb"]


@pytest.mark.parametrize("ranks", [2, 4])
def test_power_law_shards_are_nnz_balanced(ranks):
    """bench.py --config c3 --gpus 2/4 --verify: the generated shards are cut
    nnz-balanced, every rank's nnz within 1 % of nnz / N, and the
    gathered y matches the oracle over the whole matrix."""
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--steps", "3", "--warmup", "1",
           "--trials", "1", "--rows", "500000", "--config", "c3", "--formats", "auto", "--verify", "--no-cpu"]
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
    assert d["verify_max_rel"] is not None and d["verify_max_rel"] <= 1e-12, d["verify_max_rel"]


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

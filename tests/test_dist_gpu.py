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


@pytest.mark.parametrize("config,fmts", [("c2", "css,csr"), ("c2", "bin,csr"), ("c3", "auto,ss")])
def test_two_rank_bench_flow(config, fmts):
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--rows", "150000", "--config", config,
           "--formats", fmts, "--verify", "--no-cpu"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["m"] == 300000 and d["collective_ms"] is not None
    assert d["verify_max_rel"] is not None and d["verify_max_rel"] <= 1e-12, d["verify_max_rel"]
    assert d["iterative"] is not None and d["iterative"]["ms_per_iter"] > 0

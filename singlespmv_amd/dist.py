"""Multi-GPU plumbing of the SpMV path: one process per GPU over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" in the
CPU tests).

The path shards by rows: every rank owns an nnz-balanced row
range and keeps global column indices; x is replicated once by a broadcast
(setup, untimed -- x is fixed across calls, src/main.cpp:36-102); a rank's y
slice is complete after its local SpMV, and the full y is assembled with one
all_gather when the caller needs it.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def row_range(m: int, rank: int, world: int, row_ptr=None) -> Tuple[int, int]:
    """[r0, r1) of `rank`: nnz-balanced when the global row_ptr is known
    (spmv_partition_rows), otherwise equal row blocks (uniform generators)."""
    if row_ptr is not None:
        from . import partition_rows
        cuts = partition_rows(row_ptr, world)
        return int(cuts[rank]), int(cuts[rank + 1])
    per = (m + world - 1) // world
    return min(m, rank * per), min(m, (rank + 1) * per)


def generated_cuts(spec, world: int) -> np.ndarray:
    """nnz-balanced cut rows of a synthetic matrix (SURVEY §8e "Partition":
    cuts[k] = first row with row_ptr[r] >= k*nnz/world, as spmv_partition_rows
    and dist.cpp's spmv_dist_layout cut a caller's CSR).  The row lengths are
    a function of (seed, row) alone, so the global row_ptr comes from the
    generator without building any entries; a uniform matrix (equal rows,
    equal nnz) is cut into equal row blocks directly."""
    from . import GEN_UNIFORM, generate_row_ptr, partition_rows
    if world <= 1:
        return np.array([0, spec.m], np.int64)
    if spec.kind == GEN_UNIFORM:
        per = (spec.m + world - 1) // world
        return np.minimum(np.arange(world + 1, dtype=np.int64) * per, spec.m)
    return partition_rows(generate_row_ptr(spec), world)


def shard_generated(spec, rank: int, world: int, cuts=None):
    """Generate only this rank's rows of a synthetic matrix: the rank's
    nnz-balanced row range (generated_cuts) and its CSR."""
    from . import generate_csr
    if cuts is None:
        cuts = generated_cuts(spec, world)
    r0, r1 = int(cuts[rank]), int(cuts[rank + 1])
    rp, col, val = generate_csr(spec, r0, r1)
    return (r0, r1), rp, col, val


def shard_csr(row_ptr, col, val, rank: int, world: int):
    """Cut a global host CSR into this rank's nnz-balanced slice."""
    m = len(row_ptr) - 1
    r0, r1 = row_range(m, rank, world, row_ptr)
    b, e = int(row_ptr[r0]), int(row_ptr[r1])
    return (r0, r1), (row_ptr[r0:r1 + 1] - b).astype(np.int64), col[b:e], val[b:e]


_CPU_COLLECTIVES = False
_FORCE_COLLECTIVES = False


def set_cpu_collectives(flag: bool) -> None:
    """Route collectives through host copies (gloo rehearsal with several
    ranks on one GPU); RCCL runs keep device tensors."""
    global _CPU_COLLECTIVES
    _CPU_COLLECTIVES = bool(flag)


def force_collectives(flag: bool) -> None:
    """Test hook: issue the collectives even in a world of one rank, so a
    one-GPU box runs the device-tensor RCCL branches (broadcast,
    all_gather_into_tensor) that an N > 1 job takes (RCCL refuses two ranks
    on one GPU)."""
    global _FORCE_COLLECTIVES
    _FORCE_COLLECTIVES = bool(flag)


def _dist_on():
    import torch.distributed as dist
    return dist.is_initialized() and (dist.get_world_size() > 1 or _FORCE_COLLECTIVES)


def replicate_x(x, src: int = 0):
    """Broadcast x from `src` to every rank (RCCL/gloo broadcast), in place."""
    import torch.distributed as dist
    if _dist_on():
        if _CPU_COLLECTIVES and x.is_cuda:
            h = x.cpu()
            dist.broadcast(h, src=src)
            x.copy_(h)
        else:
            dist.broadcast(x, src=src)
    return x


def max_over_ranks(values, device):
    """Element-wise max of a short list of floats over all ranks."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64,
                     device="cpu" if _CPU_COLLECTIVES else device)
    if _dist_on():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def sum_over_ranks(values, device):
    """Element-wise sum of a short list of floats over all ranks."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64,
                     device="cpu" if _CPU_COLLECTIVES else device)
    if _dist_on():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def gather_floats(values, device):
    """Every rank's short list of floats (equal lengths), in rank order."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64,
                     device="cpu" if _CPU_COLLECTIVES else device)
    if not _dist_on():
        return [[float(v) for v in t.tolist()]]
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [[float(v) for v in p.tolist()] for p in parts]


def gather_y(y_local, rows_per_rank: int):
    """All-gather equal, padded y slices into the full y (length
    world * rows_per_rank; the caller trims the padding)."""
    import torch
    import torch.distributed as dist
    if not _dist_on():
        return y_local
    world = dist.get_world_size()
    if y_local.numel() < rows_per_rank:
        pad = torch.zeros(rows_per_rank - y_local.numel(), dtype=y_local.dtype, device=y_local.device)
        y_local = torch.cat([y_local, pad])
    if _CPU_COLLECTIVES and y_local.is_cuda:
        parts = [torch.empty(rows_per_rank, dtype=y_local.dtype) for _ in range(world)]
        dist.all_gather(parts, y_local.cpu())
        return torch.cat(parts).to(y_local.device)
    out = torch.empty(world * rows_per_rank, dtype=y_local.dtype, device=y_local.device)
    dist.all_gather_into_tensor(out, y_local.contiguous())
    return out


def allgather_into(x, y_local):
    """Iterative use (y -> next x): all-gather every rank's
    equal y slice straight into the replicated x (length world * slice)."""
    import torch
    import torch.distributed as dist
    if not _dist_on():
        x[: y_local.numel()].copy_(y_local)
        return x
    if _CPU_COLLECTIVES and y_local.is_cuda:
        parts = [torch.empty(y_local.numel(), dtype=y_local.dtype) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, y_local.cpu())
        x.copy_(torch.cat(parts).to(x.device))
        return x
    dist.all_gather_into_tensor(x, y_local.contiguous())
    return x

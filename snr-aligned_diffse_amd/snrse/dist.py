"""Multi-GPU utterance sharding: one process per GPU, no data-path
collective.  Utterances are independent, so each rank enhances a contiguous shard; RCCL
(torch.distributed 'nccl' on ROCm) is used only to take the max wall time over ranks and
to gather the per-utterance metrics at the end.  'gloo' runs the same code on CPU (tests).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None):
    """(rank, world, device) from torchrun's env; single process skips process-group init."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        be = backend or ("nccl" if use_gpu else "gloo")
        if be == "nccl":
            dist.init_process_group(be, device_id=dev)
        else:
            dist.init_process_group(be)
    return rank, world, dev


def shard_range(n: int, rank: int, world: int):
    """Contiguous balanced shard [start, stop) of n utterances for `rank`."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_over_ranks(value: float, device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def gather_metrics(values, n_total: int, rank: int, world: int, device):
    """All ranks' per-utterance metric rows -> [n_total, k] float64 tensor on every rank,
    ordered by utterance index (rank r holds rows shard_range(n_total, r, world))."""
    vals = torch.as_tensor(values, dtype=torch.float64, device=device)
    if vals.dim() == 1:
        vals = vals[:, None]
    if not (dist.is_available() and dist.is_initialized()) or world == 1:
        return vals
    k = vals.shape[1]
    cap = shard_range(n_total, 0, world)[1]  # largest shard
    pad = torch.full((cap, k), float("nan"), dtype=torch.float64, device=device)
    pad[: vals.shape[0]] = vals
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    rows = []
    for r in range(world):
        a, b = shard_range(n_total, r, world)
        rows.append(bufs[r][: b - a])
    return torch.cat(rows, 0)

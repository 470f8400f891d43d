"""Multi-GPU utterance sharding: one process per GPU, no data-path
collective.  Utterances are independent, so each rank enhances a contiguous shard; RCCL
(torch.distributed 'nccl' on ROCm) is used only to take the max wall time over ranks and
to gather the per-utterance metrics at the end.  'gloo' runs the same code on CPU (tests).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def oversubscribed(world: int) -> bool:
    """More ranks than visible GPUs (a rehearsal of the N-rank launch on a smaller box): ranks then
    share devices round-robin and the collectives run on gloo (RCCL needs one rank per device).
    torch.cuda.device_count() does not initialise the GPU."""
    n = torch.cuda.device_count()
    return 0 < n < world


def init_from_env(backend: str | None = None):
    """(rank, world, device) from torchrun's env; single process skips process-group init."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if use_gpu and oversubscribed(world):
        local %= torch.cuda.device_count()
        backend = backend or "gloo"
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


def _coll_device(device):
    """gloo collectives take host tensors."""
    return torch.device("cpu") if dist.get_backend() == "gloo" else device


def max_over_ranks(value: float, device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=_coll_device(device))
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
    out_dev, device = device, _coll_device(device)
    vals = vals.to(device)
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
    return torch.cat(rows, 0).to(out_dev)


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(rank, world, port, fn, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    fn(*args)


def spawn_ranks(world: int, fn, args=(), poll_s: float = 0.5) -> int:
    """Run fn(*args) in `world` fresh processes (multiprocessing 'spawn'), rank r on GPU r, with
    torchrun's environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT).
    The caller must not have initialised the GPU (children are new interpreters, nothing is exec'd
    over a GPU-initialised process).  If a rank fails, the others are terminated instead of being
    left waiting in a collective.  Returns 0 or the first failing rank's exit code."""
    import time

    import torch.multiprocessing as mp
    port = free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_entry, args=(r, world, port, fn, args)) for r in range(world)]
    for p in procs:
        p.start()
    rc = 0
    while any(p.is_alive() for p in procs):
        bad = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.is_alive():
                    p.terminate()
            break
        time.sleep(poll_s)
    for p in procs:
        p.join()
        if rc == 0 and p.exitcode:
            rc = p.exitcode
    return rc

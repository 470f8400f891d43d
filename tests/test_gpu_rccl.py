"""The RCCL ('nccl' backend) branch of snrse.dist on a real device: a world-size-1 process group over
RCCL runs the same max-over-ranks all_reduce and metric all_gather that bench.py / evaluate use after
the timed region (snrse/dist.py), on HIP tensors.  World sizes > 1 need one GPU per rank, which the
single-GPU test box does not have; their logic is covered by the gloo world-2 tests (test_dist_gloo.py)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as dist

    from snrse import dist as sd
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        backend = dist.get_backend()
        t = sd.max_over_ranks(3.5, dev)
        rows = [[float(i), 2.0 * i] for i in range(5)]
        allm = sd.gather_metrics(rows, 5, 0, 1, dev)
        # gather_metrics returns early at world 1; run its collective path explicitly as well
        pad = torch.arange(10, dtype=torch.float64, device=dev).reshape(5, 2)
        bufs = [torch.empty_like(pad)]
        dist.all_gather(bufs, pad)
        dist.barrier()
        q.put((backend, t, allm.cpu().tolist(), bool(torch.equal(bufs[0], pad)), str(allm.device)))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_collectives(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    backend, t, rows, gathered, dev = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl"
    assert t == 3.5
    assert rows == [[float(i), 2.0 * i] for i in range(5)]
    assert gathered and dev.startswith("cuda")

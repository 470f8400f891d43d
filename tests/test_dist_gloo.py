"""world_size-2 gloo run of the utterance-sharding path (CPU): shards cover every utterance
exactly once, the max-over-ranks time and the metric gather are what rank 0 reports."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from snrse import dist as sd
    r, w, dev = sd.init_from_env("gloo")
    a, b = sd.shard_range(n_total, r, w)
    metrics = [[float(i), float(i) * 0.5] for i in range(a, b)]  # stand-in per-utterance metrics
    t = sd.max_over_ranks(1.0 + r, dev)
    allm = sd.gather_metrics(metrics, n_total, r, w, dev)
    q.put((r, a, b, t, allm.numpy().tolist()))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_sharding_ranges():
    from snrse.dist import shard_range
    for n in (1, 7, 32, 256, 257):
        for w in (1, 2, 3, 8):
            covered = []
            for r in range(w):
                a, b = shard_range(n, r, w)
                covered += list(range(a, b))
            assert covered == list(range(n))


def test_gloo_world2_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_total = 7
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, a0, b0, t0, m0), (r1, a1, b1, t1, m1) = res
    assert (a0, b0, a1, b1) == (0, 4, 4, 7)
    assert t0 == t1 == 2.0
    assert m0 == m1 == [[float(i), float(i) * 0.5] for i in range(n_total)]


def _eval_worker(rank, world, port, root, out, q):
    """evaluate() on gloo with a stand-in model and metric (the HIP parts are GPU-tested in
    test_metrics.py): each rank enhances its shard, the rows meet in one all_gather, rank 0 writes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import numpy as np

    from snrse import dist as sd
    from snrse import evaluate as ev
    r, w, _ = sd.init_from_env("gloo")

    class _SDE:
        _T = 1.0

    class _Model:
        sde = _SDE()
        seen = []

        def enhance(self, x, y, **kw):
            self.seen.append(kw["N"])
            return (0.5 * y[0]).numpy()

    ev.score_files = lambda xh, x, y, sr=16000, pesq_fn=None: [float("nan"), float(len(x)), float(r), float(xh[0])]
    m = _Model()
    data = ev.evaluate(m, root, out, N=30, rank=r, world=w)
    q.put((r, len(m.seen), data["si_sdr"], data["si_sir"]))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_gloo_world2_evaluate_sharded(tmp_path):
    import numpy as np

    from snrse import audio
    root = tmp_path / "t"
    for d in ("clean", "noisy"):
        os.makedirs(root / d)
    for k in range(5):
        sig = np.full(1000 + 10 * k, 0.25, np.float32)
        audio.write_wav(str(root / "clean" / f"u{k}.wav"), sig, bits=32)
        audio.write_wav(str(root / "noisy" / f"u{k}.wav"), sig, bits=32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    out = str(tmp_path / "out")
    procs = [ctx.Process(target=_eval_worker, args=(r, 2, port, str(root), out, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, sdr0, sir0), (r1, n1, sdr1, sir1) = res
    assert (n0, n1) == (3, 2)                       # contiguous shards of the 5 files
    assert sdr0 == sdr1 == [1000.0 + 10 * k for k in range(5)]  # every row, in file order
    assert sir0 == [0.0, 0.0, 0.0, 1.0, 1.0]        # which rank scored each file
    lines = open(os.path.join(out, "_results.csv")).read().splitlines()
    assert len(lines) == 6 and lines[1].startswith("u0.wav,nan,1000.0,0.0,")


def _spawned_child(path):
    """What bench.py's --gpus N launcher runs per rank, on gloo: init from the env it was given."""
    from snrse import dist as sd
    r, w, dev = sd.init_from_env("gloo")
    t = sd.max_over_ranks(0.5 * (r + 1), dev)
    allm = sd.gather_metrics([[float(r)]] * 3, 3 * w, r, w, dev)
    if r == 0:
        with open(path, "w") as f:
            f.write(f"{w} {t} {allm[:, 0].tolist()}")
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def _failing_child():
    raise SystemExit(3)


def test_spawn_ranks_world2(tmp_path):
    """snrse.dist.spawn_ranks -- the launcher behind `bench.py --gpus N` -- starts N ranks with the
    torchrun environment; a failing rank's code is returned."""
    from snrse import dist as sd
    path = str(tmp_path / "r0.txt")
    assert sd.spawn_ranks(2, _spawned_child, (path,)) == 0
    assert open(path).read() == "2 1.0 [0.0, 0.0, 0.0, 1.0, 1.0, 1.0]"
    assert sd.spawn_ranks(2, _failing_child) == 3


def _deep_eval_worker(rank, world, port, root, out, q):
    """deep_evaluate() (the deep_eval.py SNR sweep) on gloo with a stand-in model: each rank enhances
    the nine SNR variants of its files, the rows meet in one all_gather, rank 0 writes the tables."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from snrse import deep_evaluate as de
    from snrse import dist as sd
    r, w, _ = sd.init_from_env("gloo")

    class _SDE:
        _T = 1.0

    class _Model:
        sde = _SDE()
        seen = []

        def enhance(self, x, y, **kw):
            self.seen.append(kw["noise_rms"])
            return (0.5 * y[0]).numpy()

    m = _Model()
    data = de.deep_evaluate(m, root, out, N=30, rank=r, world=w, batched=False, verbose=False)
    q.put((r, len(m.seen), data["filename"], data["pesq_-5"], sorted(set(round(v, 6) for v in m.seen))))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_gloo_world2_deep_evaluate_sharded(tmp_path):
    import numpy as np

    from snrse import audio
    root = tmp_path / "t"
    for d in ("clean", "noisy"):
        os.makedirs(root / d)
    for k in range(3):
        sig = np.full(800 + 10 * k, 0.25, np.float32)
        audio.write_wav(str(root / "clean" / f"u{k}.wav"), sig, bits=32)
        audio.write_wav(str(root / "noisy" / f"u{k}.wav"), sig * 1.5, bits=32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    out = str(tmp_path / "out")
    procs = [ctx.Process(target=_deep_eval_worker, args=(r, 2, port, str(root), out, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, f0, p0, rms0), (r1, n1, f1, p1, rms1) = res
    assert (n0, n1) == (2 * 9, 1 * 9)                # contiguous shards, nine variants per file
    assert f0 == f1 == ["u0.wav", "u1.wav", "u2.wav"] and len(p0) == 3
    assert rms0 == sorted(round(10 ** ((5 - s) / 20), 6) for s in range(0, 41, 5))  # deep_eval.py:118
    lines = open(os.path.join(out, "_results_deep.csv")).read().splitlines()
    assert lines[0] == "filename," + ",".join(f"pesq_{s - 5}" for s in range(0, 41, 5)) and len(lines) == 4
    for s in range(0, 41, 5):
        assert os.path.exists(os.path.join(out, "{0:02d}".format(s - 5), "u2.wav"))
    txt = open(os.path.join(out, "_avg_results_deep.txt")).read().splitlines()
    assert txt[0].startswith("PESQ_-5: ") and txt[-1].startswith("PESQ_35: ") and len(txt) == 9

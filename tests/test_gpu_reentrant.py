"""Reentrancy of the C-ABI ("stateless and reentrant per stream"): two host threads,
each issuing on its own HIP stream through its own launch context (snrse_ctx: switches, split-K
workspace, read-backs; snrse.ops.LaunchContext), run NCSN++ evaluations and split-K convs concurrently
and get the outputs of the serial run."""
import threading

import pytest
import torch

from conftest import fnormal, formula_sd

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu() if not a.is_complex() else a.detach().cpu().to(torch.complex128), \
        b.detach().double().cpu() if not b.is_complex() else b.detach().cpu().to(torch.complex128)
    return float((a - b).abs().pow(2).mean().sqrt() / (b.abs().pow(2).mean().sqrt() + 1e-30))


def _run_threads(fns):
    errs, outs = [], [None] * len(fns)
    barrier = threading.Barrier(len(fns))

    def body(k):
        try:
            s = torch.cuda.Stream()
            barrier.wait()
            with torch.cuda.stream(s):
                outs[k] = fns[k]()
            s.synchronize()
        except Exception as e:  # noqa: BLE001 - re-raised in the main thread
            errs.append(e)

    ts = [threading.Thread(target=body, args=(k,)) for k in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "thread did not finish"
    if errs:
        raise errs[0]
    return outs


@pytest.mark.parametrize("dt", ["fp32", "fp16", "bf16"])
def test_two_threads_network_evaluations_match_serial(gpu, dt):
    from snrse import ncsnpp
    sd = {k: torch.from_numpy(v) for k, v in formula_sd("ncsnpp").items()}
    net = ncsnpp.NCSNppHIP(sd, dtype={"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[dt],
                           device=gpu)
    ins = []
    for k in range(2):
        x = torch.from_numpy(fnormal(f"reentrant.x{k}", (2, 2, 256, 64), complex_=True)) * 0.5
        ins.append((x[:, 0].contiguous().to(gpu), x[:, 1].contiguous().to(gpu),
                    torch.tensor([0.4 + 0.2 * k, 0.7], device=gpu)))
    reps = 4
    serial = [[net.dnn(*ins[k]).clone() for _ in range(reps)] for k in range(2)]
    torch.cuda.synchronize()

    def make(k):
        return lambda: [net.dnn(*ins[k]).clone() for _ in range(reps)]

    conc = _run_threads([make(0), make(1)])
    tol = 1e-6 if dt == "fp32" else 2e-3  # up to the order of the f64 GroupNorm-statistics atomics
    for k in range(2):
        for r in range(reps):
            assert _rel(conc[k][r], serial[k][0]) < tol, (k, r, _rel(conc[k][r], serial[k][0]))


def test_two_threads_splitk_convs_use_their_own_contexts(gpu):
    """Low-resolution fp32 convs whose tile grid underfills the chip split K into each thread's own
    workspace (read-back "last_ksplit" > 1 in that thread's context) and match the serial outputs."""
    from snrse import ops
    g = torch.Generator(device=gpu).manual_seed(5)
    cases = []
    for k in range(2):
        x = torch.randn(2, 8, 16, 256, device=gpu, generator=g)
        w = torch.randn(256, 9 * 256, device=gpu, generator=g) / 48
        bias = torch.randn(256, device=gpu, generator=g)
        cases.append((x, w, bias))
    serial = [ops.conv2d(x, w, 3, 256, bias=b) for x, w, b in cases]
    torch.cuda.synchronize()

    def make(k):
        def f():
            x, w, b = cases[k]
            outs = [ops.conv2d(x, w, 3, 256, bias=b) for _ in range(8)]
            return outs, ops.get_option("last_ksplit"), ops.context(gpu).ptr
        return f

    (o0, ks0, c0), (o1, ks1, c1) = _run_threads([make(0), make(1)])
    assert ks0 > 1 and ks1 > 1, (ks0, ks1)
    assert c0 != c1 and c0 != ops.context(gpu).ptr
    for k, outs in ((0, o0), (1, o1)):
        for o in outs:
            assert _rel(o, serial[k]) < 1e-6

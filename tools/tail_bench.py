#!/usr/bin/env python3
"""Micro-benchmarks of the C2 network's low-resolution tail launches (levels 4-6 of the B = 32, 256 x 512
pyramid) that profiles/r05a_c2_dispatch_shapes.jsonl showed far above their work: the 4 x 8 level 1x1 GEMM
with multi-image wave tiles (NIN_3 of the mid-block attention), the pyramid heads of the 8 x 16 / 4 x 8 /
16 x 32 levels (option head_small), the time-embedding MLP + Dense_0 table, the 4-channel pyramid FIRs
and the level-4 attention.  HIP events on the launch stream, mean of `reps` back-to-back launches.
Usage: python tools/tail_bench.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))
import torch  # noqa: E402

from snrse import ops  # noqa: E402


def timed(run, reps):
    run()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main(reps=50):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    ops.context(dev)  # this thread's launch context (with its split-K workspace, as the network runs)
    B = 32
    # 1x1 GEMM + statistics on the 4 x 8 level (wave tiles spanning two images)
    for (H, W, Cin) in [(4, 8, 256), (8, 16, 256)]:
        x = torch.randn(B, H, W, Cin, device=dev, generator=g).bfloat16()
        w = (torch.randn(256, Cin, device=dev, generator=g) * 0.05).bfloat16()
        bias = torch.randn(256, device=dev, generator=g)
        res = torch.randn(B, H, W, 256, device=dev, generator=g).bfloat16()

        def run():
            st = ops.new_stats(B, 256)
            ops.conv2d(x, w, 1, 256, bias=bias, res=res, out_scale=0.7071, stats=st)
        us = timed(run, reps)
        emit(op="conv1x1_stats", shape=[B, H, W, Cin], kernel=ops.kernel_name(ops.get_option("last_kernel")),
             ksplit=ops.get_option("last_ksplit"), us=us)
    # pyramid heads (GroupNorm + SiLU fused where the kernel takes it)
    for (H, W) in [(4, 8), (8, 16), (16, 32)]:
        C = 256
        x = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
        w = (torch.randn(4, 9 * C, device=dev, generator=g) * 0.05).bfloat16()
        wp = torch.cat([w, w.new_zeros(12, 9 * C)], 0).contiguous()
        bias = torch.randn(4, device=dev, generator=g)
        res = torch.randn(B, H, W, 4, device=dev, generator=g)
        sums, _ = ops.gn_stats(x)
        gam, bet = torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g) * 0.2
        for hs in (0, 1, 2):
            ops.set_option("head_small", hs)
            try:
                if ops.head_ok(x):
                    def run():
                        gn = ops.gn_scale_shift(sums, gam, bet, H * W)
                        ops.conv2d(x, wp, 3, 4, bias=bias, res=res, out_f32=True, gn=gn)
                else:
                    def run():
                        a = ops.gn_apply(x, None, sums, gam, bet, act=True)
                        ops.conv2d(a, wp, 3, 4, bias=bias, res=res, out_f32=True)
                us = timed(run, reps)
                emit(op="pyramid_head(+gn)", shape=[B, H, W, C], head_small=hs,
                     kernel=ops.kernel_name(ops.get_option("last_kernel")), us=us)
            finally:
                ops.set_option("head_small", 1)
    # time embedding: MLP + all Dense_0 rows (R = 10880 for the shipped NCSN++)
    t = torch.rand(B, device=dev, generator=g) * 0.9 + 0.05
    Wg = torch.randn(128, device=dev, generator=g) * 16
    W1, b1 = torch.randn(512, 256, device=dev, generator=g) * 0.05, torch.randn(512, device=dev, generator=g)
    W2, b2 = torch.randn(512, 512, device=dev, generator=g) * 0.05, torch.randn(512, device=dev, generator=g)
    Wd, bd = torch.randn(10880, 512, device=dev, generator=g) * 0.05, torch.randn(10880, device=dev, generator=g)
    te = ops.temb_mlp(t, Wg, W1, b1, W2, b2)
    emit(op="temb_mlp", B=B, us=timed(lambda: ops.temb_mlp(t, Wg, W1, b1, W2, b2), reps))
    emit(op="temb_dense", B=B, R=10880, us=timed(lambda: ops.temb_dense(te, Wd, bd), reps))
    # exactness vs fp64 torch
    e = torch.log(t)[:, None] * Wg[None, :] * 2 * torch.pi
    emb = torch.cat([torch.sin(e), torch.cos(e)], 1).double()
    ref = torch.nn.functional.silu(emb @ W1.double().t() + b1.double()) @ W2.double().t() + b2.double()
    refd = torch.nn.functional.silu(ref) @ Wd.double().t() + bd.double()
    dn = ops.temb_dense(te, Wd, bd)
    emit(op="temb_check", mlp_max_abs=float((te.double() - ref).abs().max()),
         dense_max_abs=float((dn.double() - refd).abs().max()), dense_ref_rms=float(refd.pow(2).mean().sqrt()))
    # 4-channel f32 pyramid FIRs, every level transition
    for (H, W) in [(256, 512), (128, 256), (64, 128), (32, 64), (16, 32), (8, 16)]:
        p = torch.randn(B, H, W, 4, device=dev, generator=g)
        emit(op="fir_down", shape=[B, H, W, 4], us=timed(lambda: ops.fir(p, "down"), reps))
        q = torch.randn(B, H // 2, W // 2, 4, device=dev, generator=g)
        emit(op="fir_up", shape=[B, H // 2, W // 2, 4], us=timed(lambda: ops.fir(q, "up"), reps))
    # attention (level 4: L = 512; mid block: L = 32)
    for L in (512, 32):
        qkv = torch.randn(B, L, 768, device=dev, generator=g).bfloat16()
        emit(op="attention", B=B, L=L, us=timed(lambda: ops.attention(qkv, 256), reps))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)

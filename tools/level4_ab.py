#!/usr/bin/env python3
"""Low-resolution ResBlock convs: the halo GEMM with the fused GroupNorm+SiLU (8 x 32 tiles) against the
LDS-DMA GEMM path it replaces there (gn_act pass + conv_glds_kernel with split-K + finalize).  HIP events on
the launch stream, median of --reps, interleaved rounds.  Usage: python tools/level4_ab.py [--reps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))

import torch  # noqa: E402

from snrse import ops  # noqa: E402

# (B, C0, C1, Cout, H, W): level 4 (16 x 32) Conv_0 / Conv_1, up-path cat Conv_0, level 3 for reference
SHAPES = [(32, 256, 0, 256, 16, 32), (32, 256, 256, 256, 16, 32), (32, 256, 0, 256, 32, 64)]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for B, C0, C1, Co, H, W in SHAPES:
        x0 = torch.randn(B, H, W, C0, device=dev, generator=g).bfloat16()
        x1 = torch.randn(B, H, W, C1, device=dev, generator=g).bfloat16() if C1 else None
        w = (torch.randn(Co, 9 * (C0 + C1), device=dev, generator=g) / 40).bfloat16()
        bias = torch.zeros(Co, device=dev)
        sc = torch.rand(B, C0 + C1, device=dev, generator=g) + 0.5
        sh = torch.randn(B, C0 + C1, device=dev, generator=g)
        st = ops.new_stats(B, Co)
        row = {"shape": [B, C0, C1, Co, H, W]}

        def halo():
            ops.set_option("conv_variant", 0)
            return ops.conv2d(x0, w, 3, Co, bias=bias, src1=x1, stats=st, gn=(sc, sh))

        def glds():
            act = ops.gn_act(x0, x1, sc, sh)
            ops.set_option("conv_variant", 2)
            return ops.conv2d(act, w, 3, Co, bias=bias, stats=st)

        for r in range(a.rounds):
            for name, fn in (("halo", halo), ("glds", glds)):
                ms = timed(fn, a.reps)
                row[f"{name}_us"] = min(ms * 1e3, row.get(f"{name}_us", 1e30))
        ops.set_option("conv_variant", 0)
        d = (halo().float() - glds().float()).abs().max().item()
        ops.set_option("conv_variant", 0)
        row["max_abs_diff"] = d
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

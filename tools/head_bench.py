#!/usr/bin/env python3
"""Micro-benchmark of the bf16 pyramid heads (conv_head_part_kernel / conv_head_kernel, option head_part: GroupNorm+SiLU fused 3x3 conv C -> 4, f32 output + the
upsampled pyramid residual, ncsnpp.py:345-366) on the C2 level shapes; HIP events on the launch stream.  Bytes per
launch: the bf16 input once + 16 B read (residual) + 16 B written per pixel.  Usage: python tools/head_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))
import torch  # noqa: E402

from snrse import ops  # noqa: E402

SHAPES = [(32, 256, 512, 128), (32, 128, 256, 128), (32, 64, 128, 256)]


def main(reps=20):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for B, H, W, C in SHAPES:
        x = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
        w = (torch.randn(4, 9 * C, device=dev, generator=g) * 0.05).bfloat16()
        wp = torch.cat([w, w.new_zeros(12, 9 * C)], 0).contiguous()
        bias = torch.randn(4, device=dev, generator=g)
        res = torch.randn(B, H, W, 4, device=dev, generator=g)
        sums, _ = ops.gn_stats(x)
        gn = ops.gn_scale_shift(sums, torch.rand(C, device=dev, generator=g) + 0.5,
                                torch.randn(C, device=dev, generator=g) * 0.2, H * W)
        run = lambda: ops.conv2d(x, wp, 3, 4, bias=bias, res=res, out_f32=True, gn=gn)  # noqa: E731
        outs = {}
        for rnd in range(2):  # interleaved rounds of the two head forms (option head_part)
            for part in (1, 0):
                ops.set_option("head_part", part)
                outs[part] = run()
                kern = ops.kernel_name(ops.get_option("last_kernel"))
                s = torch.cuda.current_stream()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(reps):
                    run()
                e1.record(s)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / reps * 1e3
                nbytes = B * H * W * (2 * C + 32)
                print(json.dumps({"shape": [B, H, W, C], "round": rnd, "head_part": part, "kernel": kern, "us": us,
                                  "TBps": nbytes / us / 1e6, "frac_of_8TBps": nbytes / us / 1e6 / 8}), flush=True)
        ops.set_option("head_part", 1)
        d = (outs[1] - outs[0]).abs().max().item() / outs[0].abs().max().item()
        print(json.dumps({"shape": [B, H, W, C], "part_vs_taps_max_rel": d}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A/B of the bf16 input conv forms (option ic_lds: 1 = input rows staged in LDS, 2 = the same with the channels split over wave pairs,
0 = streaming neighbour loads) on
the C2 shape [32, 256, 512] (HIP events on the launch stream, interleaved).  HBM bytes per launch: 16 B read + 256 B
(h) + 16 B (pyramid) written per pixel.  Usage: python tools/ic_bench.py [--reps 20] [--rounds 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))
import torch  # noqa: E402

from snrse import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shape", default="32,256,512")
    a = ap.parse_args()
    B, F, T = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.complex(torch.randn(B, F, T, device=dev, generator=g), torch.randn(B, F, T, device=dev, generator=g))
    y = torch.complex(torch.randn(B, F, T, device=dev, generator=g), torch.randn(B, F, T, device=dev, generator=g))
    wp = torch.cat([torch.randn(128, 36, device=dev, generator=g) / 6, torch.zeros(128, 28, device=dev)], 1)
    wp = wp.bfloat16().contiguous()
    bias = torch.randn(128, device=dev, generator=g) * 0.1
    nbytes = B * F * T * (16 + 256 + 16)
    for r in range(a.rounds):
        for v in (0, 1, 2, 3):
            ops.set_option("ic_lds", v)
            ops.input_conv(x, y, wp, bias)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                ops.input_conv(x, y, wp, bias)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            print(json.dumps({"round": r, "ic_lds": v, "shape": [B, F, T], "us": ms * 1e3,
                              "TBps": nbytes / ms / 1e9, "frac_of_8TBps": nbytes / ms / 1e9 / 8}), flush=True)
    ops.set_option("ic_lds", 3)


if __name__ == "__main__":
    main()

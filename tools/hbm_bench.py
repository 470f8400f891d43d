#!/usr/bin/env python3
"""Micro-benchmark of the HBM-bound kernels of one NCSN++ evaluation at the C2 shapes (B=32, 4 s):
gn_resample down / up at every level, the fused input conv, gn_act.  HIP events on the launch stream,
median of --reps; achieved = algorithmic bytes (each tensor read or written once) / time.
Usage: python tools/hbm_bench.py [--reps 20] [--only down,up,input,act,head,copy] [--levels 0,1]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))

import torch  # noqa: E402

from snrse import ops  # noqa: E402

B = 32
LEVELS = [(256, 512, 128), (128, 256, 128), (64, 128, 256), (32, 64, 256), (16, 32, 256), (8, 16, 256), (4, 8, 256)]


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
    ap.add_argument("--only", default="down,up,input,act")
    ap.add_argument("--resample-variant", type=int, default=0)
    ap.add_argument("--nt", type=int, default=0)
    ap.add_argument("--down-rows", type=int, default=4, help="option resample_down_rows (1, 2, 4)")
    ap.add_argument("--levels", default="", help="comma list of pyramid levels for down / up / head (default all)")
    a = ap.parse_args()
    ops.set_option("resample_down_rows", a.down_rows)
    ops.set_option("resample_variant", a.resample_variant)
    ops.set_option("resample_nt", a.nt)
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    only = a.only.split(",")
    rows = []
    tot = {}
    for kind in ("down", "up"):
        if kind not in only:
            continue
        lv = range(0, 6) if kind == "down" else range(1, 7)
        if a.levels:
            lv = [int(v) for v in a.levels.split(",") if int(v) in lv]
        for li in lv:
            H, W, C = LEVELS[li]
            x = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
            sc = torch.rand(B, C, device=dev, generator=g) + 0.5
            sh = torch.randn(B, C, device=dev, generator=g)
            ms = timed(lambda: ops.gn_resample(x, sc, sh, act=True, mode=kind, want_raw=True), a.reps)
            f = 0.25 if kind == "down" else 4.0
            byt = x.numel() * 2 * (1 + 2 * f)
            rows.append({"kernel": f"gn_resample_{kind}", "variant": a.resample_variant, "down_rows": a.down_rows, "shape": [B, H, W, C], "us": ms * 1e3,
                         "bytes": byt, "TBps": byt / ms / 1e9})
            tot.setdefault(kind, [0.0, 0.0])
            tot[kind][0] += byt
            tot[kind][1] += ms
            del x
    if "copy" in only:  # achievable-rate references: torch copy (read + write) and fill (write only)
        x = torch.randn(B, 256, 512, 128, device=dev, generator=g).bfloat16()
        y = torch.empty_like(x)
        ms = timed(lambda: y.copy_(x), a.reps)
        rows.append({"kernel": "torch_copy", "shape": list(x.shape), "us": ms * 1e3, "bytes": 2 * x.numel() * 2,
                     "TBps": 4 * x.numel() / ms / 1e9})
        ms = timed(lambda: y.fill_(1.0), a.reps)
        rows.append({"kernel": "torch_fill", "shape": list(x.shape), "us": ms * 1e3, "bytes": x.numel() * 2,
                     "TBps": 2 * x.numel() / ms / 1e9})
        del x, y
    if "input" in only:
        from snrse import ncsnpp  # noqa: F401
        F, T = 256, 512
        x = torch.randn(B, F, T, dtype=torch.complex64, device=dev)
        y = torch.randn(B, F, T, dtype=torch.complex64, device=dev)
        w = (torch.randn(128, 64, device=dev) / 8).bfloat16()
        bias = torch.zeros(128, device=dev)
        ms = timed(lambda: ops.input_conv(x, y, w, bias), a.reps)
        byt = B * F * T * (16 + 256 + 16)  # x, y read; h bf16 + pyramid f32 written
        rows.append({"kernel": "input_conv", "shape": [B, F, T], "us": ms * 1e3, "bytes": byt,
                     "TBps": byt / ms / 1e9})
    if "head" in only:  # level pyramid head: SiLU(GN(h)) -> conv3x3 C -> 4 (f32) + upsampled pyramid
        for li in ([int(v) for v in a.levels.split(",")] if a.levels else range(0, 4)):
            H, W, C = LEVELS[li]
            x = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
            sc = torch.rand(B, C, device=dev, generator=g) + 0.5
            sh = torch.randn(B, C, device=dev, generator=g)
            w = (torch.randn(16, 9 * C, device=dev, generator=g) / 48).bfloat16()
            w[4:] = 0
            bias = torch.zeros(4, device=dev)
            r = torch.randn(B, H, W, 4, device=dev, generator=g)
            assert ops.head_ok(x)
            ms = timed(lambda: ops.conv2d(x, w, 3, 4, bias=bias, res=r, out_f32=True, gn=(sc, sh)), a.reps)
            byt = x.numel() * 2 + 2 * r.numel() * 4
            rows.append({"kernel": "conv_head_gn", "shape": [B, H, W, C], "us": ms * 1e3, "bytes": byt,
                         "TBps": byt / ms / 1e9})
            del x, r
    if "act" in only:
        for li in (4, 5, 6):
            H, W, C = LEVELS[li]
            x0 = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
            x1 = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
            sc = torch.rand(B, 2 * C, device=dev, generator=g) + 0.5
            sh = torch.randn(B, 2 * C, device=dev, generator=g)
            ms = timed(lambda: ops.gn_act(x0, x1, sc, sh), a.reps)
            byt = 4 * x0.numel() * 2
            rows.append({"kernel": "gn_act", "shape": [B, H, W, 2 * C], "us": ms * 1e3, "bytes": byt,
                         "TBps": byt / ms / 1e9})
    for r in rows:
        print(json.dumps(r), flush=True)
    for k, (byt, ms) in tot.items():
        print(json.dumps({"kernel": f"gn_resample_{k}", "variant": a.resample_variant, "all_levels_us": ms * 1e3, "bytes": byt,
                          "TBps": byt / ms / 1e9}), flush=True)


if __name__ == "__main__":
    main()

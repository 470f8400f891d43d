"""Micro-bench of the split-bf16 fp32 GEMM (conv_x3_kernel) on the C2 NCSN++ conv shapes, per x3_tile
option, against the exact-fp32 kernel: HIP events, median of --reps.  GPU only.
Output: one JSON line per (shape, variant) with ms and fp32-equivalent TFLOP/s."""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snr-aligned_diffse_amd")]
from snrse import ops  # noqa: E402

# (B, C0, C1, Cout, H, W) of the C2 levels 0-3 (Appendix B of SURVEY.md)
SHAPES = [(32, 128, 0, 128, 256, 512), (32, 128, 128, 128, 256, 512), (32, 128, 0, 128, 128, 256),
          (32, 256, 0, 256, 64, 128), (32, 256, 256, 256, 64, 128), (32, 256, 0, 256, 32, 64)]


def time_call(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="0,1,3")
    ap.add_argument("--exact", type=int, default=1)
    ap.add_argument("--gn", type=int, default=0, help="1: fused GroupNorm+SiLU on the x3h variants (x3_tile 0)")
    ap.add_argument("--spread", default="2", help="x3_spread settings to run each split variant with")
    ap.add_argument("--shapes", default="", help="comma list of SHAPES indices (default all)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    sel = [SHAPES[int(i)] for i in args.shapes.split(",")] if args.shapes else SHAPES
    for B, C0, C1, Co, H, W in sel:
        x0 = torch.randn(B, H, W, C0, device=dev, generator=g)
        x1 = torch.randn(B, H, W, C1, device=dev, generator=g) if C1 else None
        w = torch.randn(Co, 9 * (C0 + C1), device=dev, generator=g) / math.sqrt(9 * (C0 + C1))
        ws = ops.split_weight(w)
        b = torch.randn(Co, device=dev, generator=g)
        out = torch.empty(B, H, W, Co, device=dev)
        st = ops.new_stats(B, Co)
        flops = 2.0 * B * H * W * Co * 9 * (C0 + C1)
        spreads = list(map(int, args.spread.split(",")))
        variants = [("x3", t, sp) for t in map(int, args.tiles.split(",")) for sp in spreads]
        variants += [("exact", 0, 0)] if args.exact else []
        gn = None
        if args.gn:
            sc = torch.rand(B, C0 + C1, device=dev, generator=g) + 0.5
            gn = (sc, torch.randn(B, C0 + C1, device=dev, generator=g) * 0.1)
            variants = [("x3gn", 0, sp) for sp in spreads] + variants
        ref = None
        for kind, t, sp in variants:
            ops.set_option("x3_tile", t)
            ops.set_option("x3_spread", sp)
            wt = w if kind == "exact" else ws
            kw = {"gn": gn} if kind.startswith("x3gn") else {}
            fn = lambda: ops.conv2d(x0, wt, 3, Co, bias=b, src1=x1, out=out, stats=st, **kw)  # noqa: E731
            ms = time_call(fn, args.reps)
            fn()
            torch.cuda.synchronize()
            o = out.clone() if ref is None else out
            if ref is None:
                ref = o
            err = float((o - ref).pow(2).mean().sqrt() / ref.pow(2).mean().sqrt())
            print(json.dumps({"shape": [B, C0, C1, Co, H, W], "kind": kind, "tile": t, "spread": sp, "ms": ms,
                              "tflops": flops / ms / 1e9, "kernel": ops.kernel_name(ops.get_option("last_kernel")),
                              "ksplit": ops.get_option("last_ksplit"), "rel_vs_first": err}), flush=True)
        ops.set_option("x3_tile", 0)
        ops.set_option("x3_spread", 2)
        del x0, x1, out, ref


if __name__ == "__main__":
    main()

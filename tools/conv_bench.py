#!/usr/bin/env python3
"""Micro-benchmark of the conv GEMM variants on the NCSN++ shapes (interleaved A/B in one
process, HIP events on the launch stream).  Usage: python tools/conv_bench.py [--reps 10]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))

import torch  # noqa: E402

from snrse import ops  # noqa: E402

DT = torch.float16  # the 16-bit format (--dtype)

# (B, C0, C1, Cout, H, W, ksize, Csc) — the dominant per-NFE shapes at 4 s
SHAPES = [
    (32, 128, 0, 128, 256, 512, 3, 0),
    (32, 128, 128, 128, 256, 512, 3, 0),   # up-path cat Conv_0
    (32, 128, 0, 128, 256, 512, 3, 128),   # Conv_1 + 1x1 shortcut (Cin != Cout block)
    (32, 256, 0, 256, 128, 256, 3, 0),
    (32, 256, 0, 256, 64, 128, 3, 0),
    (32, 256, 256, 256, 32, 64, 3, 0),
    (32, 256, 0, 768, 16, 32, 1, 0),
    (32, 128, 0, 128, 256, 512, 3, 256),   # 7: up-path Conv_1 at level 0: shortcut over cat(h, skip) = 256 channels
    (32, 256, 0, 256, 128, 256, 3, 512),   # 8: the same at level 1
    (32, 128, 0, 128, 128, 256, 3, 256),   # 9: level-1 up-path Conv_1 (RB 67-68: 128 couts, cat shortcut)
    (32, 256, 0, 256, 128, 256, 3, 256),   # 10: RB 65 Conv_1 (up-sampling block: FIR'd shortcut, Csc = Cin)
    (32, 256, 0, 256, 64, 128, 3, 512),    # 11: level-2 up-path Conv_1 (RB 60-61)
]


def _gn_pair(B, C, dev, g):
    """(scale, shift) views of one [2, B, C] tensor, the layout ops.gn_scale_shift returns."""
    ss = torch.empty(2, B, C, device=dev)
    ss[0] = torch.rand(B, C, device=dev, generator=g) + 0.5
    ss[1] = torch.randn(B, C, device=dev, generator=g)
    return ss[0], ss[1]


def run(shape, variant, reps, dev, gn=False, opt=None):
    B, C0, C1, Co, H, W, k, Csc = shape
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(B, H, W, C0, device=dev, generator=g).to(DT)
    x1 = torch.randn(B, H, W, C1, device=dev, generator=g).to(DT) if C1 else None
    sc = torch.randn(B, H, W, Csc, device=dev, generator=g).to(DT) if Csc else None
    w = (torch.randn(Co, k * k * (C0 + C1), device=dev, generator=g) / 30).to(DT)
    ws = (torch.randn(Co, Csc, device=dev, generator=g) / 16).to(DT) if Csc else None
    bias = torch.zeros(Co, device=dev)
    st = ops.new_stats(B, Co)
    gnp = None
    if gn and k == 3:
        gnp = _gn_pair(B, C0 + C1, dev, g)
    if opt:
        ops.set_option(opt[0], opt[1])
    else:
        ops.set_option("conv_variant", variant)
    out = ops.conv2d(x0, w, k, Co, bias=bias, src1=x1, sc=sc, sc_wgt=ws, stats=st, gn=gnp)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.conv2d(x0, w, k, Co, bias=bias, src1=x1, sc=sc, sc_wgt=ws, out=out, stats=st, gn=gnp)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    fl = 2.0 * B * H * W * Co * (k * k * (C0 + C1) + Csc)
    return out, ts[len(ts) // 2], fl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="5")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--shapes", default="", help="comma list of SHAPES indices (default all)")
    ap.add_argument("--gn", action="store_true", help="fused GroupNorm+SiLU prologue (halo kernels)")
    ap.add_argument("--option", default="", help="A/B an option instead of conv_variant: --variants are its values")
    ap.add_argument("--dtype", default="fp16", choices=("fp16", "bf16"))
    a = ap.parse_args()
    global DT
    DT = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    dev = torch.device("cuda")
    res = []
    sel = [SHAPES[int(i)] for i in a.shapes.split(",")] if a.shapes else SHAPES
    for sh in sel:
        outs = {}
        row = {"shape": sh}
        for rnd in range(a.rounds):  # interleaved A/B rounds: clocks drift between launches
            for v in [int(x) for x in a.variants.split(",")]:
                out, ms, fl = run(sh, v, a.reps, dev, gn=a.gn, opt=(a.option, v) if a.option else None)
                outs[v] = out.float()
                ms = min(ms, row.get(f"v{v}_ms", ms))
                row[f"v{v}_ms"] = ms
                row[f"v{v}_tflops"] = fl / ms / 1e9
        if len(outs) > 1:
            ks = list(outs)
            d = (outs[ks[0]] - outs[ks[1]]).abs().max().item()
            row["max_abs_diff"] = d
        res.append(row)
        if a.option:
            row["option"] = a.option
        print(json.dumps(row), flush=True)
    ops.set_option("conv_variant", 0)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Interval timeline of the ping-pong halo GEMM (csrc/conv_pp.hip) from the -DSNRSE_STAMPS build.

  python tools/pp_stamps.py --build        # here: lib/var_ppstamps/libsnrse_hip.so
  python tools/pp_stamps.py [--tpw 4]      # on the GPU box: per sub-phase work / barrier-wait cycles

Every wave stamps s_memtime before each sub-phase wait and after its barrier.  A wave's interval
sequence is known (half 1 starts with one idle interval; per tile and chunk V then M; the last tile's
epilogue V; idle padding), so each sub-phase's work (previous barrier exit -> next wait start) and wait
(wait start -> barrier exit) is attributed to M / V / V-with-epilogue.  Stamps serialize the waves
around them: read the shares, not the lengths."""
import argparse
import ctypes
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "snr-aligned_diffse_amd")
sys.path.insert(0, PKG)
LIB = os.path.join(PKG, "lib", "var_ppstamps", "libsnrse_hip.so")


def kinds(half, nh, C, K):
    seq = ["idle"] if half else []
    for tl in range(nh):
        for c in range(C):
            seq.append("Vepi" if (c == 0 and tl > 0) else "V")
            seq.append("M")
    if nh:
        seq.append("Vend")
    seq += ["idle"] * (K - len(seq))
    return seq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--tpw", type=int, default=4)
    ap.add_argument("--B", type=int, default=32)
    a = ap.parse_args()
    if a.build:
        from snrse.build import build_library
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        print(build_library(force=True, extra_flags=("-DSNRSE_STAMPS",), lib=LIB))
        return
    os.environ["SNRSE_LIB"] = LIB
    import numpy as np
    import torch
    from snrse import _lib, ops
    dev = torch.device("cuda")
    B, H, W, C = a.B, 256, 512, 128
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, H, W, C, device=dev, generator=g).bfloat16()
    w = (torch.randn(C, 9 * C, device=dev, generator=g) / 34).bfloat16()
    bias = torch.zeros(C, device=dev)
    ss = torch.empty(2, B, C, device=dev)
    ss[0] = 1.0
    ss[1] = 0.1
    temb = torch.randn(B, C, device=dev, generator=g)
    tiles = B * (H // 4) * (W // 64)
    nblk = (tiles + 2 * a.tpw - 1) // (2 * a.tpw)
    buf = torch.zeros(nblk * 8 * 256, dtype=torch.int64, device=dev)
    lib = _lib.load()
    lib.snrse_debug_set_stamps.argtypes = [ctypes.c_void_p]
    lib.snrse_debug_set_stamps(buf.data_ptr())
    ops.set_option("conv_variant", 6)
    ops.set_option("pp_tiles", a.tpw)
    st = ops.new_stats(B, C)
    for _ in range(3):
        ops.conv2d(x, w, 3, C, bias=bias, temb=temb, stats=st, gn=(ss[0], ss[1]))
    torch.cuda.synchronize()
    s = buf.view(nblk, 8, 256).cpu().numpy().astype(np.int64)
    Cc = C // 32
    K = max(2 * Cc * ((2 * a.tpw + 1) // 2) + 1, 2 * Cc * (2 * a.tpw // 2) + 2)
    acc = {}
    for blk in range(1, nblk - 1):  # full blocks only
        for wv in range(8):
            half = wv >> 2
            seq = kinds(half, a.tpw, Cc, K)
            st_ = s[blk, wv]
            for k, kind in enumerate(seq):
                for sp in range(3):
                    i = 2 * (3 * k + sp)  # st[i]: wait start, st[i + 1]: barrier exit of sub-phase (k, sp)
                    if i + 2 >= 256 or st_[i + 2] == 0:
                        continue
                    wait = st_[i + 1] - st_[i]
                    work = st_[i + 2] - st_[i + 1]
                    key = (half, kind, sp)
                    d = acc.setdefault(key, [0, 0.0, 0.0])
                    d[0] += 1
                    d[1] += work
                    d[2] += wait
    rows = []
    for (half, kind, sp), (n, wk, wt) in sorted(acc.items()):
        rows.append({"half": half, "interval": kind, "subphase": sp, "n": n, "work_cyc": round(wk / n),
                     "wait_cyc": round(wt / n)})
    tot = {}
    for r in rows:
        t = tot.setdefault((r["half"], r["interval"]), [0, 0])
        t[0] += r["work_cyc"]
        t[1] += r["wait_cyc"]
    out = {"shape": [B, H, W, C], "tpw": a.tpw, "rows": rows,
           "per_interval": {f"h{h}_{k}": {"work": v[0], "wait": v[1]} for (h, k), v in tot.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Segment timeline of the halo conv kernel from the -DSNRSE_STAMPS diagnostic build.

  python tools/conv_stamps.py --build          # here: builds lib/stamps/libsnrse_hip.so
  python tools/conv_stamps.py [--shape 0]      # on the GPU box: prints per-segment shares

Each wave records s_memtime at: kernel start (0), prologue done (1), per phase q the end of
the phase-start wait+barrier (2+2q) and the end of its MFMA section (3+2q), epilogue start
(28) and end (29).  The stamp build's run time is not the product's (stamps fence overlaps):
read shares, not lengths.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "snr-aligned_diffse_amd")
sys.path.insert(0, PKG)
STAMP_LIB = os.path.join(PKG, "lib", "stamps", "libsnrse_hip.so")


def _gn_pair(B, C, dev, g):
    """(scale, shift) views of one [2, B, C] tensor, the layout ops.gn_scale_shift returns."""
    import torch
    ss = torch.empty(2, B, C, device=dev)
    ss[0] = torch.rand(B, C, device=dev, generator=g) + 0.5
    ss[1] = torch.randn(B, C, device=dev, generator=g)
    return ss[0], ss[1]


PHASE_LIB = os.path.join(PKG, "lib", "stamps_phase", "libsnrse_hip.so")


def build():
    from snrse import build as b
    for lib, flags in ((STAMP_LIB, ("-DSNRSE_STAMPS",)), (PHASE_LIB, ("-DSNRSE_STAMPS", "-DSNRSE_STAMPS_PHASE"))):
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        print(b.build_library(force=True, extra_flags=flags, lib=lib))


def v8_phase_report(s, shape, ms):
    """v8 phase stamps (-DSNRSE_STAMPS_PHASE): chunk 1 of each workgroup's first tile, taps 0..5:
    2+4t L start, 3+4t L end (before barrier 1), 4+4t after barrier 1, 5+4t M end; per wave group."""
    import numpy as np
    s = s[:, :8]
    s = s[s[:, 0, 29] != 0]
    out = {"shape": shape, "variant": 8, "ms": ms, "phase_stamps": True}
    for gname, ws in (("waves0-3", slice(0, 4)), ("waves4-7", slice(4, 8))):
        g = s[:, ws]
        rows = []
        for t in range(6):
            L = (g[:, :, 3 + 4 * t] - g[:, :, 2 + 4 * t]).mean()
            b1 = (g[:, :, 4 + 4 * t] - g[:, :, 3 + 4 * t]).mean()
            M = (g[:, :, 5 + 4 * t] - g[:, :, 4 + 4 * t]).mean()
            b2 = (g[:, :, 2 + 4 * (t + 1)] - g[:, :, 5 + 4 * t]).mean() if t < 5 else float("nan")
            rows.append({"tap": t, "L": round(float(L)), "wait_b1": round(float(b1)), "M": round(float(M)),
                         "wait_b2": round(float(b2)) if t < 5 else None})
        out[gname] = rows
    return out


def v6_report(s, shape, ms, nw=4, variant=6):
    """v6 / v8 stamps: 0 start, 1 prologue done, 2+2t / 3+2t epilogue start / end of local tile t
    (t < 13), 28 loop end, 29 kernel end; nw waves per workgroup (v6: 4, v8: 8)."""
    import numpy as np
    s = s[:, :nw]
    s = s[s[:, 0, 29] != 0]
    rel = s - s[:, :, :1]
    out = {"shape": shape, "variant": variant, "ms": ms, "workgroups": int(s.shape[0]),
           "wave_total_mean": float(rel[:, :, 29].mean()), "prologue": float(rel[:, :, 1].mean())}
    mains, epis = [], []
    prev = rel[:, :, 1]
    for t in range(13):
        st, en = rel[:, :, 2 + 2 * t], rel[:, :, 3 + 2 * t]
        ok = en > 0
        if not ok.any():
            break
        mains.append(float((st - prev)[ok].mean()))
        epis.append(float((en - st)[ok].mean()))
        prev = np.where(ok, en, prev)
    out["tile_main"] = [round(x) for x in mains]
    out["tile_epilogue"] = [round(x) for x in epis]
    out["tail"] = float((rel[:, :, 29] - rel[:, :, 28]).mean())
    cu = (s[:, 0, 31] << 16) | (s[:, 0, 30] & 0xFF00)
    out["workgroups_per_cu"] = float(s.shape[0] / len(np.unique(cu)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--shapes", default="0")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--stats", default="1", help="comma list of 0/1: fuse GN statistics")
    ap.add_argument("--gn", action="store_true", help="fused GroupNorm+SiLU prologue")
    ap.add_argument("--phase", action="store_true", help="v8 phase-level stamp build")
    a = ap.parse_args()
    if a.build:
        return build()
    os.environ["SNRSE_LIB"] = PHASE_LIB if a.phase else STAMP_LIB
    import numpy as np
    import torch
    from snrse import _lib, ops
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from conv_bench import SHAPES

    lib = _lib.load()
    lib.snrse_debug_set_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda")
    for si in [int(x) for x in a.shapes.split(",")]:
        B, C0, C1, Co, H, W, k, Csc = SHAPES[si]
        g = torch.Generator(device=dev).manual_seed(0)
        x0 = torch.randn(B, H, W, C0, device=dev, generator=g).bfloat16()
        x1 = torch.randn(B, H, W, C1, device=dev, generator=g).bfloat16() if C1 else None
        sc = torch.randn(B, H, W, Csc, device=dev, generator=g).bfloat16() if Csc else None
        w = (torch.randn(Co, k * k * (C0 + C1), device=dev, generator=g) / 30).bfloat16()
        ws = (torch.randn(Co, Csc, device=dev, generator=g) / 16).bfloat16() if Csc else None
        bias = torch.zeros(Co, device=dev)
        gnp = None
        if a.gn:
            gnp = _gn_pair(B, C0 + C1, dev, g)
        nblk = B * (H // 4) * (W // 64) * (Co // 128)
        nblk = max(nblk, 1024)  # v6 is persistent: gridDim = min(tiles, 2 x CUs)
        buf = torch.zeros(nblk * 8 * 32, dtype=torch.int64, device=dev)
        for v, use_st in [(int(x), int(y)) for x in a.variants.split(",") for y in a.stats.split(",")]:
            ops.set_option("conv_variant", v)
            st = ops.new_stats(B, Co) if use_st else None
            lib.snrse_debug_set_stamps(None)
            out = ops.conv2d(x0, w, k, Co, bias=bias, src1=x1, sc=sc, sc_wgt=ws, stats=st, gn=gnp)
            for _ in range(3):
                ops.conv2d(x0, w, k, Co, bias=bias, src1=x1, sc=sc, sc_wgt=ws, out=out, stats=st, gn=gnp)
            buf.zero_()
            lib.snrse_debug_set_stamps(buf.data_ptr())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.conv2d(x0, w, k, Co, bias=bias, src1=x1, sc=sc, sc_wgt=ws, out=out, stats=st, gn=gnp)
            e1.record()
            torch.cuda.synchronize()
            lib.snrse_debug_set_stamps(None)
            ms = e0.elapsed_time(e1)
            s = buf.view(nblk, 8, 32).cpu().numpy().astype(np.int64)
            if v == 8 and a.phase:
                print(json.dumps(v8_phase_report(s, SHAPES[si], ms)), flush=True)
                continue
            if v in (6, 8):
                print(json.dumps(v6_report(s, SHAPES[si], ms, nw=4 if v == 6 else 8, variant=v)), flush=True)
                continue
            s = s[:, :4] if v == 5 else s  # v5 workgroups have 4 waves
            cin = C0 + C1
            kt = 32 if v == 5 else 64
            nq = 3 * (cin // kt) + (Csc // kt)
            t0 = s[:, :, 0]
            rel = s - t0[:, :, None]
            seg = {"prologue": rel[:, :, 1]}
            prev = rel[:, :, 1]
            waits, comps = [], []
            for q in range(nq):
                waits.append(rel[:, :, 2 + 2 * q] - prev)
                comps.append(rel[:, :, 3 + 2 * q] - rel[:, :, 2 + 2 * q])
                prev = rel[:, :, 3 + 2 * q]
            seg["tail_to_epi"] = rel[:, :, 28] - prev
            seg["epilogue"] = rel[:, :, 29] - rel[:, :, 28]
            if v == 5:  # finer epilogue stamps: 26 after half 0, 27 after half 1 (before the stats flush)
                seg["epi_half0"] = rel[:, :, 26] - rel[:, :, 28]
                seg["epi_half1"] = rel[:, :, 27] - rel[:, :, 26]
                seg["epi_flush_store"] = rel[:, :, 29] - rel[:, :, 27]
            res = {"shape": SHAPES[si], "variant": v, "stats": use_st, "ms": ms, "nq": nq,
                   "wave_total_mean": float(rel[:, :, 29].mean())}
            res.update({k_: float(v_.mean()) for k_, v_ in seg.items()})
            res["wait_per_phase"] = [round(float(x.mean())) for x in waits]
            res["mfma_per_phase"] = [round(float(x.mean())) for x in comps]
            res["wait_per_phase_by_wave"] = [[round(float(x[:, wv].mean())) for wv in range(s.shape[1])] for x in waits[:3]]
            # gaps between consecutive blocks on one CU (dispatch + tail effects)
            hw = s[:, 0, 30]
            xcc = s[:, 0, 31]
            cu = (xcc << 16) | (hw & 0xFF00)
            start, end = s[:, :, 0].min(1), s[:, :, 29].max(1)
            gaps = []
            for key in np.unique(cu)[:64]:
                idx = np.where(cu == key)[0]
                o = idx[np.argsort(start[idx])]
                if len(o) > 1:
                    gaps.extend((start[o[1:]] - end[o[:-1]]).tolist())
            res["block_lifetime_mean"] = float((end - start).mean())
            res["inter_block_gap_median"] = float(np.median(gaps)) if gaps else None
            res["blocks_per_cu_mean"] = float(nblk / len(np.unique(cu)))
            print(json.dumps(res), flush=True)
    ops.set_option("conv_variant", 0)


if __name__ == "__main__":
    main()

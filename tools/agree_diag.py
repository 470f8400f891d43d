#!/usr/bin/env python3
"""Diagnostic of the C2 bf16-vs-fp32x3 agreement (tests/test_gpu_c2_path.py::test_c2_bf16_vs_fp32x3_agreement_at_c2_size):
is a low per-clip SI-SDR a property of the clip (bf16 rounding amplified along its 60-NFE trajectory) or of its batch
position?  Runs the 32 C2 clips through bf16 and fp32x3 in the bench order and rolled by 5 (the Philox draws follow the
batch position, so the roll also changes each clip's noise).  Writes gpurun_out/agree_diag.json.  Usage: python tools/agree_diag.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "snr-aligned_diffse_amd")]
import paritycheck  # noqa: E402
from conftest import formula_sd  # noqa: E402
from snrse import ncsnpp, sampler  # noqa: E402
from snrse.enhance import PCEnhancer  # noqa: E402
from test_gpu_c2_path import _clips  # noqa: E402


def run(y, dt, gemm):
    sd = {k: torch.from_numpy(v) for k, v in formula_sd("ncsnpp").items()}
    net = ncsnpp.NCSNppHIP(sd, dtype=dt, gemm=gemm)
    enh = PCEnhancer(net, sampler.SDESpec("ouve", theta=1.5, sigma_min=0.05, sigma_max=0.5), N=30)
    xh, _ = enh(y, sampler.NoiseSource(seed=7919 + 102))
    out = xh.detach().double().cpu()
    del enh, net
    torch.cuda.empty_cache()
    return out


def main():
    dev = torch.device("cuda:0")
    y, _ = _clips(32, 4.0, 0)
    yg = torch.from_numpy(y).to(dev)
    res = {}
    b, x = run(yg, torch.bfloat16, "exact"), run(yg, torch.float32, "x3")
    res["bench_order"] = paritycheck.waveform_agreement(b, x, per_clip=True)
    perm = torch.roll(torch.arange(32), 5)  # position p holds clip perm[p]
    br, xr = run(yg[perm.to(dev)], torch.bfloat16, "exact"), run(yg[perm.to(dev)], torch.float32, "x3")
    inv = torch.argsort(perm)
    res["rolled_by_5_in_clip_order"] = paritycheck.waveform_agreement(br[inv], xr[inv], per_clip=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "agree_diag.json"), "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res.items():
        if isinstance(v, dict):
            print(k, json.dumps({kk: vv for kk, vv in v.items() if kk != "per_clip"}))
            print("   si_sdr", v["per_clip"]["si_sdr_db"])


if __name__ == "__main__":
    main()

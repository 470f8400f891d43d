#!/usr/bin/env python3
"""Three-way C2 agreement: the benched batch (B = 32 synthetic 4 s clips as bench.py makes them,
N = 30 PC steps = 60 NFE, OUVE, Philox seed 7919 + 102) through the bf16 headline network, the fp32x3 parity mode and
the EXACT fp32 mode (v_mfma_f32_16x16x4_f32 GEMMs, the reference's fp32 network arithmetic: sgmse-bbed/sgmse/model.py:824,
sampling/__init__.py:54-75).  Per clip: SI-SDR of bf16 vs fp32, x3 vs fp32 and bf16 vs x3 (the reference's formula,
sgmse/util/other.py:71-75) and, per network evaluation, the relative RMS distance of the PC state x (complex spectrogram)
from the fp32 run's -- so a low-agreement clip shows which side leaves the fp32 trajectory and at which NFE.  Also pins
the fp32 leg to the reference golden pc_ouve.npz (N = 5).  Writes gpurun_out/agree3.json.
Usage: python tools/agree3.py [--out PATH]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "snr-aligned_diffse_amd")]
import paritycheck  # noqa: E402
from conftest import formula_sd  # noqa: E402
from snrse import ncsnpp, ops, sampler  # noqa: E402
from snrse.enhance import PCEnhancer  # noqa: E402
from test_gpu_c2_path import _clips  # noqa: E402


class RecordingPC(PCEnhancer):
    """PCEnhancer that keeps the PC state x entering every network evaluation (the whole batch, on the device)."""

    def _iter(self, Y, noise):
        net, rec = self.net, self.rec

        def step(x, tv, coef, z, seed, off):
            rec.append(x.detach().clone())
            pyr = net.pyramid(x, Y, tv)
            xo, xm, _ = ops.score_update(pyr, net.W["out_w"], net.W["out_b"], tv, self.score_mode, x, Y,
                                         coef=coef, noise=z, seed=seed, offset=off)
            return xo, xm

        return sampler.pc_sample_iter(step, Y, self.sde, N=self.N, eps=self.eps, snr=self.snr,
                                      predictor=self.predictor, corrector=self.corrector,
                                      corrector_steps=self.corrector_steps, noise=noise)


def run(y, dt, gemm):
    sd = {k: torch.from_numpy(v) for k, v in formula_sd("ncsnpp").items()}
    net = ncsnpp.NCSNppHIP(sd, dtype=dt, gemm=gemm)
    enh = RecordingPC(net, sampler.SDESpec("ouve", theta=1.5, sigma_min=0.05, sigma_max=0.5), N=30)
    enh.rec = []
    t0 = time.time()
    xh, nfe = enh(y, sampler.NoiseSource(seed=7919 + 102))
    torch.cuda.synchronize()
    assert nfe == 60
    states = torch.stack(enh.rec)  # [60, B, F, T] complex64
    out = xh.detach().double().cpu()
    del enh, net
    torch.cuda.empty_cache()
    return out, states, time.time() - t0


def state_dist(a, b):
    """[NFE, B] relative RMS of the state difference a - b against b."""
    d = (a - b).abs().pow(2).mean((2, 3)).sqrt()
    n = b.abs().pow(2).mean((2, 3)).sqrt()
    return (d / n).double().cpu()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "agree3.json"))
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    y, _ = _clips(32, 4.0, 0)
    yg = torch.from_numpy(y).to(dev)
    res = {"config": "C2: B=32 synthetic 4 s clips (bench.py's), N=30 PC (reverse_diffusion + ald, 60 NFE), OUVE, "
                     "formula weights, Philox seed 8021"}
    wav, st, secs = {}, {}, {}
    for name, dt, gemm in (("fp32", torch.float32, "exact"), ("x3", torch.float32, "x3"), ("bf16", torch.bfloat16, "exact")):
        wav[name], st[name], secs[name] = run(yg, dt, gemm)
    res["seconds"] = secs
    for pa, pb in (("bf16", "fp32"), ("x3", "fp32"), ("bf16", "x3")):
        r = paritycheck.waveform_agreement(wav[pa], wav[pb], per_clip=True)
        res[f"{pa}_vs_{pb}"] = r
    dist = {f"{p}_vs_fp32": state_dist(st[p], st["fp32"]) for p in ("bf16", "x3")}
    # per clip: the state distance at NFE 1, 10, 20, ..., 60 and the first NFE where it exceeds 1e-2 / 1e-1
    traj = {}
    for k, d in dist.items():
        rows = []
        for b in range(d.shape[1]):
            col = d[:, b]
            first = {f"first_nfe_gt_{t:g}": (int((col > t).nonzero()[0, 0]) + 1 if bool((col > t).any()) else None)
                     for t in (0.01, 0.1)}
            rows.append({"clip": b, "at_nfe": {str(i): round(float(col[i - 1]), 6) for i in (1, 10, 20, 30, 40, 50, 60)},
                         **first})
        traj[k] = rows
    res["state_rel_rms_vs_fp32"] = traj
    # the fp32 leg against the reference golden (N = 5, injected noise)
    sd = {k: torch.from_numpy(v) for k, v in formula_sd("ncsnpp").items()}
    res["fp32_pc_vs_golden"] = paritycheck.pc_vs_golden(dev, ncsnpp.NCSNppHIP(sd, dtype=torch.float32, gemm="exact"))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    for k in ("bf16_vs_fp32", "x3_vs_fp32", "bf16_vs_x3"):
        v = res[k]
        print(k, json.dumps({kk: vv for kk, vv in v.items() if kk not in ("per_clip", "bounds")}))
        print("   si_sdr", v["per_clip"]["si_sdr_db"])
    print("fp32 vs golden", json.dumps(res["fp32_pc_vs_golden"]))


if __name__ == "__main__":
    main()

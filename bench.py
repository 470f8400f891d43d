#!/usr/bin/env python3
"""Benchmark: utterances/sec of the PC reverse-diffusion enhancement path on MI355X.

One "step" = ScoreModel.enhance() on one batch of B synthetic 4 s / 16 kHz noisy clips:
device STFT + exponent transform -> prior -> N=30 PC steps (reverse_diffusion predictor +
ALD corrector = 60 NCSN++ NFEs, each fused with its SDE update) -> iSTFT.  Inputs are
resident in HBM before the timed region.  Multi-GPU: one process per GPU (torchrun), each
rank enhances its own batch (weak scaling, utterance sharding, no collective in the data
path); RCCL is used for the max-over-ranks time and the final metric gather only.

Prints ONE JSON line (rank 0).  See DESIGN.md §Measurement for the roofline definition.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "utterances/sec (4 s @16 kHz, N=30 PC steps) at 1/2/4/8 MI355X; PESQ delta vs ref"
PEAK = {"bf16": 2.5e15, "fp32": 157.3e12}  # dense MFMA peaks (MI355X_MICROARCH.md)
SR = 16000


def synth_clips(n, seconds, seed0):
    """SURVEY.md §8(d) recipe: harmonic 'speech' + white noise at SNR -5..35 dB, peak 0.9."""
    L = int(seconds * SR)
    t = np.arange(L) / SR
    out = np.empty((n, L), dtype=np.float32)
    snrs = np.arange(-5, 40, 5)
    for i in range(n):
        rng = np.random.Generator(np.random.PCG64(seed0 + i))
        ph = rng.uniform(0, 2 * np.pi, 5)
        c = 0.1 * sum(np.sin(2 * np.pi * f * t + p) for f, p in zip((200, 400, 800, 1600, 3200), ph))
        c = c * (0.5 + 0.5 * np.sin(2 * np.pi * 3 * t))
        nz = rng.standard_normal(L)
        snr = snrs[(seed0 + i) % len(snrs)]
        nz *= np.sqrt(np.mean(c ** 2) / np.mean(nz ** 2) / 10 ** (snr / 10))
        y = c + nz
        out[i] = 0.9 * y / np.abs(y).max()
    return out


def formula_weights():
    from snrse import formula
    with open(os.path.join(ROOT, "tests", "golden", "state_dict_keys.json")) as f:
        shapes = {k: tuple(s) for k, s in json.load(f)["ncsnpp"]}
    return {k: torch.from_numpy(v) for k, v in formula.formula_state_dict(shapes).items()}


def snrnet_formula(dev):
    """SNRNet (sgmse/backbones/snrnet.py) with formula weights of the reference architecture."""
    from snrse import formula
    from sgmse.backbones import SNRNet
    with open(os.path.join(ROOT, "tests", "golden", "state_dict_keys.json")) as f:
        shapes = {"snrnet." + k: tuple(s) for k, s in json.load(f)["snrnet"]}
    sd = {k[len("snrnet."):]: torch.from_numpy(v) for k, v in formula.formula_state_dict(shapes).items()}
    net = SNRNet()
    net.load_state_dict(sd)
    return net


def cpu_baseline(seconds=4.0, nfe=2, threads=None):
    """Oracle (CPU restatement) on a bounded sample: 1 clip, `nfe` NCSN++ evaluations + the
    STFT/iSTFT and SDE updates, extrapolated to 60 NFE per utterance."""
    from oracle import ncsnpp_ref, spec_ref
    threads = threads or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = ncsnpp_ref.state_dict_to_torch({k: v.numpy() for k, v in formula_weights().items()})
    y = synth_clips(1, seconds, 10_000)
    t0 = time.perf_counter()
    Y = spec_ref.spec_fwd(spec_ref.stft(y / np.abs(y).max()))
    Y = torch.from_numpy(spec_ref.pad_spec(Y).astype(np.complex64))[:, None]
    t_front = time.perf_counter() - t0
    x = Y.clone()
    tt = torch.tensor([0.5])
    with torch.no_grad():
        ncsnpp_ref.ncsnpp_forward(torch.cat([x, Y], 1), tt, sd)  # warm-up
        t0 = time.perf_counter()
        for _ in range(nfe):
            s = -ncsnpp_ref.ncsnpp_forward(torch.cat([x, Y], 1), tt, sd)
            x = x + 0.01 * s + 0.01 * torch.randn_like(x)
        t_nfe = (time.perf_counter() - t0) / nfe
    t0 = time.perf_counter()
    spec_ref.istft(spec_ref.spec_back(x[0, 0].numpy()), y.shape[1])
    t_back = time.perf_counter() - t0
    t_utt = 60 * t_nfe + t_front + t_back
    return {"value": 1.0 / t_utt, "unit": "utt/s", "cores": threads, "kind": "port",
            "sample": f"1 synthetic 4 s clip: {nfe} timed NCSN++ fp32 NFEs (+1 warm-up) at [1,2,256,512] "
                      f"+ STFT/iSTFT, extrapolated to 60 NFE/utt ({t_nfe:.2f} s/NFE)"}


def conv_flops(src0, src1, ksize, cout, sc, sc1):
    B, H, W, C0 = src0.shape
    cin = C0 + (0 if src1 is None else src1.shape[3])
    k = ksize * ksize * cin + (0 if sc is None else sc.shape[3]) + (0 if sc1 is None else sc1.shape[3])
    return 2.0 * B * H * W * cout * k


class ConvProbe:
    """HIP events on the launch stream around every halo-path conv launch (bf16 3x3, Cout % 128 == 0,
    H % 4 == 0, W % 64 == 0; ops.halo_ok) during one extra enhance() pass after the timed region,
    grouped by the kernel that ran (snrse_get_option "last_kernel").  achieved = algorithmic FLOPs of
    the dominant kernel's launches / their summed event time, i.e. mean FLOPs per launch / mean
    launch duration (the quantity rocprofv3 --stats reports as AverageNs for that kernel)."""

    def __init__(self):
        self.rec = []

    def install(self, ops):
        orig = ops.conv2d
        probe = self

        def wrapped(src0, wgt, ksize, cout, *a, **kw):
            # bf16: the halo-path convs; fp32 parity mode (C5): every 3x3 conv with Cout >= 64
            big = ops.halo_ok(src0, ksize, cout) or (src0.dtype == torch.float32 and ksize == 3 and cout >= 64)
            if not big:
                return orig(src0, wgt, ksize, cout, *a, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = orig(src0, wgt, ksize, cout, *a, **kw)
            e1.record()
            probe.rec.append((conv_flops(src0, kw.get("src1"), ksize, cout, kw.get("sc"), kw.get("sc1")), e0, e1,
                              ops.kernel_name(ops.get_option("last_kernel"))))
            return out

        ops.conv2d = wrapped
        self.orig, self.ops = orig, ops

    def uninstall(self):
        self.ops.conv2d = self.orig

    def summary(self):
        """{kernel: [flops, ms, launches]} over the probed pass."""
        torch.cuda.synchronize()
        by = {}
        for fl, e0, e1, k in self.rec:
            d = by.setdefault(k, [0.0, 0.0, 0])
            d[0] += fl
            d[1] += e0.elapsed_time(e1)
            d[2] += 1
        return by


def pmc_traffic(kernel_prefix):
    """HBM bytes per launch of the dominant kernel from the committed PMC profile
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py: FETCH_SIZE x 2 per the gfx950
    correction + WRITE_SIZE); None when absent."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("kernel", "").startswith(kernel_prefix):
            return d.get("bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    ap.add_argument("--N", type=int, default=30, help="PC steps")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--conv-variant", type=int, default=0, help="snrse conv_variant option (0 = auto)")
    ap.add_argument("--config", choices=["c2", "c4"], default="c2",
                    help="c2: PC sampler (default, the headline line); c4: one-step SNR-aligned path "
                         "(SNRNet estimate + 1 preconditioned NFE, sebridge_v3)")
    args = ap.parse_args()

    from snrse import dist as sdist
    rank, world, dev = sdist.init_from_env()
    dist = None
    if world > 1:
        import torch.distributed as dist

    from snrse import ncsnpp, ops, sampler
    from snrse.enhance import PCEnhancer

    ops.set_option("conv_variant", args.conv_variant)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    net = ncsnpp.NCSNppHIP(formula_weights(), dtype=dtype, device=dev)
    enh = PCEnhancer(net, sampler.SDESpec("ouve", theta=1.5, sigma_min=0.05, sigma_max=0.5), N=args.N)
    B = args.batch
    y = torch.from_numpy(synth_clips(B, args.seconds, 1000 * rank)).to(dev)
    noise = lambda it: sampler.NoiseSource(seed=7919 * (rank + 1) + it)  # noqa: E731
    if args.config == "c4":
        from snrse.enhance import SNRAlignedEnhancer
        snr_net = snrnet_formula(dev)
        one = SNRAlignedEnhancer(net, snr_fn=lambda spec: (lambda g: g / (1 - g))(snr_net.forward_complex(spec)[:, 0]),
                                 fixed_snr=0.17783, sigma_max=0.5)
        enh = lambda yy, nz: (one(yy, seed=nz.seed)[0], 1)  # noqa: E731

    for w in range(args.warmup):
        enh(y, noise(w))
        if rank == 0:
            print(f"[bench] warmup step {w + 1}/{args.warmup} done", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        xh, nfe = enh(y, noise(100 + k))
        if rank == 0 and args.steps > 1:
            print(f"[bench] step {k + 1}/{args.steps} enqueued", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = sdist.max_over_ranks(time.perf_counter() - t0, dev)
    # per-utterance output RMS of the last step, gathered over RCCL (the one metric gather)
    rms = xh.pow(2).mean(dim=1).sqrt().double().cpu().tolist()
    allm = sdist.gather_metrics(rms, B * world, rank, world, dev)
    value = args.steps * B * world / elapsed

    roof = None
    if not args.no_probe:
        probe = ConvProbe()
        probe.install(ops)
        try:
            enh(y, noise(999))
        finally:
            probe.uninstall()
        by = probe.summary()
        kname = max(by, key=lambda k: by[k][1])  # the halo kernel with the most time in the step
        fl, ms, n = by[kname]
        ach = fl / (ms * 1e-3) if ms > 0 else 0.0
        peak = PEAK[args.dtype]
        traffic, tsrc = pmc_traffic(kname)
        roof = {"bound": "mfma", "achieved": ach / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s",
                "frac": ach / peak, "traffic": traffic, "kernel": kname, "launches_per_step": n,
                "avg_launch_us": ms * 1e3 / max(n, 1), "flop_per_launch": fl / max(n, 1),
                "kernel_ms_per_step": ms, "traffic_source": tsrc,
                "other_halo_kernels": {k: {"launches": v[2], "ms": v[1], "tflops": v[0] / max(v[1], 1e-9) / 1e9}
                                       for k, v in by.items() if k != kname}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        cpu = cpu_baseline()

    n_frames = 1 + int(args.seconds * SR) // 128
    T_frames = (n_frames + 63) // 64 * 64
    cfg = "C4" if args.config == "c4" else "C2" if (args.seconds == 4.0 and args.dtype == "bf16") else (
        "C5" if args.seconds >= 30 and args.dtype == "fp32" else "custom")
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "utt/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (SURVEY §8d harmonic+noise clips; formula weights of the NCSN++ architecture)",
            "config": {"workload": (f"{cfg}: B={B} {args.seconds:g} s/16 kHz clips per GPU, one-step SNR-aligned "
                                    f"enhancement (SNRNet estimate + 1 sebridge_v3 NFE at t_hat), NCSN++ nf=128")
                       if args.config == "c4" else
                       (f"{cfg}: B={B} {args.seconds:g} s/16 kHz clips per GPU, N={args.N} PC steps "
                        f"(reverse_diffusion + ald, {nfe} NFE/utt), OUVE SDE, NCSN++ nf=128"),
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": T_frames,
                       "parallelism": f"dp{world} (utterance sharding)"},
            "roofline": roof, "cpu_baseline": cpu,
            "output_rms_mean": float(allm.mean()),
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

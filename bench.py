#!/usr/bin/env python3
"""Benchmark: utterances/sec of the PC reverse-diffusion enhancement path on MI355X.

One "step" = ScoreModel.enhance() on one batch of B synthetic 4 s / 16 kHz noisy clips:
device STFT + exponent transform -> prior -> N=30 PC steps (reverse_diffusion predictor +
ALD corrector = 60 NCSN++ NFEs, each fused with its SDE update) -> iSTFT.  Inputs are
resident in HBM before the timed region.

Multi-GPU (`--gpus N`): one process per GPU.  Launched by torchrun (RANK / WORLD_SIZE in the
environment) the ranks are torchrun's; otherwise bench.py starts the N ranks itself
(snrse.dist.spawn_ranks, before anything touches the GPU).  Each rank enhances its own batch
(weak scaling, utterance sharding, no collective in the data path); RCCL is used for the
max-over-ranks time and the final metric gather only.

Configs (BASELINE.json): c2 (default, the headline line), c4 (SNR-aligned one-step path),
c5 (30 s clips, N=200, fp32), and `--gpus 0` = c1 (the reference's CPU plumbing case, run by the
CPU oracle: no GPU).  Prints ONE JSON line (rank 0).  See DESIGN.md §4 for the roofline definition.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import math
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "utterances/sec (4 s @16 kHz, N=30 PC steps) at 1/2/4/8 MI355X; PESQ delta vs ref"
PEAK = {"fp16": 2.5e15, "bf16": 2.5e15, "fp32": 157.3e12,  # dense MFMA peaks (MI355X_MICROARCH.md)
        "fp32x3": 2.5e15 / 3}  # split-bf16 fp32 GEMM: three dense bf16 MFMA products per fp32 product
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


def _shapes(kind):
    with open(os.path.join(ROOT, "tests", "golden", "state_dict_keys.json")) as f:
        return json.load(f)[kind]


def formula_weights():
    from snrse import formula
    shapes = {k: tuple(s) for k, s in _shapes("ncsnpp")}
    return {k: torch.from_numpy(v) for k, v in formula.formula_state_dict(shapes).items()}


def snrnet_formula_sd():
    from snrse import formula
    shapes = {"snrnet." + k: tuple(s) for k, s in _shapes("snrnet")}
    return {k[len("snrnet."):]: torch.from_numpy(v) for k, v in formula.formula_state_dict(shapes).items()}


def snrnet_formula(dev):
    """SNRNet (sgmse/backbones/snrnet.py) with formula weights of the reference architecture."""
    from sgmse.backbones import SNRNet
    net = SNRNet()
    net.load_state_dict(snrnet_formula_sd())
    return net


# ----------------------------------------------------------------------------- CPU baseline
def cpu_threads():
    """Host threads this process may actually run on: the affinity mask, capped by a cgroup-v2 CPU
    quota (a GPU box shares its host; os.cpu_count() reports the whole machine there, and torch
    threads beyond the quota only time-slice)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _stable_malloc():
    """glibc serves the oracle's large activations (> the adaptive mmap threshold, at most 32 MB) by fresh mmaps,
    page-faulted on every NFE, while smaller ones move to the heap as the threshold adapts, so the NFE time drifts
    over a run (round 5, profiles/r05c_cpu_full_n30.json: 2.2-2.4 s for the first NFEs, 1.4-1.9 s for the last).
    All allocations from the heap, never trimmed: steady NFE times, and the sample extrapolates the full run."""
    try:
        libc = ctypes.CDLL("libc.so.6")
        libc.mallopt(-4, 0)          # M_MMAP_MAX: no mmapped chunks
        libc.mallopt(-1, 1 << 30)    # M_TRIM_THRESHOLD: keep freed heap memory
    except (OSError, AttributeError):
        pass


def _cpu_env():
    _stable_malloc()
    threads = cpu_threads()
    torch.set_num_threads(threads)
    return {"cores": threads, "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count()}


def _complex_noise(gen):
    def noise(shape):  # torch.randn_like on complex64: each part N(0, 1/2)
        return torch.complex(torch.randn(shape, generator=gen), torch.randn(shape, generator=gen)) * math.sqrt(0.5)
    return noise


def cpu_baseline(seconds=4.0, n_steps=4, full=False, N=30, warm=2):
    """The oracle (CPU restatement of the reference path, pinned to the reference goldens) on the
    host: one synthetic `seconds` clip, STFT + exponent transform -> prior -> `n_steps` PC steps with
    the reference's reverse_diffusion + ALD algebra (sde_ref.pc_sample: 2 fp32 NCSN++ NFEs per step)
    -> spec_back + iSTFT.  The per-NFE time (step algebra included) is extrapolated to N steps
    (2N NFE).  full=True also runs the whole N=30 utterance once and reports it beside the
    extrapolation.  `warm` untimed NFEs first: the first evaluations of a process run slower (allocator and
    oneDNN primitive caches; round 4's single warm-up NFE left the extrapolation 1.3x the full run's per-NFE
    time, profiles/r04b_cpu_full_n30.json); each timed NFE's duration is in the record."""
    from oracle import ncsnpp_ref, sde_ref, spec_ref
    env = _cpu_env()
    sd = ncsnpp_ref.state_dict_to_torch({k: v.numpy() for k, v in formula_weights().items()})
    y = synth_clips(1, seconds, 10_000)
    gen = torch.Generator().manual_seed(0)
    noise = _complex_noise(gen)
    sde = sde_ref.OUVE(theta=1.5, sigma_min=0.05, sigma_max=0.5, N=30)

    nfe_times = []

    def score_fn(x, t, Y):  # ScoreModel.forward, model_type 'bbed' (model.py:488-489)
        t0 = time.perf_counter()
        out = -ncsnpp_ref.ncsnpp_forward(torch.cat([x, Y], 1), torch.full((x.shape[0],), float(t)), sd)
        nfe_times.append(time.perf_counter() - t0)
        return out

    def front():
        nf = np.abs(y).max()
        Y = spec_ref.spec_fwd(spec_ref.stft(y / nf))
        return torch.from_numpy(spec_ref.pad_spec(Y).astype(np.complex64))[:, None], nf

    def back(x, nf):
        return spec_ref.istft(spec_ref.spec_back(x[0, 0].numpy()), y.shape[1]) * nf

    with torch.no_grad():
        t0 = time.perf_counter()
        Y, nf = front()
        t_front = time.perf_counter() - t0
        for _ in range(warm):  # warm-up NFEs (allocator, oneDNN primitive cache)
            score_fn(Y, 0.5, Y)
        nfe_times.clear()
        t0 = time.perf_counter()
        x, nfe = sde_ref.pc_sample(sde, score_fn, Y, noise, N=n_steps, eps=0.03, snr=0.5)
        t_loop = time.perf_counter() - t0
        t0 = time.perf_counter()
        back(x, nf)
        t_back = time.perf_counter() - t0
        t_nfe = t_loop / nfe
        t_utt = t_front + 2 * N * t_nfe + t_back
        whole = n_steps == N  # the whole utterance measured, nothing extrapolated
        res = {"value": 1.0 / t_utt, "unit": "utt/s", "cores": env["cores"], "kind": "port",
               "sample": (f"1 synthetic {seconds:g} s clip through the oracle (CPU restatement, fp32): STFT + "
                          f"transform, {n_steps} reverse_diffusion+ALD PC steps ({nfe} NCSN++ NFEs at "
                          f"[1,2,256,{Y.shape[-1]}] with the reference step algebra) + iSTFT; "
                          + (f"the whole N={N} utterance timed in this run ({t_nfe:.2f} s/NFE)" if whole else
                             f"{t_nfe:.2f} s/NFE extrapolated to N={N} ({2 * N} NFE/utt)")),
               "seconds": t_front + t_loop + t_back, "extrapolated": not whole,
               "s_per_nfe": t_nfe, "nfe_seconds": [round(v, 3) for v in nfe_times], "warmup_nfe": warm,
               "cpu_model": env["cpu_model"], "os_cpu_count": env["os_cpu_count"]}
        if full:
            nfe_times.clear()
            t0 = time.perf_counter()
            Y, nf = front()
            x, nfe_full = sde_ref.pc_sample(sde, score_fn, Y, noise, N=30, eps=0.03, snr=0.5)
            back(x, nf)
            t_full = time.perf_counter() - t0
            res["full_utterance"] = {"N": 30, "nfe": nfe_full, "seconds": t_full, "utt_per_s": 1.0 / t_full,
                                     "extrapolated_seconds": t_utt, "measured_over_extrapolated": t_full / t_utt,
                                     "nfe_seconds_mean": sum(nfe_times) / len(nfe_times),
                                     "nfe_seconds": [round(v, 3) for v in nfe_times]}
    return res


def c1_clip():
    """C1's '4 s VBD utterance': the three dataset utterances held in tests/golden/enhance_snrnet_c4.npz
    (reference dataset/VBD*, 16 kHz int16) concatenated and cut at 4 s."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "enhance_snrnet_c4.npz"), allow_pickle=False)
    return (np.concatenate(list(g["noisy_i16"]))[: 4 * SR].astype(np.float32) / 32768.0)[None]


def oracle_one_step(y, sd, ssd, noise, fixed_snr=0.17783, sigma_max=0.5):
    """The reference's SNR-aligned one-step enhance (model.py:713-833, sebridge_v3 + snr_conditioned
    'true') through the oracle on the CPU: y [1, L] numpy -> (x_hat [L], t_hat)."""
    from oracle import ncsnpp_ref, snrnet_ref, spec_ref
    nf0 = float(np.abs(y).max())
    raw = spec_ref.stft(y / nf0)
    T16 = raw.shape[-1] + (16 - raw.shape[-1] % 16) % 16
    R = np.zeros((1, 256, T16), np.complex64)
    R[..., : raw.shape[-1]] = raw
    Rt = torch.from_numpy(R)
    g = snrnet_ref.snrnet_forward(torch.stack([Rt.real, Rt.imag], 1), ssd)
    est = float(g[0, 0] / (1 - g[0, 0]))
    t_hat = snrnet_ref.snap_t(est, fixed_snr)
    norm = nf0 * snrnet_ref.normfac(t_hat, fixed_snr)
    Y = torch.from_numpy(spec_ref.pad_spec(spec_ref.spec_fwd(spec_ref.stft(y / norm))).astype(np.complex64))[:, None]
    X = Y + noise(Y.shape) * sigma_max * t_hat
    tt = torch.tensor([t_hat], dtype=torch.float32)
    c_skip = 0.25 / ((t_hat - 0.001) ** 2 + 0.25)
    c_out = 0.5 * (t_hat - 0.001) / math.sqrt(0.25 + t_hat ** 2)
    s = c_skip * X + c_out * ncsnpp_ref.ncsnpp_forward(torch.cat([X, Y], 1), tt, sd)
    return spec_ref.istft(spec_ref.spec_back(s[0, 0].numpy()), y.shape[1]) * norm, t_hat


def cpu_baseline_train(frames=256, steps=1):
    """--config train's CPU leg: the oracle's consistency-training step (oracle/train_ref.py: the loss of
    model.py:361-390 on the NCSN++ restatement, torch autograd backward, pinned to the reference's own
    autograd by tests/test_oracle_golden.py::test_train_step) + torch.optim.Adam over the trainable tensors,
    for ONE [256, frames] spectrogram pair per step (the GPU leg's per-sample work), after one warm-up step."""
    from oracle import ncsnpp_ref, train_ref
    env = _cpu_env()
    sd = ncsnpp_ref.state_dict_to_torch({k: v.numpy() for k, v in formula_weights().items()})
    gen = torch.Generator().manual_seed(0)
    noise = _complex_noise(gen)
    x = noise((1, 1, 256, frames)) * 0.4
    y = x + noise((1, 1, 256, frames)) * 0.4
    params = [v for k, v in sd.items() if k not in train_ref.FROZEN]
    for v in params:
        v.requires_grad_(True)
    opt = torch.optim.Adam(params, lr=1e-4)

    def step(n):
        opt.zero_grad(set_to_none=True)
        loss = train_ref.consistency_loss(sd, x, y, noise(x.shape), torch.tensor([n]))
        loss.backward()
        opt.step()
        return loss

    step(5)
    t0 = time.perf_counter()
    for i in range(steps):
        step(3 + i)
    el = (time.perf_counter() - t0) / steps
    return {"value": 1.0 / el, "unit": "samples/s", "cores": env["cores"], "kind": "port",
            "sample": (f"{steps} oracle consistency-training step(s) (CPU restatement, fp32) on ONE [256, {frames}] "
                       f"spectrogram pair: 2 NCSN++ evaluations + autograd backward + torch Adam; {el:.2f} s/sample"),
            "cpu_model": env["cpu_model"], "os_cpu_count": env["os_cpu_count"]}


def cpu_baseline_c4(seconds=4.0, n=3):
    """C4's CPU leg: `n` synthetic clips through the oracle's one-step SNR-aligned enhance (SNRNet
    estimate + one fp32 NCSN++ evaluation + STFT / iSTFT), after one warm-up clip."""
    from oracle import ncsnpp_ref
    env = _cpu_env()
    sd = ncsnpp_ref.state_dict_to_torch({k: v.numpy() for k, v in formula_weights().items()})
    ssd = {k: v.float() for k, v in snrnet_formula_sd().items()}
    ys = synth_clips(n + 1, seconds, 20_000)
    noise = _complex_noise(torch.Generator().manual_seed(2))
    with torch.no_grad():
        oracle_one_step(ys[:1], sd, ssd, noise)
        t0 = time.perf_counter()
        for k in range(1, n + 1):
            oracle_one_step(ys[k:k + 1], sd, ssd, noise)
        el = time.perf_counter() - t0
    return {"value": n / el, "unit": "utt/s", "cores": env["cores"], "kind": "port",
            "sample": (f"{n} synthetic {seconds:g} s clips through the oracle (CPU restatement, fp32): SNRNet "
                       f"estimate + t_hat snap + one preconditioned NCSN++ NFE + STFT / iSTFT each"),
            "cpu_model": env["cpu_model"], "os_cpu_count": env["os_cpu_count"]}


def run_c1(args):
    """configs[0]: the reference's CPU-runnable case, --gpus 0.  One 4 s VBD utterance, sebridge_v3,
    exponent transform, SNR from SNRNet, on PyTorch CPU via the oracle: the one-step enhance
    (model.py:713-833; N is ignored on this branch) timed `--steps` times, plus one N=5 PC run
    (10 NFE, model.py:756-768 arithmetic) as the plumbing check of the sampler path."""
    from oracle import ncsnpp_ref, sde_ref, spec_ref
    env = _cpu_env()
    sd = ncsnpp_ref.state_dict_to_torch({k: v.numpy() for k, v in formula_weights().items()})
    ssd = {k: v.float() for k, v in snrnet_formula_sd().items()}
    y = c1_clip()
    noise = _complex_noise(torch.Generator().manual_seed(1))

    def one_step():
        return oracle_one_step(y, sd, ssd, noise)

    with torch.no_grad():
        for _ in range(args.warmup):
            one_step()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            xh, t_hat = one_step()
        el = time.perf_counter() - t0
        Y = torch.from_numpy(spec_ref.pad_spec(spec_ref.spec_fwd(spec_ref.stft(y / np.abs(y).max())))
                             .astype(np.complex64))[:, None]
        t1 = time.perf_counter()
        xp, ns = sde_ref.pc_sample(sde_ref.OUVE(1.5, 0.05, 0.5, N=5), lambda x, t, Yc: -ncsnpp_ref.ncsnpp_forward(
            torch.cat([x, Yc], 1), torch.full((1,), float(t)), sd), Y, noise, N=5)
        t_pc = time.perf_counter() - t1
    value = args.steps / el
    cpu = {"value": value, "unit": "utt/s", "cores": env["cores"], "kind": "port",
           "sample": f"C1 itself: {args.steps} one-step enhancements of the 4 s VBD clip",
           "cpu_model": env["cpu_model"], "os_cpu_count": env["os_cpu_count"]}
    line = {"metric": METRIC, "value": value, "unit": "utt/s", "n_gpus": 0, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "VBD dataset utterances (reference dataset/, via tests/golden) cut to 4 s; formula weights",
            "config": {"workload": ("C1: one 4 s VBD utterance, sebridge_v3 + snr_conditioned (SNRNet estimate), "
                                    "exponent transform, one-step enhance on PyTorch CPU (oracle restatement; "
                                    "--gpus 0 plumbing, no GPU)"),
                       "global_batch": 1, "per_gpu_batch": 1, "seq_len": 512, "parallelism": "none (CPU)"},
            "roofline": None, "cpu_baseline": cpu, "t_hat": float(t_hat),
            "output_rms": float(np.sqrt(np.mean(np.asarray(xh, np.float64) ** 2))),
            "pc_n5_plumbing": {"nfe": ns, "seconds": t_pc, "finite": bool(torch.isfinite(torch.view_as_real(xp)).all())}}
    print(json.dumps(line), flush=True)


# ----------------------------------------------------------------------------- roofline probe
def conv_flops(src0, src1, ksize, cout, sc, sc1):
    B, H, W, C0 = src0.shape
    cin = C0 + (0 if src1 is None else src1.shape[3])
    k = ksize * ksize * cin + (0 if sc is None else sc.shape[3]) + (0 if sc1 is None else sc1.shape[3])
    return 2.0 * B * H * W * cout * k


class ConvProbe:
    """HIP events on the launch stream around every conv call during one extra enhance() pass after the
    timed region, recorded by the library itself around the call's kernel launches (snrse_ctx_probe_begin:
    events without the system-scope fence, so no cache write-back sits inside a bracket -- torch.cuda.Event
    pairs read ~7 % long on the fp32 path, profiles/r03g_c5_probe_vs_rocprof.json).  The big convs (bf16:
    the halo-path 3x3 convs, ops.halo_ok; fp32 parity mode: every 3x3 conv with Cout >= 64) are grouped by
    the kernel that ran.  achieved = algorithmic FLOPs of the dominant kernel's launches / their summed
    event time, i.e. mean FLOPs per launch / mean launch duration (what rocprofv3 --stats reports as
    AverageNs; a split-K call's bracket also holds its conv_splitk_finalize)."""

    CAP = 4096

    def __init__(self, all_threads=False):
        self.rec = []
        self.chunks = []
        self.all_threads = all_threads  # also the other threads' contexts (the autograd worker's backward)

    def install(self, ops):
        orig = ops.conv2d
        probe = self

        def wrapped(src0, wgt, ksize, cout, *a, **kw):
            big = ops.halo_ok(src0, ksize, cout) or (src0.dtype == torch.float32 and ksize == 3 and cout >= 64)
            probe.rec.append(conv_flops(src0, kw.get("src1"), ksize, cout, kw.get("sc"), kw.get("sc1")) if big else None)
            out = orig(src0, wgt, ksize, cout, *a, **kw)
            # launches of this call: sources beyond 2 GiB (fp32 level 0 at B = 32) run as image-range chunks
            probe.chunks.append(max(1, ops._opt(src0, "last_chunks")) if big else 1)
            return out

        ops.conv2d = wrapped
        self.orig, self.ops = orig, ops
        ops.probe_begin(self.CAP, all_threads=self.all_threads)

    def uninstall(self):
        self.ops.conv2d = self.orig

    def summary(self):
        """{kernel: [flops, ms, launches]} over the probed pass (launches: kernel launches, counting each
        image-range chunk of a call whose sources exceed 2 GiB)."""
        ms, kern = self.ops.probe_read(self.CAP, all_threads=self.all_threads)
        self.ops.probe_begin(0, all_threads=self.all_threads)
        if len(ms) != min(len(self.rec), self.CAP):
            raise RuntimeError(f"probe: {len(ms)} timed calls for {len(self.rec)} conv2d calls")
        if os.environ.get("SNRSE_PROBE_DUMP"):  # per-call record for tools/probe_reconcile.py
            with open(os.environ["SNRSE_PROBE_DUMP"], "w") as f:
                json.dump({"ms": ms, "kernel": kern, "flops": self.rec[:len(ms)], "launches": self.chunks[:len(ms)]}, f)
        by = {}
        for fl, t, k, nl in zip(self.rec, ms, kern, self.chunks):
            if fl is None:
                continue
            d = by.setdefault(self.ops.kernel_name(k), [0.0, 0.0, 0])
            d[0] += fl
            d[1] += t
            d[2] += nl
        return by


def pmc_traffic(kernel_prefix, tag, dtype=None):
    """HBM bytes per launch of the dominant kernel from the committed PMC profile
    (profiles/*_pmc_traffic.json, tools/pmc_traffic.py: FETCH_SIZE x 2 per the gfx950 correction +
    WRITE_SIZE) for this config tag and 16-bit format (profiles before round 6 carry no dtype: bf16);
    None when absent."""
    def newest_first(path):  # profiles/rNN<suffix>_...: round, then suffix length, then suffix (v < ak)
        tag = os.path.basename(path).split("_")[0]
        m = re.match(r"r(\d+)([a-z]*)$", tag)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, tag)

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), key=newest_first, reverse=True):
        with open(path) as f:
            d = json.load(f)
        if (d.get("kernel", "").startswith(kernel_prefix) and d.get("config", "c2") == tag
                and (dtype is None or d.get("dtype", "bf16") == dtype)):
            return d.get("bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


# ----------------------------------------------------------------------------- training step
def run_train(args):
    """consistency-training steps of the SNR-aligned sebridge_v3 model (model.py:361-390,
    loss mse) on the HIP forward + backward kernels, fused Adam + EMA (model.py:99-106): synthetic
    complex spectrogram pairs [B, 1, 256, T] (the data module's training crop, num_frames 256), fp32 as
    the reference trains.  One step = training_step -> loss.backward() -> optimizer_step -> zero_grad."""
    from sgmse.model import ScoreModel
    from snrse import ops
    from snrse import train as strain
    strain.set_gemm("x3" if args.dtype == "fp32x3" else "exact")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    hp = dict(backbone="ncsnpp", sde="ouve", model_type="sebridge_v3", snr_conditioned="true", theta=1.5,
              sigma_min=0.05, sigma_max=0.5, N=30, compute_dtype="fp32", fixed_snr=0.17783, loss_type="mse")
    m = ScoreModel(**hp)
    m.dnn.load_state_dict(formula_weights())
    m = m.cuda().train()
    opt = m.configure_optimizers()
    B, T = args.batch, args.frames
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(B, 1, 256, T, dtype=torch.complex64, device=dev, generator=g) * 0.4)
    y = x + torch.randn(B, 1, 256, T, dtype=torch.complex64, device=dev, generator=g) * 0.4

    def step(i):
        loss = m.training_step((x, y), i)
        loss.backward()
        m.optimizer_step(opt)
        opt.zero_grad(set_to_none=False)
        return loss

    for w in range(args.warmup):
        step(w)
    torch.cuda.synchronize()
    probe = ConvProbe(all_threads=True)  # the backward's dgrad convs run on the autograd worker thread
    t0 = time.perf_counter()
    for k in range(args.steps):
        loss = step(args.warmup + k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    probe.install(ops)
    try:
        step(999)
    finally:
        probe.uninstall()
    by = probe.summary()
    roof = None
    if by:
        kname = max(by, key=lambda k: by[k][1])
        fl, ms, n = by[kname]
        pk = PEAK["fp32x3"] if kname.startswith("conv_x3") else PEAK["fp32"]  # split-bf16 GEMMs: bf16 peak / 3
        roof = {"bound": "mfma", "achieved": fl / (ms * 1e-3) / 1e12, "peak": pk / 1e12, "unit": "TFLOP/s",
                "frac": fl / (ms * 1e-3) / pk, "traffic": None, "kernel": kname,
                "launches_per_pass": n, "avg_launch_us": ms * 1e3 / max(n, 1), "scope": "3x3 convs of the step (forward and dgrad)"}
    line = {"metric": "consistency-training samples/s (sebridge_v3, loss mse, fp32)", "value": args.steps * B / el,
            "gemm": "split-bf16 forward / input-gradient GEMMs (fp32x3)" if args.dtype == "fp32x3" else "exact fp32",
            "unit": "samples/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic complex spectrogram pairs; formula weights of the NCSN++ architecture",
            "config": {"workload": (f"§8(f)2 training step: B={B} x [256, {T}] spectrogram pairs, two NCSN++ "
                                    "evaluations + backward + fused Adam/EMA"), "global_batch": B, "per_gpu_batch": B,
                       "seq_len": T, "parallelism": "dp1"},
            "roofline": roof, "cpu_baseline": None, "loss": float(loss)}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_train(frames=T)
    print(json.dumps(line), flush=True)


# ----------------------------------------------------------------------------- GPU bench
# rocprofv3 --kernel-trace --marker-trace --selected-regions collects only between roctxProfilerResume(0) and
# roctxProfilerPause(0); the roctx library is loaded before anything touches the GPU (loaded later, or without
# --marker-trace, the region collected nothing: profiles/r06d_roctx_region_check.txt)
_ROCTX = None
if os.environ.get("SNRSE_ROCTX") == "1":
    import ctypes as _ct
    _ROCTX = _ct.CDLL("librocprofiler-sdk-roctx.so")
    _ROCTX.roctxProfilerResume.argtypes = [_ct.c_uint64]
    _ROCTX.roctxProfilerPause.argtypes = [_ct.c_uint64]


def roctx_region():
    """f(True) / f(False): roctxProfilerResume(0) / roctxProfilerPause(0) around the timed steps when SNRSE_ROCTX=1, so
    the rocprof summary holds exactly the timed kernels; a no-op otherwise."""
    if _ROCTX is None:
        return lambda on: None
    return lambda on: (_ROCTX.roctxProfilerResume if on else _ROCTX.roctxProfilerPause)(0)


# c2 / c4: the configuration's 16-bit arithmetic, in IEEE fp16 since round 6 (same bytes and MFMA rate as bf16;
# bf16 misses SURVEY 8(c)'s 1e-2 parity bound, fp16 meets it: DESIGN.md 9, profiles/r06a_bf16_attribution.jsonl)
CONFIG_DEFAULTS = {"c2": dict(batch=32, N=30, seconds=4.0, dtype="fp16"),
                   "c4": dict(batch=32, N=30, seconds=4.0, dtype="fp16"),
                   "c5": dict(batch=1, N=200, seconds=30.0, dtype="fp32"),
                   "train": dict(batch=8, N=30, seconds=4.0, dtype="fp32")}


def run(args):
    from snrse import dist as sdist
    rank, world, dev = sdist.init_from_env()
    if world != max(args.gpus, 1):
        raise SystemExit(f"bench: --gpus {args.gpus} but the process group has {world} ranks")
    dist = None
    if world > 1:
        import torch.distributed as dist

    from snrse import ncsnpp, ops, sampler
    from snrse.enhance import PCEnhancer

    ops.set_option("conv_variant", args.conv_variant)
    dtype = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(args.dtype, torch.float32)
    net = ncsnpp.NCSNppHIP(formula_weights(), dtype=dtype, device=dev, gemm="x3" if args.dtype == "fp32x3" else "exact")
    sde = sampler.SDESpec("ouve", theta=1.5, sigma_min=0.05, sigma_max=0.5)
    enh = PCEnhancer(net, sde, N=args.N, streams=args.streams, stagger=bool(args.stagger))
    probe_enh = PCEnhancer(net, sde, N=min(args.N, 2))  # kernel durations do not depend on N
    B = args.batch
    y = torch.from_numpy(synth_clips(B, args.seconds, 1000 * rank)).to(dev)
    noise = lambda it: sampler.NoiseSource(seed=7919 * (rank + 1) + it)  # noqa: E731
    if args.config == "c4":
        from snrse.enhance import SNRAlignedEnhancer
        snr_net = snrnet_formula(dev)
        one = SNRAlignedEnhancer(net, snr_fn=lambda spec: (lambda g: g / (1 - g))(snr_net.forward_complex(spec)[:, 0]),
                                 fixed_snr=0.17783, sigma_max=0.5)
        enh = probe_enh = lambda yy, nz: (one(yy, seed=nz.seed)[0], 1)  # noqa: E731

    for w in range(args.warmup):
        enh(y, noise(w))
        if rank == 0:
            print(f"[bench] warmup step {w + 1}/{args.warmup} done", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    region = roctx_region()  # (rocprofv3 --selected-regions: the kernel summary brackets exactly the timed steps)
    region(True)
    t0 = time.perf_counter()
    for k in range(args.steps):
        xh, nfe = enh(y, noise(100 + k))
        if rank == 0 and args.steps > 1:
            print(f"[bench] step {k + 1}/{args.steps} enqueued", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    region(False)
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
            probe_enh(y, noise(999))
        finally:
            probe.uninstall()
        by = probe.summary()
        per_kernel = {k: {"launches": v[2], "ms": v[1], "tflops": v[0] / max(v[1], 1e-9) / 1e9,
                          "frac": v[0] / max(v[1], 1e-9) * 1e3 / PEAK[args.dtype]} for k, v in by.items()}
        # (rounds 4-5 ran the ResBlock 3x3 convs on two kernels split by shape, reported as one family -- the sum of
        # their FLOPs over the sum of their launch times; since round 5 one kernel, conv_halo5_kernel, runs them all)
        fam = [k for k in ("conv_halo5_kernel", "conv_halo10_kernel") if k in by]
        if len(fam) == 2:
            by["+".join(fam)] = [sum(by[k][i] for k in fam) for i in range(3)]
            for k in fam:
                by.pop(k)
        kname = max(by, key=lambda k: by[k][1])  # the conv kernel (family) with the most time in the pass
        fl, ms, n = by[kname]
        ach = fl / (ms * 1e-3) if ms > 0 else 0.0
        peak = PEAK[args.dtype]
        tdt = args.dtype if args.dtype in ("fp16", "bf16") else None
        traffic, tsrc = pmc_traffic(kname, args.config, tdt)
        if traffic is None and "+" in kname:  # no family profile: its first kernel's launches
            traffic, tsrc = pmc_traffic(kname.split("+")[0], args.config, tdt)
        roof = {"bound": "mfma", "achieved": ach / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s",
                "frac": ach / peak, "traffic": traffic, "kernel": kname, "launches_per_pass": n,
                "avg_launch_us": ms * 1e3 / max(n, 1), "flop_per_launch": fl / max(n, 1),
                "kernel_ms_per_pass": ms, "traffic_source": tsrc,
                "per_kernel": per_kernel}

    parity = None
    if rank == 0 and not args.no_parity:
        # the timed network object itself on the reference's N=5 OUVE PC run (paritycheck.py), after the
        # timed region: pins the benched code's numerics in the same JSON line
        import paritycheck
        if args.dtype == "fp32x3":  # the golden's [2, 256, 64] grid is small: force the benched halo kernel
            ops.set_option("x3_tile", 4)  # (conv_x3h_kernel + fused GroupNorm) wherever its shape allows
        try:
            if args.config == "c4":  # the timed SNR-aligned path on the reference's C4 run
                r = paritycheck.c4_vs_golden(dev, net)
            else:
                r = paritycheck.pc_vs_golden(dev, net)
        finally:
            ops.set_option("x3_tile", 0)
        if args.config == "c4":
            parity = {k: r[k] for k in ("check", "dtype", "rel_rms", "t_hat_abs_err", "tol_rel", "ok")}
            parity["golden"] = "tests/golden/enhance_snrnet_c4.npz"
        else:
            parity = {k: r[k] for k in ("check", "dtype", "rel_rms", "abs_rms", "golden_rms", "tol_rel", "ok")}
            parity["golden"] = "tests/golden/pc_ouve.npz"
        if r["dtype"] in ("fp32", "fp32x3") and "abs_rms" in r:  # the north star's 1e-4 absolute RMS bound
            parity["tol_abs"] = 1e-4
            parity["ok"] = bool(parity["ok"] and r["abs_rms"] < 1e-4)

    # The same C2 workload in the fp32x3 parity mode (split-bf16 fp32 GEMMs: within the north star's 1e-4
    # RMS) beside the bf16 headline, single-GPU default runs only: one warm-up step, then K3 = max(3, --steps)
    # timed steps on the timed run's clips and noise seeds, the dominant x3 kernel's probe fraction, its own
    # N=5 PC golden check (halo kernel forced at the golden's size) and the C2-size agreement of the timed
    # bf16 output with the x3 output of the same clips and Philox seed (c2_agreement)
    pmode = None
    if (world == 1 and args.config == "c2" and args.dtype in ("fp16", "bf16") and not args.no_parity_mode
            and args.seconds == 4.0 and args.N == 30):
        del enh, probe_enh, net
        torch.cuda.empty_cache()
        fcost = None
        if args.dtype == "fp16":
            # what the fp16 headline costs against the bf16 form of the same kernels (round 6): one warm-up + 3 timed
            # bf16 steps on the same clips and seeds, and bf16's own N=5 PC golden error beside fp16's
            import paritycheck
            netb = ncsnpp.NCSNppHIP(formula_weights(), dtype=torch.bfloat16, device=dev)
            enhb = PCEnhancer(netb, sde, N=args.N)
            enhb(y, noise(50))
            torch.cuda.synchronize()
            tb = time.perf_counter()
            for k in range(3):
                enhb(y, noise(100 + k))
            torch.cuda.synchronize()
            vb = 3 * B / (time.perf_counter() - tb)
            fcost = {"what": "the same C2 step with bf16 activations / weights / MFMA operands (same kernels)",
                     "bf16_value": vb, "bf16_steps": 3, "fp16_over_bf16": value / vb}
            if not args.no_parity:
                rb = paritycheck.pc_vs_golden(dev, netb)
                fcost["bf16_pc_rel_rms"] = rb["rel_rms"]
                fcost["fp16_pc_rel_rms"] = parity["rel_rms"] if parity else None
                fcost["tol_rel"] = paritycheck.TOL["pc"]["fp16"]
            del enhb, netb
            torch.cuda.empty_cache()
        net3 = ncsnpp.NCSNppHIP(formula_weights(), dtype=torch.float32, device=dev, gemm="x3")
        enh3 = PCEnhancer(net3, sde, N=args.N)
        K3 = max(3, args.steps)
        enh3(y, noise(50))
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        for k in range(K3):
            xh3, _ = enh3(y, noise(100 + k))  # the 16-bit timed steps' seeds
        torch.cuda.synchronize()
        el3 = time.perf_counter() - t3
        pmode = {"dtype": "fp32x3", "value": K3 * B / el3, "unit": "utt/s", "ms_per_step": el3 / K3 * 1e3,
                 "steps": K3, "warmup": 1, "format_cost": fcost,
                 "note": ("fp32 activations / storage / accumulation, ResBlock and input convs as "
                          "split-bf16 GEMMs (bench.py --dtype fp32x3 for the full line)")}
        # the x3 output for the 16-bit timed run's last seed (100 + steps - 1): the K3-th timed step when
        # K3 == steps, else one more untimed step
        if K3 != args.steps:
            xh3, _ = enh3(y, noise(100 + args.steps - 1))
        import paritycheck
        pmode["c2_agreement"] = paritycheck.waveform_agreement(
            xh, xh3, bounds=paritycheck.C2_AGREE16 if args.dtype == "fp16" else paritycheck.C2_AGREE)
        pmode["c2_agreement"]["what"] = (f"timed {args.dtype} C2 output vs fp32x3 on the same {B} clips and Philox seed "
                                         f"(N={args.N}, {nfe} NFE/utt)")
        if not args.no_probe:
            probe = ConvProbe()
            probe.install(ops)
            try:
                PCEnhancer(net3, sde, N=2)(y, noise(999))
            finally:
                probe.uninstall()
            by = probe.summary()
            kn = max(by, key=lambda k: by[k][1])
            fl, ms, n = by[kn]
            pmode["roofline"] = {"kernel": kn, "bound": "mfma", "achieved": fl / (ms * 1e-3) / 1e12,
                                 "peak": PEAK["fp32x3"] / 1e12, "unit": "TFLOP/s (fp32-equivalent)",
                                 "frac": fl / (ms * 1e-3) / PEAK["fp32x3"], "launches_per_pass": n,
                                 "avg_launch_us": ms * 1e3 / max(n, 1)}
        if not args.no_parity:
            ops.set_option("x3_tile", 4)
            try:
                r3 = paritycheck.pc_vs_golden(dev, net3)
            finally:
                ops.set_option("x3_tile", 0)
            pmode["parity"] = {"abs_rms": r3["abs_rms"], "rel_rms": r3["rel_rms"], "tol_abs": 1e-4,
                               "ok": bool(r3["ok"] and r3["abs_rms"] < 1e-4), "golden": "tests/golden/pc_ouve.npz",
                               "kernels": "x3_tile=4: conv_x3h_kernel forced wherever its shape allows"}
            r30 = paritycheck.pc_vs_golden(dev, net3)  # the dispatch the timed steps ran (x3_tile 0)
            pmode["parity"]["timed_dispatch"] = {"abs_rms": r30["abs_rms"], "rel_rms": r30["rel_rms"],
                                                 "ok": bool(r30["ok"] and r30["abs_rms"] < 1e-4)}
            pmode["parity"]["ok"] = bool(pmode["parity"]["ok"] and pmode["parity"]["timed_dispatch"]["ok"])
        del enh3, net3
        torch.cuda.empty_cache()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        # the whole N = 30 utterance (60 NFE, ~25 s on the box's 16 host threads): measured in the same run as the GPU
        # line, nothing extrapolated (rounds 3-5 timed 4 steps and extrapolated, validated by a stored full run)
        cpu = cpu_baseline(n_steps=30)
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c5":
        cpu = cpu_baseline(seconds=args.seconds, n_steps=1, N=args.N, warm=1)  # 2 NFEs of a 30 s clip
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c4":
        cpu = cpu_baseline_c4(seconds=args.seconds)

    n_frames = 1 + int(args.seconds * SR) // 128
    T_frames = (n_frames + 63) // 64 * 64
    tag = args.config.upper()
    if args.config == "c2" and (args.seconds != 4.0 or args.N != 30):
        tag = "custom"
    elif args.config == "c2" and args.dtype == "fp32":
        tag = "C2-fp32"  # the C2 workload in the exact fp32 parity mode (the north star's 1e-4 tolerance)
    elif args.config == "c2" and args.dtype == "fp32x3":
        tag = "C2-fp32x3"  # the same parity mode on the split-bf16 fp32 GEMMs
    if rank == 0:
        if args.config == "c4":
            wl = (f"C4: B={B} {args.seconds:g} s/16 kHz clips per GPU, one-step SNR-aligned enhancement "
                  f"(SNRNet estimate + 1 sebridge_v3 NFE at t_hat), NCSN++ nf=128")
        else:
            wl = (f"{tag}: B={B} {args.seconds:g} s/16 kHz clips per GPU, N={args.N} PC steps "
                  f"(reverse_diffusion + ald, {nfe} NFE/utt), OUVE SDE, NCSN++ nf=128, {args.dtype}")
        line = {
            "metric": METRIC, "value": value, "unit": "utt/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (SURVEY §8d harmonic+noise clips; formula weights of the NCSN++ architecture)",
            "config": {"workload": wl, "global_batch": B * world, "per_gpu_batch": B, "seq_len": T_frames,
                       "parallelism": f"dp{world} (utterance sharding)"},
            "roofline": roof, "cpu_baseline": cpu, "parity": parity,
            "output_rms_mean": float(allm.mean()),
        }
        if pmode is not None:
            line["parity_mode"] = pmode
        if sdist.oversubscribed(world):  # a launcher rehearsal: ranks share the visible GPU(s)
            line["oversubscribed"] = {"ranks": world, "devices": torch.cuda.device_count(),
                                      "note": "ranks share devices; collectives on gloo; not a scaling figure"}
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="GPUs (ranks); 0 = C1, the CPU plumbing case")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=["c2", "c4", "c5", "train"], default="c2",
                    help="c2: PC sampler, B=32 4 s fp16 (default, the headline line); c4: one-step SNR-aligned "
                         "path (SNRNet estimate + 1 preconditioned NFE, sebridge_v3); c5: 30 s clips, N=200, fp32; "
                         "train: the consistency-training step (SURVEY §8(f) 2)")
    ap.add_argument("--frames", type=int, default=256, help="spectrogram frames of a training sample (--config train)")
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU")
    ap.add_argument("--N", type=int, default=None, help="PC steps")
    ap.add_argument("--seconds", type=float, default=None)
    ap.add_argument("--dtype", choices=["fp16", "bf16", "fp32", "fp32x3"], default=None,
                    help="fp16 (c2 / c4 default); bf16 (the same kernels on bf16); fp32 (exact fp32 MFMA GEMMs); "
                         "fp32x3 (fp32 activations, split-bf16 GEMMs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-parity-mode", action="store_true",
                    help="skip the fp32x3 parity-mode step timed beside the default 16-bit C2 line")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the post-run parity check of the benched network vs tests/golden/pc_ouve.npz")
    ap.add_argument("--conv-variant", type=int, default=0, help="snrse conv_variant option (0 = auto)")
    ap.add_argument("--streams", type=int, default=1,
                    help="PC-sampler lanes per GPU, each on its own HIP stream (snrse.enhance.PCEnhancer)")
    ap.add_argument("--stagger", type=int, default=1,
                    help="with --streams > 1: start each lane half a network evaluation after the previous one")
    ap.add_argument("--cpu-full", default=None, metavar="PATH",
                    help="only run the CPU baseline with one full N=30 utterance and write it to PATH")
    args = ap.parse_args()
    for k, v in CONFIG_DEFAULTS[args.config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    if args.cpu_full:
        res = cpu_baseline(full=True)
        with open(args.cpu_full, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res), flush=True)
        return 0
    if args.gpus == 0:
        run_c1(args)
        return 0
    if args.config == "train":
        run_train(args)
        return 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # start the N ranks here (no torchrun); nothing in this process has touched the GPU
        from snrse import dist as sdist
        return sdist.spawn_ranks(args.gpus, run, (args,))
    run(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Batched, device-resident ScoreModel.enhance() (reference sgmse/model.py:702-839).

Two branches, as the reference:
  * PC sampler (model_type 'bbed', snr_conditioned 'false', model.py:756-768): STFT ->
    exponent transform -> pad -> prior -> N x (corrector, predictor), each NFE fused with its
    SDE update -> iSTFT.  2 NFE per step for reverse_diffusion + ald.
  * one-step SNR-aligned (model_type 'sebridge_v3', snr_conditioned 'true',
    model.py:713-740, 810-825): t_hat from the SNR (estimator or oracle rms) snapped to the
    t_30 grid, X_T = Y + sigma_max t_hat Z, one preconditioned NFE.
Utterances are processed as a batch (the reference loops B=1); per-utterance scalars
(norm factors, t_hat) stay per batch element.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import ops, sampler

T_30 = (0.001 ** (1 / 7) + (np.arange(1, 31) - 1) / 29 * (1 - 0.001 ** (1 / 7))) ** 7  # model.py:22-23


def snap_t(est_snr, fixed_snr):
    """calculate_snr_direct + nearest t_30 (model.py:627-629, 810-817), per utterance."""
    t = np.asarray(est_snr, dtype=np.float64) / (10 ** 0.25 * fixed_snr)
    return T_30[np.abs(T_30[None, :] - t.reshape(-1, 1)).argmin(axis=1)]


def normfac(t_hat, fixed_snr):
    """calculate_normfac_direct at est_snr_ = 10^0.25 fixed_snr t_hat (model.py:631-634, 734-736)."""
    s = 10 ** 0.25 * fixed_snr * np.asarray(t_hat, dtype=np.float64)
    return 2.040166 * (0.240253 + 0.759747 * fixed_snr ** 2) ** 0.5 / np.sqrt(1 + s ** 2)


def pad_frames(T, mult=64):
    return T + ((mult - T % mult) % mult)


TRANSFORM_MODES = {"exponent": 1, "none": 0}  # fused spec_fwd/spec_back (|c|^0.5 e^{i angle} 0.15) or raw


def transform_mode(transform):
    if transform not in TRANSFORM_MODES:
        raise NotImplementedError(f"transform_type {transform!r} is not built for the HIP path")
    return TRANSFORM_MODES[transform]


class PCEnhancer:
    """PC-sampler enhancement of a batch of noisy waveforms with an NCSNppHIP network.

    streams > 1 splits the batch into that many lanes, each on its own HIP stream with its own
    GroupNorm-statistics arena and split-K workspace, and issues their network evaluations
    alternately (sampler.pc_sample_lockstep): one lane's latency-bound low-resolution levels overlap
    the other lane's full-resolution GEMMs.  stagger: lane k starts when lane k-1's first evaluation
    has reached the middle of the network (an event recorded between its down and up paths), so the
    lanes run half an evaluation apart instead of in phase.  The noise draws are the whole-batch ones
    (LaneNoise), so the result equals the single-stream run."""

    def __init__(self, net, sde: sampler.SDESpec, N=30, eps=0.03, snr=0.5, predictor="reverse_diffusion",
                 corrector="ald", corrector_steps=1, score_mode=0, transform="exponent", streams=1, stagger=True):
        self.net, self.sde, self.N, self.eps, self.snr = net, sde, N, eps, snr
        self.mode = transform_mode(transform)
        self.predictor, self.corrector, self.corrector_steps = predictor, corrector, corrector_steps
        self.score_mode = score_mode
        self.streams = int(streams)
        self.stagger = bool(stagger)
        self._lane_streams = {}

    def _iter(self, Y, noise):
        net = self.net

        def step(x, tv, coef, z, seed, off):
            pyr = net.pyramid(x, Y, tv)
            xo, xm, _ = ops.score_update(pyr, net.W["out_w"], net.W["out_b"], tv, self.score_mode, x, Y,
                                         coef=coef, noise=z, seed=seed, offset=off)
            return xo, xm

        def score_tensor(x, tv):
            return net.score(x, Y, tv, self.score_mode)

        return sampler.pc_sample_iter(step, Y, self.sde, N=self.N, eps=self.eps, snr=self.snr,
                                      predictor=self.predictor, corrector=self.corrector,
                                      corrector_steps=self.corrector_steps, noise=noise, score_tensor=score_tensor)

    def sample(self, Y, noise: sampler.NoiseSource | None = None):
        B = Y.shape[0]
        noise = noise or sampler.NoiseSource()
        nl = min(self.streams, B)
        if nl <= 1:
            it = self._iter(Y, noise)
            while True:
                try:
                    next(it)
                except StopIteration as e:
                    return e.value
        cur = torch.cuda.current_stream(Y.device)
        bounds = [(B * h // nl, B * (h + 1) // nl) for h in range(nl)]
        lanes, lane_noise = [], []
        for h, (a, b) in enumerate(bounds):
            s = self._lane_streams.get((Y.device, h))
            if s is None:
                s = self._lane_streams[(Y.device, h)] = torch.cuda.Stream(device=Y.device)
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                Yh = Y[a:b].contiguous()
                lane_noise.append(sampler.LaneNoise(noise, a, b, B))
                lanes.append((s, self._iter(Yh, lane_noise[-1])))
        starts = None
        if self.stagger:
            # lane k's first launch waits for lane k-1's first evaluation to pass the bottleneck
            evs = [torch.cuda.Event() for _ in range(nl - 1)]

            def arm(k):
                if k + 1 < nl:
                    self.net.mid_hook = lambda: evs[k].record(torch.cuda.current_stream())

            def start(k):
                if k > 0:
                    torch.cuda.current_stream().wait_event(evs[k - 1])
                arm(k)

            starts = start
        res = sampler.pc_sample_lockstep(lanes, on_first=starts)
        self.net.mid_hook = None
        noise.i = lane_noise[0].i  # the parent has now supplied the lanes' draws (as the one-stream run does)
        for (s, _), (x, _) in zip(lanes, res):
            cur.wait_stream(s)
            x.record_stream(cur)
        return torch.cat([x for x, _ in res]), res[0][1]

    def __call__(self, y, noise=None):
        """y [B, L] f32 device -> (x_hat [B, L] f32, nfe)."""
        B, L = y.shape
        nf = ops.absmax(y)  # norm_factor = max|y| (model.py:726)
        T = 1 + L // 128
        Y = ops.stft(y, 1.0, tpad=pad_frames(T), mode=self.mode, in_div=nf)
        x, nfe = self.sample(Y, noise)
        return ops.istft(x, L, mode=self.mode, out_scale=nf), nfe

class SNRAlignedEnhancer:
    """One-step SNR-aligned enhancement of a batch (C4: model_type 'sebridge_v3',
    snr_conditioned 'true'; model.py:713-740, 810-833), the reference's per-utterance loop as one
    batched pass: y / max|y| -> raw STFT padded to 16 frames -> SNR estimate (`snr_fn`, e.g.
    SNRNet's forward_complex -> g / (1 - g), or oracle noise/clean rms) -> t_hat snapped to t_30
    -> Y = spec_fwd(STFT(y / (max|y| normfac))) -> X_T = Y + sigma_max t_hat Z -> one
    preconditioned NCSN++ evaluation at t_hat (c_skip x + c_out dnn, score mode 1) -> iSTFT x
    max|y| normfac.  The per-utterance scalars (t_hat, normfac) are host float64 as in the
    reference (one B-element copy).  Returns (x_hat [B, L], t_hat numpy [B])."""

    def __init__(self, net, snr_fn=None, fixed_snr=0.17783, sigma_max=0.5, transform="exponent"):
        self.net, self.snr_fn = net, snr_fn
        self.mode = transform_mode(transform)
        self.fixed_snr, self.sigma_max = float(fixed_snr), float(sigma_max)

    def __call__(self, y, est_snr=None, noise=None, seed=0):
        B, L = y.shape
        nf = ops.absmax(y)
        if est_snr is None:
            T16 = pad_frames(1 + L // 128, 16)
            raw = ops.stft(y, 1.0, tpad=T16, mode=0, in_div=nf)  # no spec transform (model.py:715-719)
            est_snr = self.snr_fn(raw).reshape(B).double().cpu().numpy()
        t_hat = snap_t(est_snr, self.fixed_snr)
        div = nf * torch.from_numpy(normfac(t_hat, self.fixed_snr)).to(nf.device, torch.float32)
        Y = ops.stft(y, 1.0, tpad=pad_frames(1 + L // 128), mode=self.mode, in_div=div)
        coef = torch.zeros(B, 4, dtype=torch.float32)
        coef[:, 1] = 1.0
        coef[:, 3] = torch.from_numpy(self.sigma_max * t_hat).float()
        X_T = ops.axpby_noise(coef.to(Y.device), y=Y, noise=noise, seed=seed)
        tv = torch.from_numpy(t_hat).to(Y.device, torch.float32)
        sample = self.net.score(X_T, Y, tv, 1)
        return ops.istft(sample.contiguous(), L, mode=self.mode, out_scale=div.contiguous()), t_hat

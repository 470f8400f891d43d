"""Predictor-corrector reverse-diffusion sampler driven by the fused HIP kernels.

Restates the reference loop (sampling/__init__.py:54-75, timesteps_space 84-91) with every
per-element update done by snrse_score_update (network output head + score + step in one
kernel) or snrse_sde_update (arbitrary score tensors).  Per-step scalars (t, stepsize, SDE
std / diffusion, step sizes) are host float64 tables computed once per call and uploaded
as one device tensor, so the loop issues no host<->device synchronisation.

Step algebra (all elementwise on complex64, per-utterance scalars a, by, c, s):
  x_mean = a x + by y + c score,   x = x_mean + s z
  ALD corrector (correctors.py:69-81):   a=1, by=0, c=e, s=sqrt(2e), e = 2 (snr std(t))^2
  reverse diffusion (predictors.py:75-80 with SDE.discretize sdes.py:86-91, RSDE 132-140):
      OUVE drift theta (y - x):  a = 1 + theta dt, by = -theta dt, c = G^2, s = G
      BBED / PROPOSED_1 drift (y - x)/(1 - t): a = 1 + dt/(1-t), by = -dt/(1-t), c = G^2, s = G
      with G = g(t) sqrt(dt), dt = stepsize
  Euler-Maruyama (predictors.py:46-52): dt = -1/N,
      a = 1 - theta dt (OUVE) | 1 - dt/(1-t) (BBED), by = -(a - 1), c = -g^2 dt, s = g sqrt(-dt)
  prior (sdes.py:225-232 / 298-304): x = y + std(T) z
"""
from __future__ import annotations

import math

import numpy as np
import scipy.special as sc
import torch

from . import ops


class SDESpec:
    """Scalar side of an SDE (float64 host math)."""

    def __init__(self, kind, **kw):
        self.kind = kind
        if kind == "ouve":
            self.theta = float(kw.get("theta", 1.5))
            self.sigma_min = float(kw.get("sigma_min", 0.05))
            self.sigma_max = float(kw.get("sigma_max", 0.5))
            self.logsig = math.log(self.sigma_max / self.sigma_min)
            self.T = float(kw.get("T", 1.0))
        elif kind == "bbed":
            self.k = float(kw.get("k", 2.6))
            self.theta = float(kw.get("theta", 0.52))
            self.logk = math.log(self.k)
            self.Eilog = float(sc.expi(-2 * self.logk))
            self.T = float(kw.get("T", 0.999))
        elif kind == "proposed_1":
            # BBED in the (sigma_min, sigma_max) parameterisation, sdes.py:314-392
            self.sigma_min = float(kw.get("sigma_min", 1.0))
            self.sigma_max = float(kw.get("sigma_max", 1.0))
            self.theta = float(kw.get("theta", 0.53))
            self.logsig = math.log(self.sigma_max / self.sigma_min)
            self.ratio = self.sigma_max / self.sigma_min
            self.Eilog = float(sc.expi(-2 * self.logsig))
            self.T = float(kw.get("T", 0.99))
        else:
            raise ValueError(f"SDE kind {kind} unknown")

    def g(self, t):
        if self.kind == "ouve":
            return self.sigma_min * (self.sigma_max / self.sigma_min) ** t * math.sqrt(2 * self.logsig)
        if self.kind == "proposed_1":  # sdes.py:359-361: sigma = sigma_max * t (linear in t, as written)
            return self.sigma_max * t * math.sqrt(self.theta)
        return self.k ** t * math.sqrt(self.theta)

    def std(self, t):
        if self.kind == "ouve":
            a = self.sigma_min ** 2 * math.exp(-2 * self.theta * t) * (math.exp(2 * (self.theta + self.logsig) * t) - 1)
            return math.sqrt(a * self.logsig / (self.theta + self.logsig))
        if self.kind == "proposed_1":  # sdes.py:371-378
            Eis = float(sc.expi(2 * (t - 1) * self.logsig)) - self.Eilog
            k = 2 * self.sigma_max ** 2 * self.logsig
            var = self.sigma_min ** 2 * (self.ratio ** (2 * t) - 1 + t) + k * (1 - t) * Eis
        else:
            Eis = float(sc.expi(2 * (t - 1) * self.logk)) - self.Eilog
            h = 2 * self.k ** 2 * self.logk
            var = (self.k ** (2 * t) - 1 + t) + h * (1 - t) * Eis
        v = var * (1 - t) * self.theta
        return math.sqrt(v) if v >= 0 else float("nan")

    def drift_coef(self, t):
        """drift = kappa (y - x)."""
        return self.theta if self.kind == "ouve" else 1.0 / (1.0 - t)


def timesteps(T, N, eps):
    # torch.linspace in float32, exactly as the reference (sampling/__init__.py:84-86)
    return torch.linspace(T, eps, N, dtype=torch.float32).double().numpy()


def build_schedule(sde: SDESpec, N, eps, predictor, corrector, snr, corrector_steps, probability_flow=False):
    """List of ('corr'|'pred', t, (a, by, c, s)) in execution order + prior coefficient.
    `probability_flow` is accepted and ignored, as in the reference: its Predictor builds the reverse
    SDE without the flag (predictors.py:18), so the PC updates never change with it."""
    ts = timesteps(sde.T, N, eps)
    steps = []
    for i in range(N):
        t = float(ts[i])
        stepsize = float(ts[i] - ts[i + 1]) if i != N - 1 else float(ts[-1])
        if corrector == "ald":
            e = (snr * sde.std(t)) ** 2 * 2
            for _ in range(corrector_steps):
                steps.append(("corr", t, (1.0, 0.0, e, math.sqrt(e * 2))))
        elif corrector == "langevin":
            for _ in range(corrector_steps):
                steps.append(("langevin", t, None))
        elif corrector != "none":
            raise ValueError(f"Corrector with name '{corrector}' unknown.")
        kap = sde.drift_coef(t)
        if predictor == "reverse_diffusion":
            G = sde.g(t) * math.sqrt(stepsize)
            steps.append(("pred", t, (1.0 + kap * stepsize, -kap * stepsize, G * G, G)))
        elif predictor == "euler_maruyama":
            dt = -1.0 / N
            g = sde.g(t)
            steps.append(("pred", t, (1.0 - kap * dt, kap * dt, -g * g * dt, g * math.sqrt(-dt))))
        elif predictor == "none":
            steps.append(("none", t, None))
        else:
            raise ValueError(f"Predictor with name '{predictor}' unknown.")
    prior = (0.0, 1.0, 0.0, sde.std(sde.T))
    n_corr = 0 if corrector == "none" else corrector_steps
    return steps, prior, N * (n_corr + 1)


class NoiseSource:
    """Draw i of the sampler: injected tensor (parity mode) or in-kernel Philox (seed, offset)."""

    def __init__(self, seed=0, tape=None):
        self.seed, self.tape, self.i = int(seed), tape, 0

    def next(self, numel):
        i = self.i
        self.i += 1
        if self.tape is not None:
            return self.tape(i), 0
        return None, i * numel


class LaneNoise(NoiseSource):
    """The draws of batch rows [a, b) of a parent NoiseSource over the whole batch: the tape's row slice,
    or the parent's Philox counters of those elements (offset i * numel(batch) + a * numel(row)), so a
    half-batch run on its own stream draws exactly the numbers the whole-batch run would."""

    def __init__(self, parent: NoiseSource, a, b, rows):
        super().__init__(parent.seed, None)
        self.parent_tape, self.a, self.b, self.rows = parent.tape, a, b, rows
        self.i = parent.i  # continue where the parent's earlier draws left off

    def next(self, numel):
        i = self.i
        self.i += 1
        if self.parent_tape is not None:
            return self.parent_tape(i)[self.a:self.b].contiguous(), 0
        row = numel // (self.b - self.a)
        return None, i * row * self.rows + self.a * row


def pc_sample(score_step, Y, sde: SDESpec, N=30, eps=0.03, snr=0.5, predictor="reverse_diffusion",
              corrector="ald", corrector_steps=1, noise: NoiseSource | None = None, denoise=True,
              score_tensor=None, Y_prior=None, probability_flow=False):
    """Run the PC loop.  Y: complex64 [B, F, T] (device).
    score_step(x, t_vec, coef_row, z, seed, offset) -> (x_new, x_mean) runs the network + fused step;
    score_tensor(x, t_vec) -> complex score (only needed for the Langevin corrector).
    Returns (x_result, nfe)."""
    it = pc_sample_iter(score_step, Y, sde, N=N, eps=eps, snr=snr, predictor=predictor, corrector=corrector,
                        corrector_steps=corrector_steps, noise=noise, denoise=denoise, score_tensor=score_tensor,
                        Y_prior=Y_prior, probability_flow=probability_flow)
    while True:
        try:
            next(it)
        except StopIteration as e:
            return e.value


def pc_sample_lockstep(lanes, on_first=None):
    """Run several PC loops (one per half-batch) with their launches interleaved step by step, each
    on its own HIP stream and split-K workspace: `lanes` = [(stream, pc_sample_iter generator)].
    While one lane's network evaluation is in its latency-bound low-resolution levels, the other
    lane's full-resolution GEMMs fill the chip.  on_first(k) runs on lane k's stream before its first
    step (the enhancer's stagger).  Returns [(x_result, nfe)] in lane order."""
    out = [None] * len(lanes)
    live = list(range(len(lanes)))
    first = [True] * len(lanes)
    while live:
        for k in list(live):
            stream, it = lanes[k]
            dev = stream.device
            with torch.cuda.stream(stream):
                ops.use_workspace_lane(k, dev)
                if first[k]:
                    first[k] = False
                    if on_first is not None:
                        on_first(k)
                try:
                    next(it)
                except StopIteration as e:
                    out[k] = e.value
                    live.remove(k)
    ops.use_workspace_lane(0, lanes[0][0].device)
    return out


def pc_sample_iter(score_step, Y, sde: SDESpec, N=30, eps=0.03, snr=0.5, predictor="reverse_diffusion",
                   corrector="ald", corrector_steps=1, noise: NoiseSource | None = None, denoise=True,
                   score_tensor=None, Y_prior=None, probability_flow=False):
    """pc_sample as a generator: yields after issuing each step (one network evaluation + its fused SDE
    update), returns (x_result, nfe) through StopIteration."""
    noise = noise or NoiseSource()
    steps, prior, ns = build_schedule(sde, N, eps, predictor, corrector, snr, corrector_steps, probability_flow)
    B = Y.shape[0]
    dev = Y.device
    numel = Y.numel()
    coefs = [c for _, _, c in steps if c is not None] + [prior]
    ctab = torch.tensor(np.repeat(np.asarray(coefs, dtype=np.float32)[:, None, :], B, axis=1), device=dev)
    ttab = torch.tensor(np.repeat(np.asarray([t for _, t, _ in steps], dtype=np.float32)[:, None], B, axis=1),
                        device=dev)
    z, off = noise.next(numel)
    x = ops.axpby_noise(ctab[-1], y=Y if Y_prior is None else Y_prior, noise=z, seed=noise.seed, offset=off)
    x_mean = x
    ci = 0
    for si, (kind, t, cf) in enumerate(steps):
        tv = ttab[si]
        if kind in ("corr", "pred"):
            z, off = noise.next(numel)
            x, x_mean = score_step(x, tv, ctab[ci], z, noise.seed, off)
            ci += 1
            yield
        elif kind == "langevin":
            grad = score_tensor(x, tv)
            z, off = noise.next(numel)
            if z is None:  # Langevin needs the noise norm: materialise the draw
                z = ops.axpby_noise(torch.tensor([[0.0, 0.0, 0.0, 1.0]] * B, device=dev, dtype=torch.float32),
                                    like=Y, seed=noise.seed, offset=off)
            gn = torch.linalg.vector_norm(grad.reshape(B, -1), dim=-1).mean()
            nn_ = torch.linalg.vector_norm(z.reshape(B, -1), dim=-1).mean()
            e = (snr * nn_ / gn) ** 2 * 2
            row = torch.stack([torch.ones_like(e), torch.zeros_like(e), e, torch.sqrt(e * 2)]).float()
            x, x_mean = ops.sde_update(x, row.expand(B, 4).contiguous(), score=grad, noise=z)
            yield
        else:  # NonePredictor
            x_mean = x
    return (x_mean if denoise else x), ns

"""CPU oracle (TEST INFRASTRUCTURE ONLY) — SDEs and the predictor-corrector sampler.

Restates:
  OUVESDE           sdes.py:149-232  (drift 192-200, _mean 202-205, _std 207-220, prior 225-232)
  BBED              sdes.py:240-304  (drift 275-279, _mean 282-285, _std 287-293, prior 298-304)
  SDE.discretize    sdes.py:73-91;   RSDE.discretize 132-140
  ReverseDiffusionPredictor.update_fn   predictors.py:75-80
  AnnealedLangevinDynamics.update_fn    correctors.py:69-81
  LangevinCorrector.update_fn           correctors.py:45-56
  get_pc_sampler / pc_sampler           sampling/__init__.py:28-80, timesteps_space 84-91
Noise is injected through `noise(shape)` (reference: torch.randn_like) so runs are
reproducible across devices.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.special as sc
import torch


class OUVE:
    def __init__(self, theta=1.5, sigma_min=0.05, sigma_max=0.5, N=30):
        self.theta, self.sigma_min, self.sigma_max, self.N = theta, sigma_min, sigma_max, N
        self.logsig = math.log(sigma_max / sigma_min)
        self.T = 1.0

    def g(self, t):
        return self.sigma_min * (self.sigma_max / self.sigma_min) ** t * math.sqrt(2 * self.logsig)

    def drift(self, x, t, y):
        return self.theta * (y - x)

    def std(self, t):
        a = self.sigma_min ** 2 * np.exp(-2 * self.theta * t) * (np.exp(2 * (self.theta + self.logsig) * t) - 1)
        return np.sqrt(a * self.logsig / (self.theta + self.logsig))

    def mean(self, x0, t, y):
        e = np.exp(-self.theta * t)
        return e * x0 + (1 - e) * y

    def prior_std(self):
        return float(self.std(1.0))


class BBED:
    def __init__(self, T=0.999, k=2.6, theta=0.52, N=30):
        self.T, self.k, self.theta, self.N = T, k, theta, N
        self.logk = math.log(k)
        self.Eilog = sc.expi(-2 * self.logk)

    def g(self, t):
        return self.k ** t * math.sqrt(self.theta)

    def drift(self, x, t, y):
        return (y - x) / (1.0 - t)

    def std(self, t):
        t = np.asarray(t, dtype=np.float64)
        Eis = sc.expi(2 * (t - 1) * self.logk) - self.Eilog
        h = 2 * self.k ** 2 * self.logk
        var = (self.k ** (2 * t) - 1 + t) + h * (1 - t) * Eis
        return np.sqrt(var * (1 - t) * self.theta)

    def mean(self, x0, t, y):
        return x0 * (1 - t) + y * t

    def prior_std(self):
        return float(self.std(self.T))


class PROPOSED_1:
    """sdes.py:314-392: BBED in the (sigma_min, sigma_max) parameterisation, restated as written
    (diffusion sigma_max * t * sqrt(theta), sdes.py:359-361; std sdes.py:371-378)."""

    def __init__(self, T=0.99, sigma_min=1.0, sigma_max=1.0, theta=0.53, N=30):
        self.T, self.sigma_min, self.sigma_max, self.theta, self.N = T, sigma_min, sigma_max, theta, N
        self.logsig = math.log(sigma_max / sigma_min)
        self.ratio = sigma_max / sigma_min
        self.Eilog = sc.expi(-2 * self.logsig)

    def g(self, t):
        return self.sigma_max * t * math.sqrt(self.theta)

    def drift(self, x, t, y):
        return (y - x) / (1.0 - t)

    def std(self, t):
        t = np.asarray(t, dtype=np.float64)
        Eis = sc.expi(2 * (t - 1) * self.logsig) - self.Eilog
        k = 2 * self.sigma_max ** 2 * self.logsig
        var = self.sigma_min ** 2 * (self.ratio ** (2 * t) - 1 + t) + k * (1 - t) * Eis
        return np.sqrt(var * (1 - t) * self.theta)

    def mean(self, x0, t, y):
        return x0 * (1 - t) + y * t

    def prior_std(self):
        return float(self.std(self.T))


def pc_sample(sde, score_fn, Y, noise, predictor="reverse_diffusion", corrector="ald",
              N=None, eps=0.03, snr=0.5, corrector_steps=1, denoise=True):
    """pc_sampler (sampling/__init__.py:54-75) for a batch Y (complex [B,1,F,T]).
    t is handled per step as a python float (every batch element shares it)."""
    N = sde.N if N is None else N
    xt = Y + noise(Y.shape) * sde.prior_std()
    ts = torch.linspace(sde.T, eps, N, dtype=torch.float32).double().numpy()
    x_mean = xt
    for i in range(N):
        t = float(ts[i])
        stepsize = float(ts[i] - ts[i + 1]) if i != N - 1 else float(ts[-1])
        # corrector
        if corrector == "ald":
            std = float(sde.std(t))
            for _ in range(corrector_steps):
                grad = score_fn(xt, t, Y)
                z = noise(xt.shape)
                step = (snr * std) ** 2 * 2
                x_mean = xt + step * grad
                xt = x_mean + z * math.sqrt(step * 2)
        elif corrector == "langevin":
            for _ in range(corrector_steps):
                grad = score_fn(xt, t, Y)
                z = noise(xt.shape)
                gn = torch.linalg.vector_norm(grad.reshape(grad.shape[0], -1), dim=-1).mean()
                nn_ = torch.linalg.vector_norm(z.reshape(z.shape[0], -1), dim=-1).mean()
                step = (snr * nn_ / gn) ** 2 * 2
                x_mean = xt + step * grad
                xt = x_mean + z * torch.sqrt(step * 2)
        elif corrector != "none":
            raise ValueError(corrector)
        # predictor
        if predictor == "reverse_diffusion":
            f = sde.drift(xt, t, Y) * stepsize
            G = sde.g(t) * math.sqrt(stepsize)
            rev_f = f - G ** 2 * score_fn(xt, t, Y)
            z = noise(xt.shape)
            x_mean = xt - rev_f
            xt = x_mean + G * z
        elif predictor == "euler_maruyama":
            dt = -1.0 / N
            z = noise(xt.shape)
            g = sde.g(t)
            f = sde.drift(xt, t, Y) - g ** 2 * score_fn(xt, t, Y)
            x_mean = xt + f * dt
            xt = x_mean + g * math.sqrt(-dt) * z
        elif predictor == "none":
            x_mean = xt  # NonePredictor returns (x, x)  (predictors.py:93-94)
        else:
            raise ValueError(predictor)
    n_corr = 0 if corrector == "none" else corrector_steps  # NoneCorrector.n_steps = 0
    return (x_mean if denoise else xt), N * (n_corr + 1)

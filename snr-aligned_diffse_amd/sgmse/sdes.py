"""SDEs of the enhancement path — reference API (sgmse/sdes.py:20-392).

`OUVESDE`, `BBED` and `PROPOSED_1` keep the reference's method names and shapes (sde, marginal_prob,
_mean, _std, prior_sampling, discretize, reverse, copy, N, T) so user code and the
samplers interoperate.  The per-element work of the samplers does not go through these
methods: `spec()` hands the scalar side (float64 host math) to snrse.sampler, whose fused
HIP kernels apply the same algebra.

Defined behaviour where the reference breaks:
  * BBED._std stays in the input's float dtype (the reference round-trips through numpy
    float64 and returns complex128 samples that the network then rejects);
  * BBED.sde broadcasts a [B] time vector over [B, 1, F, T] (the reference only works for B=1);
  * BBED._std(1.0) is NaN exactly as in the reference (0 * inf).
"""
from __future__ import annotations

import abc
import math
import warnings

import numpy as np
import scipy.special as sc
import torch

from snrse.sampler import SDESpec

from .util.registry import Registry

SDERegistry = Registry("SDE")


def _bc(t, x):
    t = torch.as_tensor(t, device=x.device if torch.is_tensor(x) else None)
    if t.dim() == 0:
        return t
    return t.reshape(-1, *([1] * (x.dim() - 1)))


class SDE(abc.ABC):
    def __init__(self, N):
        super().__init__()
        self.N = N

    @abc.abstractmethod
    def sde(self, x, t, *args): ...

    @abc.abstractmethod
    def marginal_prob(self, x, t, *args): ...

    @abc.abstractmethod
    def prior_sampling(self, shape, *args): ...

    def prior_logp(self, z):
        raise NotImplementedError("prior_logp is not implemented (reference sdes.py:234-235, 306-307)")

    @abc.abstractmethod
    def spec(self) -> SDESpec: ...

    def discretize(self, x, t, y, stepsize):
        """Euler-Maruyama discretisation (sdes.py:73-91): f = drift dt, G = g sqrt(dt)."""
        drift, diffusion = self.sde(x, t, y)
        dt = torch.as_tensor(stepsize, device=t.device, dtype=torch.float32)
        return drift * dt, diffusion * torch.sqrt(dt)

    def reverse(oself, score_model, probability_flow=False):
        """Reverse-time SDE (sdes.py:93-142)."""
        N, T, sde_fn, discretize_fn = oself.N, oself.T, oself.sde, oself.discretize

        class RSDE:
            def __init__(self):
                self.N = N
                self.T = T
                self.probability_flow = probability_flow

            def sde(self, x, t, *args):
                p = self.rsde_parts(x, t, *args)
                return p["total_drift"], p["diffusion"]

            def rsde_parts(self, x, t, *args):
                sde_drift, sde_diffusion = sde_fn(x, t, *args)
                score = score_model(x, t, *args)
                g = _bc(sde_diffusion, x)
                score_drift = -g ** 2 * score * (0.5 if self.probability_flow else 1.0)
                diffusion = torch.zeros_like(sde_diffusion) if self.probability_flow else sde_diffusion
                return {"total_drift": sde_drift + score_drift, "diffusion": diffusion, "sde_drift": sde_drift,
                        "sde_diffusion": sde_diffusion, "score_drift": score_drift, "score": score}

            def discretize(self, x, t, y, stepsize):
                f, G = discretize_fn(x, t, y, stepsize)
                if torch.is_complex(G):
                    G = G.imag
                rev_f = f - _bc(G, x) ** 2 * score_model(x, t, y) * (0.5 if self.probability_flow else 1.0)
                rev_G = torch.zeros_like(G) if self.probability_flow else G
                return rev_f, rev_G

        return RSDE()

    @abc.abstractmethod
    def copy(self): ...


@SDERegistry.register("ouve")
class OUVESDE(SDE):
    @staticmethod
    def add_argparse_args(parser):
        parser.add_argument("--sde-n", type=int, default=1000, help="The number of timesteps in the SDE discretization.")
        parser.add_argument("--theta", type=float, default=1.5, help="The constant stiffness of the Ornstein-Uhlenbeck process.")
        parser.add_argument("--sigma-min", type=float, default=0.05, help="The minimum sigma to use.")
        parser.add_argument("--sigma-max", type=float, default=0.5, help="The maximum sigma to use.")
        return parser

    def __init__(self, theta, sigma_min, sigma_max, N=1000, **ignored_kwargs):
        """dx = theta (y - x) dt + sigma(t) dw, sigma(t) = sigma_min (sigma_max/sigma_min)^t sqrt(2 log(sigma_max/sigma_min))."""
        super().__init__(N)
        self.theta, self.sigma_min, self.sigma_max = theta, sigma_min, sigma_max
        self.logsig = np.log(self.sigma_max / self.sigma_min)
        self._T = 1

    def copy(self):
        # as the reference (sdes.py:185-186): the copy starts from the constructor's _T = 1, so
        # eval.py's `model.sde._T = reverse_starting_point` does not reach get_pc_sampler (model.py:552)
        return OUVESDE(self.theta, self.sigma_min, self.sigma_max, N=self.N)

    @property
    def T(self):
        return self._T

    def sde(self, x, t, y):
        drift = self.theta * (y - x)
        sigma = self.sigma_min * (self.sigma_max / self.sigma_min) ** t
        return drift, sigma * np.sqrt(2 * self.logsig)

    def _mean(self, x0, t, y):
        e = torch.exp(-self.theta * t)[:, None, None, None]
        return e * x0 + (1 - e) * y

    def _std(self, t):
        s, th, ls = self.sigma_min, self.theta, self.logsig
        return torch.sqrt(s ** 2 * torch.exp(-2 * th * t) * (torch.exp(2 * (th + ls) * t) - 1) * ls / (th + ls))

    def marginal_prob(self, x0, t, y):
        return self._mean(x0, t, y), self._std(t)

    def prior_sampling(self, shape, y):
        if shape != y.shape:
            warnings.warn(f"Target shape {shape} does not match shape of y {y.shape}! Ignoring target shape.")
        std = self._std(torch.ones((y.shape[0],), device=y.device))
        z = torch.randn_like(y)
        return y + z * std[:, None, None, None], z

    def spec(self):
        return SDESpec("ouve", theta=self.theta, sigma_min=self.sigma_min, sigma_max=self.sigma_max, T=float(self._T))


@SDERegistry.register("bbed")
class BBED(SDE):
    @staticmethod
    def add_argparse_args(parser):
        parser.add_argument("--sde-n", type=int, default=30, help="The number of timesteps in the SDE discretization.")
        parser.add_argument("--T_sampling", type=float, default=0.999, help="The T so that t < T during sampling.")
        parser.add_argument("--k", type=float, default=2.6, help="base factor for diffusion term")
        parser.add_argument("--theta", type=float, default=0.52, help="root scale factor for diffusion term.")
        return parser

    def __init__(self, T_sampling=0.999, k=2.6, theta=0.52, N=1000, **kwargs):
        """dx = (y - x)/(Tc - t) dt + sqrt(theta) k^t dw (Brownian bridge, exploding diffusion)."""
        super().__init__(N)
        self.k, self.logk, self.theta = k, np.log(k), theta
        self.Eilog = sc.expi(-2 * self.logk)
        self.T = T_sampling
        self.Tc = 1

    def copy(self):
        return BBED(self.T, self.k, self.theta, N=self.N)

    def sde(self, x, t, y):
        tb = _bc(t, x)
        drift = (y - x) / (self.Tc - tb)
        return drift, (self.k ** t) * np.sqrt(self.theta)

    def _mean(self, x0, t, y):
        time = (t / self.Tc)[:, None, None, None]
        return x0 * (1 - time) + y * time

    def _std(self, t):
        t64 = t.detach().cpu().double().numpy()
        Eis = sc.expi(2 * (t64 - 1) * self.logk) - self.Eilog
        h = 2 * self.k ** 2 * self.logk
        var = ((self.k ** (2 * t64) - 1 + t64) + h * (1 - t64) * Eis) * (1 - t64) * self.theta
        return torch.sqrt(torch.as_tensor(var, device=t.device)).to(t.dtype if t.is_floating_point() else torch.float32)

    def marginal_prob(self, x0, t, y):
        return self._mean(x0, t, y), self._std(t)

    def prior_sampling(self, shape, y):
        if shape != y.shape:
            warnings.warn(f"Target shape {shape} does not match shape of y {y.shape}! Ignoring target shape.")
        std = self._std(self.T * torch.ones((y.shape[0],), device=y.device))
        z = torch.randn_like(y)
        return y + z * std[:, None, None, None], z

    def spec(self):
        return SDESpec("bbed", k=self.k, theta=self.theta, T=float(self.T))


@SDERegistry.register("proposed_1")
class PROPOSED_1(SDE):
    """BBED in the (sigma_min, sigma_max) parameterisation (reference sdes.py:312-392; k = sigma_max /
    sigma_min).  As written there, the diffusion is sigma_max * t * sqrt(theta) (linear in t, sdes.py:359)
    while the marginal std uses the exponential form (sdes.py:371-378); both are kept as written."""

    @staticmethod
    def add_argparse_args(parser):
        parser.add_argument("--sde-n", type=int, default=1000, help="The number of timesteps in the SDE discretization.")
        parser.add_argument("--T_sampling", type=float, default=0.99, help="The T so that t < T during sampling in the train step.")
        parser.add_argument("--sigma-min", type=float, default=1, help="The minimum sigma to use. Set it to 1 and dont change it.")
        parser.add_argument("--sigma-max", type=float, default=1, help="This is k, the base of diffusion term, when sigma min is 1.")
        parser.add_argument("--theta", type=float, default=0.53, help="This rescales the diffusion term")
        return parser

    def __init__(self, T_sampling=0.99, sigma_min=1.0, sigma_max=1.0, theta=0.53, N=1000, **kwargs):
        super().__init__(N)
        self.sigma_min, self.sigma_max, self.theta = sigma_min, sigma_max, theta
        self.logsig = np.log(self.sigma_max / self.sigma_min)
        self.ratio = self.sigma_max / self.sigma_min
        self.Eilog = sc.expi(-2 * self.logsig)
        self.T = T_sampling
        self.Tc = 1

    def copy(self):
        return PROPOSED_1(self.T, self.sigma_min, self.sigma_max, self.theta, N=self.N)

    def sde(self, x, t, y):
        tb = _bc(t, x)
        drift = (y - x) / (self.Tc - tb)
        return drift, (self.sigma_max * t) * np.sqrt(self.theta)

    def _mean(self, x0, t, y):
        time = (t / self.Tc)[:, None, None, None]
        return x0 * (1 - time) + y * time

    def _std(self, t):
        t64 = t.detach().cpu().double().numpy()
        Eis = sc.expi(2 * (t64 - 1) * self.logsig) - self.Eilog
        k = 2 * self.sigma_max ** 2 * self.logsig
        var = (self.sigma_min ** 2 * (self.ratio ** (2 * t64) - 1 + t64) + k * (1 - t64) * Eis) * (1 - t64) * self.theta
        return torch.sqrt(torch.as_tensor(var, device=t.device)).to(t.dtype if t.is_floating_point() else torch.float32)

    def marginal_prob(self, x0, t, y):
        return self._mean(x0, t, y), self._std(t)

    def prior_sampling(self, shape, y):
        if shape != y.shape:
            warnings.warn(f"Target shape {shape} does not match shape of y {y.shape}! Ignoring target shape.")
        std = self._std(self.T * torch.ones((y.shape[0],), device=y.device))
        z = torch.randn_like(y)
        return y + z * std[:, None, None, None], z

    def spec(self):
        return SDESpec("proposed_1", sigma_min=self.sigma_min, sigma_max=self.sigma_max, theta=self.theta,
                       T=float(self.T))


def sde_spec(sde) -> SDESpec:
    if hasattr(sde, "spec"):
        return sde.spec()
    raise TypeError(f"no scalar spec for SDE {type(sde).__name__}")


__all__ = ["SDERegistry", "SDE", "OUVESDE", "BBED", "PROPOSED_1", "math"]

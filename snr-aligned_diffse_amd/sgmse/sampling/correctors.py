"""Correctors — reference API (sampling/correctors.py:8-94); updates run on snrse_sde_update."""
import abc
import math

import torch

from snrse import ops

from ..util.registry import Registry
from .predictors import _noise_seed

CorrectorRegistry = Registry("Corrector")


class Corrector(abc.ABC):
    def __init__(self, sde, score_fn, snr, n_steps):
        super().__init__()
        self.rsde = sde.reverse(score_fn)
        self.score_fn = score_fn
        self.snr = snr
        self.n_steps = n_steps

    @abc.abstractmethod
    def update_fn(self, x, t, *args):
        """One corrector update -> (x, x_mean)."""


def _flat(x):
    return x.reshape(x.shape[0], x.shape[-2], x.shape[-1]).contiguous()


@CorrectorRegistry.register(name="langevin")
class LangevinCorrector(Corrector):
    def update_fn(self, x, t, *args):
        """step = 2 (snr ||z|| / ||grad||)^2 (batch means), x_mean = x + step grad (correctors.py:45-56)."""
        x_mean = x
        B = x.shape[0]
        for _ in range(self.n_steps):
            grad = self.score_fn(x, t, *args)
            unit = torch.tensor([[0.0, 0.0, 0.0, 1.0]] * B, device=x.device)
            z = ops.axpby_noise(unit, like=_flat(x), seed=_noise_seed())
            gn = torch.linalg.vector_norm(grad.reshape(B, -1), dim=-1).mean()
            nn_ = torch.linalg.vector_norm(z.reshape(B, -1), dim=-1).mean()
            e = (self.snr * nn_ / gn) ** 2 * 2
            row = torch.stack([torch.ones_like(e), torch.zeros_like(e), e, torch.sqrt(e * 2)]).float()
            xo, xm = ops.sde_update(_flat(x), row.expand(B, 4).contiguous(), score=_flat(grad), noise=z)
            x, x_mean = xo.reshape(x.shape), xm.reshape(x.shape)
        return x, x_mean


@CorrectorRegistry.register(name="ald")
class AnnealedLangevinDynamics(Corrector):
    """The original annealed Langevin dynamics corrector of NCSN/NCSNv2 (correctors.py:59-81)."""

    def __init__(self, sde, score_fn, snr, n_steps):
        super().__init__(sde, score_fn, snr, n_steps)
        self.sde = sde

    def update_fn(self, x, t, y):
        B = x.shape[0]
        std = self.sde.spec().std(float(t.reshape(-1)[0]))
        e = (self.snr * std) ** 2 * 2
        coef = torch.tensor([[1.0, 0.0, e, math.sqrt(2 * e)]] * B, device=x.device)
        x_mean = x
        for _ in range(self.n_steps):
            grad = self.score_fn(x, t, y)
            xo, xm = ops.sde_update(_flat(x), coef, score=_flat(grad), seed=_noise_seed())
            x, x_mean = xo.reshape(x.shape), xm.reshape(x.shape)
        return x, x_mean


@CorrectorRegistry.register(name="none")
class NoneCorrector(Corrector):
    def __init__(self, *args, **kwargs):
        self.snr = 0
        self.n_steps = 0

    def update_fn(self, x, t, *args):
        return x, x

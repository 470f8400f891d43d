"""Predictors — reference API (sampling/predictors.py:9-94); updates run on snrse_sde_update."""
import abc
import math

import torch

from snrse import ops

from ..util.registry import Registry

PredictorRegistry = Registry("Predictor")


def _noise_seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class Predictor(abc.ABC):
    def __init__(self, sde, score_fn, probability_flow=False):
        super().__init__()
        self.sde = sde
        # as the reference (predictors.py:18): the reverse SDE is built WITHOUT probability_flow, so the
        # flag is stored but changes nothing in the updates below
        self.rsde = sde.reverse(score_fn)
        self.score_fn = score_fn
        self.probability_flow = probability_flow

    @abc.abstractmethod
    def update_fn(self, x, t, *args):
        """One predictor update -> (x, x_mean)."""

    def debug_update_fn(self, x, t, *args):
        raise NotImplementedError(f"Debug update function not implemented for predictor {self}.")

    def _step(self, x, y, score, a, by, c, s):
        B = x.shape[0]
        coef = torch.tensor([[a, by, c, s]] * B, device=x.device, dtype=torch.float32)
        xv = x.reshape(B, x.shape[-2], x.shape[-1]).contiguous()
        yv = None if y is None else y.reshape(xv.shape).contiguous()
        sv = score.reshape(xv.shape).contiguous()
        xo, xm = ops.sde_update(xv, coef, y=yv, score=sv, seed=_noise_seed())
        return xo.reshape(x.shape), xm.reshape(x.shape)


@PredictorRegistry.register("euler_maruyama")
class EulerMaruyamaPredictor(Predictor):
    def update_fn(self, x, t, *args):
        """x_mean = x + f dt, x = x_mean + g sqrt(-dt) z with dt = -1/N (predictors.py:46-52).
        Extra positional args beyond y (the pc loop's stepsize) are ignored; the reference's
        loop passes it through to sde.sde() and fails."""
        y = args[0]
        sp = self.sde.spec()
        tt = float(t.reshape(-1)[0])
        dt = -1.0 / self.rsde.N
        kap, g = sp.drift_coef(tt), sp.g(tt)
        score = self.score_fn(x, t, y)
        return self._step(x, y, score, 1.0 - kap * dt, kap * dt, -g * g * dt, g * math.sqrt(-dt))


@PredictorRegistry.register("reverse_diffusion")
class ReverseDiffusionPredictor(Predictor):
    def update_fn(self, x, t, y, stepsize):
        """rev_f = f - G^2 score, x_mean = x - rev_f, x = x_mean + G z (predictors.py:75-80)."""
        sp = self.sde.spec()
        tt = float(t.reshape(-1)[0])
        st = float(stepsize)
        kap = sp.drift_coef(tt)
        G = sp.g(tt) * math.sqrt(st)
        score = self.score_fn(x, t, y)
        return self._step(x, y, score, 1.0 + kap * st, -kap * st, G * G, G)


@PredictorRegistry.register("none")
class NonePredictor(Predictor):
    def __init__(self, *args, **kwargs):
        pass

    def update_fn(self, x, t, *args):
        return x, x

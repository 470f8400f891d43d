"""Samplers — reference API (sgmse/sampling/__init__.py:28-91).

get_pc_sampler returns a closure that runs the predictor-corrector loop of the reference
(prior, linspace(T, eps, N), corrector then predictor per step, return the last x_mean and
the NFE count).  When score_fn is a ScoreModel whose score is the HIP NCSN++ network, each
NFE is fused with its SDE update (snrse_score_update); any other score_fn is evaluated as a
plain callable and the update runs on snrse_sde_update.  Noise: in-kernel Philox seeded from
torch's default generator (so torch.manual_seed reproduces a run on the same device), or an
explicit `noise_tape(i) -> complex tensor` for bit-level parity runs.
"""
import torch

from snrse import sampler as _s

from .correctors import Corrector, CorrectorRegistry
from .predictors import Predictor, PredictorRegistry, ReverseDiffusionPredictor

__all__ = ["PredictorRegistry", "CorrectorRegistry", "Predictor", "Corrector", "get_pc_sampler",
           "get_ode_sampler", "timesteps_space", "ReverseDiffusionPredictor"]


def timesteps_space(sdeT, sdeN, eps, device, type="linear"):
    """linspace(T, eps, N) (sampling/__init__.py:84-91); other types are not used by the reference."""
    return torch.linspace(sdeT, eps, sdeN, device=device)


def get_pc_sampler(predictor_name, corrector_name, sde, score_fn, Y, Y_prior=None, denoise=True, eps=3e-2,
                   snr=0.1, corrector_steps=1, probability_flow: bool = False, intermediate=False,
                   timestep_type=None, noise_tape=None, seed=None, **kwargs):
    PredictorRegistry.get_by_name(predictor_name)  # ValueError on unknown names, as the reference
    CorrectorRegistry.get_by_name(corrector_name)
    if intermediate:
        raise NotImplementedError("intermediate=True refers to an undefined sampler in the reference "
                                  "(sampling/__init__.py:77-78)")

    def pc_sampler(Y_prior=Y_prior, timestep_type=timestep_type):
        with torch.no_grad():
            if not Y.is_cuda:
                raise RuntimeError("pc_sampler: HIP device tensors required (no CPU fallback)")
            B = Y.shape[0]
            Yc = Y.to(torch.complex64).reshape(B, Y.shape[-2], Y.shape[-1]).contiguous()
            Yp = None if Y_prior is None else Y_prior.to(torch.complex64).reshape(Yc.shape).contiguous()
            sd = seed if seed is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
            src = _s.NoiseSource(seed=sd, tape=noise_tape)
            fused = getattr(score_fn, "fused_score_step", None)
            if fused is not None:
                step = fused(Yc)
            else:
                from snrse import ops

                def step(x, tv, coef, z, sd_, off):
                    sc = score_fn(x[:, None], tv, Yc[:, None]).reshape(x.shape).to(torch.complex64).contiguous()
                    return ops.sde_update(x, coef, y=Yc, score=sc, noise=z, seed=sd_, offset=off)

            def score_tensor(x, tv):
                return score_fn(x[:, None], tv, Yc[:, None]).reshape(x.shape).to(torch.complex64).contiguous()

            x, ns = _s.pc_sample(step, Yc, sde.spec(), N=sde.N, eps=eps, snr=snr, predictor=predictor_name,
                                 corrector=corrector_name, corrector_steps=corrector_steps, noise=src,
                                 denoise=denoise, score_tensor=score_tensor, Y_prior=Yp,
                                 probability_flow=probability_flow)
            return x[:, None], ns

    return pc_sampler


def get_ode_sampler(sde, score_fn, y, Y_prior=None, inverse_scaler=None, denoise=True, rtol=1e-5, atol=1e-5,
                    timestep_type=None, method="RK45", eps=3e-2, device="cuda", **kwargs):
    """Probability-flow ODE sampler (sampling/__init__.py:95-171): prior sample at T, integrate
    dx/dt = f(x, t, y) - 1/2 g(t)^2 score(x, t, y) from T down to eps with adaptive RK45, then
    (denoise) one noise-free ReverseDiffusion step at eps with stepsize 0.03.  Returns
    (x complex64 shaped like y, nfev).  The integrator is `snrse.ode.rk45_solve` -- scipy's RK45
    restated on the device state (no host round trip of the spectrogram per evaluation); the
    score is whatever `score_fn` runs (the HIP NCSN++ for a ScoreModel).  Extra kwargs are
    accepted and ignored (scipy warns about them and ignores them too)."""
    from snrse.ode import rk45_solve

    if method != "RK45":
        raise NotImplementedError(f"ODE method {method!r}: only RK45 (the reference default) is built")
    predictor = ReverseDiffusionPredictor(sde, score_fn, probability_flow=False)
    rsde = sde.reverse(score_fn, probability_flow=True)
    T = float(sde.T)

    def ode_sampler(z=None, Y_prior=Y_prior, **kw):
        with torch.no_grad():
            yp = y if Y_prior is None else Y_prior
            if not y.is_cuda:
                raise RuntimeError("ode_sampler: HIP device tensors required (no CPU fallback)")
            xt, _ = sde.prior_sampling(yp.shape, yp)
            x0 = xt.to(yp.device)
            B = y.shape[0]

            def drift(t, xs):
                xc = xs.reshape(y.shape).to(torch.complex64)
                vec_t = torch.ones(B, device=xc.device) * t
                return rsde.sde(xc, vec_t, y)[0]

            res = rk45_solve(drift, T, eps, x0, rtol=rtol, atol=atol)
            x = res.y.reshape(y.shape).to(torch.complex64)
            if denoise:
                vec_eps = torch.ones(B, device=x.device) * eps
                _, x = predictor.update_fn(x, vec_eps, y, 0.03)
            if inverse_scaler is not None:
                x = inverse_scaler(x)
            return x, res.nfev

    return ode_sampler

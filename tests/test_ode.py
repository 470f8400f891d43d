"""Probability-flow ODE sampler (sampling/__init__.py:95-171).

CPU: snrse.ode.rk45_solve (scipy's RK45 restated on device tensors) against
scipy.integrate.solve_ivp itself -- same nfev, same accepted/rejected step sequence, same
solution -- on complex probability-flow-shaped ODEs and a stiff-ish real one.  Parity anchor:
the reference pins scipy 1.8.0 (requirements.txt); the installed scipy (1.15) differs only in
clipping the initial step to the interval, which `clip_initial` reproduces and which does not
bind in the 1.8.0-mode cases below (asserted).

GPU: get_ode_sampler with the HIP NCSN++ score against the reference's own loop shape
(scipy RK45 over host numpy copies, calling the same score), same prior sample.
"""
import math

import numpy as np
import pytest
import torch
from scipy import integrate

from snrse.ode import rk45_solve, select_initial_step


def _pf_problem(n=96, seed=0):
    """dx/dt = theta (y - x) - 1/2 g(t)^2 s(x, t), OUVE g, Gaussian score s = -(x - y)/std(t)^2."""
    rng = np.random.default_rng(seed)
    y = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 0.5
    x0 = y + 0.5 * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / math.sqrt(2)
    theta, smin, smax = 1.5, 0.05, 0.5
    lg = math.log(smax / smin)

    def g(t):
        return smin * (smax / smin) ** t * math.sqrt(2 * lg)

    def std(t):
        return math.sqrt(smin ** 2 * (math.exp(2 * t * lg) - math.exp(-2 * theta * t)) * lg / (theta + lg))

    def f_np(t, x):
        return theta * (y - x) - 0.5 * g(t) ** 2 * (-(x - y) / std(t) ** 2)

    yt = torch.from_numpy(y)

    def f_t(t, x):
        return theta * (yt - x) - 0.5 * g(t) ** 2 * (-(x - yt) / std(t) ** 2)

    return x0, f_np, f_t


@pytest.mark.parametrize("rtol,atol", [(1e-5, 1e-5), (1e-3, 1e-3), (1e-7, 1e-9)])
def test_rk45_matches_scipy_complex(rtol, atol):
    x0, f_np, f_t = _pf_problem()
    T, eps = 1.0, 0.03
    ref = integrate.solve_ivp(f_np, (T, eps), x0.astype(np.complex64), rtol=rtol, atol=atol, method="RK45")
    assert ref.status == 0
    # the 1.8.0-mode initial step equals 1.15's clipped one here
    y0 = torch.from_numpy(x0.astype(np.complex64)).to(torch.complex128)
    f0 = f_t(T, y0)
    h_18 = select_initial_step(lambda t, y: f_t(t, y), T, y0, f0, -1.0, rtol, atol)
    h_15 = select_initial_step(lambda t, y: f_t(t, y), T, y0, f0, -1.0, rtol, atol, t_bound=eps, clip_initial=True)
    assert h_18 == h_15
    res = rk45_solve(f_t, T, eps, torch.from_numpy(x0.astype(np.complex64)), rtol=rtol, atol=atol)
    assert res.status == 0 and res.t == eps
    assert res.nfev == ref.nfev
    assert res.nfev == 2 + 6 * (res.n_accepted + res.n_rejected)
    np.testing.assert_allclose(res.y.numpy(), ref.y[:, -1], rtol=1e-10, atol=1e-12)


def test_rk45_rejections_match_scipy():
    """Stiff-ish real ODE (step rejections happen) with the 1.15 initial-step clip."""
    lam = 60.0

    def f_np(t, y):
        return -lam * (y - np.cos(3 * t)) + 0.1 * y ** 2

    def f_t(t, y):
        return -lam * (y - math.cos(3 * t)) + 0.1 * y ** 2

    y0 = np.array([2.0, -1.0, 0.5])
    ref = integrate.solve_ivp(f_np, (0.0, 0.7), y0, rtol=1e-6, atol=1e-8, method="RK45")
    res = rk45_solve(f_t, 0.0, 0.7, torch.from_numpy(y0), rtol=1e-6, atol=1e-8, clip_initial=True)
    assert res.n_rejected > 0
    assert res.nfev == ref.nfev
    np.testing.assert_allclose(res.y.numpy(), ref.y[:, -1], rtol=1e-9, atol=1e-12)


def test_rk45_edge_cases():
    # no integration interval: finished at once.  scipy 1.15 evaluates only f(t0); 1.8.0 (the
    # reference's pin) also runs the initial-step probe
    y0 = torch.ones(4, dtype=torch.complex64)
    ref = integrate.solve_ivp(lambda t, y: -y, (0.5, 0.5), y0.numpy(), method="RK45")
    res = rk45_solve(lambda t, y: -y, 0.5, 0.5, y0, clip_initial=True)
    assert res.status == 0 and torch.equal(res.y, y0.to(torch.complex128))
    assert res.nfev == ref.nfev == 1
    assert rk45_solve(lambda t, y: -y, 0.5, 0.5, y0).nfev == 2
    with pytest.raises(ValueError):
        rk45_solve(lambda t, y: -y, 0.0, 1.0, y0, rtol=0.0)


@pytest.mark.gpu
def test_ode_sampler_hip_vs_scipy_loop():
    from test_gpu_dropin import score_model
    from conftest import fnormal

    from sgmse import sampling

    dev = torch.device("cuda")
    m = score_model("bbed", dtype="fp32")
    sde = m.sde.copy()
    Y = (torch.from_numpy(fnormal("ode.y", (1, 1, 256, 64), True)) * 0.3).to(dev)
    rtol = atol = 1e-3

    torch.manual_seed(7)
    sampler = sampling.get_ode_sampler(sde, m, Y, rtol=rtol, atol=atol, eps=0.03, denoise=False)
    x_hip, nfe_hip = sampler()

    # the reference's loop (sampling/__init__.py:130-164): scipy RK45 over host numpy copies
    torch.manual_seed(7)
    xt, _ = sde.prior_sampling(Y.shape, Y)
    rsde = sde.reverse(m, probability_flow=True)

    def ode_func(t, x):
        xx = torch.from_numpy(x.reshape(Y.shape)).to(dev).type(torch.complex64)
        vec_t = torch.ones(Y.shape[0], device=dev) * t
        return rsde.sde(xx, vec_t, Y)[0].detach().cpu().numpy().reshape(-1)

    sol = integrate.solve_ivp(ode_func, (sde.T, 0.03), xt.detach().cpu().numpy().reshape(-1), rtol=rtol, atol=atol,
                              method="RK45")
    x_ref = torch.tensor(sol.y[:, -1]).reshape(Y.shape).type(torch.complex64)
    assert nfe_hip == sol.nfev, (nfe_hip, sol.nfev)
    err = float((x_hip.cpu() - x_ref).abs().pow(2).mean().sqrt() / x_ref.abs().pow(2).mean().sqrt())
    assert err < 1e-5, err
    # denoise step on top: one noise-free reverse-diffusion update, finite, same shape
    torch.manual_seed(7)
    x_dn, _ = sampling.get_ode_sampler(sde, m, Y, rtol=rtol, atol=atol, eps=0.03)()
    assert x_dn.shape == Y.shape and torch.isfinite(torch.view_as_real(x_dn)).all()


@pytest.mark.gpu
def test_enhance_ode_branch():
    """ScoreModel.enhance(sampler_type='ode') (model.py:762-763): the eval.py kwargs (atol, rtol,
    timestep_type, correct_stepsize) flow through to the device RK45; output is a finite waveform
    of the input length."""
    from test_gpu_dropin import score_model

    m = score_model("bbed", dtype="fp32")
    L = 9000
    y = (0.1 * torch.sin(torch.arange(L) * 0.05) + 0.01 * torch.randn(L, generator=torch.Generator().manual_seed(1)))
    x_hat = m.enhance(y[None], y[None], sampler_type="ode", N=30, atol=1e-3, rtol=1e-3, timestep_type="linear",
                      correct_stepsize=False)
    assert x_hat.shape == (L,) and np.isfinite(x_hat).all()

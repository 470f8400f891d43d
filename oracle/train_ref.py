"""CPU oracle (TEST INFRASTRUCTURE ONLY) — the consistency-training loss of ScoreModel._step for the
SNR-aligned sebridge_v3 model and its gradients, fp32 torch on the CPU.

Restates:
  grid t_n, t_{n+1} (Karras rho = 7 on N = 30, eps 1e-3)   model.py:298-302 / 366-370
  mu_t, 'true':  H(H^-1(x) (1 - t) + H^-1(y) t)              model.py:372-376
  mu_t, 'fixed': H(x0 + (H^-1(y) - x0) fixed_snr t)          model.py:304-312
  x_t = mu_t + t sigma_max z                                  model.py:313-314 / 377-378
  preconditioned forward c_skip x + c_out F(x, y, t)          model.py:536-541 (sigma_data 0.5, eps 1e-3)
  loss 'mse' / 'sqrt_mse' = mean_b 0.5 sum |f(t_n+1) - f(t_n)|^2    model.py:315-326 / 379-390
on the NCSN++ restatement oracle.ncsnpp_ref.ncsnpp_forward (H = the exponent spectrogram transform,
data_module.py:241-267); torch autograd differentiates it w.r.t. every trainable parameter (all but the
frozen GaussianFourierProjection W).  Pinned by tests/golden/train_step.npz, which tools/gen_golden.py
computes from the reference's own NCSNpp module (tests/test_oracle_golden.py::test_train_step).
Used by tests/ and by bench.py's --config train cpu_baseline leg only.
"""
from __future__ import annotations

import torch

from . import ncsnpp_ref

SIGMA_MAX, N_GRID, RHO, EPS_T, T_END = 0.5, 30, 7, 0.001, 1.0
SIGMA_DATA, EPS_PRE = 0.5, 0.001
SPEC_FACTOR, SPEC_EXP = 0.15, 0.5
FROZEN = ("all_modules.0.W",)


def grid_t(n):
    """t_n of the consistency grid for integer grid indices n (model.py:298-302)."""
    n = torch.as_tensor(n, dtype=torch.float64)
    a, b = EPS_T ** (1 / RHO), T_END ** (1 / RHO)
    return (a + ((n - 1) / (N_GRID - 1)) * (b - a)) ** RHO


def spec_fwd(s):
    return s.abs() ** SPEC_EXP * torch.exp(1j * s.angle()) * SPEC_FACTOR


def spec_back(s):
    s = s / SPEC_FACTOR
    return s.abs() ** (1.0 / SPEC_EXP) * torch.exp(1j * s.angle())


def precond_forward(sd, xx, t, yy):
    """ScoreModel.forward for sebridge_v3 (model.py:536-541): t [B, 1, 1, 1]."""
    c_skip = SIGMA_DATA ** 2 / ((t - EPS_PRE) ** 2 + SIGMA_DATA ** 2)
    c_out = (SIGMA_DATA * (t - EPS_PRE)) / ((SIGMA_DATA ** 2 + t ** 2) ** 0.5)
    return c_skip * xx + c_out * ncsnpp_ref.ncsnpp_forward(torch.cat([xx, yy], 1), t.reshape(-1), sd)


def consistency_loss(sd, x, y, z, n, branch="true", loss_type="mse", fixed_snr=0.17783):
    """x, y, z complex64 [B, 1, F, T] (clean, noisy, unit normal draw); n [B] grid indices in 1..29."""
    B = x.shape[0]
    t_n = grid_t(n).float().reshape(B, 1, 1, 1)
    t_n1 = grid_t(torch.as_tensor(n) + 1).float().reshape(B, 1, 1, 1)
    if branch == "true":
        xb, yb = spec_back(x), spec_back(y)
        mu_n, mu_n1 = (spec_fwd(xb * (1 - tt) + yb * tt) for tt in (t_n, t_n1))
    elif branch == "fixed":
        x0 = spec_back(x)
        d = (spec_back(y) - x0) * fixed_snr
        mu_n, mu_n1 = (spec_fwd(x0 + d * tt) for tt in (t_n, t_n1))
    else:
        raise ValueError(branch)
    zz = z * SIGMA_MAX
    f1 = precond_forward(sd, mu_n1 + t_n1 * zz, t_n1, mu_n1)
    f0 = precond_forward(sd, mu_n + t_n * zz, t_n, mu_n)
    if loss_type == "mse":
        err = f1 - f0
    elif loss_type == "sqrt_mse":
        sq = lambda f: f.abs() ** 0.5 * torch.exp(1j * f.angle())  # noqa: E731
        err = sq(f1) - sq(f0)
    else:
        raise ValueError(loss_type)
    losses = torch.square(err.abs())
    return torch.mean(0.5 * torch.sum(losses.reshape(B, -1), dim=-1))


def loss_and_grads(sd, x, y, z, n, branch="true", loss_type="mse", fixed_snr=0.17783):
    """(loss, {name: grad}) for every trainable tensor of the torch state dict `sd` (modified in place:
    requires_grad set, grads cleared)."""
    names = [k for k in sd if k not in FROZEN]
    for k, v in sd.items():
        v.requires_grad_(k not in FROZEN)
        v.grad = None
    loss = consistency_loss(sd, x, y, z, n, branch, loss_type, fixed_snr)
    loss.backward()
    return loss.detach(), {k: sd[k].grad for k in names}

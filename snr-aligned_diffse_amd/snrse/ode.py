"""Device-resident Dormand-Prince RK45 for the probability-flow ODE sampler.

The reference integrates the probability-flow ODE with `scipy.integrate.solve_ivp(...,
method='RK45')` on host numpy copies of the state (sgmse/sampling/__init__.py:95-171; scipy
pinned to 1.8.0 in requirements.txt).  Here the same algorithm runs on the device tensors: the
state stays complex128 in HBM (scipy promotes the complex64 state to complex128), every stage
combination is a device op, and only the scalar error norm of each attempted step crosses to
the host (step acceptance).  Restated from scipy 1.8.0's `RungeKutta` / `RK45`:

* tableau: Dormand-Prince 5(4), FSAL (`RK45.A/B/C/E`), error estimator order 4, error exponent
  -1/5, SAFETY 0.9, MIN_FACTOR 0.2, MAX_FACTOR 10;
* initial step (`common.select_initial_step`, Hairer-Norsett-Wanner II.4):
  h0 = 0.01 d0/d1 (1e-6 when d0 or d1 < 1e-5), h1 = (0.01/max(d1, d2))^(1/5) (max(1e-6,
  1e-3 h0) when both <= 1e-15), h = min(100 h0, h1); scipy >= 1.12 also clips h0 and h to the
  interval length and max_step (`clip_initial=True` reproduces that);
* step (`RungeKutta._step_impl`): min_step = 10 ulp(t); clip to t_bound; error norm
  = RMS(|h K^T E| / (atol + rtol max(|y|, |y_new|))); accept when < 1;
* `rk_step`: 5 stage evaluations + f(t+h, y_new) (FSAL) per attempted step, so
  nfev = 2 + 6 x attempts, as `solve_ivp(...).nfev` counts.

Test infrastructure checks it against scipy itself (tests/test_ode.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable

import numpy as np
import torch

# Dormand-Prince 5(4) (scipy RK45.A / B / C / E)
_A = [
    [],
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
]
_B = [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84]
_C = [0.0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0]
_E = [-71 / 57600, 0.0, 71 / 16695, -71 / 1920, 17253 / 339200, -22 / 525, 1 / 40]
_ORDER = 4  # error estimator order
_EXP = -1.0 / (_ORDER + 1)
SAFETY, MIN_FACTOR, MAX_FACTOR = 0.9, 0.2, 10.0


@dataclass
class OdeResult:
    y: torch.Tensor      # final state (the dtype the solver worked in)
    t: float
    nfev: int
    status: int          # 0 reached t_bound, -1 step size fell below 10 ulp(t)
    message: str
    n_accepted: int
    n_rejected: int


def _rms(x: torch.Tensor) -> float:
    """np.linalg.norm(x) / sqrt(x.size) (scipy common.norm), complex-aware, one host sync."""
    return math.sqrt(float(x.abs().double().pow(2).sum()) / x.numel())


def _lincomb(ks, coefs):
    """sum_i coefs[i] * ks[i], in stage order (the order of numpy's dot over K[:s])."""
    acc = None
    for k, c in zip(ks, coefs):
        if c == 0.0:
            continue
        acc = k * c if acc is None else acc + k * c
    return acc if acc is not None else torch.zeros_like(ks[0])


def select_initial_step(fun, t0, y0, f0, direction, rtol, atol, t_bound=None, max_step=math.inf,
                        clip_initial=False):
    scale = atol + y0.abs() * rtol
    d0 = _rms(y0 / scale)
    d1 = _rms(f0 / scale)
    h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    interval = abs(t_bound - t0) if t_bound is not None else math.inf
    if clip_initial:
        if interval == 0.0:
            return 0.0
        h0 = min(h0, interval)
    y1 = y0 + (h0 * direction) * f0
    f1 = fun(t0 + h0 * direction, y1)
    d2 = _rms((f1 - f0) / scale) / h0
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = max(1e-6, h0 * 1e-3)
    else:
        h1 = (0.01 / max(d1, d2)) ** (1 / (_ORDER + 1))
    if clip_initial:
        return min(100 * h0, h1, interval, max_step)
    return min(100 * h0, h1)


def rk45_solve(fun: Callable[[float, torch.Tensor], torch.Tensor], t0: float, t_bound: float, y0: torch.Tensor,
               rtol: float = 1e-3, atol: float = 1e-6, max_step: float = math.inf, first_step=None,
               clip_initial: bool = False) -> OdeResult:
    """solve_ivp(fun, (t0, t_bound), y0, method='RK45') on device tensors; returns the final state.

    `fun(t, y)` receives a python float and a tensor shaped like y0 (the solver's dtype) and
    returns dy/dt of the same shape (any float/complex dtype: it is promoted like scipy does)."""
    if not (rtol > 0 and atol >= 0):
        raise ValueError("rtol must be > 0 and atol >= 0")
    if rtol < 100 * np.finfo(float).eps:
        rtol = 100 * np.finfo(float).eps  # scipy validate_tol
    dtype = torch.complex128 if y0.is_complex() else torch.float64
    y = y0.to(dtype)
    nfev = 0

    def f_eval(t, yy):
        nonlocal nfev
        nfev += 1
        return fun(float(t), yy).to(dtype)

    t = float(t0)
    direction = float(np.sign(t_bound - t0)) if t_bound != t0 else 1.0
    f = f_eval(t, y)
    if first_step is None:
        h_abs = select_initial_step(f_eval, t, y, f, direction, rtol, atol, t_bound, max_step, clip_initial)
    else:
        h_abs = float(first_step)
    n_acc = n_rej = 0
    status, message = None, ""
    if y.numel() == 0 or t == t_bound:
        status = 0
    while status is None:
        min_step = 10 * abs(np.nextafter(t, direction * np.inf) - t)
        h_abs = max_step if h_abs > max_step else (min_step if h_abs < min_step else h_abs)
        accepted = rejected = False
        while not accepted:
            if h_abs < min_step:
                status, message = -1, "Required step size is less than spacing between numbers."
                break
            h = h_abs * direction
            t_new = t + h
            if direction * (t_new - t_bound) > 0:
                t_new = t_bound
            h = t_new - t
            h_abs = abs(h)
            K = [f]
            for s in range(1, 6):
                K.append(f_eval(t + _C[s] * h, y + _lincomb(K, _A[s]) * h))
            y_new = y + h * _lincomb(K, _B)
            f_new = f_eval(t + h, y_new)
            K.append(f_new)
            scale = atol + torch.maximum(y.abs(), y_new.abs()) * rtol
            err = _rms(_lincomb(K, _E) * h / scale)
            if err < 1:
                factor = MAX_FACTOR if err == 0 else min(MAX_FACTOR, SAFETY * err ** _EXP)
                if rejected:
                    factor = min(1.0, factor)
                h_abs *= factor
                accepted = True
                n_acc += 1
            else:
                h_abs *= max(MIN_FACTOR, SAFETY * err ** _EXP)
                rejected = True
                n_rej += 1
        if status is not None:
            break
        t, y, f = t_new, y_new, f_new
        if direction * (t - t_bound) >= 0:
            status = 0
    return OdeResult(y=y, t=t, nfev=nfev, status=status, message=message or "The solver successfully reached "
                     "the end of the integration interval.", n_accepted=n_acc, n_rejected=n_rej)

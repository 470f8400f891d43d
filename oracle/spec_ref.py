"""CPU oracle (TEST INFRASTRUCTURE ONLY) — STFT front end and iSTFT back end, numpy fp64.

Restates the reference's spectrogram glue:
  get_window('hann')                   data_module.py:13-19 (periodic Hann, 510)
  SpecsDataModule.stft / istft         data_module.py:269-297 (n_fft 510, hop 128, center=True,
                                       reflect pad, onesided) -> torch.stft / torch.istft
  spec_fwd / spec_back ('exponent')    data_module.py:241-267 (e = 0.5, factor 0.15)
  pad_spec / pad_spec_16               util/other.py:83-99
torch.stft/istft's published algorithm (torch==1.10.2 pinned by requirements.txt):
frames of the reflect-padded signal times the window, real DFT keeping bins 0..n_fft/2;
the inverse is a C2R inverse DFT (imaginary parts of DC / Nyquist dropped), windowed
overlap-add divided by the summed squared window, trimmed by n_fft/2 and to `length`.
"""
from __future__ import annotations

import numpy as np

N_FFT = 510
HOP = 128
F_BINS = N_FFT // 2 + 1  # 256
SPEC_FACTOR = 0.15
SPEC_EXP = 0.5


def hann(n=N_FFT):
    i = np.arange(n)
    return 0.5 - 0.5 * np.cos(2 * np.pi * i / n)  # periodic


def n_frames(length):
    return 1 + length // HOP


def stft(sig: np.ndarray) -> np.ndarray:
    """sig [B, L] real -> complex [B, 256, 1 + L//128]."""
    sig = np.atleast_2d(np.asarray(sig, dtype=np.float64))
    B, L = sig.shape
    pad = N_FFT // 2
    xp = np.pad(sig, ((0, 0), (pad, pad)), mode="reflect")
    T = n_frames(L)
    idx = np.arange(T)[:, None] * HOP + np.arange(N_FFT)[None, :]
    frames = xp[:, idx] * hann()[None, None, :]  # [B, T, n_fft]
    k = np.arange(F_BINS)
    n = np.arange(N_FFT)
    basis = np.exp(-2j * np.pi * np.outer(n, k) / N_FFT)  # [n_fft, F]
    return np.einsum("btn,nf->bft", frames, basis)


def istft(spec: np.ndarray, length: int) -> np.ndarray:
    """spec complex [B, 256, T] -> real [B, length]."""
    spec = np.asarray(spec, dtype=np.complex128)
    if spec.ndim == 2:
        spec = spec[None]
    B, F, T = spec.shape
    n = np.arange(N_FFT)
    k = np.arange(F)
    w_k = np.full(F, 2.0)
    w_k[0] = 1.0
    w_k[-1] = 1.0  # Nyquist bin (n_fft even)
    re = spec.real.copy()
    im = spec.imag.copy()
    im[:, 0, :] = 0.0
    im[:, -1, :] = 0.0
    ang = 2 * np.pi * np.outer(k, n) / N_FFT  # [F, n]
    frames = (np.einsum("bft,fn->btn", re * w_k[None, :, None], np.cos(ang))
              - np.einsum("bft,fn->btn", im * w_k[None, :, None], np.sin(ang))) / N_FFT
    win = hann()
    frames *= win[None, None, :]
    total = N_FFT + HOP * (T - 1)
    y = np.zeros((B, total))
    env = np.zeros(total)
    for f in range(T):
        y[:, f * HOP:f * HOP + N_FFT] += frames[:, f]
        env[f * HOP:f * HOP + N_FFT] += win ** 2
    start = N_FFT // 2
    y = y[:, start:start + length]
    env = env[start:start + length]
    out = np.zeros_like(y)
    ok = env > 1e-11
    out[:, ok] = y[:, ok] / env[ok]
    if out.shape[1] < length:  # torch.istft zero-pads to `length`
        out = np.pad(out, ((0, 0), (0, length - out.shape[1])))
    return out


def spec_fwd(spec):
    a = np.abs(spec)
    return a ** SPEC_EXP * np.exp(1j * np.angle(spec)) * SPEC_FACTOR


def spec_back(spec):
    spec = spec / SPEC_FACTOR
    return np.abs(spec) ** (1.0 / SPEC_EXP) * np.exp(1j * np.angle(spec))


def pad_spec(Y, mult=64):
    T = Y.shape[-1]
    n = (mult - T % mult) if T % mult else 0
    pad = [(0, 0)] * (Y.ndim - 1) + [(0, n)]
    return np.pad(Y, pad)


def specs_item(x: np.ndarray, y: np.ndarray, num_frames: int = 256, normalize: str = "noisy", fixed_snr: float = 1.0,
               start: int | None = None):
    """Specs.__getitem__ (data_module.py:47-84) on decoded mono clips x, y [L]: mix, crop at
    `start` (the centred start when None) or zero-pad (pad//2 left), normalise, STFT, spec_fwd.
    -> (X, Y) complex [256, num_frames]."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    y = x + (y - x) * fixed_snr
    target = (num_frames - 1) * HOP
    cur = x.shape[-1]
    pad = max(target - cur, 0)
    if pad == 0:
        s = int((cur - target) / 2) if start is None else start
        x, y = x[s:s + target], y[s:s + target]
    else:
        x = np.pad(x, (pad // 2, pad // 2 + pad % 2))
        y = np.pad(y, (pad // 2, pad // 2 + pad % 2))
    nf = {"noisy": np.abs(y).max(), "clean": np.abs(x).max(), "not": 1.0}[normalize]
    return spec_fwd(stft((x / nf)[None])[0]), spec_fwd(stft((y / nf)[None])[0])

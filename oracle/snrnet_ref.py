"""CPU oracle (TEST INFRASTRUCTURE ONLY) — SNR estimator, functional torch.

Restates SNRNet.forward (snrnet.py:47-97) over a plain state_dict, with the bidirectional
LSTM written out cell by cell (torch.nn.LSTM gate order i, f, g, o; one layer, hidden 128,
batch_first), and the SNR->t / normalisation glue of ScoreModel.enhance:
  calculate_snr_direct     model.py:627-629
  calculate_normfac_direct model.py:631-634
  t_30 grid                model.py:22-23
  t snapping               model.py:810-817
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

T_30 = (0.001 ** (1 / 7) + (np.arange(1, 31) - 1) / 29 * (1 - 0.001 ** (1 / 7))) ** 7


def _lstm_dir(x, sd, suffix, reverse):
    Wih, Whh = sd["blstm.weight_ih_l0" + suffix], sd["blstm.weight_hh_l0" + suffix]
    b = sd["blstm.bias_ih_l0" + suffix] + sd["blstm.bias_hh_l0" + suffix]
    B, S, _ = x.shape
    H = Whh.shape[1]
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    out = [None] * S
    order = range(S - 1, -1, -1) if reverse else range(S)
    for s in order:
        g = x[:, s] @ Wih.T + h @ Whh.T + b
        i, f, gg, o = g.split(H, dim=1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        out[s] = h
    return torch.stack(out, dim=1)


def snrnet_forward(x: torch.Tensor, sd: dict) -> torch.Tensor:
    """x [B, 2, 256, T] (T multiple of 16) -> [B, 1] in (0, 1)."""
    B, _, Fq, T = x.shape
    nclu = T // 16
    xs = x.permute(0, 3, 1, 2).reshape(-1, 16, 2, Fq).permute(0, 2, 3, 1)  # [B*T/16, 2, 256, 16]
    f = F.conv2d(xs, sd["conv5x5_1.weight"], sd["conv5x5_1.bias"], padding=2)
    f = F.max_pool2d(f, 2)
    f = F.conv2d(f, sd["conv3x3_1.weight"], sd["conv3x3_1.bias"], padding=1)
    f = F.max_pool2d(f, (2, 1))
    feats = []
    for i, pool in ((1, 8), (2, 7), (3, 5), (4, 1)):
        g = F.conv2d(f, sd[f"convt_{i}.weight"], sd[f"convt_{i}.bias"])
        feats.append(F.max_pool2d(g, (1, pool)))
    f = torch.cat(feats, 1).squeeze(3).squeeze(2).reshape(B, nclu, -1)
    fw = _lstm_dir(f, sd, "", False)
    bw = _lstm_dir(f, sd, "_reverse", True)
    h = torch.cat([fw, bw], dim=2)
    stats = torch.cat([h.mean(1), h.std(1), h.min(1).values, h.max(1).values], dim=1)
    return torch.sigmoid(F.linear(stats, sd["fc.weight"], sd["fc.bias"]))


def snap_t(est_snr: float, fixed_snr: float) -> float:
    t = est_snr / (10 ** 0.25 * fixed_snr)
    return float(T_30[np.abs(T_30 - t).argmin()])


def normfac(t_hat: float, fixed_snr: float) -> float:
    s = 10 ** 0.25 * fixed_snr * t_hat
    return 2.040166 * (0.240253 + 0.759747 * fixed_snr ** 2) ** 0.5 / ((1 + s ** 2) ** 0.5)

"""Spectrogram padding helpers and the SI-SDR / SNR metrics (reference util/other.py:71-99)."""
import numpy as np
import torch


def pad_spec(Y, mult=64):
    """Zero-pad the last (frame) axis to a multiple of 64 (the U-Net down-samples 2^6x)."""
    T = Y.size(3)
    n = (mult - T % mult) % mult
    return torch.nn.functional.pad(Y, (0, n, 0, 0)) if n else Y


def pad_spec_16(Y):
    return pad_spec(Y, 16)


def si_sdr(s, s_hat):
    alpha = np.dot(s_hat, s) / np.linalg.norm(s) ** 2
    return 10 * np.log10(np.linalg.norm(alpha * s) ** 2 / np.linalg.norm(alpha * s - s_hat) ** 2)


def snr_dB(s, n):
    s_power = np.sum(np.abs(s) ** 2) / len(s)
    n_power = np.sum(np.abs(n) ** 2) / len(n)
    return 10 * np.log10(s_power / n_power)


def mean_std(data):
    data = np.asarray(data, dtype=np.float64)
    data = data[~np.isnan(data)]
    return np.mean(data), np.std(data)

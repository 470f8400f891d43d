"""CPU tests of the host-side agreement logic bench.py writes into its line (paritycheck.waveform_agreement:
parity_mode.c2_agreement, bounded by paritycheck.C2_AGREE16 for the fp16 headline, C2_AGREE for bf16): per-clip SI-SDR as the reference computes it
(sgmse/util/other.py:71-75) and the distribution bounds (median, clips below 25 dB, floor, mean relative RMS; the
fp32x3-vs-exact-fp32 bounds)."""
import math

import numpy as np
import torch

import paritycheck


def _pair(n, snr_db, seed=0, L=4000):
    g = torch.Generator().manual_seed(seed)
    ref = torch.randn(n, L, generator=g, dtype=torch.float64)
    noise = torch.randn(n, L, generator=g, dtype=torch.float64)
    scale = torch.as_tensor(10 ** (-np.asarray(snr_db, dtype=np.float64) / 20))[:, None]
    noise *= (ref.norm(dim=1, keepdim=True) / noise.norm(dim=1, keepdim=True)) * scale
    return ref + noise, ref


def test_si_sdr_matches_the_reference_formula():
    est, ref = _pair(3, [10.0, 20.0, 30.0])
    r = paritycheck.waveform_agreement(est, ref, per_clip=True)
    for k in range(3):
        e, x = est[k], ref[k]
        alpha = float((e * x).sum() / (x * x).sum())
        want = 10 * math.log10(float((alpha * x).pow(2).sum() / (alpha * x - e).pow(2).sum()))
        assert abs(r["per_clip"]["si_sdr_db"][k] - want) < 0.01
    assert abs(r["si_sdr_db_median"] - 20.0) < 0.5


def test_fp16_bounds():
    """C2_AGREE16 (the default): the fp16 headline's measured distribution passes, an 11.9 dB clip (the bf16 outlier
    trajectory) or a shifted median fails."""
    snr = np.full(32, 49.7)
    snr[3] = 35.6  # the measured fp16 minimum (profiles/r06a_bench_fp16_line.json)
    est, ref = _pair(32, snr)
    assert paritycheck.waveform_agreement(est, ref)["ok"]
    snr[0] = 11.9
    est, ref = _pair(32, snr)
    assert not paritycheck.waveform_agreement(est, ref)["ok"]
    est, ref = _pair(32, np.full(32, 36.0))
    assert not paritycheck.waveform_agreement(est, ref)["ok"]


def test_bounds_accept_one_outlier_and_reject_a_shifted_distribution():
    """C2_AGREE (bf16)."""
    snr = np.full(32, 32.0)
    snr[0] = 11.9  # the measured outlier, bf16 against exact fp32 (profiles/r05f_agree3.json)
    est, ref = _pair(32, snr)
    ok = paritycheck.waveform_agreement(est, ref, bounds=paritycheck.C2_AGREE)
    assert ok["ok"] and ok["clips_below_25db"] == 1 and ok["si_sdr_db_min"] < 12.5
    # every clip 24 dB: median and clip-count bounds fail
    est, ref = _pair(32, np.full(32, 24.0))
    assert not paritycheck.waveform_agreement(est, ref, bounds=paritycheck.C2_AGREE)["ok"]
    # a second clip below 25 dB (a regression that hits more than the one known trajectory)
    snr2 = snr.copy()
    snr2[5] = 20.0
    est, ref = _pair(32, snr2)
    assert not paritycheck.waveform_agreement(est, ref, bounds=paritycheck.C2_AGREE)["ok"]
    # the outlier itself falling below the 10 dB floor
    snr3 = snr.copy()
    snr3[0] = 8.0
    est, ref = _pair(32, snr3)
    assert not paritycheck.waveform_agreement(est, ref, bounds=paritycheck.C2_AGREE)["ok"]
    # NaN output anywhere
    est, ref = _pair(32, np.full(32, 32.0))
    est[5, 7] = float("nan")
    assert not paritycheck.waveform_agreement(est, ref, bounds=paritycheck.C2_AGREE)["ok"]


def test_x3_vs_fp32_bounds():
    b = paritycheck.C2_X3_VS_FP32
    est, ref = _pair(32, np.full(32, 78.0))  # the measured floor of fp32x3 against exact fp32
    assert paritycheck.waveform_agreement(est, ref, bounds=b)["ok"]
    snr = np.full(32, 85.0)
    snr[3] = 50.0
    est, ref = _pair(32, snr)
    assert not paritycheck.waveform_agreement(est, ref, bounds=b)["ok"]

"""deep_eval.py's SNR sweep (deep_eval.py:103-163) on the HIP path: the nine SNR variants of a file
enhanced as one batch must match the reference's per-variant ScoreModel.enhance loop (B=1) on the same
injected noise, for the PC sampler (model_type 'bbed') and the SNR-aligned one-step path (sebridge_v3,
oracle SNR = noise_rms / clean_rms).  fp32, 1e-4 relative RMS per variant."""
import os

import numpy as np
import pytest
import torch

from conftest import fnormal
from test_gpu_dropin import score_model

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


def _clip(L, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(L) / 16000.0
    x = (0.2 * np.sin(2 * np.pi * 440.0 * t) * np.hanning(L)).astype(np.float32)
    y = (x + 0.05 * rng.standard_normal(L)).astype(np.float32)
    return x, y


def _tape(tag, V, T, gpu):
    def tape(i):
        return torch.from_numpy(fnormal(f"{tag}.{i}", (V, 256, T), complex_=True)).to(gpu)
    return tape


@pytest.mark.parametrize("kind", ["bbed_pc", "sebridge_v3_oracle"])
def test_snr_sweep_batched_matches_per_variant_enhance(gpu, kind):
    from snrse import deep_evaluate as de
    L = 12000
    x, y = _clip(L, 1)
    ys, noise_rms = de.snr_variants(x, y)
    T = L // 128 + 1
    T = T + (64 - T % 64) % 64
    tape = _tape(f"de.{kind}", 9, T, gpu)
    if kind == "bbed_pc":
        m = score_model("bbed", dtype="fp32")
        kw = dict(sampler_type="pc", N=2, oracle=False)
    else:
        m = score_model("sebridge_v3", "true", fixed_snr=0.17783, dtype="fp32")
        kw = dict(sampler_type="pc", N=30, oracle=True)
    xb = de.enhance_variants(m, ys, noise_rms, 1.0, batched=True, noise_tape=tape, **kw)
    xr = de.enhance_variants(m, ys, noise_rms, 1.0, batched=False, noise_tape=tape, **kw)
    assert xb.shape == xr.shape == (9, L)
    errs = [rel(xb[k], xr[k]) for k in range(9)]
    assert max(errs) < 1e-4, errs
    assert np.isfinite(xb).all()


def test_deep_evaluate_end_to_end(gpu, tmp_path):
    """The driver: nine directories of 16-bit PCM files, _results_deep.csv / _avg_results_deep.txt with
    the reference's columns, si_sdr columns (optional here, commented out in the reference) equal to the
    numpy energy ratios of the written-out waveforms' source."""
    from snrse import audio
    from snrse import deep_evaluate as de
    from test_metrics import np_energy_ratios
    root = tmp_path / "t"
    for d in ("clean", "noisy"):
        os.makedirs(root / d)
    for k in range(2):
        x, y = _clip(9000 + 2000 * k, 10 + k)
        audio.write_wav(str(root / "clean" / f"f{k}.wav"), x, bits=32)
        audio.write_wav(str(root / "noisy" / f"f{k}.wav"), y, bits=32)
    m = score_model("bbed", dtype="fp32")
    outs = []
    orig = de.enhance_variants

    def rec(*a, **kw):
        r = orig(*a, **kw)
        outs.append(r)
        return r

    de.enhance_variants = rec
    try:
        data = de.deep_evaluate(m, str(root), str(tmp_path / "o"), N=2, si_sdr=True, verbose=False)
    finally:
        de.enhance_variants = orig
    assert data["filename"] == ["f0.wav", "f1.wav"] and len(outs) == 2
    for k in range(2):
        x, _ = audio.load(str(root / "clean" / f"f{k}.wav"))
        y, _ = audio.load(str(root / "noisy" / f"f{k}.wav"))
        ys, _ = de.snr_variants(x[0].numpy(), y[0].numpy())
        for j, lab in enumerate(de.LABELS):
            xh, _ = audio.load(str(tmp_path / "o" / "{0:02d}".format(lab) / f"f{k}.wav"))
            pcm = np.clip(np.round(outs[k][j] * 32768.0), -32768, 32767) / 32768.0
            np.testing.assert_array_equal(xh[0].numpy(), pcm.astype(np.float32))
            ref = np_energy_ratios(outs[k][j], x[0].numpy(), ys[j] - x[0].numpy())
            assert abs(data[f"si_sdr_{lab}"][k] - ref[0]) < 1e-4
    head = open(tmp_path / "o" / "_results_deep.csv").read().splitlines()[0].split(",")
    assert head[:10] == ["filename"] + [f"pesq_{s}" for s in de.LABELS]
    assert len(open(tmp_path / "o" / "_avg_results_deep.txt").read().splitlines()) == 9

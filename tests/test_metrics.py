"""Metric layer: eval.py:94-170 on the HIP path.

CPU: the reference's numpy energy_ratios / si_sdr (utils.py:10-35, sgmse/util/other.py:71-75)
restated in the test against the C-ABI symbol's closed form (expansion through six dot
products), the mean ± std formatting, the table writer.  GPU: snrse_energy_ratios against the
numpy restatement (1e-9 dB on well-conditioned inputs), and the evaluate() driver end to end on a
two-file tree with a formula-weight ScoreModel (N=2): written WAVs, CSV rows, metrics re-scored
from the written files.  PESQ: the `pesq` package is absent here, so the column is NaN
(the reference's own failure value) -- PESQ parity is unverified.
"""
import os

import numpy as np
import pytest
import torch

from snrse import audio, evaluate


def np_energy_ratios(s_hat, s, n):
    """utils.py:10-35 verbatim arithmetic (numpy, float64)."""
    s_hat, s, n = (np.asarray(v, np.float64) for v in (s_hat, s, n))
    a_s = np.dot(s_hat, s) / np.linalg.norm(s) ** 2
    tgt = a_s * s
    a_n = np.dot(s_hat, n) / np.linalg.norm(n) ** 2
    noi = a_n * n
    art = s_hat - tgt - noi
    sdr = 10 * np.log10(np.linalg.norm(tgt) ** 2 / np.linalg.norm(noi + art) ** 2)
    sir = 10 * np.log10(np.linalg.norm(tgt) ** 2 / np.linalg.norm(noi) ** 2)
    sar = 10 * np.log10(np.linalg.norm(tgt) ** 2 / np.linalg.norm(art) ** 2)
    return sdr, sir, sar


def closed_form(s_hat, s, n):
    """The kernel's six-dot-product expansion, in numpy (what snrse_energy_ratios computes)."""
    h, x, z = (np.asarray(v, np.float64) for v in (s_hat, s, n))
    ss, nn, hh, hs, hn, sn = x @ x, z @ z, h @ h, h @ x, h @ z, x @ z
    a_s, a_n = hs / ss, hn / nn
    tgt, noi = a_s * a_s * ss, a_n * a_n * nn
    dist = hh - 2 * a_s * hs + a_s * a_s * ss
    art = hh + tgt + noi - 2 * a_s * hs - 2 * a_n * hn + 2 * a_s * a_n * sn
    return 10 * np.log10(tgt / dist), 10 * np.log10(tgt / noi), 10 * np.log10(tgt / art)


def _sigs(L, seed, snr_db):
    rng = np.random.default_rng(seed)
    s = np.sin(np.arange(L) * 0.01) + 0.3 * rng.standard_normal(L)
    n = rng.standard_normal(L) * 10 ** (-snr_db / 20)
    s_hat = 0.9 * s + 0.3 * n + 0.01 * rng.standard_normal(L)
    return s_hat.astype(np.float32), s.astype(np.float32), n.astype(np.float32)


@pytest.mark.parametrize("snr_db", [-5.0, 10.0, 30.0])
def test_closed_form_matches_reference_arithmetic(snr_db):
    sh, s, n = _sigs(16000, 1, snr_db)
    np.testing.assert_allclose(closed_form(sh, s, n), np_energy_ratios(sh, s, n), rtol=0, atol=1e-8)


def test_print_mean_std_and_tables(tmp_path):
    assert evaluate.print_mean_std([1.0, float("nan"), 3.0]) == "2.00 ± 1.00"
    assert evaluate.print_mean_std([1.0, 2.0], decimal=3) == "1.500 ± 0.500"
    data = {"filename": ["a.wav", "b.wav"], "pesq": [float("nan")] * 2, "si_sdr": [1.5, 2.5],
            "si_sir": [3.0, 4.0], "si_sar": [5.0, 6.0]}
    evaluate.write_tables(data, str(tmp_path))
    lines = open(tmp_path / "_results.csv").read().splitlines()
    assert lines[0] == "filename,pesq,si_sdr,si_sir,si_sar" and lines[1].startswith("a.wav,nan,1.5,")
    assert "SI-SDR: 2.00 ± 0.50" in open(tmp_path / "_avg_results.txt").read()


@pytest.mark.gpu
def test_energy_ratios_kernel_vs_numpy():
    from snrse import ops
    rows = [_sigs(64000, k, db) for k, db in enumerate([-5.0, 0.0, 12.0, 35.0])]
    sh, s, n = (torch.from_numpy(np.stack([r[i] for r in rows])).cuda() for i in range(3))
    out = ops.energy_ratios(sh, s, n).cpu().numpy()
    ref = np.array([np_energy_ratios(*r) for r in rows])
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-6)
    only = ops.energy_ratios(sh, s).cpu().numpy()
    np.testing.assert_allclose(only[:, 0], ref[:, 0], rtol=0, atol=1e-6)
    assert np.isnan(only[:, 1:]).all()
    with pytest.raises(RuntimeError):
        ops.energy_ratios(sh.cpu(), s.cpu(), n.cpu())


@pytest.mark.gpu
def test_evaluate_driver_end_to_end(tmp_path):
    from test_gpu_dropin import score_model

    root = tmp_path / "test"
    for d in ("clean", "noisy"):
        os.makedirs(root / d)
    rng = np.random.default_rng(3)
    for k in range(2):
        L = 12000 + 3000 * k
        c = (0.2 * np.sin(np.arange(L) * (0.02 + 0.01 * k))).astype(np.float32)
        y = (c + 0.05 * rng.standard_normal(L)).astype(np.float32)
        audio.write_wav(str(root / "clean" / f"f{k}.wav"), c, bits=32)
        audio.write_wav(str(root / "noisy" / f"f{k}.wav"), y, bits=32)
    m = score_model("bbed", dtype="fp32")
    outs = []
    enhance = m.enhance

    def recording_enhance(x, y, **kw):
        r = enhance(x, y, **kw)
        outs.append(r)
        return r

    m.enhance = recording_enhance
    out = tmp_path / "out"
    data = evaluate.evaluate(m, str(root), str(out), N=2)
    assert data["filename"] == ["f0.wav", "f1.wav"] and len(outs) == 2
    assert np.isnan(data["pesq"]).all() == (evaluate._pesq_fn() is None)
    for k in range(2):
        xh, _ = audio.load(str(out / "all" / f"f{k}.wav"))
        x, _ = audio.load(str(root / "clean" / f"f{k}.wav"))
        y, _ = audio.load(str(root / "noisy" / f"f{k}.wav"))
        assert xh.shape == x.shape
        # the file holds the 16-bit PCM of the enhanced float waveform (formula weights: clipped)
        pcm = np.clip(np.round(outs[k] * 32768.0), -32768, 32767) / 32768.0
        np.testing.assert_array_equal(xh[0].numpy(), pcm.astype(np.float32))
        ref = np_energy_ratios(outs[k], x[0].numpy(), (y - x)[0].numpy())
        np.testing.assert_allclose([data["si_sdr"][k], data["si_sir"][k], data["si_sar"][k]], ref, atol=1e-5)
    assert (out / "_results.csv").exists() and (out / "_avg_results.txt").exists()


def test_deep_eval_snr_variants_match_reference_arithmetic():
    """deep_eval.py:108-118 in torch float32 (the reference's tensors) vs snr_variants."""
    from snrse import deep_evaluate as de
    rng = np.random.default_rng(5)
    x = rng.standard_normal(999).astype(np.float32) * 0.1
    y = (x + rng.standard_normal(999).astype(np.float32) * 0.05).astype(np.float32)
    ys, noise_rms = de.snr_variants(x, y)
    xt, yt = torch.from_numpy(x)[None], torch.from_numpy(y)[None]
    y0 = yt - xt
    for k, S in enumerate(range(0, 41, 5)):
        ref = (xt + y0 * 10 ** (-S / 20)).numpy()[0]
        np.testing.assert_array_equal(ys[k], ref)
        assert noise_rms[k] == 10 ** ((-S + 5) / 20)
    assert de.LABELS == (-5, 0, 5, 10, 15, 20, 25, 30, 35)
    assert ["{0:02d}".format(v) for v in de.LABELS][:3] == ["-5", "00", "05"]

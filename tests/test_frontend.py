"""Audio IO + Specs batching front-end (data_module.py:22-176, 221-321).

CPU: snrse.audio.load against Python's `wave` module (PCM 8/16/24/32) and numpy (float WAV),
torchaudio.load's normalisation.  GPU: Specs / Specs_SNR items and Specs.batch against the oracle
restatement (oracle/spec_ref.specs_item) on synthetic clips written to a temporary dataset tree
(clips shorter than the crop -> zero pad, longer -> centred crop), SpecsDataModule.setup and its
DataLoaders.  Tolerance: raw fp32 STFT vs the fp64 oracle 1e-5 relative RMS; after the
|X|^0.5 transform 5e-4: the synthetic two-tone clips have sparse spectra (and the padded one
exact-zero regions) whose fp32 rounding noise the square root lifts -- an fp32 emulation of the
oracle itself lands at 1.8e-4 on them (broadband speech stays under 2e-5: test_gpu_kernels).
"""
TOL_RAW, TOL_FWD = 1e-5, 5e-4
import os
import struct
import wave

import numpy as np
import pytest
import torch

from snrse import audio


def _pcm_write(path, ints, bits, ch):
    with wave.open(path, "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(bits // 8)
        w.setframerate(16000)
        if bits == 24:
            b = np.asarray(ints, np.int32).reshape(-1)
            raw = np.stack([b & 0xff, (b >> 8) & 0xff, (b >> 16) & 0xff], 1).astype(np.uint8).tobytes()
        elif bits == 8:
            raw = (np.asarray(ints) + 128).astype(np.uint8).tobytes()
        else:
            raw = np.asarray(ints).astype(f"<i{bits // 8}").tobytes()
        w.writeframes(raw)


@pytest.mark.parametrize("bits,ch", [(16, 1), (16, 2), (24, 1), (32, 2), (8, 1)])
def test_wav_pcm_matches_wave_module(tmp_path, bits, ch):
    rng = np.random.default_rng(bits + ch)
    lim = 2 ** (bits - 1)
    ints = rng.integers(-lim, lim, size=(1001, ch))
    ints[0] = -lim
    ints[1] = lim - 1
    p = str(tmp_path / "a.wav")
    _pcm_write(p, ints, bits, ch)
    x, sr = audio.load(p)
    assert sr == 16000 and x.dtype == torch.float32 and tuple(x.shape) == (ch, 1001)
    with wave.open(p, "rb") as w:
        assert w.getnframes() == 1001 and w.getnchannels() == ch
    np.testing.assert_allclose(x.numpy(), (ints.T / lim).astype(np.float32), rtol=0, atol=0)


def test_wav_float_roundtrip_and_errors(tmp_path):
    x = np.tanh(np.random.default_rng(0).standard_normal((500, 2))).astype(np.float32) * 0.9
    p = str(tmp_path / "f.wav")
    audio.write_wav(p, x, 22050, bits=32)
    y, sr = audio.load(p)
    assert sr == 22050 and np.array_equal(y.numpy(), x.T)
    p16 = str(tmp_path / "i.wav")
    audio.write_wav(p16, x[:, 0], bits=16)
    y16, _ = audio.load(p16)
    assert np.abs(y16.numpy()[0] - x[:, 0]).max() <= 0.5 / 32768 + 1e-7
    bad = tmp_path / "bad.wav"
    bad.write_bytes(b"RIFX" + struct.pack("<I", 4) + b"WAVE")
    with pytest.raises(ValueError):
        audio.load(str(bad))


def _clip(L, seed, scale):
    rng = np.random.default_rng(seed)
    t = np.arange(L) / 16000.0
    c = 0.1 * np.sin(2 * np.pi * 440 * t) + 0.05 * np.sin(2 * np.pi * 1250 * t + seed)
    n = rng.standard_normal(L) * scale
    return c, c + n


def _tree(root, lengths):
    """<root>/{train,valid,valid2,test}/{clean,noisy}/*.wav (+ valid/active_rms.txt)."""
    clips = {}
    for sub in ("train", "valid", "valid2", "test"):
        for d in ("clean", "noisy"):
            os.makedirs(os.path.join(root, sub, d), exist_ok=True)
        rms = []
        for i, L in enumerate(lengths):
            c, y = _clip(L, i, 0.02 * (i + 1))
            name = f"p{i:03d}.wav"
            audio.write_wav(os.path.join(root, sub, "clean", name), c, bits=32)
            audio.write_wav(os.path.join(root, sub, "noisy", name), y, bits=32)
            clips[(sub, i)] = (c.astype(np.float32), y.astype(np.float32))
            rms.append(f"{name}\t{0.07 + i:.4f}\t{0.01 * (i + 1):.4f}\n")
        if sub == "valid":
            with open(os.path.join(root, sub, "active_rms.txt"), "w") as f:
                f.writelines(rms)
    return clips


def _rel(a, b):
    a = np.asarray(a, np.complex128)
    b = np.asarray(b, np.complex128)
    return float(np.sqrt(np.mean(np.abs(a - b) ** 2) / np.mean(np.abs(b) ** 2)))


@pytest.mark.gpu
@pytest.mark.parametrize("normalize,fixed_snr", [("noisy", 1.0), ("clean", 0.5), ("not", 1.0)])
def test_specs_items_and_batch_vs_oracle(tmp_path, normalize, fixed_snr):
    from oracle import spec_ref
    from sgmse.data_module import Specs, SpecsDataModule

    clips = _tree(str(tmp_path), [20000, 40000, 32640, 50001])
    dm = SpecsDataModule(base_dir=str(tmp_path))
    ds = Specs(str(tmp_path), "test", False, False, 256, normalize=normalize, spec_transform=dm.spec_fwd,
               stft_kwargs=dm.istft_kwargs, fixed_snr=fixed_snr)
    assert len(ds) == 4
    refs = [spec_ref.specs_item(*clips[("test", i)], normalize=normalize, fixed_snr=fixed_snr) for i in range(4)]
    for i in range(4):
        X, Y = ds[i]
        assert X.shape == (1, 256, 256) and X.dtype == torch.complex64 and X.is_cuda
        tol = TOL_FWD
        assert _rel(X[0].cpu(), refs[i][0]) < tol and _rel(Y[0].cpu(), refs[i][1]) < tol
    Xb, Yb = ds.batch([3, 0, 2])
    assert Xb.shape == (3, 1, 256, 256)
    for k, i in enumerate([3, 0, 2]):
        tol = TOL_FWD
        assert _rel(Xb[k, 0].cpu(), refs[i][0]) < tol and _rel(Yb[k, 0].cpu(), refs[i][1]) < tol
    # raw STFT (spec_transform=None): the un-transformed spectrogram at the fp32 STFT bound
    raw = Specs(str(tmp_path), "test", False, False, 256, normalize=normalize, spec_transform=None,
                stft_kwargs=dm.istft_kwargs, fixed_snr=fixed_snr)
    Xr, Yr = raw.batch([0, 1])
    for k in range(2):
        xr, yr = spec_ref.specs_item(*clips[("test", k)], normalize=normalize, fixed_snr=fixed_snr)
        assert _rel(Xr[k, 0].cpu(), spec_ref.spec_back(xr)) < TOL_RAW
        assert _rel(Yr[k, 0].cpu(), spec_ref.spec_back(yr)) < TOL_RAW


@pytest.mark.gpu
def test_datamodule_setup_loaders_and_specs_snr(tmp_path):
    from oracle import spec_ref
    from sgmse.data_module import SpecsDataModule

    clips = _tree(str(tmp_path), [20000, 40000, 32640, 50001])
    dm = SpecsDataModule(base_dir=str(tmp_path), batch_size=2)
    dm.setup()
    X, Y, s, n = dm.valid_set[1]
    assert abs(s - 1.07) < 1e-9 and abs(n - 0.02) < 1e-9
    ref = spec_ref.specs_item(*clips[("valid", 1)])
    assert _rel(X[0].cpu(), ref[0]) < TOL_FWD
    batches = list(dm.test_dataloader())
    assert len(batches) == 2 and batches[0][0].shape == (2, 1, 256, 256)
    np.random.seed(0)
    Xt, Yt = dm.train_set[3]  # random crop of the 50001-sample clip: same start as the reference's draw
    np.random.seed(0)
    start = int(np.random.uniform(0, 50001 - 255 * 128))
    ref = spec_ref.specs_item(*clips[("train", 3)], start=start)
    assert _rel(Xt[0].cpu(), ref[0]) < TOL_FWD and _rel(Yt[0].cpu(), ref[1]) < TOL_FWD

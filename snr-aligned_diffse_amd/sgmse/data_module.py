"""SpecsDataModule — the spectrogram front/back end of the reference (data_module.py:178-297),
importable without pytorch_lightning / torchaudio (checkpoints unpickle it by qualified name,
model.py:45,93).  stft / istft / spec_fwd / spec_back run on the HIP kernels for device
tensors (n_fft 510, hop 128, periodic Hann, center=True, the 'exponent' transform).

Front-end: `Specs` / `Specs_SNR` (data_module.py:22-176) read the clean /
noisy WAV pairs (snrse.audio, torchaudio.load semantics), crop or zero-pad to num_frames on the
host (the only per-clip host work: index arithmetic on the decoded samples) and run the
mix / normalisation / STFT / spectrogram transform as device kernels.  `Specs.batch(indices)`
does that for a whole batch in one upload, one absmax, one fused STFT+transform launch per
signal, so batches reach the sampler at device speed.
"""
from __future__ import annotations

from glob import glob
from os.path import join

import numpy as np
import torch

from snrse import audio, ops


def get_window(window_type, window_length):
    if window_type == "sqrthann":
        return torch.sqrt(torch.hann_window(window_length, periodic=True))
    if window_type == "hann":
        return torch.hann_window(window_length, periodic=True)
    raise NotImplementedError(f"Window type {window_type} not implemented!")


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("Specs: the front-end runs on the HIP device (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


class Specs(torch.utils.data.Dataset):
    """Clean/noisy pairs -> (X, Y) complex64 [1, 256, num_frames] on the device
    (data_module.py:22-90): y = x + (y - x) fixed_snr; crop (random start when shuffle_spec,
    centred otherwise) or zero-pad (pad//2 left) to (num_frames - 1) hop samples; divide by
    max|y| ('noisy'), max|x| ('clean') or 1 ('not'); STFT; spec_transform."""

    def __init__(self, data_dir, subset, dummy, shuffle_spec, num_frames, format="default", normalize="noisy",
                 spec_transform=None, stft_kwargs=None, fixed_snr=1, **ignored_kwargs):
        if format != "default":
            raise NotImplementedError(f"Directory format {format} unknown!")
        self.clean_files = sorted(glob(join(data_dir, subset) + "/clean/*.wav"))
        self.noisy_files = sorted(glob(join(data_dir, subset) + "/noisy/*.wav"))
        self.dummy, self.num_frames, self.shuffle_spec = dummy, num_frames, shuffle_spec
        self.normalize, self.spec_transform, self.fixed_snr = normalize, spec_transform, fixed_snr
        stft_kwargs = stft_kwargs or dict(n_fft=510, hop_length=128, center=True, window=get_window("hann", 510))
        assert all(k in stft_kwargs.keys() for k in ["n_fft", "hop_length", "center", "window"]), \
            "misconfigured STFT kwargs"
        self.stft_kwargs = stft_kwargs
        self.hop_length = stft_kwargs["hop_length"]
        assert stft_kwargs.get("center", None) is True, "'center' must be True for current implementation"
        if (stft_kwargs["n_fft"], self.hop_length) != (510, 128):
            raise NotImplementedError("the HIP STFT is built for n_fft=510, hop 128")

    def _crop(self, x, y):
        """Host crop / pad of one [C, L] pair (data_module.py:53-68)."""
        target_len = (self.num_frames - 1) * self.hop_length
        cur = x.shape[-1]
        pad = max(target_len - cur, 0)
        if pad == 0:
            start = int(np.random.uniform(0, cur - target_len)) if self.shuffle_spec else int((cur - target_len) / 2)
            return x[..., start:start + target_len], y[..., start:start + target_len]
        pw = (pad // 2, pad // 2 + (pad % 2))
        return (torch.nn.functional.pad(x, pw, mode="constant"), torch.nn.functional.pad(y, pw, mode="constant"))

    def _load_pair(self, i):
        x, _ = audio.load(self.clean_files[i])
        y, _ = audio.load(self.noisy_files[i])
        return x, y

    def _specs(self, xs, ys, fixed_snr, one_clip=False):
        """Device half for stacked host crops xs, ys [B, L] -> (X, Y) [B, 1, 256, num_frames].
        one_clip: the rows are the C channels of ONE clip, normalised by one max over all of them
        (y.abs().max(), data_module.py:70-75) instead of per row."""
        dev = _device()
        B = xs.shape[0]
        xy = torch.cat([xs, ys], 0).to(dev, torch.float32, non_blocking=True)
        x, y = xy[:B], xy[B:]
        if fixed_snr != 1:
            y = (x + (y - x) * fixed_snr).contiguous()
        if self.normalize == "noisy":
            nf = ops.absmax(y)
        elif self.normalize == "clean":
            nf = ops.absmax(x)
        elif self.normalize == "not":
            nf = None
        else:
            raise ValueError(f"normalize {self.normalize!r}")
        if one_clip and nf is not None and B > 1:
            nf = nf.max().reshape(1).expand(B).contiguous()
        fused = getattr(self.spec_transform, "__func__", None) is SpecsDataModule.spec_fwd and \
            self.spec_transform.__self__.transform_type == "exponent"
        mode = 1 if fused else 0
        X = ops.stft(x.contiguous(), 1.0, mode=mode, in_div=nf)
        Y = ops.stft(y.contiguous(), 1.0, mode=mode, in_div=nf)
        if not fused and self.spec_transform is not None:
            X, Y = self.spec_transform(X), self.spec_transform(Y)
        return X[:, None], Y[:, None]

    def __getitem__(self, i):
        x, y = self._load_pair(i)
        x, y = self._crop(x, y)
        X, Y = self._specs(x, y, self.fixed_snr, one_clip=True)
        return X[:, 0], Y[:, 0]  # [C, F, T] like torch.stft of a [C, L] clip

    def batch(self, indices):
        """(X, Y) [len(indices), 1, 256, num_frames] for a list of clip indices, one device pass
        (mono clips; the per-item path handles [C, L] like the reference)."""
        xs, ys = [], []
        for i in indices:
            x, y = self._crop(*self._load_pair(i))
            if x.shape[0] != 1:
                raise ValueError("Specs.batch: mono clips only")
            xs.append(x[0])
            ys.append(y[0])
        return self._specs(torch.stack(xs), torch.stack(ys), self.fixed_snr)

    def __len__(self):
        return int(len(self.clean_files) / 200) if self.dummy else len(self.clean_files)


class Specs_SNR(Specs):
    """Validation set with per-clip active RMS (data_module.py:93-176): items are (X, Y, s, n)
    with s, n the clean / noise active RMS read from <subset>/active_rms.txt (tab-separated,
    columns 1 and 2); no fixed_snr mixing.  (The reference's __len__ returns None unless dummy;
    here it is the clip count.)"""

    def __init__(self, data_dir, subset, dummy, shuffle_spec, num_frames, format="default", normalize="noisy",
                 spec_transform=None, stft_kwargs=None, **ignored_kwargs):
        super().__init__(data_dir, subset, dummy, shuffle_spec, num_frames, format=format, normalize=normalize,
                         spec_transform=spec_transform, stft_kwargs=stft_kwargs, fixed_snr=1)
        self.active_rms = join(data_dir, subset) + "/active_rms.txt"
        self.clean_rms, self.noise_rms = [], []
        with open(self.active_rms, "r") as f:
            for line in f:
                parts = line.split("\t")
                try:
                    s_, n_ = float(parts[1]), float(parts[2])
                except (IndexError, ValueError):
                    break  # the reference stops at the first malformed line
                self.clean_rms.append(s_)
                self.noise_rms.append(n_)

    def __getitem__(self, i):
        X, Y = super().__getitem__(i)
        return X, Y, self.clean_rms[i], self.noise_rms[i]


class SpecsDataModule:
    @staticmethod
    def add_argparse_args(parser):
        parser.add_argument("--base_dir", type=str, required=True, help="The base directory of the dataset.")
        parser.add_argument("--format", type=str, choices=("default", "dns"), default="default")
        parser.add_argument("--batch_size", type=int, default=4)
        parser.add_argument("--n_fft", type=int, default=510)
        parser.add_argument("--hop_length", type=int, default=128)
        parser.add_argument("--num_frames", type=int, default=256)
        parser.add_argument("--window", type=str, choices=("sqrthann", "hann"), default="hann")
        parser.add_argument("--num_workers", type=int, default=4)
        parser.add_argument("--dummy", action="store_true")
        parser.add_argument("--spec_factor", type=float, default=0.15)
        parser.add_argument("--spec_abs_exponent", type=float, default=0.5)
        parser.add_argument("--normalize", type=str, choices=("clean", "noisy", "not"), default="noisy")
        parser.add_argument("--transform_type", type=str, choices=("exponent", "log", "none"), default="exponent")
        return parser

    def __init__(self, base_dir="", format="default", batch_size=8, n_fft=510, hop_length=128, num_frames=256,
                 window="hann", num_workers=4, dummy=False, spec_factor=0.15, spec_abs_exponent=0.5, gpu=True,
                 normalize="noisy", transform_type="exponent", fixed_snr=1, **kwargs):
        self.base_dir, self.format, self.batch_size = base_dir, format, batch_size
        self.n_fft, self.hop_length, self.num_frames = n_fft, hop_length, num_frames
        self.window_type = window
        self.window = get_window(window, n_fft)
        self.num_workers, self.dummy = num_workers, dummy
        self.spec_factor, self.spec_abs_exponent = spec_factor, spec_abs_exponent
        self.gpu, self.normalize, self.transform_type = gpu, normalize, transform_type
        self.fixed_snr = fixed_snr
        self.kwargs = kwargs

    def _check(self):
        if (self.n_fft, self.hop_length, self.window_type) != (510, 128, "hann"):
            raise NotImplementedError("the HIP STFT is built for n_fft=510, hop 128, periodic Hann")
        if self.transform_type == "exponent" and (self.spec_abs_exponent, self.spec_factor) != (0.5, 0.15):
            raise NotImplementedError("the HIP transform is built for exponent 0.5, factor 0.15")
        if self.transform_type not in ("exponent", "none"):
            raise NotImplementedError(f"transform_type {self.transform_type} is not built for the HIP path")

    def hip_mode(self):
        """Spectrogram mode of the fused HIP STFT / iSTFT for this configuration: 1 = 'exponent'
        transform fused (spec_fwd / spec_back, data_module.py:241-267), 0 = raw ('none').  Raises for a
        configuration the kernels are not built for (_check)."""
        self._check()
        return 1 if self.transform_type == "exponent" else 0

    def setup(self, stage=None):
        """Datasets of data_module.py:221-240 (device-producing Specs / Specs_SNR)."""
        self._check()
        kw = dict(stft_kwargs=self.istft_kwargs, num_frames=self.num_frames, spec_transform=self.spec_fwd,
                  **self.kwargs)
        if stage == "fit" or stage is None:
            self.train_set = Specs(data_dir=self.base_dir, subset="train", dummy=self.dummy, shuffle_spec=True,
                                   format=self.format, normalize=self.normalize, fixed_snr=self.fixed_snr, **kw)
            self.valid_set = Specs_SNR(data_dir=self.base_dir, subset="valid", dummy=self.dummy, shuffle_spec=False,
                                       format=self.format, normalize=self.normalize, **kw)
            self.valid_set_2 = Specs(data_dir=self.base_dir, subset="valid2", dummy=self.dummy, shuffle_spec=False,
                                     fixed_snr=1, format=self.format, normalize=self.normalize, **kw)
        if stage == "test" or stage is None:
            self.test_set = Specs(data_dir=self.base_dir, subset="test", dummy=self.dummy, shuffle_spec=False,
                                  format=self.format, normalize=self.normalize, fixed_snr=1, **kw)

    # DataLoaders of data_module.py:299-321; items are device tensors, so loading stays in-process
    def _loader(self, ds, batch_size, shuffle):
        return torch.utils.data.DataLoader(ds, batch_size=batch_size, num_workers=0, shuffle=shuffle, drop_last=True)

    def train_dataloader(self):
        return self._loader(self.train_set, self.batch_size, True)

    def val_dataloader(self):
        return self._loader(self.valid_set, 1, False)

    def val_dataloader_2(self):
        return self._loader(self.valid_set_2, self.batch_size, False)

    def test_dataloader(self):
        return self._loader(self.test_set, self.batch_size, False)

    @property
    def stft_kwargs(self):
        return {**self.istft_kwargs, "return_complex": True}

    @property
    def istft_kwargs(self):
        return dict(n_fft=self.n_fft, hop_length=self.hop_length, window=self.window, center=True)

    def spec_fwd(self, spec):
        self._check()
        if self.transform_type == "none":
            return spec
        flat = spec.to(torch.complex64).contiguous()
        return ops.spec_transform(flat, 0)

    def spec_back(self, spec):
        self._check()
        if self.transform_type == "none":
            return spec
        flat = spec.to(torch.complex64).contiguous()
        return ops.spec_transform(flat, 1)

    def stft(self, sig):
        """sig [L] or [B, L] (device) -> complex [.., 256, 1 + L//128] (raw STFT)."""
        self._check()
        x = sig.to(torch.float32)
        one = x.dim() == 1
        x = x.reshape(1, -1) if one else x.contiguous()
        out = ops.stft(x, 1.0, mode=0)
        return out[0] if one else out

    def istft(self, spec, length=None):
        """spec complex [.., 256, T] (device) -> waveform [.., length]."""
        self._check()
        one = spec.dim() == 2
        s = spec.reshape(1, *spec.shape) if one else spec
        L = length if length is not None else self.hop_length * (s.shape[-1] - 1)
        out = ops.istft(s.to(torch.complex64).contiguous(), L, mode=0)
        return out[0] if one else out

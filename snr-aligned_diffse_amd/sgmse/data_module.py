"""SpecsDataModule — the spectrogram front/back end of the reference (data_module.py:178-297),
importable without pytorch_lightning / torchaudio (checkpoints unpickle it by qualified name,
model.py:45,93).  stft / istft / spec_fwd / spec_back run on the HIP kernels for device
tensors (n_fft 510, hop 128, periodic Hann, center=True, the 'exponent' transform); the
dataset / DataLoader half of the reference is training-side and out of scope.
"""
from __future__ import annotations

import torch

from snrse import ops


def get_window(window_type, window_length):
    if window_type == "sqrthann":
        return torch.sqrt(torch.hann_window(window_length, periodic=True))
    if window_type == "hann":
        return torch.hann_window(window_length, periodic=True)
    raise NotImplementedError(f"Window type {window_type} not implemented!")


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

    def setup(self, stage=None):
        raise NotImplementedError("training datasets are out of scope of the inference build")

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

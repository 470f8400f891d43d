"""SNR estimator backbone — reference-compatible nn.Module (snrnet.py:9-97) on the HIP runtime.

Input [B, 2, F=256, T] real/imag planes as in the reference, or (fast path) the complex
STFT [B, 256, T] passed to `forward_complex`; output [B, 1] in (0, 1).
"""
import torch
import torch.nn as nn

from snrse import ops

from .shared import BackboneRegistry


@BackboneRegistry.register("snrnet")
class SNRNet(nn.Module):
    @staticmethod
    def add_argparse_args(parser):
        return parser

    def __init__(self):
        super().__init__()
        self.convt_out = 32
        self.conv5x5_1 = nn.Conv2d(2, 32, 5, padding=2)
        self.maxpool2x2_1 = nn.MaxPool2d(2)
        self.conv3x3_1 = nn.Conv2d(32, 32, 3, padding=1)
        self.maxpool2x1_1 = nn.MaxPool2d((2, 1))
        self.convt_1 = nn.Conv2d(32, 32, (64, 1))
        self.convt_2 = nn.Conv2d(32, 32, (64, 2))
        self.convt_3 = nn.Conv2d(32, 32, (64, 4))
        self.convt_4 = nn.Conv2d(32, 32, (64, 8))
        self.maxpoolt_1 = nn.MaxPool2d((1, 8))
        self.maxpoolt_2 = nn.MaxPool2d((1, 7))
        self.maxpoolt_3 = nn.MaxPool2d((1, 5))
        self.maxpoolt_4 = nn.MaxPool2d((1, 1))
        self.blstm = nn.LSTM(128, 128, 1, batch_first=True, bidirectional=True)
        self.fc = nn.Linear(1024, 1)
        self.sigmoid = nn.Sigmoid()
        self._packed, self._key = None, None

    def _pack(self, device):
        ps = list(self.state_dict(keep_vars=True).values())
        key = (tuple(p._version for p in ps), tuple(p.data_ptr() for p in ps), str(device))
        if self._packed is None or self._key != key:
            self._packed = ops.pack_snrnet(self.state_dict(), device)
            self._key = key
        return self._packed

    def forward_complex(self, spec):
        """spec: complex64 [B, 256, T] device tensor (T % 16 == 0) -> [B, 1]."""
        return ops.snrnet(spec.contiguous(), self._pack(spec.device))[:, None]

    def forward(self, x):
        """x: [B, 2, 256, T] (real, imag planes), T % 16 == 0 -> [B, 1]."""
        if not x.is_cuda:
            raise RuntimeError("SNRNet.forward: HIP device tensors required (no CPU fallback)")
        spec = torch.complex(x[:, 0].float(), x[:, 1].float()).contiguous()
        return self.forward_complex(spec)

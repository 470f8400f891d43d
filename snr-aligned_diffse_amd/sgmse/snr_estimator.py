"""SNRModel — the SNR-estimator wrapper of the reference (snr_estimator.py:20-174), inference
half only: forward(y) -> self.dnn(y) (SNRNet on the HIP runtime), checkpoint / EMA loading
without pytorch_lightning or torch_ema."""
from __future__ import annotations

import torch
import torch.nn as nn

from .backbones.snrnet import SNRNet
from .ema import EMAState, load_checkpoint


class SNRModel(nn.Module):
    @staticmethod
    def add_argparse_args(parser):
        parser.add_argument("--lr", type=float, default=1e-4)
        parser.add_argument("--ema_decay", type=float, default=0.999)
        parser.add_argument("--num_eval_files", type=int, default=10)
        parser.add_argument("--loss_type", type=str, default="mse")
        return parser

    def __init__(self, backbone="snrnet", lr=1e-4, ema_decay=0.999, num_eval_files=10, loss_type="mse",
                 data_module_cls=None, **kwargs):
        super().__init__()
        self.dnn = SNRNet()
        self.lr, self.ema_decay, self.loss_type, self.num_eval_files = lr, ema_decay, loss_type, num_eval_files
        self.ema = EMAState(self)
        self.data_module = data_module_cls(**kwargs, gpu=kwargs.get("gpus", 0) > 0) if data_module_cls else None

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", weights_only=None, **overrides):
        return load_checkpoint(cls, checkpoint_path, map_location, weights_only, overrides)

    def train(self, mode=True, no_ema=False):
        res = super().train(mode)
        self.ema.on_train(mode, no_ema)
        return res

    def eval(self, no_ema=False):
        return self.train(False, no_ema=no_ema)

    def forward(self, y):
        return self.dnn(y)

    @torch.no_grad()
    def estimate_from_spec(self, spec):
        """SNR estimate est_gt/(1 - est_gt) from a raw complex STFT [B, 256, T16] (model.py:715-721)."""
        g = self.dnn.forward_complex(spec)[:, 0]
        return g / (1 - g)

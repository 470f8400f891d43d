"""EMA shadow weights and PyTorch-Lightning checkpoint loading without PL / torch_ema.

The reference stores `checkpoint['ema'] = ExponentialMovingAverage.state_dict()` (torch_ema
0.3; model.py:109-118): shadow copies of the requires_grad parameters in
`ScoreModel.parameters()` order, and `eval(no_ema=False)` copies them over the live weights
(model.py:120-131).  EMAState reproduces that contract.
"""
from __future__ import annotations

import os
import warnings

import torch


class EMAState:
    def __init__(self, module: torch.nn.Module, decay=0.999):
        self.module = module
        self.decay = decay
        self.num_updates = None
        self.shadow_params = None
        self.collected_params = None
        self.error_loading = False

    def _params(self):
        return [p for p in self.module.parameters() if p.requires_grad]

    def load_state_dict(self, sd):
        params = self._params()
        shadow = sd["shadow_params"]
        if len(shadow) != len(params):
            raise ValueError(f"EMA state has {len(shadow)} shadow tensors, model has {len(params)} trainable")
        for s, p in zip(shadow, params):
            if tuple(s.shape) != tuple(p.shape):
                raise ValueError(f"EMA shadow shape {tuple(s.shape)} != parameter {tuple(p.shape)}")
        self.decay = sd.get("decay", self.decay)
        self.num_updates = sd.get("num_updates")
        self.shadow_params = [s.detach().clone() for s in shadow]

    def on_train(self, mode: bool, no_ema: bool):
        """train(False) without no_ema swaps the EMA weights in; train(True) restores."""
        if self.shadow_params is None:
            return
        params = self._params()
        if not mode and not no_ema:
            if self.collected_params is None:
                self.collected_params = [p.detach().clone() for p in params]
            with torch.no_grad():
                for s, p in zip(self.shadow_params, params):
                    p.copy_(s.to(p.device, p.dtype))
        elif mode and self.collected_params is not None:
            with torch.no_grad():
                for c, p in zip(self.collected_params, params):
                    p.copy_(c.to(p.device, p.dtype))
            self.collected_params = None


def load_checkpoint(cls, path, map_location="cpu", weights_only=None, overrides=None):
    """PL-style `load_from_checkpoint`: hyper_parameters -> __init__, state_dict, ema."""
    if weights_only is None:
        weights_only = os.environ.get("SNRSE_TRUST_CHECKPOINT", "0") != "1"
    try:
        ckpt = torch.load(path, map_location=map_location, weights_only=weights_only)
    except Exception as e:  # pickled classes in hyper_parameters (data_module_cls) need a full load
        raise RuntimeError(f"could not load {path} with weights_only={weights_only} ({e}); if you trust this "
                           "checkpoint pass weights_only=False or set SNRSE_TRUST_CHECKPOINT=1") from e
    hp = dict(ckpt.get("hyper_parameters", {}))
    hp.update(overrides or {})
    from .data_module import SpecsDataModule
    dm = hp.get("data_module_cls")
    if dm is None or isinstance(dm, str) or getattr(dm, "__name__", "") == "SpecsDataModule":
        hp["data_module_cls"] = SpecsDataModule
    model = cls(**hp)
    missing, unexpected = model.load_state_dict(ckpt["state_dict"], strict=False)
    if missing:
        raise RuntimeError(f"checkpoint is missing parameters: {missing[:5]} ...")
    if unexpected:
        warnings.warn(f"ignoring unexpected checkpoint entries: {unexpected[:5]} ...")
    if ckpt.get("ema") is not None:
        model.ema.load_state_dict(ckpt["ema"])
    else:
        model.ema.error_loading = True
        warnings.warn("EMA state_dict not found in checkpoint!")
    return model

"""NCSN++ score network — reference-compatible nn.Module, executed by the HIP runtime.

Parameter names, shapes and registration order match the reference NCSNpp
(sgmse/backbones/ncsnpp.py:36-245): `output_layer.*` first, then `all_modules.{0..76}.*`
(647 state-dict tensors, `all_modules.0.W` frozen), so checkpoints and EMA shadow lists
load unchanged.  `forward(x, time_cond)` (ncsnpp.py:247-404) packs the weights once per
parameter version into the device layout of snrse.ncsnpp.NCSNppHIP and runs there; there
is no CPU path.  Submodules are parameter holders only.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from snrse import ncsnpp as _hip

from .shared import BackboneRegistry


class GaussianFourierProjection(nn.Module):
    def __init__(self, embedding_size=256, scale=1.0):
        super().__init__()
        self.W = nn.Parameter(torch.randn(embedding_size) * scale, requires_grad=False)


class NIN(nn.Module):
    def __init__(self, in_dim, num_units):
        super().__init__()
        self.W = nn.Parameter(torch.zeros(in_dim, num_units))
        self.b = nn.Parameter(torch.zeros(num_units))


class ResnetBlockBigGANpp(nn.Module):
    def __init__(self, in_ch, out_ch=None, temb_dim=512, up=False, down=False):
        super().__init__()
        out_ch = out_ch or in_ch
        self.GroupNorm_0 = nn.GroupNorm(min(in_ch // 4, 32), in_ch, eps=1e-6)
        self.up, self.down = up, down
        self.Conv_0 = nn.Conv2d(in_ch, out_ch, 3, padding=1)
        self.Dense_0 = nn.Linear(temb_dim, out_ch)
        self.GroupNorm_1 = nn.GroupNorm(min(out_ch // 4, 32), out_ch, eps=1e-6)
        self.Dropout_0 = nn.Dropout(0.0)
        self.Conv_1 = nn.Conv2d(out_ch, out_ch, 3, padding=1)
        if in_ch != out_ch or up or down:
            self.Conv_2 = nn.Conv2d(in_ch, out_ch, 1)
        self.in_ch, self.out_ch = in_ch, out_ch


class AttnBlockpp(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.GroupNorm_0 = nn.GroupNorm(min(channels // 4, 32), channels, eps=1e-6)
        self.NIN_0 = NIN(channels, channels)
        self.NIN_1 = NIN(channels, channels)
        self.NIN_2 = NIN(channels, channels)
        self.NIN_3 = NIN(channels, channels)


class Combine(nn.Module):
    def __init__(self, dim1, dim2):
        super().__init__()
        self.Conv_0 = nn.Conv2d(dim1, dim2, 1)


@BackboneRegistry.register("ncsnpp")
class NCSNpp(nn.Module):
    """NCSN++ (nf=128, ch_mult=(1,1,2,2,2,2,2), BigGAN blocks, FIR, attention at 16, output /
    input skip pyramids) with complex [B, 2, F, T] input and [B, 1, F, T] output."""

    SUPPORTED = dict(scale_by_sigma=True, nonlinearity="swish", nf=128, ch_mult=(1, 1, 2, 2, 2, 2, 2),
                     num_res_blocks=2, attn_resolutions=(16,), resamp_with_conv=True, conditional=True,
                     fir=True, fir_kernel="song", skip_rescale=True, resblock_type="biggan",
                     progressive="output_skip", progressive_input="input_skip", progressive_combine="sum",
                     embedding_type="fourier")

    @staticmethod
    def add_argparse_args(parser):
        return parser

    def __init__(self, nf=128, ch_mult=(1, 1, 2, 2, 2, 2, 2), num_res_blocks=2, attn_resolutions=(16,),
                 image_size=256, fourier_scale=16, compute_dtype="fp32", **kw):
        super().__init__()
        for k, v in kw.items():
            if k in self.SUPPORTED and v != self.SUPPORTED[k] and not (isinstance(v, (list, tuple))
                                                                    and tuple(v) == tuple(self.SUPPORTED[k])):
                raise NotImplementedError(f"NCSNpp option {k}={v!r} is not built for the HIP path")
        self.cfg = dict(nf=nf, ch_mult=tuple(ch_mult), num_res_blocks=num_res_blocks,
                        attn_resolutions=tuple(attn_resolutions), image_size=image_size)
        _hip.check_topology(**self.cfg)  # the executor is built for the shipped topology only
        self.compute_dtype = compute_dtype
        self.output_layer = nn.Conv2d(4, 2, 1)
        mods = []
        self._plan = _hip.build_plan(**self.cfg)
        for m in self._plan:
            if m.kind == "gfp":
                mods.append(GaussianFourierProjection(nf, fourier_scale))
            elif m.kind == "linear":
                mods.append(nn.Linear(m.cin, m.cout))
            elif m.kind == "conv3x3":
                mods.append(nn.Conv2d(m.cin, m.cout, 3, padding=1))
            elif m.kind == "rb":
                mods.append(ResnetBlockBigGANpp(m.cin, m.cout, 4 * nf, up=m.up, down=m.down))
            elif m.kind == "attn":
                mods.append(AttnBlockpp(m.cin))
            elif m.kind == "combine":
                mods.append(Combine(4, m.cout))
            elif m.kind == "gn":
                mods.append(nn.GroupNorm(min(m.cin // 4, 32), m.cin, eps=1e-6))
        self.all_modules = nn.ModuleList(mods)
        self._hip_net = None
        self._hip_key = None

    # ---------------------------------------------------------------- device executor
    def _param_key(self):
        ps = list(self.state_dict(keep_vars=True).values())
        return (self.compute_dtype, tuple(p._version for p in ps), tuple(p.data_ptr() for p in ps))

    def hip(self, device=None) -> _hip.NCSNppHIP:
        """The packed device executor for the current parameters (re-packed on change)."""
        key = self._param_key()
        if self._hip_net is None or self._hip_key != key:
            dt = {"bf16": torch.bfloat16, torch.bfloat16: torch.bfloat16, "fp16": torch.float16,
                  torch.float16: torch.float16}.get(self.compute_dtype, torch.float32)
            gemm = "x3" if self.compute_dtype == "fp32x3" else "exact"  # split-bf16 fp32 GEMMs
            dev = device or (torch.device("cuda", torch.cuda.current_device()))
            self._hip_net = _hip.NCSNppHIP(self.state_dict(), dtype=dt, device=dev, gemm=gemm, **self.cfg)
            self._hip_key = key
        return self._hip_net

    def forward(self, x, time_cond):
        """x: complex [B, 2, F, T] (x_t and y), time_cond: [B] -> complex [B, 1, F, T]."""
        if not x.is_cuda:
            raise RuntimeError("NCSNpp.forward: HIP device tensors required (no CPU fallback); "
                               "move inputs with .cuda()")
        net = self.hip(x.device)
        x = x.to(torch.complex64)
        x0 = x[:, 0].contiguous()
        x1 = x[:, 1].contiguous()
        t = time_cond.reshape(-1).to(device=x.device, dtype=torch.float32).contiguous()
        return net.dnn(x0, x1, t)[:, None]

"""CPU oracle (TEST INFRASTRUCTURE ONLY) — NCSN++ score network, functional form.

Restates, over a plain state_dict (same keys as the reference module):
  * GaussianFourierProjection      layerspp.py:32-43
  * temb MLP                       ncsnpp.py:256-275
  * FIR resampling (upfirdn2d)     up_or_down_sampling.py:195-257, op/upfirdn2d.py:159-200
  * ResnetBlockBigGANpp            layerspp.py:244-276
  * AttnBlockpp + NIN              layerspp.py:77-93, layers.py:546-555
  * Combine ('sum')                layerspp.py:54-61
  * NCSNpp.forward                 ncsnpp.py:247-404 (config: nf=128, ch_mult=(1,1,2,2,2,2,2),
                                   2 res blocks, attn at 16, biggan, output_skip, input_skip,
                                   sum, fourier embedding, skip_rescale)
Works in float32 (parity) or float64 (high-precision reference).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

INV_SQRT2 = 1.0 / math.sqrt(2.0)
_K1 = (1.0, 3.0, 3.0, 1.0)


def _fir2d(dtype):
    k = torch.tensor(_K1, dtype=dtype)
    k2 = torch.outer(k, k)
    return k2 / k2.sum()  # _setup_kernel: outer product, normalised to sum 1


def fir_down2(x: torch.Tensor) -> torch.Tensor:
    """downsample_2d(x, [1,3,3,1], 2): pad (1,1) each axis, 4x4 FIR, stride 2."""
    C = x.shape[1]
    w = _fir2d(x.dtype).flip(0, 1).expand(C, 1, 4, 4)
    return F.conv2d(F.pad(x, (1, 1, 1, 1)), w, stride=2, groups=C)


def fir_up2(x: torch.Tensor) -> torch.Tensor:
    """upsample_2d(x, [1,3,3,1], 2): zero-insert x2, pad (2,1), 4x4 FIR with gain 4."""
    B, C, H, W = x.shape
    u = x.new_zeros(B, C, 2 * H, 2 * W)
    u[:, :, ::2, ::2] = x
    w = (_fir2d(x.dtype) * 4.0).flip(0, 1).expand(C, 1, 4, 4)
    return F.conv2d(F.pad(u, (2, 1, 2, 1)), w, groups=C)


def group_norm(x, sd, pre):
    C = x.shape[1]
    return F.group_norm(x, min(C // 4, 32), sd[pre + ".weight"], sd[pre + ".bias"], eps=1e-6)


def conv(x, sd, pre, pad):
    return F.conv2d(x, sd[pre + ".weight"], sd[pre + ".bias"], padding=pad)


def resblock(x, temb, sd, pre, up=False, down=False):
    """ResnetBlockBigGANpp.forward (layerspp.py:244-276), fir=True, skip_rescale=True."""
    in_ch = x.shape[1]
    out_ch = sd[pre + ".Conv_0.weight"].shape[0]
    h = F.silu(group_norm(x, sd, pre + ".GroupNorm_0"))
    if up:
        h, x = fir_up2(h), fir_up2(x)
    elif down:
        h, x = fir_down2(h), fir_down2(x)
    h = conv(h, sd, pre + ".Conv_0", 1)
    h = h + F.linear(F.silu(temb), sd[pre + ".Dense_0.weight"], sd[pre + ".Dense_0.bias"])[:, :, None, None]
    h = F.silu(group_norm(h, sd, pre + ".GroupNorm_1"))
    h = conv(h, sd, pre + ".Conv_1", 1)
    if in_ch != out_ch or up or down:
        x = conv(x, sd, pre + ".Conv_2", 0)
    return (x + h) * INV_SQRT2


def nin(x, sd, pre):
    """NIN: y[b,o,h,w] = sum_i x[b,i,h,w] W[i,o] + b[o]  (layers.py:546-555)."""
    return torch.einsum("bihw,io->bohw", x, sd[pre + ".W"]) + sd[pre + ".b"][None, :, None, None]


def attn_block(x, sd, pre):
    """AttnBlockpp.forward (layerspp.py:77-93), skip_rescale=True."""
    B, C, H, W = x.shape
    h = group_norm(x, sd, pre + ".GroupNorm_0")
    q, k, v = nin(h, sd, pre + ".NIN_0"), nin(h, sd, pre + ".NIN_1"), nin(h, sd, pre + ".NIN_2")
    s = torch.einsum("bcl,bcm->blm", q.reshape(B, C, H * W), k.reshape(B, C, H * W)) * (C ** -0.5)
    p = torch.softmax(s, dim=-1)
    o = torch.einsum("blm,bcm->bcl", p, v.reshape(B, C, H * W)).reshape(B, C, H, W)
    return (x + nin(o, sd, pre + ".NIN_3")) * INV_SQRT2


def temb_mlp(t, sd):
    """GFP(log t) -> Linear -> SiLU -> Linear  (ncsnpp.py:256-275, layerspp.py:39-43)."""
    W = sd["all_modules.0.W"]
    proj = torch.log(t)[:, None] * W[None, :] * 2 * math.pi
    e = torch.cat([torch.sin(proj), torch.cos(proj)], dim=-1)
    e = F.linear(e, sd["all_modules.1.weight"], sd["all_modules.1.bias"])
    return F.linear(F.silu(e), sd["all_modules.2.weight"], sd["all_modules.2.bias"])


CH_MULT = (1, 1, 2, 2, 2, 2, 2)
NF = 128
NUM_RES = 2
ATTN_RES = (16,)


def ncsnpp_forward(xc: torch.Tensor, t: torch.Tensor, sd: dict) -> torch.Tensor:
    """NCSNpp.forward (ncsnpp.py:247-404). xc: complex [B,2,F,T]; t: [B] -> complex [B,1,F,T]."""
    dt = sd["output_layer.weight"].dtype
    x = torch.cat([xc[:, 0:1].real, xc[:, 0:1].imag, xc[:, 1:2].real, xc[:, 1:2].imag], 1).to(dt)
    t = t.to(dt)
    temb = temb_mlp(t, sd)
    m = 3  # module index after GFP, Dense, Dense
    mod = lambda i: f"all_modules.{i}"  # noqa: E731
    nres = len(CH_MULT)
    pyr_in = x
    hs = [conv(x, sd, mod(m), 1)]
    m += 1
    for lvl in range(nres):
        for _ in range(NUM_RES):
            h = resblock(hs[-1], temb, sd, mod(m))
            m += 1
            if h.shape[-2] in ATTN_RES:
                h = attn_block(h, sd, mod(m))
                m += 1
            hs.append(h)
        if lvl != nres - 1:
            h = resblock(hs[-1], temb, sd, mod(m), down=True)
            m += 1
            pyr_in = fir_down2(pyr_in)
            h = conv(pyr_in, sd, mod(m) + ".Conv_0", 0) + h  # Combine(method='sum')
            m += 1
            hs.append(h)
    h = hs[-1]
    h = resblock(h, temb, sd, mod(m)); m += 1  # noqa: E702
    h = attn_block(h, sd, mod(m)); m += 1  # noqa: E702
    h = resblock(h, temb, sd, mod(m)); m += 1  # noqa: E702
    pyr = None
    for lvl in reversed(range(nres)):
        for _ in range(NUM_RES + 1):
            h = resblock(torch.cat([h, hs.pop()], 1), temb, sd, mod(m))
            m += 1
        if h.shape[-2] in ATTN_RES:
            h = attn_block(h, sd, mod(m))
            m += 1
        ph = conv(F.silu(group_norm(h, sd, mod(m))), sd, mod(m + 1), 1)
        m += 2
        pyr = ph if lvl == nres - 1 else fir_up2(pyr) + ph
        if lvl != 0:
            h = resblock(h, temb, sd, mod(m), up=True)
            m += 1
    assert not hs and m == 77
    h = pyr / t[:, None, None, None]
    h = conv(h, sd, "output_layer", 0)
    h = h.permute(0, 2, 3, 1).contiguous()
    if h.dtype == torch.float64:
        return torch.view_as_complex(h)[:, None]
    return torch.view_as_complex(h.float())[:, None]


def state_dict_to_torch(sd_np: dict, dtype=torch.float32) -> dict:
    return {k: torch.as_tensor(v).to(dtype) for k, v in sd_np.items()}

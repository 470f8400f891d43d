"""Per-tensor-class attribution of the 16-bit headline's error, by CPU emulation.

The NCSN++ forward of oracle/ncsnpp_ref.py (reference ncsnpp.py:247-404) restated with a rounding hook at every
point where the HIP bf16 path (snrse/ncsnpp.py) holds a tensor in 16 bits.  Each point belongs to one class:

  w      conv / NIN weights (the packed GEMM B operands; Combine and the output layer stay fp32 there)
  op     GEMM A operands produced by a GroupNorm(+SiLU) transform (halo staging of Conv_0 / Conv_1 / the pyramid
         heads, gn_apply / gn_resample outputs, the attention's GroupNorm output)
  store  stored activations written by a GEMM epilogue (Conv_0 output, ResBlock / attention outputs, the skip
         stack, the input conv output) -- also the residual / shortcut operand the next blocks read
  raw    the raw FIR'd shortcut input of up / down ResBlocks (gn_resample's second output)
  attn   q, k, v (the QKV GEMM's stored output), the softmax probabilities fed to the PV MFMA, the attention output
  inp    the input conv's operand (x, y complex64 -> 16 bits)

Every class is rounded to `fmt[class]` in {"bf16", "fp16", "fp32"} (fp32 = not rounded).  Runs the reference's
one-NFE golden (ncsnpp_full.npz) and its N = 5 OUVE PC golden (pc_ouve.npz, 10 NFE with the recorded draws) and
prints relative / absolute RMS against them, plus the largest magnitude every class held (fp16 range check).
Usage: [EMU_SD=state_dict] python tools/bf16_attrib.py [preset ...]   (presets below; default: all).
Test infrastructure: reads oracle/ and tests/golden; nothing on the product path imports it."""
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "snr-aligned_diffse_amd")]
torch.set_num_threads(int(os.environ.get("EMU_THREADS", "8")))
from conftest import fnormal, golden  # noqa: E402
from oracle import sde_ref  # noqa: E402
from oracle.ncsnpp_ref import (ATTN_RES, CH_MULT, INV_SQRT2, NUM_RES, fir_down2, fir_up2,  # noqa: E402
                               state_dict_to_torch, temb_mlp)
from snrse import formula  # noqa: E402
from test_oracle_golden import Tape  # noqa: E402

CLASSES = ("w", "op", "store", "raw", "attn", "inp")
FMT = {c: "bf16" for c in CLASSES}
MAXABS = {c: 0.0 for c in CLASSES}
MINW = [float("inf")]


def R(cls, x):
    MAXABS[cls] = max(MAXABS[cls], float(x.abs().max()))
    f = FMT[cls]
    if f == "bf16":
        return x.to(torch.bfloat16).float()
    if f == "fp16":
        return x.to(torch.float16).float()
    return x


def Wr(w):
    nz = w.abs()[w != 0]
    if nz.numel():
        MINW[0] = min(MINW[0], float(nz.min()))
    return R("w", w)


def gn(x, sd, pre):
    C = x.shape[1]
    return F.group_norm(x, min(C // 4, 32), sd[pre + ".weight"], sd[pre + ".bias"], eps=1e-6)


def conv(a, sd, pre, pad):
    return F.conv2d(a, Wr(sd[pre + ".weight"]), sd[pre + ".bias"], padding=pad)


def resblock(x, temb, sd, pre, up=False, down=False):
    """layerspp.py:244-276 with the HIP path's 16-bit points (snrse/ncsnpp.py _resblock)."""
    in_ch, out_ch = x.shape[1], sd[pre + ".Conv_0.weight"].shape[0]
    h = F.silu(gn(x, sd, pre + ".GroupNorm_0"))
    xs = x
    if up or down:
        fir = fir_up2 if up else fir_down2
        h, xs = fir(h), R("raw", fir(x))
    h = conv(R("op", h), sd, pre + ".Conv_0", 1)
    h = R("store", h + F.linear(F.silu(temb), sd[pre + ".Dense_0.weight"], sd[pre + ".Dense_0.bias"])[:, :, None, None])
    h = conv(R("op", F.silu(gn(h, sd, pre + ".GroupNorm_1"))), sd, pre + ".Conv_1", 1)
    if in_ch != out_ch or up or down:
        xs = conv(xs, sd, pre + ".Conv_2", 0)
    return (xs + h) * INV_SQRT2


def nin(x, sd, pre):
    return torch.einsum("bihw,io->bohw", x, Wr(sd[pre + ".W"])) + sd[pre + ".b"][None, :, None, None]


def attn_block(x, sd, pre):
    B, C, H, W = x.shape
    h = R("op", gn(x, sd, pre + ".GroupNorm_0"))
    q, k, v = (R("attn", nin(h, sd, pre + f".NIN_{i}")) for i in range(3))
    s = torch.einsum("bcl,bcm->blm", q.reshape(B, C, H * W), k.reshape(B, C, H * W)) * (C ** -0.5)
    p = R("attn", torch.softmax(s, dim=-1))
    o = R("attn", torch.einsum("blm,bcm->bcl", p, v.reshape(B, C, H * W)).reshape(B, C, H, W))
    return (x + nin(o, sd, pre + ".NIN_3")) * INV_SQRT2


def forward(xc, t, sd):
    x = torch.cat([xc[:, 0:1].real, xc[:, 0:1].imag, xc[:, 1:2].real, xc[:, 1:2].imag], 1).float()
    temb = temb_mlp(t.float(), sd)
    m = 3
    mod = lambda i: f"all_modules.{i}"  # noqa: E731
    nres = len(CH_MULT)
    pyr_in = x
    hs = [R("store", conv(R("inp", x), sd, mod(m), 1))]
    m += 1
    for lvl in range(nres):
        for _ in range(NUM_RES):
            h = resblock(hs[-1], temb, sd, mod(m))
            m += 1
            if h.shape[-2] in ATTN_RES:
                h = attn_block(R("store", h), sd, mod(m))
                m += 1
            hs.append(R("store", h))
        if lvl != nres - 1:
            h = resblock(hs[-1], temb, sd, mod(m), down=True)
            m += 1
            pyr_in = fir_down2(pyr_in)
            h = F.conv2d(pyr_in, sd[mod(m) + ".Conv_0.weight"], sd[mod(m) + ".Conv_0.bias"]) + h
            m += 1
            hs.append(R("store", h))
    h = hs[-1]
    h = R("store", resblock(h, temb, sd, mod(m))); m += 1  # noqa: E702
    h = R("store", attn_block(h, sd, mod(m))); m += 1  # noqa: E702
    h = R("store", resblock(h, temb, sd, mod(m))); m += 1  # noqa: E702
    pyr = None
    for lvl in reversed(range(nres)):
        for _ in range(NUM_RES + 1):
            h = R("store", resblock(torch.cat([h, hs.pop()], 1), temb, sd, mod(m)))
            m += 1
        if h.shape[-2] in ATTN_RES:
            h = R("store", attn_block(h, sd, mod(m)))
            m += 1
        ph = conv(R("op", F.silu(gn(h, sd, mod(m)))), sd, mod(m + 1), 1)
        m += 2
        pyr = ph if lvl == nres - 1 else fir_up2(pyr) + ph
        if lvl != 0:
            h = R("store", resblock(h, temb, sd, mod(m), up=True))
            m += 1
    assert not hs and m == 77
    h = F.conv2d(pyr / t[:, None, None, None], sd["output_layer.weight"], sd["output_layer.bias"])
    return torch.view_as_complex(h.permute(0, 2, 3, 1).contiguous())[:, None]


_SD = None


def weights():
    """The formula weights, or EMU_SD=path: an NCSN++ state dict (.safetensors, or a torch file read with
    weights_only=True; a Lightning checkpoint's 'state_dict' with its 'dnn.' prefix is accepted) -- the maxabs
    columns then say how far that checkpoint's activations sit from the 16-bit formats' ranges."""
    global _SD
    if _SD is None:
        path = os.environ.get("EMU_SD")
        if path:
            if path.endswith(".safetensors"):
                from safetensors.torch import load_file
                sd = load_file(path)
            else:
                sd = torch.load(path, map_location="cpu", weights_only=True)
                sd = sd.get("state_dict", sd)
            sd = {k[4:] if k.startswith("dnn.") else k: v for k, v in sd.items()}
            _SD = state_dict_to_torch({k: v.float().numpy() for k, v in sd.items() if torch.is_tensor(v)})
        else:
            with open(os.path.join(ROOT, "tests", "golden", "state_dict_keys.json")) as f:
                shapes = {k: tuple(s) for k, s in json.load(f)["ncsnpp"]}
            _SD = state_dict_to_torch(formula.formula_state_dict(shapes))
    return _SD


def rel(a, b):
    a, b = torch.as_tensor(a).to(torch.complex128), torch.as_tensor(b).to(torch.complex128)
    return float((a - b).abs().pow(2).mean().sqrt() / b.abs().pow(2).mean().sqrt()), \
        float((a - b).abs().pow(2).mean().sqrt())


def run_nfe():
    g = golden("ncsnpp_full.npz")
    x = torch.from_numpy(fnormal("golden.ncsnpp.x", (2, 2, 256, 64), complex_=True)) * 0.5
    out = forward(x, torch.tensor([0.5, 0.8]), weights())
    return rel(out[:, 0], torch.from_numpy(g["out"][:, 0]))


def run_pc():
    g = golden("pc_ouve.npz")
    Y = torch.from_numpy(fnormal("golden.pc.Y", (2, 1, 256, 64), complex_=True)) * 0.5
    sde = sde_ref.OUVE(1.5, 0.05, 0.5, N=5)
    sd = weights()

    def score_fn(x, t, y):
        return -forward(torch.cat([x, y], 1), torch.full((x.shape[0],), t, dtype=torch.float32), sd)

    xr, _ = sde_ref.pc_sample(sde, score_fn, Y, Tape("golden.pc.noise"))
    return rel(xr[:, 0], torch.from_numpy(g["out"][:, 0]))


def preset(name):
    """name: 'all:bf16', 'all:fp16', 'fp32:<cls>' (that class fp32, rest bf16), 'only:<cls>' (only that class bf16),
    'fp16:<cls>' (that class fp16, rest bf16), or 'c1=f1,c2=f2' (explicit, unnamed classes bf16)."""
    f = {c: "bf16" for c in CLASSES}
    if name.startswith("all:"):
        f = {c: name[4:] for c in CLASSES}
    elif name.startswith("fp32:"):
        for c in name[5:].split("+"):
            f[c] = "fp32"
    elif name.startswith("fp16:"):
        for c in name[5:].split("+"):
            f[c] = "fp16"
    elif name.startswith("only:"):
        f = {c: "fp32" for c in CLASSES}
        for c in name[5:].split("+"):
            f[c] = "bf16"
    else:
        for kv in name.split(","):
            k, v = kv.split("=")
            f[k] = v
    return f


DEFAULT = ["all:fp32", "all:bf16"] + [f"only:{c}" for c in CLASSES] + [f"fp32:{c}" for c in CLASSES] + ["all:fp16"]

if __name__ == "__main__":
    which = sys.argv[1:] or DEFAULT
    for name in which:
        FMT.update(preset(name))
        for c in CLASSES:
            MAXABS[c] = 0.0
        t0 = time.time()
        nfe_rel, nfe_abs = run_nfe()
        pc_rel, pc_abs = run_pc() if os.environ.get("EMU_PC", "1") == "1" else (float("nan"), float("nan"))
        print(json.dumps({"preset": name, "fmt": dict(FMT), "nfe_rel": nfe_rel, "nfe_abs": nfe_abs, "pc_rel": pc_rel,
                          "pc_abs": pc_abs, "maxabs": {k: round(v, 3) for k, v in MAXABS.items()},
                          "min_nonzero_w": MINW[0], "seconds": round(time.time() - t0, 1)}), flush=True)

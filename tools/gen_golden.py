#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ by running the REFERENCE modules.

Runs only in the build container (it reads /root/reference, which does not exist on
the GPU box).  The reference's own torch modules produce every expected output here:

  sgmse.backbones.ncsnpp.NCSNpp            (ncsnpp.py:36-404)
  sgmse.backbones.ncsnpp_utils.layerspp     (ResnetBlockBigGANpp 214-276, AttnBlockpp 64-93,
                                             GaussianFourierProjection 32-43)
  sgmse.backbones.ncsnpp_utils.up_or_down_sampling (upsample_2d/downsample_2d 195-257)
  sgmse.backbones.snrnet.SNRNet             (snrnet.py:47-97)
  sgmse.sdes.{OUVESDE,BBED,PROPOSED_1}      (sdes.py:149-392)
  sgmse.sampling.get_pc_sampler             (sampling/__init__.py:28-80)

Import recipe: stub torch.utils.cpp_extension.load before importing, so
the op/ package does not JIT-compile CUDA; the CPU paths never touch the stub.

Modules that do not import here (sgmse.model / data_module need pytorch_lightning,
torchaudio) are restated from source text for the STFT / transform / preconditioning
glue, citing the lines.  Inputs and injected noise come from snrse.formula so the tests
can regenerate them instead of storing them.  Only outputs are stored.
"""
from __future__ import annotations

import json
import math
import os
import sys
import wave

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/sgmse-bbed"
OUT = os.path.join(REPO, "tests", "golden")

# snrse/formula.py is loaded by file path: putting the build's package directory on sys.path would
# let its regular `sgmse` package shadow the reference's namespace package of the same name.
import importlib.util  # noqa: E402

_spec = importlib.util.spec_from_file_location(
    "snrse_formula", os.path.join(REPO, "snr-aligned_diffse_amd", "snrse", "formula.py"))
formula = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(formula)

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
import torch.utils.cpp_extension as _ce  # noqa: E402

_ce.load = lambda *a, **k: None
sys.path.insert(0, REF)
from sgmse.backbones import BackboneRegistry  # noqa: E402
from sgmse.backbones.ncsnpp_utils import layerspp, up_or_down_sampling  # noqa: E402
from sgmse.backbones.snrnet import SNRNet  # noqa: E402
from sgmse import sdes as ref_sdes  # noqa: E402
from sgmse import sampling as ref_sampling  # noqa: E402

torch.set_num_threads(8)


def load_formula(module: torch.nn.Module, prefix: str = ""):
    sd = module.state_dict()
    shapes = {prefix + k: tuple(v.shape) for k, v in sd.items()}
    vals = formula.formula_state_dict(shapes)
    module.load_state_dict({k: torch.from_numpy(vals[prefix + k]) for k in sd})
    return module


def fnormal(name, shape, complex_=False):
    return torch.from_numpy(formula.normal_tensor(name, shape, complex_))


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def t2n(x):
    return x.detach().cpu().numpy()


# ---------------------------------------------------------------------------------
def gen_keys():
    net = BackboneRegistry.get_by_name("ncsnpp")()
    keys = [[k, list(v.shape)] for k, v in net.state_dict().items()]
    frozen = [n for n, p in net.named_parameters() if not p.requires_grad]
    trainable_order = [n for n, p in net.named_parameters() if p.requires_grad]
    snr = SNRNet()
    skeys = [[k, list(v.shape)] for k, v in snr.state_dict().items()]
    with open(os.path.join(OUT, "state_dict_keys.json"), "w") as f:
        json.dump({"ncsnpp": keys, "ncsnpp_frozen": frozen,
                   "ncsnpp_trainable_order": trainable_order, "snrnet": skeys}, f)
    print("wrote state_dict_keys.json", len(keys), len(skeys))


def gen_fir():
    x = fnormal("golden.fir.x", (2, 8, 16, 32))
    k = [1, 3, 3, 1]
    up = up_or_down_sampling.upsample_2d(x, k, factor=2)
    dn = up_or_down_sampling.downsample_2d(x, k, factor=2)
    save("fir.npz", up=t2n(up), down=t2n(dn))


def gen_blocks():
    act = torch.nn.SiLU()
    out = {}
    cfgs = {
        "plain": dict(in_ch=128, out_ch=128, up=False, down=False, hw=(8, 16)),
        "cin_ne_cout": dict(in_ch=128, out_ch=256, up=False, down=False, hw=(8, 8)),
        "down": dict(in_ch=128, out_ch=128, up=False, down=True, hw=(8, 16)),
        "up": dict(in_ch=256, out_ch=256, up=True, down=False, hw=(4, 8)),
        "cat384": dict(in_ch=384, out_ch=256, up=False, down=False, hw=(4, 8)),
    }
    for name, c in cfgs.items():
        rb = layerspp.ResnetBlockBigGANpp(act=act, in_ch=c["in_ch"], out_ch=c["out_ch"],
                                          temb_dim=512, up=c["up"], down=c["down"],
                                          dropout=0.0, fir=True, fir_kernel=[1, 3, 3, 1],
                                          skip_rescale=True, init_scale=0.0).eval()
        load_formula(rb, f"rb_{name}.")
        x = fnormal(f"golden.rb_{name}.x", (2, c["in_ch"]) + c["hw"])
        temb = fnormal(f"golden.rb_{name}.temb", (2, 512))
        with torch.no_grad():
            y = rb(x, temb)
            gn = act(rb.GroupNorm_0(x))
        out[f"{name}_out"] = t2n(y)
        if name == "plain":
            out[f"{name}_gn0silu"] = t2n(gn)
    save("resblocks.npz", **out)


def gen_attn():
    blk = layerspp.AttnBlockpp(channels=256, skip_rescale=True, init_scale=0.0).eval()
    load_formula(blk, "attn.")
    x = fnormal("golden.attn.x", (2, 256, 16, 8))
    with torch.no_grad():
        y = blk(x)
    save("attn.npz", out=t2n(y))


def gen_ncsnpp():
    net = BackboneRegistry.get_by_name("ncsnpp")().eval()
    load_formula(net)
    x = fnormal("golden.ncsnpp.x", (2, 2, 256, 64), complex_=True) * 0.5
    t = torch.tensor([0.5, 0.8], dtype=torch.float32)
    with torch.no_grad():
        # temb path pieces (ncsnpp.py:256-275)
        m = net.all_modules
        temb = m[0](torch.log(t))
        temb = m[2](torch.nn.functional.silu(m[1](temb)))
        y = net(x, t)
    save("ncsnpp_full.npz", out=t2n(y), temb=t2n(temb), t=t2n(t))


def gen_sde():
    ts = torch.tensor([0.03, 0.2, 0.5, 0.8, 0.999], dtype=torch.float32)
    ou = ref_sdes.OUVESDE(theta=1.5, sigma_min=0.05, sigma_max=0.5, N=30)
    ou1 = ref_sdes.OUVESDE(theta=1.5, sigma_min=0.05, sigma_max=1.0, N=30)
    bb = ref_sdes.BBED(T_sampling=0.999, k=2.6, theta=0.52, N=30)
    p1 = ref_sdes.PROPOSED_1(T_sampling=0.99, sigma_min=1.0, sigma_max=2.6, theta=0.52, N=30)
    p1b = ref_sdes.PROPOSED_1(T_sampling=0.99, sigma_min=0.5, sigma_max=3.0, theta=0.53, N=30)
    x = fnormal("golden.sde.x", (5, 1, 4, 4), complex_=True)
    y = fnormal("golden.sde.y", (5, 1, 4, 4), complex_=True)
    out = {"t": t2n(ts)}
    for nm, s in (("ouve", ou), ("ouve_smax1", ou1), ("bbed", bb), ("proposed_1", p1), ("proposed_1b", p1b)):
        d, g = s.sde(x, ts[:, None, None, None], y)
        out[f"{nm}_drift"] = t2n(d)
        out[f"{nm}_g"] = t2n(torch.as_tensor(g)).reshape(-1)
        out[f"{nm}_std"] = t2n(s._std(ts)).astype(np.float64)
        out[f"{nm}_mean"] = t2n(s._mean(x, ts, y))
    save("sde.npz", **out)


class _NoiseTape:
    """Monkeypatches torch.randn_like so the reference sampler consumes formula noise
    (draw i is normal_tensor(f"{tag}.{i}") with torch's complex convention)."""

    def __init__(self, tag):
        self.tag, self.i, self._orig = tag, 0, None

    def __enter__(self):
        self._orig = torch.randn_like

        def fake(x, *a, **k):
            z = fnormal(f"{self.tag}.{self.i}", tuple(x.shape), complex_=torch.is_complex(x))
            self.i += 1
            return z.to(x.dtype) if not torch.is_complex(x) else z.to(x.dtype)

        torch.randn_like = fake
        return self

    def __exit__(self, *exc):
        torch.randn_like = self._orig


def gen_pc_ouve():
    net = BackboneRegistry.get_by_name("ncsnpp")().eval()
    load_formula(net)
    Y = fnormal("golden.pc.Y", (2, 1, 256, 64), complex_=True) * 0.5
    sde = ref_sdes.OUVESDE(theta=1.5, sigma_min=0.05, sigma_max=0.5, N=5)

    def score_fn(x, t, y):  # ScoreModel.forward, model_type='bbed' (model.py:485-489)
        return -net(torch.cat([x, y], dim=1), t)

    sampler = ref_sampling.get_pc_sampler("reverse_diffusion", "ald", sde=sde, score_fn=score_fn,
                                          Y=Y, eps=0.03, snr=0.5, corrector_steps=1)
    with torch.no_grad(), _NoiseTape("golden.pc.noise") as tape:
        xr, ns = sampler()
    save("pc_ouve.npz", out=t2n(xr), ns=np.int64(ns), draws=np.int64(tape.i))


def gen_pc_variants():
    """Sampler arithmetic with a cheap analytic score (no network): every predictor /
    corrector pairing, OUVE and BBED, so the SDE/PC kernels are pinned independently."""
    Y = fnormal("golden.pcv.Y", (2, 1, 16, 8), complex_=True)

    def score_fn(x, t, y):
        return -(x - y) * 0.7 + 0.1 * y

    out = {}
    # 'euler_maruyama' is not pinned: the reference's pc loop passes `stepsize` as a 4th
    # positional argument that EulerMaruyamaPredictor forwards into sde.sde() -> TypeError
    # (sampling/__init__.py:72, predictors.py:46-49, sdes.py:192).
    cases = [("ouve", "reverse_diffusion", "ald"), ("ouve", "reverse_diffusion", "langevin"),
             ("ouve", "reverse_diffusion", "none"), ("ouve", "none", "ald"),
             ("bbed", "reverse_diffusion", "ald"), ("proposed_1", "reverse_diffusion", "ald")]
    for sde_name, pred, corr in cases:
        if sde_name == "ouve":
            sde = ref_sdes.OUVESDE(theta=1.5, sigma_min=0.05, sigma_max=0.5, N=6)
            Yc = Y
        elif sde_name == "bbed":  # BBED works only for B=1 in the reference (sdes.py:276), see DESIGN.md
            sde = ref_sdes.BBED(T_sampling=0.999, k=2.6, theta=0.52, N=6)
            Yc = Y[:1]
        else:  # PROPOSED_1: the same (y - x)/(Tc - t) drift without the [B] reshape (sdes.py:357): B=1 as well
            sde = ref_sdes.PROPOSED_1(T_sampling=0.99, sigma_min=1.0, sigma_max=2.6, theta=0.52, N=6)
            Yc = Y[:1]
        sampler = ref_sampling.get_pc_sampler(pred, corr, sde=sde, score_fn=score_fn, Y=Yc,
                                              eps=0.03, snr=0.5, corrector_steps=1)
        tag = f"golden.pcv.{sde_name}.{pred}.{corr}"
        with torch.no_grad(), _NoiseTape(tag) as tape:
            xr, ns = sampler()
        key = f"{sde_name}__{pred}__{corr}"
        out[key] = t2n(xr).astype(np.complex128)
        out[key + "__ns"] = np.int64(ns)
        out[key + "__draws"] = np.int64(tape.i)
    save("pc_variants.npz", **out)


def read_wav(path):
    with wave.open(path) as w:
        assert w.getsampwidth() == 2 and w.getnchannels() == 1
        raw = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2")
    return raw.copy()


def stft_ref(sig):  # SpecsDataModule.stft: data_module.py:269-278, 291-293 (window 13-19)
    win = torch.hann_window(510, periodic=True)
    return torch.stft(sig, n_fft=510, hop_length=128, window=win, center=True, return_complex=True)


def istft_ref(spec, length):  # data_module.py:295-297
    win = torch.hann_window(510, periodic=True)
    return torch.istft(spec, n_fft=510, hop_length=128, window=win, center=True, length=length)


def spec_fwd_ref(spec):  # data_module.py:241-254, exponent 0.5, factor 0.15
    return spec.abs() ** 0.5 * torch.exp(1j * spec.angle()) * 0.15


def spec_back_ref(spec):  # data_module.py:256-267
    spec = spec / 0.15
    return spec.abs() ** (1 / 0.5) * torch.exp(1j * spec.angle())


def pad_spec_ref(Y, m=64):  # util/other.py:83-99
    T = Y.size(3)
    n = (m - T % m) if T % m else 0
    return torch.nn.functional.pad(Y, (0, n, 0, 0))


def gen_stft():
    base = "/root/reference/dataset/VBD_SNR-5/valid2"
    noisy = read_wav(f"{base}/noisy/p232_001.wav")
    clean = read_wav(f"{base}/clean/p232_001.wav")
    y = torch.from_numpy(noisy.astype(np.float32) / 32768.0)[None]  # torchaudio.load scaling
    nf = y.abs().max()
    Y = stft_ref(y / nf)
    Yf = spec_fwd_ref(Y)
    back = istft_ref(spec_back_ref(Yf), y.shape[1])
    # istft of a network-sized (T padded to 64) spectrogram, as to_audio does (model.py:612-613)
    Ypad = pad_spec_ref(Yf[:, None])[:, 0]
    Ypad = Ypad + 0.01 * fnormal("golden.stft.pert", tuple(Ypad.shape), complex_=True)
    wav_pad = istft_ref(spec_back_ref(Ypad[0]), y.shape[1])
    save("stft.npz", noisy_i16=noisy, clean_i16=clean, stft=t2n(Y), spec_fwd=t2n(Yf),
         roundtrip=t2n(back), istft_padded=t2n(wav_pad))


def gen_snrnet():
    net = SNRNet().eval()
    load_formula(net, "snrnet.")
    x = fnormal("golden.snrnet.x", (2, 2, 256, 64))
    with torch.no_grad():
        y = net(x)
    save("snrnet.npz", out=t2n(y))


T_30 = (0.001 ** (1 / 7) + (np.arange(1, 31) - 1) / 29 * (1 - 0.001 ** (1 / 7))) ** 7  # model.py:22-23


def gen_sebridge_enhance():
    """ScoreModel.enhance, model_type='sebridge_v3', snr_conditioned='true', oracle SNR
    (model.py:702-839), restated glue around the reference NCSNpp module."""
    net = BackboneRegistry.get_by_name("ncsnpp")().eval()
    load_formula(net)
    base = "/root/reference/dataset/VBD_SNR-5/valid"
    noisy = read_wav(f"{base}/noisy/p232_001.wav")
    with open(f"{base}/active_rms.txt") as f:
        _, clean_rms, noise_rms = f.readline().split("\t")
    clean_rms, noise_rms = float(clean_rms), float(noise_rms)
    fixed_snr, sigma_max = 0.17783, 0.5
    y = torch.from_numpy(noisy.astype(np.float32) / 32768.0)[None]
    T_orig = y.size(1)
    est_snr = torch.FloatTensor([noise_rms / clean_rms])  # model.py:722-724
    norm_factor = y.abs().max().item()
    t_ = (est_snr / (10 ** 0.25 * fixed_snr)).numpy()  # calculate_snr_direct 627-629
    t_ = T_30[np.abs(T_30 - t_).argmin()]
    est_snr_ = torch.FloatTensor([10 ** 0.25 * fixed_snr * t_])
    normfac_ = (2.040166) * (0.240253 + 0.759747 * fixed_snr ** 2) ** 0.5 / ((1 + est_snr_ ** 2) ** 0.5)
    norm_factor = norm_factor * normfac_
    y = y / norm_factor
    Y = pad_spec_ref(torch.unsqueeze(spec_fwd_ref(stft_ref(y)), 0))
    vec_t = torch.ones(1, 1, 1, 1) * float(t_)
    Z = fnormal("golden.enh.Z", tuple(Y.shape), complex_=True) * sigma_max * float(t_)
    X_T = Y + Z
    eps, sd = 0.001, 0.5  # sebridge_v3 preconditioning, model.py:536-541
    c_skip = sd ** 2 / ((vec_t - eps) ** 2 + sd ** 2)
    c_out = (sd * (vec_t - eps)) / ((sd ** 2 + vec_t ** 2) ** 0.5)
    with torch.no_grad():
        sample = c_skip * X_T + c_out * net(torch.cat([X_T, Y], dim=1), vec_t.reshape(1))
        x_hat = istft_ref(spec_back_ref(sample.squeeze()), T_orig) * norm_factor
    save("enhance_sebridge.npz", x_hat=t2n(x_hat).reshape(-1), t_hat=np.float64(t_),
         norm_factor=t2n(norm_factor).reshape(-1), score=t2n(sample))
    save("enhance_inputs.npz", noisy_valid_i16=noisy)


C4_FILES = ["VBD_SNR-5/valid/noisy/p232_001.wav", "VBD_SNR-5/train2/noisy/p286_001.wav",
            "VBD/train/noisy/p226_001.wav"]
C4_LEN = 27861
C4_FC_BIAS_SHIFT = 2.1


def pad_spec_16_ref(Y):  # util/other.py:92-99
    return pad_spec_ref(Y, 16)


def gen_snr_enhance():
    """C4: ScoreModel.enhance, sebridge_v3, snr_conditioned='true', oracle=False -- the SNR comes from
    the reference SNRNet on the raw STFT (model.py:713-721), then t_hat / normfac / noise / one
    preconditioned NCSNpp evaluation / iSTFT as model.py:726-833.  Three dataset utterances cropped to
    one length (so the GPU test can also run them as one batch), each processed at B=1 as the
    reference does; noise draw k is formula noise golden.c4.Z.{k}."""
    net = BackboneRegistry.get_by_name("ncsnpp")().eval()
    load_formula(net)
    snr_net = SNRNet().eval()
    load_formula(snr_net, "snrnet.")
    # formula weights put every clip's estimate at ~0.4 (t_hat snaps to 1.0 for all); shifting the
    # output bias moves the estimates into the middle of the t_30 grid so the clips get distinct t_hat
    with torch.no_grad():
        snr_net.fc.bias -= C4_FC_BIAS_SHIFT
    fixed_snr, sigma_max = 0.17783, 0.5
    out = {"noisy_i16": [], "x_hat": [], "t_hat": [], "est_snr": [], "est_gt": []}
    for k, rel in enumerate(C4_FILES):
        noisy = read_wav(f"/root/reference/dataset/{rel}")[:C4_LEN]
        y = torch.from_numpy(noisy.astype(np.float32) / 32768.0)[None]
        T_orig = y.size(1)
        with torch.no_grad():
            y_chk = y / y.abs().max().item()
            Yc = torch.view_as_real(stft_ref(y_chk)).permute(0, 3, 1, 2)
            Yc = pad_spec_16_ref(Yc)
            est_gt = snr_net(Yc)
            est_snr = est_gt / (1 - est_gt)
        norm_factor = y.abs().max().item()
        t_ = (est_snr / (10 ** 0.25 * fixed_snr)).numpy()
        t_ = T_30[np.abs(T_30 - t_).argmin()]
        est_snr_ = torch.FloatTensor([10 ** 0.25 * fixed_snr * t_])
        normfac_ = (2.040166) * (0.240253 + 0.759747 * fixed_snr ** 2) ** 0.5 / ((1 + est_snr_ ** 2) ** 0.5)
        norm_factor = norm_factor * normfac_
        yn = y / norm_factor
        Y = pad_spec_ref(torch.unsqueeze(spec_fwd_ref(stft_ref(yn)), 0))
        vec_t = torch.ones(1, 1, 1, 1) * float(t_)
        Z = fnormal(f"golden.c4.Z.{k}", tuple(Y.shape), complex_=True) * sigma_max * float(t_)
        X_T = Y + Z
        eps, sd = 0.001, 0.5
        c_skip = sd ** 2 / ((vec_t - eps) ** 2 + sd ** 2)
        c_out = (sd * (vec_t - eps)) / ((sd ** 2 + vec_t ** 2) ** 0.5)
        with torch.no_grad():
            sample = c_skip * X_T + c_out * net(torch.cat([X_T, Y], dim=1), vec_t.reshape(1))
            x_hat = istft_ref(spec_back_ref(sample.squeeze()), T_orig) * norm_factor
        out["noisy_i16"].append(noisy)
        out["x_hat"].append(t2n(x_hat).reshape(-1))
        out["t_hat"].append(float(t_))
        out["est_snr"].append(float(est_snr.reshape(-1)[0]))
        out["est_gt"].append(float(est_gt.reshape(-1)[0]))
    save("enhance_snrnet_c4.npz", **{k: np.asarray(v) for k, v in out.items()})


TRAIN_SHAPE = (2, 256, 64)  # B, F, T of the consistency-step golden (the reference trains on 256-frame crops)
TRAIN_N = [3, 17]          # grid indices n (torch.randint(1, 30) in the reference)
TRAIN_FULL = ["output_layer.weight", "output_layer.bias", "all_modules.1.bias", "all_modules.3.bias",
              "all_modules.4.GroupNorm_0.weight", "all_modules.4.GroupNorm_0.bias", "all_modules.4.Conv_0.bias",
              "all_modules.4.Dense_0.bias", "all_modules.7.Conv_0.weight", "all_modules.21.NIN_0.b",
              "all_modules.21.GroupNorm_0.weight", "all_modules.33.NIN_3.b", "all_modules.75.weight",
              "all_modules.76.weight", "all_modules.76.bias", "all_modules.74.Conv_2.bias"]
TRAIN_HEAD = 96            # leading elements kept of every other gradient tensor
TRAIN_FIXED_SNR = 0.17783  # fixed_snr of the 'fixed' branch (the C4 configuration's value)


def gen_train_step():
    """the consistency-training loss of ScoreModel._step, sebridge_v3 with
    snr_conditioned='true' (model.py:361-390) and 'fixed' (model.py:293-326; keys prefixed fixed_), both
    with the preconditioned forward of model.py:521-541, restated around the
    REFERENCE NCSNpp module (formula weights) and differentiated by torch autograd on the CPU.  Both loss
    types; the loss, every gradient's (sum, sum of squares, max |g|), the full gradient of a few tensors and
    the first TRAIN_HEAD elements of every other one are stored."""
    net = BackboneRegistry.get_by_name("ncsnpp")().train()
    load_formula(net)
    B, Fq, T = TRAIN_SHAPE
    x = fnormal("golden.train.x", (B, 1, Fq, T), complex_=True) * 0.4
    y = fnormal("golden.train.y", (B, 1, Fq, T), complex_=True) * 0.4 + x
    z = fnormal("golden.train.z", (B, 1, Fq, T), complex_=True)
    sigma_max, N, roh, eps, Tt = 0.5, 30, 7, 0.001, 1
    n = torch.tensor(TRAIN_N).reshape(B, 1, 1, 1)
    t_n = (eps ** (1 / roh) + ((n - 1) / (N - 1)) * (Tt ** (1 / roh) - eps ** (1 / roh))) ** roh
    t_n1 = (eps ** (1 / roh) + ((n) / (N - 1)) * (Tt ** (1 / roh) - eps ** (1 / roh))) ** roh
    zz = z * sigma_max
    # snr_conditioned 'true' (model.py:372-376): mu_t = H(H^-1(x)(1 - t) + H^-1(y) t)
    mus_true = [spec_fwd_ref(spec_back_ref(x) * (1 - tt) + spec_back_ref(y) * tt) for tt in (t_n, t_n1)]
    # snr_conditioned 'fixed' (model.py:304-312): mu_t = H(x_ori + (H^-1(y) - x_ori) fixed_snr t)
    x_ori = spec_back_ref(x)
    y0_snr = (spec_back_ref(y) - x_ori) * TRAIN_FIXED_SNR
    mus_fixed = [spec_fwd_ref(x_ori + y0_snr * tt) for tt in (t_n, t_n1)]

    def forward(xx, t, yy):  # ScoreModel.forward, snr_conditioned 'true', sebridge_v3 (model.py:536-541)
        e_, sd = 0.001, 0.5
        c_skip = sd ** 2 / ((t - e_) ** 2 + sd ** 2)
        c_out = (sd * (t - e_)) / ((sd ** 2 + t ** 2) ** 0.5)
        return c_skip * xx + c_out * net(torch.cat([xx, yy], dim=1), t.squeeze(3).squeeze(2).squeeze(1))

    out = {"n": np.asarray(TRAIN_N), "t_n": t2n(t_n).reshape(-1), "t_n1": t2n(t_n1).reshape(-1),
           "fixed_snr": np.float64(TRAIN_FIXED_SNR),
           "full_keys": np.asarray(TRAIN_FULL), "head": np.int64(TRAIN_HEAD)}
    names = [k for k, p in net.named_parameters() if p.requires_grad]
    out["names"] = np.asarray(names)
    for branch, lt in (("true", "mse"), ("true", "sqrt_mse"), ("fixed", "mse"), ("fixed", "sqrt_mse")):
        mu_t_n, mu_t_n1 = mus_true if branch == "true" else mus_fixed
        x_t_n = mu_t_n + t_n * zz
        x_t_n1 = mu_t_n1 + t_n1 * zz
        lt_key = lt if branch == "true" else f"fixed_{lt}"
        net.zero_grad()
        f_theta = forward(x_t_n1, t_n1, mu_t_n1)
        f_theta_minus = forward(x_t_n, t_n, mu_t_n)
        if lt == "mse":
            err = f_theta - f_theta_minus
        else:
            sq = lambda f: f.abs() ** 0.5 * torch.exp(1j * f.angle())  # noqa: E731
            err = sq(f_theta) - sq(f_theta_minus)
        losses = torch.square(err.abs())
        loss = torch.mean(0.5 * torch.sum(losses.reshape(losses.shape[0], -1), dim=-1))
        loss.backward()
        params = dict(net.named_parameters())
        g = {k: params[k].grad.detach().double() for k in names}
        out[f"{lt_key}_loss"] = np.float64(loss.item())
        out[f"{lt_key}_gsum"] = np.asarray([float(g[k].sum()) for k in names])
        out[f"{lt_key}_gsq"] = np.asarray([float((g[k] ** 2).sum()) for k in names])
        out[f"{lt_key}_gmax"] = np.asarray([float(g[k].abs().max()) for k in names])
        for k in TRAIN_FULL:
            out[f"{lt_key}_full__{k}"] = t2n(g[k].float())
        out[f"{lt_key}_head"] = np.concatenate([t2n(g[k].float()).reshape(-1)[:TRAIN_HEAD] for k in names])
    save("train_step.npz", **out)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["keys", "fir", "blocks", "attn", "ncsnpp", "sde", "pc_ouve",
                             "pc_variants", "stft", "snrnet", "sebridge", "c4", "train"]
    table = {"keys": gen_keys, "fir": gen_fir, "blocks": gen_blocks, "attn": gen_attn,
             "ncsnpp": gen_ncsnpp, "sde": gen_sde, "pc_ouve": gen_pc_ouve,
             "pc_variants": gen_pc_variants, "stft": gen_stft, "snrnet": gen_snrnet,
             "sebridge": gen_sebridge_enhance, "c4": gen_snr_enhance, "train": gen_train_step}
    for w in which:
        torch.manual_seed(0)
        table[w]()

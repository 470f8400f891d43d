"""Pin the CPU oracle against golden vectors produced by the reference's own modules
(tools/gen_golden.py).  CPU only."""
import math

import numpy as np
import pytest
import torch

from conftest import (fnormal, formula_attn_sd, formula_block_sd, formula_sd, golden,
                      state_dict_keys)
from oracle import ncsnpp_ref, sde_ref, snrnet_ref, spec_ref

torch.set_num_threads(min(8, torch.get_num_threads()))


def T(a, dt=torch.float32):
    return torch.as_tensor(a).to(dt)


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.sqrt(np.mean(np.abs(a - b) ** 2)) / (np.sqrt(np.mean(np.abs(b) ** 2)) + 1e-30))


def test_fir():
    g = golden("fir.npz")
    x = T(fnormal("golden.fir.x", (2, 8, 16, 32)))
    np.testing.assert_allclose(ncsnpp_ref.fir_up2(x).numpy(), g["up"], atol=2e-6)
    np.testing.assert_allclose(ncsnpp_ref.fir_down2(x).numpy(), g["down"], atol=2e-6)


BLOCKS = {
    "plain": (128, 128, False, False, (8, 16)),
    "cin_ne_cout": (128, 256, False, False, (8, 8)),
    "down": (128, 128, False, True, (8, 16)),
    "up": (256, 256, True, False, (4, 8)),
    "cat384": (384, 256, False, False, (4, 8)),
}


@pytest.mark.parametrize("name", list(BLOCKS))
def test_resblock(name):
    cin, cout, up, down, hw = BLOCKS[name]
    g = golden("resblocks.npz")
    sd = {("b." + k): T(v) for k, v in formula_block_sd(f"rb_{name}.", cin, cout, up, down).items()}
    x = T(fnormal(f"golden.rb_{name}.x", (2, cin) + hw))
    temb = T(fnormal(f"golden.rb_{name}.temb", (2, 512)))
    y = ncsnpp_ref.resblock(x, temb, sd, "b", up=up, down=down)
    assert rel(y.numpy(), g[f"{name}_out"]) < 1e-5


def test_attn():
    g = golden("attn.npz")
    sd = {("a." + k): T(v) for k, v in formula_attn_sd("attn.").items()}
    x = T(fnormal("golden.attn.x", (2, 256, 16, 8)))
    y = ncsnpp_ref.attn_block(x, sd, "a")
    assert rel(y.numpy(), g["out"]) < 1e-5


def test_state_dict_layout():
    keys = state_dict_keys()
    assert len(keys["ncsnpp"]) == 647
    assert keys["ncsnpp_frozen"] == ["all_modules.0.W"]
    assert len(keys["ncsnpp_trainable_order"]) == 646


@pytest.fixture(scope="module")
def ncsnpp_sd():
    return ncsnpp_ref.state_dict_to_torch(formula_sd("ncsnpp"))


def test_ncsnpp_full(ncsnpp_sd):
    g = golden("ncsnpp_full.npz")
    x = torch.from_numpy(fnormal("golden.ncsnpp.x", (2, 2, 256, 64), complex_=True)) * 0.5
    t = torch.tensor([0.5, 0.8])
    np.testing.assert_allclose(ncsnpp_ref.temb_mlp(t, ncsnpp_sd).numpy(), g["temb"], rtol=1e-5, atol=1e-5)
    y = ncsnpp_ref.ncsnpp_forward(x, t, ncsnpp_sd)
    assert rel(y.numpy(), g["out"]) < 1e-5


def test_sde_tables():
    g = golden("sde.npz")
    ts = g["t"].astype(np.float64)
    x = fnormal("golden.sde.x", (5, 1, 4, 4), complex_=True)
    y = fnormal("golden.sde.y", (5, 1, 4, 4), complex_=True)
    sdes = {"ouve": sde_ref.OUVE(1.5, 0.05, 0.5), "ouve_smax1": sde_ref.OUVE(1.5, 0.05, 1.0),
            "bbed": sde_ref.BBED(0.999, 2.6, 0.52), "proposed_1": sde_ref.PROPOSED_1(0.99, 1.0, 2.6, 0.52),
            "proposed_1b": sde_ref.PROPOSED_1(0.99, 0.5, 3.0, 0.53)}
    for nm, s in sdes.items():
        np.testing.assert_allclose(s.std(ts), g[f"{nm}_std"], rtol=2e-6)
        np.testing.assert_allclose([s.g(t) for t in ts], g[f"{nm}_g"], rtol=2e-6)
        d = s.drift(x, ts[:, None, None, None], y)
        np.testing.assert_allclose(d, g[f"{nm}_drift"], rtol=2e-5, atol=1e-5)
        m = s.mean(x, ts[:, None, None, None], y)
        np.testing.assert_allclose(m, g[f"{nm}_mean"], rtol=2e-5, atol=1e-6)
    # known answers recorded in SURVEY.md §8(a) a17
    bb = sdes["bbed"]
    np.testing.assert_allclose(bb.std(np.array([0.03, 0.5, 0.999])), [0.124815, 0.491685, 0.058908], atol=2e-6)
    assert math.isnan(float(bb.std(1.0)))
    np.testing.assert_allclose(sdes["ouve"].std(1.0), 0.388983, atol=2e-6)
    np.testing.assert_allclose(sdes["ouve_smax1"].std(1.0), 0.816252, atol=2e-6)
    # PROPOSED_1 with sigma_min = 1, sigma_max = k is BBED's marginal std (sdes.py:312-329)
    np.testing.assert_allclose(sdes["proposed_1"].std(ts), bb.std(ts), rtol=1e-12)


class Tape:
    def __init__(self, tag, dtype=torch.complex64):
        self.tag, self.i, self.dtype = tag, 0, dtype

    def __call__(self, shape):
        z = torch.from_numpy(fnormal(f"{self.tag}.{self.i}", tuple(shape), complex_=True)).to(self.dtype)
        self.i += 1
        return z


def test_pc_variants():
    g = golden("pc_variants.npz")
    Y = torch.from_numpy(fnormal("golden.pcv.Y", (2, 1, 16, 8), complex_=True))

    def score_fn(x, t, y):
        return -(x - y) * 0.7 + 0.1 * y

    for key in [k for k in g.files if "__" in k and not k.endswith(("__ns", "__draws"))]:
        sde_name, pred, corr = key.split("__")
        sde = {"ouve": lambda: sde_ref.OUVE(1.5, 0.05, 0.5, N=6), "bbed": lambda: sde_ref.BBED(0.999, 2.6, 0.52, N=6),
               "proposed_1": lambda: sde_ref.PROPOSED_1(0.99, 1.0, 2.6, 0.52, N=6)}[sde_name]()
        # the reference promotes BBED / PROPOSED_1 runs to complex128 (sdes.py:292,303, 376,388)
        Yc = Y if sde_name == "ouve" else Y[:1].to(torch.complex128)
        tape = Tape(f"golden.pcv.{sde_name}.{pred}.{corr}", Yc.dtype)
        xr, ns = sde_ref.pc_sample(sde, score_fn, Yc, tape, predictor=pred, corrector=corr)
        assert ns == int(g[key + "__ns"]), key
        assert tape.i == int(g[key + "__draws"]), key
        # BBED: the reference rounds its per-step scalars (1-t, k**t, sqrt(dt)) to float32 while
        # the tensors run in complex128; the oracle keeps the scalars in float64.
        tol = 2e-6 if sde_name == "ouve" else 2e-5
        assert rel(xr.numpy(), g[key]) < tol, key


def test_pc_ouve_network(ncsnpp_sd):
    g = golden("pc_ouve.npz")
    Y = torch.from_numpy(fnormal("golden.pc.Y", (2, 1, 256, 64), complex_=True)) * 0.5
    sde = sde_ref.OUVE(1.5, 0.05, 0.5, N=5)

    def score_fn(x, t, y):
        tt = torch.full((x.shape[0],), t, dtype=torch.float32)
        return -ncsnpp_ref.ncsnpp_forward(torch.cat([x, y], 1), tt, ncsnpp_sd)

    tape = Tape("golden.pc.noise")
    xr, ns = sde_ref.pc_sample(sde, score_fn, Y, tape)
    assert ns == int(g["ns"]) == 10 and tape.i == int(g["draws"]) == 11
    assert rel(xr.numpy(), g["out"]) < 1e-4


def test_stft_istft():
    g = golden("stft.npz")
    y = g["noisy_i16"].astype(np.float32) / 32768.0
    y = y / np.abs(y).max()
    S = spec_ref.stft(y[None].astype(np.float32))
    assert rel(S, g["stft"]) < 1e-6
    Sf = spec_ref.spec_fwd(S)
    assert rel(Sf, g["spec_fwd"]) < 2e-5  # fp32 STFT error of small bins, amplified by |.|**0.5
    rt = spec_ref.istft(spec_ref.spec_back(Sf[0]), y.shape[0])
    np.testing.assert_allclose(rt[0], g["roundtrip"][0], atol=2e-6)
    Yp = spec_ref.pad_spec(g["spec_fwd"][:, None])[:, 0]
    Yp = Yp + 0.01 * fnormal("golden.stft.pert", Yp.shape, complex_=True)
    w = spec_ref.istft(spec_ref.spec_back(Yp[0]), y.shape[0])
    np.testing.assert_allclose(w[0], g["istft_padded"], atol=5e-6)


def test_snrnet():
    g = golden("snrnet.npz")
    sd = {k: torch.from_numpy(v) for k, v in formula_sd("snrnet", "snrnet.").items()}
    x = torch.from_numpy(fnormal("golden.snrnet.x", (2, 2, 256, 64)))
    y = snrnet_ref.snrnet_forward(x, sd)
    np.testing.assert_allclose(y.numpy(), g["out"], rtol=1e-5, atol=1e-6)


def test_snap_and_normfac():
    g = golden("enhance_sebridge.npz")
    clean_rms, noise_rms = 0.09034279194278529, 0.01521404836098084  # active_rms.txt row 1
    t = snrnet_ref.snap_t(noise_rms / clean_rms, 0.17783)
    assert abs(t - float(g["t_hat"])) < 1e-12


@pytest.mark.parametrize("branch,loss_type", [("true", "mse"), ("fixed", "sqrt_mse")])
def test_train_step(branch, loss_type):
    """oracle/train_ref.py (the consistency-training loss + autograd on the NCSN++ restatement) vs the
    reference module's own autograd (tests/golden/train_step.npz): loss, per-tensor gradient sums of
    squares and the recorded gradient heads.  The attention key biases (NIN_1.b) get an analytically zero
    gradient (softmax is invariant to a per-query constant): compared by norm, as in test_gpu_train."""
    from oracle import train_ref
    g = golden("train_step.npz")
    sd = ncsnpp_ref.state_dict_to_torch(formula_sd("ncsnpp"))
    B, Fq, Tn = 2, 256, 64
    x = torch.from_numpy(fnormal("golden.train.x", (B, 1, Fq, Tn), complex_=True)) * 0.4
    y = torch.from_numpy(fnormal("golden.train.y", (B, 1, Fq, Tn), complex_=True)) * 0.4 + x
    z = torch.from_numpy(fnormal("golden.train.z", (B, 1, Fq, Tn), complex_=True))
    key = loss_type if branch == "true" else f"fixed_{loss_type}"
    loss, grads = train_ref.loss_and_grads(sd, x, y, z, g["n"], branch, loss_type, float(g["fixed_snr"]))
    assert abs(float(loss) / float(g[f"{key}_loss"]) - 1) < 3e-5
    names = [str(k) for k in g["names"]]
    head = int(g["head"])
    got_sq = np.array([float((grads[k].double() ** 2).sum()) for k in names])
    rel_sq = np.abs(got_sq - g[f"{key}_gsq"]) / np.maximum(g[f"{key}_gsq"], 1e-30)
    for i, k in enumerate(names):
        if k.endswith("NIN_1.b"):
            sib = names.index(k.replace("NIN_1.b", "NIN_0.b"))
            assert math.sqrt(got_sq[i] / g[f"{key}_gsq"][sib]) < 1e-5, k
            rel_sq[i] = 0.0
    assert rel_sq.max() < 2e-3, names[int(np.argmax(rel_sq))]
    got_head = np.concatenate([grads[k].double().reshape(-1)[:head].numpy() for k in names])
    assert rel(got_head, g[f"{key}_head"].astype(np.float64)) < 1e-3

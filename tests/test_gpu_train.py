"""GPU parity of the consistency-training step against the reference.

tests/golden/train_step.npz holds the loss of ScoreModel._step (sebridge_v3, snr_conditioned='true',
model.py:361-390, and 'fixed', model.py:293-326) and the parameter gradients of loss.backward(), computed by tools/gen_golden.py
with the REFERENCE NCSNpp module and torch autograd on the CPU (formula weights, B=2 x 256 x 64,
n = (3, 17), formula noise).  Here the same batch runs through sgmse.model.ScoreModel._step on the
HIP kernels (forward, backward and loss all HIP, snrse/train.py).

Tolerances (fp32 on both sides, different summation orders): loss 3e-5 relative (a mean over
2 x 256 x 64 complex bins whose value is ~2.5e4, summed in a different order); gradients 1e-3
relative RMS over every tensor's stored elements and per-tensor sums of squares to 2e-3 (GroupNorm
backward and the 3x3 wgrad reduce over up to 2 x 256 x 64 pixels in a different order than the
CPU reference).  The attention KEY biases (NIN_1.b) are the exception: softmax over keys is
invariant to adding q.b to every logit of a query, so their exact gradient is zero and both sides
hold only rounding noise (~1e-7 of the query-bias gradient in the golden); for them the test checks
that the HIP gradient is that small too, relative to the sibling query-bias (NIN_0.b) gradient.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, fnormal, formula_sd, golden

pytestmark = pytest.mark.gpu

REPORT_DIR = os.environ.get("SNRSE_REPORT_DIR", os.path.join(ROOT, "gpurun_out"))


def _model(loss_type, snr_conditioned="true"):
    from sgmse.model import ScoreModel
    hp = dict(backbone="ncsnpp", sde="ouve", model_type="sebridge_v3", snr_conditioned=snr_conditioned, theta=1.5,
              sigma_min=0.05, sigma_max=0.5, N=30, compute_dtype="fp32", fixed_snr=0.17783, loss_type=loss_type)
    m = ScoreModel(**hp)
    m.dnn.load_state_dict({k: torch.from_numpy(v) for k, v in formula_sd("ncsnpp").items()})
    return m.cuda().train()


def _batch(gpu):
    g = golden("train_step.npz")
    B, Fq, T = 2, 256, 64
    x = torch.from_numpy(fnormal("golden.train.x", (B, 1, Fq, T), complex_=True)) * 0.4
    y = torch.from_numpy(fnormal("golden.train.y", (B, 1, Fq, T), complex_=True)) * 0.4 + x
    z = torch.from_numpy(fnormal("golden.train.z", (B, 1, Fq, T), complex_=True))
    return g, x.to(gpu), y.to(gpu), z.to(gpu)


@pytest.mark.parametrize("snr_conditioned,loss_type,gemm", [("true", "mse", "exact"), ("true", "sqrt_mse", "exact"),
                                                             ("fixed", "mse", "exact"), ("fixed", "sqrt_mse", "exact"),
                                                             ("true", "mse", "x3"), ("fixed", "mse", "x3")])
def test_consistency_step_loss_and_grads_vs_reference(gpu, loss_type, snr_conditioned, gemm):
    """'true': model.py:361-390; 'fixed': model.py:293-326 (mu_t = H(x_ori + (H^-1(y) - x_ori) fixed_snr t),
    golden keys prefixed fixed_, fixed_snr 0.17783).  gemm 'x3': the forward / input-gradient convs as
    split-bf16 GEMMs (snrse.train.set_gemm, bench.py --config train --dtype fp32x3), held to the exact mode's
    tolerances (measured: loss 1e-5, gradient heads 5e-5, sums of squares 2e-4 -- as the exact mode's)."""
    from snrse import train as strain
    g, x, y, z = _batch(gpu)
    m = _model(loss_type, snr_conditioned)
    if snr_conditioned == "fixed":
        assert abs(float(g["fixed_snr"]) - m.fixed_snr) < 1e-12
    key = loss_type if snr_conditioned == "true" else f"fixed_{loss_type}"
    strain.set_gemm(gemm)
    try:
        loss = m._step((x, y), 0, n=g["n"], noise=z)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        strain.set_gemm("exact")
    f = 1.0
    ref_loss = float(g[f"{key}_loss"])
    err_loss = abs(float(loss) - ref_loss) / abs(ref_loss)
    params = dict(m.dnn.named_parameters())
    names = [str(k) for k in g["names"]]
    head = int(g["head"])
    got_head, got_sq, worst = [], [], []
    for k in names:
        gr = params[k].grad
        assert gr is not None, k
        gd = gr.detach().double().cpu()
        got_head.append(gd.reshape(-1)[:head].numpy())
        got_sq.append(float((gd ** 2).sum()))
    got_head = np.concatenate(got_head)
    ref_head = g[f"{key}_head"].astype(np.float64)
    rel_head = float(np.sqrt(np.mean((got_head - ref_head) ** 2)) / np.sqrt(np.mean(ref_head ** 2)))
    ref_sq = g[f"{key}_gsq"]
    rel_sq = np.abs(np.asarray(got_sq) - ref_sq) / np.maximum(ref_sq, 1e-30)
    key_bias = {}
    for i, k in enumerate(names):
        if k.endswith("NIN_1.b"):
            sib = names.index(k.replace("NIN_1.b", "NIN_0.b"))
            key_bias[k] = math.sqrt(got_sq[i] / ref_sq[sib])
            rel_sq[i] = 0.0
    full = {}
    for k in [str(s) for s in g["full_keys"]]:
        r = g[f"{key}_full__{k}"].astype(np.float64)
        a = params[k.replace("dnn.", "")].grad.detach().double().cpu().numpy()
        full[k] = float(np.sqrt(np.mean((a - r) ** 2)) / (np.sqrt(np.mean(r ** 2)) + 1e-30))
    order = np.argsort(-rel_sq)[:5]
    worst = [(names[i], float(rel_sq[i])) for i in order]
    os.makedirs(REPORT_DIR, exist_ok=True)
    with open(os.path.join(REPORT_DIR, f"train_step_{key}_{gemm}_vs_reference.json"), "w") as fh:
        json.dump({"gemm": gemm, "loss": float(loss), "ref_loss": ref_loss, "rel_err_loss": err_loss,
                   "rel_rms_grad_heads": rel_head, "max_rel_err_grad_sumsq": float(rel_sq.max()),
                   "worst_sumsq": worst, "rel_rms_full_tensors": full,
                   "key_bias_grad_norm_over_query_bias": key_bias}, fh, indent=1)
    assert err_loss < 3e-5 * f, err_loss
    assert len(key_bias) == 4 and max(key_bias.values()) < 1e-5 * f, key_bias
    assert rel_head < 1e-3 * f, (rel_head, worst)
    assert rel_sq.max() < 2e-3 * f, worst
    assert max(full.values()) < 1e-3 * f, full


def test_fused_adam_and_ema_match_torch(gpu):
    """FusedAdam (one HIP launch) vs torch.optim.Adam on the same tensors for 3 steps, and the EMA
    shadows vs torch_ema 0.3's update rule restated (model.py:103-106)."""
    from sgmse.ema import EMAState
    from snrse.train import FusedAdam
    gen = torch.Generator(device=gpu).manual_seed(3)
    mod = torch.nn.Module()
    shapes = [(128, 128, 3, 3), (128,), (7,), (4097,)]
    mod.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(s, device=gpu, generator=gen)) for s in shapes])
    ref = [p.detach().clone().requires_grad_(True) for p in mod.ps]
    ema = EMAState(mod, 0.999)
    opt = FusedAdam(mod.parameters(), lr=1e-3, ema=ema)
    topt = torch.optim.Adam(ref, lr=1e-3)
    shadow = [p.detach().clone() for p in ref]
    for it in range(3):
        grads = [torch.randn(s, device=gpu, generator=gen) for s in shapes]
        for p, q, gr in zip(mod.ps, ref, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        opt.step()
        topt.step()
        decay = min(0.999, (1 + it + 1) / (10 + it + 1))
        with torch.no_grad():
            for s, q in zip(shadow, ref):
                s.sub_((1.0 - decay) * (s - q))
    torch.cuda.synchronize()
    for p, q in zip(mod.ps, ref):
        assert torch.allclose(p, q, rtol=1e-6, atol=1e-6)
    for s, r in zip(ema.shadow_params, shadow):
        assert torch.allclose(s, r, rtol=1e-6, atol=1e-6)
    assert ema.num_updates == 3


def test_fused_adam_missing_and_noncontiguous_grads_match_torch(gpu):
    """Per-tensor step counts (a parameter without a gradient on step 2 falls one step behind, as in
    torch.optim.Adam), EMA shadows of parameters without a gradient still move (torch_ema 0.3 updates
    every requires_grad shadow), and a non-contiguous gradient is read correctly (its contiguous copy
    stays alive until the asynchronous launch has run)."""
    from sgmse.ema import EMAState
    from snrse.train import FusedAdam
    gen = torch.Generator(device=gpu).manual_seed(4)
    mod = torch.nn.Module()
    shapes = [(64, 32), (33,), (4097,)]
    mod.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(s, device=gpu, generator=gen)) for s in shapes])
    ref = [p.detach().clone().requires_grad_(True) for p in mod.ps]
    ema = EMAState(mod, 0.999)
    opt = FusedAdam(mod.parameters(), lr=1e-3, ema=ema)
    topt = torch.optim.Adam(ref, lr=1e-3)
    shadow = [p.detach().clone() for p in ref]
    for it in range(4):
        grads = [torch.randn(s, device=gpu, generator=gen) for s in shapes]
        for k, (p, q, gr) in enumerate(zip(mod.ps, ref, grads)):
            if it == 1 and k == 1:  # no gradient for parameter 1 on step 2
                p.grad, q.grad = None, None
                continue
            if k == 0:  # a non-contiguous (transposed-view) gradient
                p.grad = gr.t().contiguous().t()
                assert not p.grad.is_contiguous()
            else:
                p.grad = gr.clone()
            q.grad = gr.clone()
        opt.step()
        topt.step()
        decay = min(0.999, (1 + it + 1) / (10 + it + 1))
        with torch.no_grad():
            for s, q in zip(shadow, ref):
                s.sub_((1.0 - decay) * (s - q))
    torch.cuda.synchronize()
    for p, q in zip(mod.ps, ref):
        assert torch.allclose(p, q, rtol=1e-6, atol=1e-6), (p - q).abs().max()
    for s, r in zip(ema.shadow_params, shadow):
        assert torch.allclose(s, r, rtol=1e-6, atol=1e-6), (s - r).abs().max()


def test_training_loop_runs_and_updates(gpu):
    """Three steps of the reference loop shape (training_step -> backward -> optimizer_step) on the HIP
    path: finite losses, every trainable parameter receives a gradient and moves, the frozen Fourier
    features do not, the EMA shadows follow."""
    g, x, y, _ = _batch(gpu)
    m = _model("mse")
    opt = m.configure_optimizers()
    w0 = m.dnn.all_modules[4].Conv_0.weight.detach().clone()
    gfp0 = m.dnn.all_modules[0].W.detach().clone()
    losses = []
    for it in range(3):
        opt.zero_grad()
        loss = m.training_step((x, y), it)
        loss.backward()
        assert all(p.grad is not None for p in m.dnn.parameters() if p.requires_grad)
        m.optimizer_step(opt)
        losses.append(float(loss))
    torch.cuda.synchronize()
    assert all(math.isfinite(v) for v in losses)
    assert not torch.equal(w0, m.dnn.all_modules[4].Conv_0.weight)
    assert torch.equal(gfp0, m.dnn.all_modules[0].W)
    assert m.ema.num_updates == 3 and len(m.ema.shadow_params) == 646


@pytest.mark.parametrize("chunked", [False, True])
def test_training_attention_vs_torch(gpu, chunked):
    """snrse.train._Attention (HIP bgemm + softmax kernels, probabilities recomputed in the backward,
    batch chunks bounded by ATTN_CHUNK_BYTES) vs torch autograd of softmax(q k^T / sqrt(C)) v in fp64."""
    from snrse import train as tr
    gen = torch.Generator(device=gpu).manual_seed(11)
    B, L, C = 3, 192, 64
    q, k, v = (torch.randn(B, L, C, device=gpu, generator=gen) for _ in range(3))
    do = torch.randn(B, L, C, device=gpu, generator=gen)
    old = tr.ATTN_CHUNK_BYTES
    if chunked:
        tr.ATTN_CHUNK_BYTES = L * L * 4  # one utterance per chunk
    try:
        qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
        o = tr._Attention.apply(qa, ka, va)
        o.backward(do)
    finally:
        tr.ATTN_CHUNK_BYTES = old
    assert len(tr._attn_chunks(B, L)) == 1 and (not chunked or L * L * 4 < old)
    qr, kr, vr = (t.double().clone().requires_grad_(True) for t in (q, k, v))
    orf = torch.softmax(qr @ kr.transpose(1, 2) / math.sqrt(C), -1) @ vr
    orf.backward(do.double())
    for got, ref in ((o, orf), (qa.grad, qr.grad), (ka.grad, kr.grad), (va.grad, vr.grad)):
        err = (got.double() - ref).norm() / ref.norm()
        assert err < 1e-5, float(err)


@pytest.mark.parametrize("case", [
    # B, C0, C1, Cout, H, W, ksize
    (2, 128, 0, 128, 16, 64, 3),
    (1, 128, 128, 256, 8, 40, 3),   # concatenated input, W not a multiple of the 32-px segment
    (2, 32, 0, 128, 9, 33, 3),      # the padded input conv (Cin 4 -> 32)
    (2, 128, 0, 4, 8, 64, 3),       # a pyramid head (Cout 4)
    (2, 256, 0, 256, 8, 16, 1),     # 1x1
])
def test_conv_wgrad_x3_vs_exact(gpu, case):
    """snrse_conv_wgrad_x3 (split-bf16 products, transposed LDS reads) vs snrse_conv_wgrad (exact f32 MFMA)
    and a float64 torch reference of the same weight gradient."""
    import torch.nn.functional as F
    from snrse import train as tr
    B, C0, C1, Co, H, W, k = case
    g = torch.Generator(device=gpu).manual_seed(sum(case))
    x0 = torch.randn(B, H, W, C0, device=gpu, generator=g)
    x1 = torch.randn(B, H, W, C1, device=gpu, generator=g) if C1 else None
    dy = torch.randn(B, H, W, Co, device=gpu, generator=g)
    Cin = C0 + C1
    outs = {}
    for name in ("snrse_conv_wgrad", "snrse_conv_wgrad_x3"):
        dw = torch.zeros(Co, k * k, Cin, device=gpu)
        tr._call(name, dy.data_ptr(), Co, x0.data_ptr(), C0, tr._p(x1), C1, B, H, W, k, dw.data_ptr())
        torch.cuda.synchronize()
        outs[name] = dw.reshape(Co, k, k, Cin).permute(0, 3, 1, 2).double().cpu()
    x = x0 if x1 is None else torch.cat([x0, x1], -1)
    xd = x.permute(0, 3, 1, 2).double().cpu()
    dyd = dy.permute(0, 3, 1, 2).double().cpu()
    ref = torch.nn.grad.conv2d_weight(xd, (Co, Cin, k, k), dyd, padding=k // 2)
    def rel(a, b):
        return float((a - b).pow(2).mean().sqrt() / b.pow(2).mean().sqrt())
    assert rel(outs["snrse_conv_wgrad"], ref) < 1e-5
    assert rel(outs["snrse_conv_wgrad_x3"], ref) < 3e-5

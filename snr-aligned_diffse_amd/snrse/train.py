"""Consistency-training step of the SNR-aligned sebridge_v3 model on the HIP kernels
(reference ScoreModel._step, sgmse/model.py:293-326 / 361-390, with the
backward pass PyTorch Lightning runs through loss.backward() and its optimizer / EMA hooks,
model.py:99-106).

Every layer of the NCSN++ network (reference sgmse/backbones/ncsnpp.py:247-404) is a
torch.autograd.Function whose forward AND backward run as HIP kernels through the C-ABI
(csrc/conv.hip, norm.hip, train.hip): conv (dgrad = the forward implicit-GEMM conv with the
transposed, flipped kernel; wgrad = snrse_conv_wgrad), GroupNorm(+SiLU) (snrse_gn_backward),
FIR up/down (the adjoint is the other FIR with the gain swapped), NIN / Linear (snrse_bgemm),
attention (materialised softmax, snrse_bgemm + snrse_softmax_*), the temb MLP, the 1/t scaling
of the output head, and the consistency loss itself (snrse_ct_loss).  torch autograd only
orders the calls and accumulates gradients, so `loss.backward()` works as in the reference and
gradients land in the nn.Parameters of sgmse.backbones.NCSNpp in the reference layout.
FusedAdam is torch.optim.Adam (+ the torch_ema 0.3 update) as one HIP launch over all tensors.

fp32 throughout (the reference trains in fp32).  Parity: tests/test_gpu_train.py against
gradients of the reference module computed by tools/gen_golden.py (tests/golden/train_step.npz).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from . import _lib, ops

INV_SQRT2 = 1.0 / math.sqrt(2.0)


def _s():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _call(name, *args):
    _lib.call(name, *args, _s())


def _pad_last(x, C):
    """Zero-pad the channel (last) dim of a contiguous tensor to C (the f32 GEMM's 32-channel K tiles)."""
    if x.shape[-1] == C:
        return x
    out = x.new_zeros(*x.shape[:-1], C)
    out[..., :x.shape[-1]] = x
    return out


def _ceil(n, m):
    return (n + m - 1) // m * m


# ----------------------------------------------------------------------------- primitives
def chan_sum(x, per_b=False, scale=1.0):
    """NHWC [B, ..., C] -> [C] (or [B, C] with per_b) sums over the pixels."""
    B, C = x.shape[0], x.shape[-1]
    HW = x.numel() // (B * C)
    out = torch.zeros((B, C) if per_b else (C,), device=x.device, dtype=torch.float32)
    _call("snrse_chan_sum", x.data_ptr(), B, HW, C, out.data_ptr() if per_b else None,
          None if per_b else out.data_ptr(), float(scale))
    return out


def axpby(x, y, a, b):
    """y <- a x + b y (in place on y); returns y."""
    _call("snrse_axpby", x.data_ptr(), y.data_ptr(), x.numel(), float(a), float(b))
    return y


def scaled(x, a):
    y = torch.empty_like(x)
    return axpby(x, y, a, 0.0)


def bgemm(A, sA, Bm, sB, M, N, K, batch=1, C=None, sC=None, bias=None, alpha=1.0, beta=0.0):
    """C(m, n) = alpha sum_k A(m, k) B(k, n) + beta C (+ bias[n]); s* = (batch, row, col) strides."""
    if C is None:
        C = torch.empty(batch, M, N, device=A.device, dtype=torch.float32)
        sC = (M * N, N, 1)
    _call("snrse_bgemm", A.data_ptr(), *sA, Bm.data_ptr(), *sB, C.data_ptr(), *sC, _p(bias), batch, M, N, K,
          float(alpha), float(beta))
    return C


# ----------------------------------------------------------------------------- conv
def _pack(w, cin_pad, rows):
    """[Cout, Cin, k, k] -> [rows][k][k][cin_pad] (the conv kernels' K-contiguous layout)."""
    co, ci, k, _ = w.shape
    p = w.detach().permute(0, 2, 3, 1)
    if cin_pad != ci:
        p = _pad_last(p.contiguous(), cin_pad)
    p = p.reshape(co, k * k * cin_pad)
    if rows != co:
        p = torch.cat([p, p.new_zeros(rows - co, p.shape[1])], 0)
    return p.contiguous()


# GEMM arithmetic of the training convs: "exact" fp32 MFMA, or "x3" -- the split-bf16 fp32 GEMMs of the
# fp32x3 mode (~2^-16 relative per product): the forward and input-gradient convs whose weight matrix has
# >= 128 rows (ops.split_weight; the Cout <= 16 pyramid heads and their likes stay exact) and every weight
# gradient (snrse_conv_wgrad_x3).
_GEMM = {"mode": "exact"}


def set_gemm(mode):
    if mode not in ("exact", "x3"):
        raise ValueError(f"snrse.train: gemm mode {mode!r}")
    _GEMM["mode"] = mode


def _wmat(wp):
    rows, k = wp.shape
    if _GEMM["mode"] == "x3" and rows % 128 == 0 and k % 32 == 0:
        return ops.split_weight(wp)
    return wp


def _rows(cout):
    if cout >= 64:
        if cout % 128:
            raise ValueError(f"conv Cout {cout}: the GEMM tiles need Cout % 128 == 0 (or Cout <= 16)")
        return cout
    if cout > 16:
        raise ValueError(f"conv Cout {cout} not supported")
    return 16


class _Conv(torch.autograd.Function):
    """out = (conv(x0 | x1, w) + b + temb[b] + res) * scale  (NHWC, 3x3 pad 1 or 1x1, f32)."""

    @staticmethod
    def forward(ctx, x0, x1, w, b, res, temb, scale):
        k = w.shape[-1]
        cout = w.shape[0]
        C0 = x0.shape[-1]
        cin = C0 + (0 if x1 is None else x1.shape[-1])
        if x1 is not None and (C0 % 32 or x1.shape[-1] % 32):
            raise ValueError("concatenated conv inputs need 32-channel multiples")
        x0p = x0 if x1 is not None else _pad_last(x0.contiguous(), _ceil(C0, 32))
        wp = _wmat(_pack(w, x0p.shape[-1] + (0 if x1 is None else x1.shape[-1]), _rows(cout)))
        out = ops.conv2d(x0p.contiguous(), wp, k, cout, bias=None if b is None else b.detach().contiguous(),
                         src1=None if x1 is None else x1.contiguous(),
                         res=None if res is None else res.detach().contiguous(), out_scale=scale,
                         temb=None if temb is None else temb.detach().contiguous())
        ctx.save_for_backward(x0p, x1, w)
        ctx.meta = (k, cout, C0, cin, scale, res is not None, temb is not None, b is not None)
        return out

    @staticmethod
    def backward(ctx, dy):
        x0p, x1, w = ctx.saved_tensors
        k, cout, C0, cin, scale, has_res, has_temb, has_b = ctx.meta
        dy = dy.contiguous()
        d = dy if scale == 1.0 else scaled(dy, scale)  # gradient of conv(x) + b + temb + res
        B, H, W_ = dy.shape[:3]
        dx0 = dx1 = dw = db = dres = dtemb = None
        if has_res and ctx.needs_input_grad[4]:
            dres = d
        if has_temb and ctx.needs_input_grad[5]:
            dtemb = chan_sum(d, per_b=True)
        if has_b and ctx.needs_input_grad[3]:
            db = chan_sum(d)
        if ctx.needs_input_grad[2]:
            cin_p = x0p.shape[-1] + (0 if x1 is None else x1.shape[-1])
            g = torch.zeros(cout, k * k, cin_p, device=dy.device, dtype=torch.float32)
            _call("snrse_conv_wgrad_x3" if _GEMM["mode"] == "x3" and cout % 4 == 0 else "snrse_conv_wgrad",
                  d.data_ptr(), cout, x0p.data_ptr(), x0p.shape[-1], _p(x1),
                  0 if x1 is None else x1.shape[-1], B, H, W_, k, g.data_ptr())
            if cin_p != cin:
                g = g[..., :cin]
            dw = g.reshape(cout, k, k, cin).permute(0, 3, 1, 2).contiguous()
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            # transposed conv = conv of dY with the flipped kernel, in / out channels swapped
            wt = w.detach().flip(2, 3).permute(1, 0, 2, 3)  # [Cin, Cout, k, k]
            cp = _ceil(cout, 32)
            dpad = _pad_last(d, cp)
            wtp = _wmat(_pack(wt.contiguous(), cp, _rows(cin)))
            dx = ops.conv2d(dpad.contiguous(), wtp, k, cin)
            if x1 is None:
                dx0 = dx
            else:
                dx0, dx1 = dx[..., :C0].contiguous(), dx[..., C0:].contiguous()
        return dx0, dx1, dw, db, dres, dtemb, None


def conv(x0, w, b=None, x1=None, res=None, temb=None, scale=1.0):
    return _Conv.apply(x0, x1, w, b, res, temb, float(scale))


# ----------------------------------------------------------------------------- GroupNorm (+SiLU)
class _GroupNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x0, x1, gamma, beta, act):
        x0 = x0.contiguous()
        x1 = None if x1 is None else x1.contiguous()
        s0, s1 = ops.gn_stats(x0, x1)
        out = ops.gn_apply(x0, x1, (s0, s1), gamma.detach().contiguous(), beta.detach().contiguous(), act=act)
        ctx.save_for_backward(x0, x1, gamma, beta, s0, s1)
        ctx.act = act
        return out

    @staticmethod
    def backward(ctx, dy):
        x0, x1, gamma, beta, s0, s1 = ctx.saved_tensors
        dy = dy.contiguous()
        B, H, W_, C0 = x0.shape
        C1 = 0 if x1 is None else x1.shape[-1]
        C = C0 + C1
        G = min(C // 4, 32)
        HW = H * W_
        mean = torch.empty(B * G, device=dy.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        _call("snrse_gn_moments", s0.data_ptr(), C0, _p(s1), C1, B, HW, G, 1e-6, mean.data_ptr(), rstd.data_ptr())
        R = torch.empty(B, C, 2, device=dy.device, dtype=torch.float32)
        dx0 = torch.empty_like(x0)
        dx1 = None if x1 is None else torch.empty_like(x1)
        dg = torch.zeros(C, device=dy.device, dtype=torch.float32)
        dbt = torch.zeros(C, device=dy.device, dtype=torch.float32)
        _call("snrse_gn_backward", x0.data_ptr(), C0, _p(x1), C1, dy.data_ptr(), B, HW, G,
              gamma.detach().contiguous().data_ptr(), beta.detach().contiguous().data_ptr(), mean.data_ptr(),
              rstd.data_ptr(), int(bool(ctx.act)), R.data_ptr(), dx0.data_ptr(), _p(dx1), dg.data_ptr(),
              dbt.data_ptr())
        return dx0, dx1, dg, dbt, None


def group_norm(x0, gamma, beta, act, x1=None):
    return _GroupNorm.apply(x0, x1, gamma, beta, bool(act))


# ----------------------------------------------------------------------------- FIR resampling
class _Fir(torch.autograd.Function):
    """upsample_2d / downsample_2d with [1,3,3,1] (up_or_down_sampling.py:195-257).  Adjoints
    (upfirdn2d backward, op/upfirdn2d.py:23-85): down^T = up / 4, up^T = 4 down."""

    @staticmethod
    def forward(ctx, x, mode):
        ctx.mode = mode
        return ops.fir(x.contiguous(), mode)

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        if ctx.mode == "down":
            g = ops.fir(dy, "up")
            return axpby(g, g, 0.25, 0.0), None
        g = ops.fir(dy, "down")
        return axpby(g, g, 4.0, 0.0), None


def fir(x, mode):
    return _Fir.apply(x, mode)


# ----------------------------------------------------------------------------- dense layers
class _Dense(torch.autograd.Function):
    """y = x Wt + b over the last dim; Wt = W^T for nn.Linear (W [out, in], in_out=False) or W for
    NIN (W [in, out], layers.py:546-555)."""

    @staticmethod
    def forward(ctx, x, W, b, in_out):
        x2 = x.contiguous().reshape(-1, x.shape[-1])
        n, din = x2.shape
        dout = W.shape[1] if in_out else W.shape[0]
        Wd = W.detach().contiguous()
        sB = (0, dout, 1) if in_out else (0, 1, din)
        y = bgemm(x2, (0, din, 1), Wd, sB, n, dout, din, bias=None if b is None else b.detach().contiguous())
        ctx.save_for_backward(x2, W)
        ctx.meta = (in_out, x.shape, b is not None)
        return y.reshape(*x.shape[:-1], dout)

    @staticmethod
    def backward(ctx, dy):
        x2, W = ctx.saved_tensors
        in_out, xshape, has_b = ctx.meta
        n, din = x2.shape
        dout = W.shape[1] if in_out else W.shape[0]
        d2 = dy.contiguous().reshape(n, dout)
        Wd = W.detach().contiguous()
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            sB = (0, 1, dout) if in_out else (0, din, 1)  # B(k = o, n = i) = W(i, o)
            dx = bgemm(d2, (0, dout, 1), Wd, sB, n, din, dout).reshape(xshape)
        if ctx.needs_input_grad[1]:
            if in_out:  # dW[i][o] = sum_n x[n][i] dy[n][o]
                dW = bgemm(x2, (0, 1, din), d2, (0, dout, 1), din, dout, n)[0]
            else:       # dW[o][i] = sum_n dy[n][o] x[n][i]
                dW = bgemm(d2, (0, 1, dout), x2, (0, din, 1), dout, din, n)[0]
        if has_b and ctx.needs_input_grad[2]:
            db = chan_sum(d2.reshape(1, n, dout))
        return dx, dW, db, None


def linear(x, W, b):
    return _Dense.apply(x, W, b, False)


def nin(x, W, b):
    return _Dense.apply(x, W, b, True)


class _SiLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        _call("snrse_silu", x.data_ptr(), y.data_ptr(), x.numel())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        _call("snrse_silu_bwd", x.data_ptr(), dy.contiguous().data_ptr(), dx.data_ptr(), x.numel(), 0)
        return dx


def silu(x):
    return _SiLU.apply(x)


class _AddScale(torch.autograd.Function):
    """(a + b) * s  (the skip_rescale residual of AttnBlockpp, layerspp.py:89-93)."""

    @staticmethod
    def forward(ctx, a, b, s):
        ctx.s = s
        out = scaled(a.contiguous(), s)
        return axpby(b.contiguous(), out, s, 1.0)

    @staticmethod
    def backward(ctx, dy):
        g = scaled(dy.contiguous(), ctx.s)
        return g, g, None


class _ScaleRows(torch.autograd.Function):
    """x[b] / s[b] (h / used_sigmas, ncsnpp.py:398-400; s carries no gradient: time_cond)."""

    @staticmethod
    def forward(ctx, x, s):
        x = x.contiguous()
        ctx.save_for_backward(s)
        y = torch.empty_like(x)
        _call("snrse_scale_rows", x.data_ptr(), s.data_ptr(), y.data_ptr(), x.shape[0], x.numel() // x.shape[0], 1)
        return y

    @staticmethod
    def backward(ctx, dy):
        (s,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        _call("snrse_scale_rows", dy.data_ptr(), s.data_ptr(), dx.data_ptr(), dy.shape[0], dy.numel() // dy.shape[0], 1)
        return dx, None


# ----------------------------------------------------------------------------- attention
ATTN_CHUNK_BYTES = 256 << 20  # transient score / probability matrices per batch chunk


def _attn_chunks(B, L):
    """Utterance ranges whose [chunk, L, L] f32 score matrix fits ATTN_CHUNK_BYTES (at least one)."""
    cb = max(1, ATTN_CHUNK_BYTES // (L * L * 4))
    return [(b0, min(B, b0 + cb)) for b0 in range(0, B, cb)]


def _attn_probs(q, k, scale):
    """P = softmax_rows(q k^T scale) of one batch chunk (the same kernels in forward and backward, so the
    recomputed probabilities are bit-identical to the forward's)."""
    B, L, Cc = q.shape
    S = bgemm(q, (L * Cc, Cc, 1), k, (L * Cc, 1, Cc), L, L, Cc, batch=B)
    P = torch.empty_like(S)
    _call("snrse_softmax_rows", S.data_ptr(), P.data_ptr(), B * L, L, float(scale))
    return P


class _Attention(torch.autograd.Function):
    """o[l] = sum_m softmax_m(q[l] . k[m] C^-1/2) v[m] per utterance (AttnBlockpp, layerspp.py:84-88);
    q, k, v [B, L, C].  Only q, k, v are kept for the backward, which recomputes the probabilities; both
    passes walk the batch in chunks whose L x L matrices stay within ATTN_CHUNK_BYTES, so memory is bounded
    for any sequence length (30 s clips: L = 16 x 236)."""

    @staticmethod
    def forward(ctx, q, k, v):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, L, Cc = q.shape
        scale = Cc ** -0.5
        o = torch.empty_like(q)
        for b0, b1 in _attn_chunks(B, L):
            P = _attn_probs(q[b0:b1], k[b0:b1], scale)
            bgemm(P, (L * L, L, 1), v[b0:b1], (L * Cc, Cc, 1), L, Cc, L, batch=b1 - b0, C=o[b0:b1],
                  sC=(L * Cc, Cc, 1))
        ctx.save_for_backward(q, k, v)
        ctx.scale = scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v = ctx.saved_tensors
        do = do.contiguous()
        B, L, Cc = q.shape
        dQ, dK, dV = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        for b0, b1 in _attn_chunks(B, L):
            n = b1 - b0
            qc, kc, vc, doc = q[b0:b1], k[b0:b1], v[b0:b1], do[b0:b1]
            P = _attn_probs(qc, kc, ctx.scale)
            dP = bgemm(doc, (L * Cc, Cc, 1), vc, (L * Cc, 1, Cc), L, L, Cc, batch=n)
            bgemm(P, (L * L, 1, L), doc, (L * Cc, Cc, 1), L, Cc, L, batch=n, C=dV[b0:b1], sC=(L * Cc, Cc, 1))
            dS = torch.empty_like(dP)
            _call("snrse_softmax_bwd_rows", P.data_ptr(), dP.data_ptr(), dS.data_ptr(), n * L, L, float(ctx.scale))
            bgemm(dS, (L * L, L, 1), kc, (L * Cc, Cc, 1), L, Cc, L, batch=n, C=dQ[b0:b1], sC=(L * Cc, Cc, 1))
            bgemm(dS, (L * L, 1, L), qc, (L * Cc, Cc, 1), L, Cc, L, batch=n, C=dK[b0:b1], sC=(L * Cc, Cc, 1))
        return dQ, dK, dV


# ----------------------------------------------------------------------------- NCSN++ (training form)
def resblock(m, x0, act_temb, x1=None, up=False, down=False):
    """ResnetBlockBigGANpp.forward (layerspp.py:244-276), fir=True, skip_rescale=True."""
    a = group_norm(x0, m.GroupNorm_0.weight, m.GroupNorm_0.bias, True, x1=x1)
    xs0, xs1 = x0, x1
    if up or down:
        mode = "up" if up else "down"
        a, xs0 = fir(a, mode), fir(x0, mode)
    dense = linear(act_temb, m.Dense_0.weight, m.Dense_0.bias)
    h = conv(a, m.Conv_0.weight, m.Conv_0.bias, temb=dense)
    a1 = group_norm(h, m.GroupNorm_1.weight, m.GroupNorm_1.bias, True)
    if hasattr(m, "Conv_2"):
        xs = conv(xs0, m.Conv_2.weight, m.Conv_2.bias, x1=xs1)
    else:
        xs = xs0
    return conv(a1, m.Conv_1.weight, m.Conv_1.bias, res=xs, scale=INV_SQRT2)


def attn_block(m, x):
    """AttnBlockpp.forward (layerspp.py:77-93)."""
    B, H, W_, Cc = x.shape
    a = group_norm(x, m.GroupNorm_0.weight, m.GroupNorm_0.bias, False)
    a2 = a.reshape(B, H * W_, Cc)
    q = nin(a2, m.NIN_0.W, m.NIN_0.b)
    k = nin(a2, m.NIN_1.W, m.NIN_1.b)
    v = nin(a2, m.NIN_2.W, m.NIN_2.b)
    o = _Attention.apply(q, k, v)
    h = nin(o, m.NIN_3.W, m.NIN_3.b).reshape(B, H, W_, Cc)
    return _AddScale.apply(x, h, INV_SQRT2)


def ncsnpp_forward(net, x, y, t):
    """NCSNpp.forward (ncsnpp.py:247-404) on complex x, y [B, F, T] (device), t [B]: the network output
    as real [B, F, T, 2] (view_as_complex of it is the reference's [B, 1, F, T] output).  Differentiable
    w.r.t. the parameters of `net` (sgmse.backbones.NCSNpp) through the HIP kernels."""
    mods = net.all_modules
    B, Fq, T = x.shape
    _, pyr_in = ops.input_pack(x.contiguous(), y.contiguous(), torch.float32)  # [B, F, T, 4]: x.re x.im y.re y.im
    gfp = torch.empty(B, 2 * mods[0].W.shape[0], device=x.device, dtype=torch.float32)
    _call("snrse_gfp", t.data_ptr(), mods[0].W.detach().contiguous().data_ptr(), B, mods[0].W.shape[0], gfp.data_ptr())
    temb = linear(gfp, mods[1].weight, mods[1].bias)
    temb = linear(silu(temb), mods[2].weight, mods[2].bias)
    act_temb = silu(temb)
    h = conv(pyr_in, mods[3].weight, mods[3].bias)
    hs = [h]
    i = 4
    plan = net._plan
    for lvl in range(7):
        for _ in range(2):
            h = resblock(mods[i], hs[-1], act_temb)
            i += 1
            if plan[i].kind == "attn":
                h = attn_block(mods[i], h)
                i += 1
            hs.append(h)
        if lvl != 6:
            h = resblock(mods[i], hs[-1], act_temb, down=True)
            pyr_in = ops.fir(pyr_in, "down")  # the input pyramid carries no gradient
            h = conv(pyr_in, mods[i + 1].Conv_0.weight, mods[i + 1].Conv_0.bias, res=h)  # Combine, 'sum'
            i += 2
            hs.append(h)
    h = hs[-1]
    h = resblock(mods[i], h, act_temb)
    h = attn_block(mods[i + 1], h)
    h = resblock(mods[i + 2], h, act_temb)
    i += 3
    pyr = None
    for lvl in reversed(range(7)):
        for _ in range(3):
            h = resblock(mods[i], h, act_temb, x1=hs.pop())
            i += 1
        if plan[i].kind == "attn":
            h = attn_block(mods[i], h)
            i += 1
        a = group_norm(h, mods[i].weight, mods[i].bias, True)
        pyr = conv(a, mods[i + 1].weight, mods[i + 1].bias, res=None if pyr is None else fir(pyr, "up"))
        i += 2
        if lvl != 0:
            h = resblock(mods[i], h, act_temb, up=True)
            i += 1
    assert i == len(mods) and not hs
    h = _ScaleRows.apply(pyr, t)  # h / used_sigmas (ncsnpp.py:398-400)
    return conv(h, net.output_layer.weight, net.output_layer.bias)  # [B, F, T, 2]


# ----------------------------------------------------------------------------- loss
class _CTLoss(torch.autograd.Function):
    """mean_b 0.5 sum |err|^2 with err = f1 - f0 or s(f1) - s(f0), f_k = cs_k x_k + co_k dnn_k
    (model.py:378-390 with the sebridge_v3 preconditioning 536-541)."""

    @staticmethod
    def forward(ctx, dnn1, dnn0, x1, x0, coef, sqrt_loss):
        B = dnn1.shape[0]
        HW = dnn1.numel() // (2 * B)
        loss_b = torch.empty(B, device=dnn1.device, dtype=torch.float64)
        g1, g0 = torch.empty_like(dnn1), torch.empty_like(dnn0)
        _call("snrse_ct_loss", dnn1.contiguous().data_ptr(), dnn0.contiguous().data_ptr(), x1.data_ptr(),
              x0.data_ptr(), coef.data_ptr(), B, HW, int(bool(sqrt_loss)), loss_b.data_ptr(), g1.data_ptr(),
              g0.data_ptr())
        ctx.save_for_backward(g1, g0)
        return loss_b.mean().to(torch.float32)

    @staticmethod
    def backward(ctx, go):
        g1, g0 = ctx.saved_tensors
        gs = float(go)  # scalar upstream gradient (1.0 from loss.backward())
        if gs != 1.0:
            g1, g0 = scaled(g1, gs), scaled(g0, gs)
        return g1, g0, None, None, None, None


# ----------------------------------------------------------------------------- the step
N_GRID, ROH, T_EPS = 30, 7, 0.001


def t_grid(n, T=1.0):
    """t_n of model.py:366-367: (eps^(1/roh) + (n-1)/(N-1) (T^(1/roh) - eps^(1/roh)))^roh, n in 1..N."""
    n = np.asarray(n, dtype=np.float64)
    return (T_EPS ** (1 / ROH) + (n - 1) / (N_GRID - 1) * (T ** (1 / ROH) - T_EPS ** (1 / ROH))) ** ROH


def precond(t):
    """sebridge_v3 c_skip, c_out (model.py:536-541), float64 host scalars."""
    eps, sd = 0.001, 0.5
    t = np.asarray(t, dtype=np.float64)
    return sd ** 2 / ((t - eps) ** 2 + sd ** 2), (sd * (t - eps)) / np.sqrt(sd ** 2 + t ** 2)


def consistency_loss(net, X, Y, n, z, sigma_max, loss_type="mse", fixed_snr=None, transform=True):
    """The consistency-training loss of one batch (model.py:361-390; with fixed_snr, the
    snr_conditioned='fixed' sebridge_v3 form of model.py:293-326).

    X, Y: clean / noisy spectrograms complex64 [B, F, T] (device, the data module's transformed specs);
    n: int grid indices [B] in 1..29 (torch.randint(1, N)); z: standard complex normal draws [B, F, T]
    (torch.randn_like(x); scaled by sigma_max here).  Returns the scalar loss tensor (autograd graph
    through the network parameters)."""
    B = X.shape[0]
    HW = X.shape[-2] * X.shape[-1]
    dev = X.device
    tn = t_grid(n, 1.0)
    tn1 = t_grid(np.asarray(n) + 1, 1.0)
    X, Y, z = X.contiguous(), Y.contiguous(), z.contiguous()
    w = lambda tt: tt if fixed_snr is None else fixed_snr * tt  # noqa: E731
    mus, xts = [], []
    for tt in (tn1, tn):
        wm = torch.tensor(w(tt), device=dev, dtype=torch.float32)
        ns = torch.tensor(tt * sigma_max, device=dev, dtype=torch.float32)
        mu, xt = torch.empty_like(X), torch.empty_like(X)
        _call("snrse_ct_perturb", X.data_ptr(), Y.data_ptr(), z.data_ptr(), wm.data_ptr(), ns.data_ptr(), B, HW,
              int(bool(transform)), mu.data_ptr(), xt.data_ptr())
        mus.append(mu)
        xts.append(xt)
    t1 = torch.tensor(tn1, device=dev, dtype=torch.float32)
    t0 = torch.tensor(tn, device=dev, dtype=torch.float32)
    dnn1 = ncsnpp_forward(net, xts[0], mus[0], t1)  # f_theta = self(x_t_n1, t_n1, mu_t_n1)
    dnn0 = ncsnpp_forward(net, xts[1], mus[1], t0)  # f_theta_minus = self(x_t_n, t_n, mu_t_n)
    cs1, co1 = precond(tn1)
    cs0, co0 = precond(tn)
    coef = torch.tensor(np.stack([cs1, co1, cs0, co0], 1), device=dev, dtype=torch.float32).contiguous()
    if loss_type not in ("mse", "sqrt_mse"):
        raise NotImplementedError(f"loss_type {loss_type!r} (the reference's sebridge_v3 branch has mse / sqrt_mse)")
    xv1 = torch.view_as_real(xts[0])
    xv0 = torch.view_as_real(xts[1])
    return _CTLoss.apply(dnn1, dnn0, xv1, xv0, coef, loss_type == "sqrt_mse")


# ----------------------------------------------------------------------------- optimizer
class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (betas, eps; no weight decay, amsgrad or maximize) whose step runs as ONE HIP
    launch over every parameter tensor that has a gradient (snrse_adam_ema; torch skips the others too),
    one launch per distinct per-tensor step count (torch's bias correction uses each tensor's own);
    `ema` (a sgmse.ema.EMAState) is updated in the same launch with torch_ema 0.3's rule,
    decay = min(decay, (1 + n) / (10 + n)), its shadows created from the parameters on first use; shadows of
    parameters without a gradient move too (torch_ema updates every requires_grad shadow)."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, ema=None):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self.ema = ema
        self._chunk_cache = {}

    def _chunks(self, ps):
        """(tensor index, start) of every 2048-element chunk of the tensors `ps`, on the device."""
        tix, starts = [], []
        for i, p in enumerate(ps):
            for s0 in range(0, p.numel(), 2048):
                tix.append(i)
                starts.append(s0)
        dev = ps[0].device
        return (torch.tensor(tix, dtype=torch.int32, device=dev), torch.tensor(starts, dtype=torch.int64, device=dev))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        shadow_of = {}
        decay = 0.0
        if self.ema is not None:
            eps_ = self.ema._params()
            if self.ema.shadow_params is None:
                self.ema.shadow_params = [p.detach().clone() for p in eps_]
            shadow_of = {id(p): s for p, s in zip(eps_, self.ema.shadow_params)}
            n_up = (0 if self.ema.num_updates is None else self.ema.num_updates) + 1
            self.ema.num_updates = n_up
            decay = min(self.ema.decay, (1 + n_up) / (10 + n_up))
        updated = set()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                    raise RuntimeError("FusedAdam: contiguous f32 HIP parameters required (no CPU fallback)")
                st = self.state[p]
                if "exp_avg" not in st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
            # torch.optim.Adam corrects every tensor with its own step count: one launch per distinct count
            # (a single one while every parameter gets a gradient on every step)
            by_step = {}
            for p in ps:
                by_step.setdefault(int(self.state[p]["step"]), []).append(p)
            keep = []
            for step, sub in by_step.items():
                # chunk tables depend only on the element counts, in order (a recycled id() cannot serve a
                # table of other sizes); a few entries at most, oldest evicted (gradient presence can vary)
                key = (str(sub[0].device),) + tuple(p.numel() for p in sub)
                if key in self._chunk_cache:
                    self._chunk_cache[key] = self._chunk_cache.pop(key)  # most recently used last
                else:
                    self._chunk_cache[key] = self._chunks(sub)
                    while len(self._chunk_cache) > 8:
                        self._chunk_cache.pop(next(iter(self._chunk_cache)))
                tix, starts = self._chunk_cache[key]
                rec = np.zeros((len(sub), 6), dtype=np.int64)
                for i, p in enumerate(sub):
                    st = self.state[p]
                    sh = shadow_of.get(id(p))
                    g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                    keep.append(g)  # a temporary copy must outlive the asynchronous launch
                    rec[i] = [p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                              st["exp_avg_sq"].data_ptr(), 0 if sh is None else sh.data_ptr(), p.numel()]
                table = torch.from_numpy(rec).to(sub[0].device)
                keep.append(table)  # the launch reads it asynchronously
                b1, b2 = group["betas"]
                _call("snrse_adam_ema", table.data_ptr(), tix.data_ptr(), starts.data_ptr(),
                      int(tix.numel()), float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                      float(1 - b1 ** step), float(math.sqrt(1 - b2 ** step)), float(decay))
            self._keep = keep
            updated.update(id(p) for p in ps)
        if self.ema is not None:
            # torch_ema 0.3 moves EVERY requires_grad shadow on every update, gradient or not:
            # s = decay s + (1 - decay) p for the parameters the fused launch did not touch
            for p, sh in zip(eps_, self.ema.shadow_params):
                if id(p) not in updated and p.requires_grad:
                    _call("snrse_axpby", p.data_ptr(), sh.data_ptr(), p.numel(), float(1 - decay), float(decay))
        return loss


__all__ = ["ncsnpp_forward", "consistency_loss", "FusedAdam", "t_grid", "precond"]

"""NCSN++ score network executed on the HIP kernels (NHWC; 16-bit -- fp16 by default, or bf16 -- or the fp32 modes).

Mirrors NCSNpp (reference sgmse/backbones/ncsnpp.py:36-404) for its shipped configuration:
nf=128, ch_mult=(1,1,2,2,2,2,2), num_res_blocks=2, attn_resolutions=(16,), BigGAN
ResBlocks with FIR [1,3,3,1] resampling, skip_rescale, output_skip / input_skip pyramids
with 'sum' combine, Gaussian-Fourier time embedding, 4-channel complex I/O.

Each ResnetBlockBigGANpp (layerspp.py:244-276) runs as
    stats(x) -> GN0+SiLU(+FIR) -> Conv_0 (+bias +Dense_0 temb)      [one MFMA GEMM]
    stats(h) -> GN1+SiLU       -> Conv_1 (+bias) [+Conv_2 1x1 shortcut as extra K]
                               -> (x + h)/sqrt(2) [+ input-skip Combine]    [one MFMA GEMM]
and AttnBlockpp (layerspp.py:77-93) as GN -> fused QKV GEMM -> flash attention -> NIN_3
GEMM with the residual epilogue.  Weights are re-packed once on the device (K-contiguous
[Cout][ky][kx][Cin]).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from . import ops

INV_SQRT2 = 1.0 / math.sqrt(2.0)
# tests flip this to compare the fused 16-bit input conv with the im2col + GEMM path
_NO_FUSED_INPUT = False


@dataclass
class Mod:
    kind: str  # gfp, linear, conv3x3, rb, attn, combine, gn
    idx: int
    cin: int = 0
    cout: int = 0
    up: bool = False
    down: bool = False
    extra: dict = field(default_factory=dict)


def build_plan(nf=128, ch_mult=(1, 1, 2, 2, 2, 2, 2), num_res_blocks=2, attn_resolutions=(16,),
               image_size=256):
    """Module list of NCSNpp.__init__ (ncsnpp.py:99-245) for the supported configuration."""
    mods = []

    def add(kind, **kw):
        mods.append(Mod(kind, len(mods), **kw))

    nres = len(ch_mult)
    res = [image_size // (2 ** i) for i in range(nres)]
    add("gfp", cout=2 * nf)
    add("linear", cin=2 * nf, cout=4 * nf)
    add("linear", cin=4 * nf, cout=4 * nf)
    add("conv3x3", cin=4, cout=nf)
    hs_c = [nf]
    in_ch = nf
    for lvl in range(nres):
        for _ in range(num_res_blocks):
            out_ch = nf * ch_mult[lvl]
            add("rb", cin=in_ch, cout=out_ch)
            in_ch = out_ch
            if res[lvl] in attn_resolutions:
                add("attn", cin=in_ch, cout=in_ch)
            hs_c.append(in_ch)
        if lvl != nres - 1:
            add("rb", cin=in_ch, cout=in_ch, down=True)
            add("combine", cin=4, cout=in_ch)
            hs_c.append(in_ch)
    in_ch = hs_c[-1]
    add("rb", cin=in_ch, cout=in_ch)
    add("attn", cin=in_ch, cout=in_ch)
    add("rb", cin=in_ch, cout=in_ch)
    for lvl in reversed(range(nres)):
        for _ in range(num_res_blocks + 1):
            out_ch = nf * ch_mult[lvl]
            skip = hs_c.pop()
            add("rb", cin=in_ch + skip, cout=out_ch, extra={"c0": in_ch, "c1": skip})
            in_ch = out_ch
        if res[lvl] in attn_resolutions:
            add("attn", cin=in_ch, cout=in_ch)
        add("gn", cin=in_ch, cout=in_ch)
        add("conv3x3", cin=in_ch, cout=4)
        if lvl != 0:
            add("rb", cin=in_ch, cout=in_ch, up=True)
    assert not hs_c
    return mods


SHIPPED = dict(nf=128, ch_mult=(1, 1, 2, 2, 2, 2, 2), num_res_blocks=2, attn_resolutions=(16,), image_size=256)


def check_topology(**cfg):
    """The executor (_pyramid) hard-codes the shipped NCSN++ topology (ncsnpp.py:45-245 with the
    defaults of the README configuration): reject any other one at construction instead of
    mis-executing a checkpoint."""
    for k, v in cfg.items():
        want = SHIPPED.get(k)
        got = tuple(v) if isinstance(v, (list, tuple)) else v
        if want is not None and got != want:
            raise NotImplementedError(f"NCSNpp {k}={v!r}: the HIP executor is built for {k}={want!r} only")


def _pack3x3(w, dt, npad=None):
    co = w.shape[0]
    p = w.permute(0, 2, 3, 1).reshape(co, -1)
    if npad is not None and npad > co:
        p = torch.cat([p, p.new_zeros(npad - co, p.shape[1])], 0)
    return p.to(dt).contiguous()


def _pack1x1(w, dt, npad=None):
    return _pack3x3(w, dt, npad)


class NCSNppHIP:
    """Device-resident packed weights + the forward executor."""

    def __init__(self, sd: dict, dtype=torch.float16, device="cuda", gemm="exact", **cfg):
        """dtype: torch.float16 (the fast path's default since round 6: fp16 activations / weights / MFMA operands,
        fp32 accumulation and statistics), torch.bfloat16 (the same kernels on bf16) or torch.float32.
        gemm (fp32 only): "exact" = v_mfma_f32_16x16x4_f32 GEMMs; "x3" = the split-bf16 GEMM
        (ops.split_weight, three bf16 products per K-tile) for every conv: the ResBlock, input and pyramid-head
        convs and (round 5) the attention projections NIN_0..3 and the attention core (split q, k, v, p)."""
        if not torch.cuda.is_available():
            raise RuntimeError("snrse: NCSNppHIP needs a HIP device (no CPU fallback)")
        if gemm not in ("exact", "x3") or (gemm == "x3" and dtype != torch.float32):
            raise ValueError(f"snrse: gemm={gemm!r} with dtype {dtype} (x3 is an fp32 mode)")
        self.dtype = dtype
        self.gemm = gemm
        self.device = torch.device(device)
        self._arena = None  # ops.StatsArena of the GroupNorm statistics, one fill per evaluation
        self._arenas = {}   # one arena per launch stream (the two-stream sampler runs evaluations concurrently)
        self.mid_hook = None  # callable run once between the down and the up path of the next evaluation
        check_topology(**cfg)
        self.plan = build_plan(**cfg)
        dev, dt = self.device, dtype
        f32 = lambda k: sd[k].detach().to(dev, torch.float32).contiguous()  # noqa: E731
        self.W = {}
        W = self.W
        W["gfp"] = f32("all_modules.0.W")
        W["l1w"], W["l1b"] = f32("all_modules.1.weight"), f32("all_modules.1.bias")
        W["l2w"], W["l2b"] = f32("all_modules.2.weight"), f32("all_modules.2.bias")
        w_in = sd["all_modules.3.weight"].detach().to(dev, torch.float32)  # [128, 4, 3, 3]
        col = w_in.permute(0, 2, 3, 1).reshape(w_in.shape[0], 36)
        W["in_w"] = torch.cat([col, col.new_zeros(col.shape[0], 28)], 1).to(dt).contiguous()
        W["in_b"] = f32("all_modules.3.bias")
        W["out_w"] = f32("output_layer.weight").reshape(2, 4).contiguous()
        W["out_b"] = f32("output_layer.bias")
        dense_w, dense_b, off = [], [], 0
        self.mw = {}
        for m in self.plan:
            pre = f"all_modules.{m.idx}"
            e = {}
            if m.kind == "rb":
                e["gn0_g"], e["gn0_b"] = f32(pre + ".GroupNorm_0.weight"), f32(pre + ".GroupNorm_0.bias")
                e["gn1_g"], e["gn1_b"] = f32(pre + ".GroupNorm_1.weight"), f32(pre + ".GroupNorm_1.bias")
                e["w0"] = _pack3x3(sd[pre + ".Conv_0.weight"].detach().to(dev), dt)
                e["b0"] = f32(pre + ".Conv_0.bias")
                e["w1"] = _pack3x3(sd[pre + ".Conv_1.weight"].detach().to(dev), dt)
                b1 = f32(pre + ".Conv_1.bias")
                if m.cin != m.cout or m.up or m.down:
                    e["w2"] = _pack1x1(sd[pre + ".Conv_2.weight"].detach().to(dev), dt)
                    b1 = b1 + f32(pre + ".Conv_2.bias")
                e["b1"] = b1.contiguous()
                dense_w.append(f32(pre + ".Dense_0.weight"))
                dense_b.append(f32(pre + ".Dense_0.bias"))
                e["temb_off"] = off
                off += m.cout
            elif m.kind == "attn":
                e["gn_g"], e["gn_b"] = f32(pre + ".GroupNorm_0.weight"), f32(pre + ".GroupNorm_0.bias")
                Ws = [sd[f"{pre}.NIN_{i}.W"].detach().to(dev, torch.float32) for i in range(4)]
                e["wqkv"] = torch.cat([Ws[0].t(), Ws[1].t(), Ws[2].t()], 0).to(dt).contiguous()
                e["bqkv"] = torch.cat([f32(f"{pre}.NIN_{i}.b") for i in range(3)]).contiguous()
                e["w3"] = Ws[3].t().to(dt).contiguous()
                e["b3"] = f32(pre + ".NIN_3.b")
            elif m.kind == "combine":
                e["w"] = f32(pre + ".Conv_0.weight").reshape(m.cout, 4).contiguous()
                e["b"] = f32(pre + ".Conv_0.bias")
            elif m.kind == "gn":
                e["g"], e["b"] = f32(pre + ".weight"), f32(pre + ".bias")
            elif m.kind == "conv3x3" and m.idx != 3:
                e["w"] = _pack3x3(sd[pre + ".weight"].detach().to(dev), dt, npad=16)
                e["b"] = f32(pre + ".bias")
            self.mw[m.idx] = e
        W["dense_w"] = torch.cat(dense_w, 0).contiguous()
        W["dense_b"] = torch.cat(dense_b, 0).contiguous()
        if gemm == "x3":
            W["in_w"] = ops.split_weight(W["in_w"])
            # the pyramid heads split too: their fused-GroupNorm halo kernel (conv_head_x3_kernel) reads the
            # fp32 input once instead of a gn_act pass + the register-staged Cout <= 16 GEMM (split heads on
            # the register-staged GEMM alone measured no faster, profiles/r03zG)
            for m in self.plan:
                e = self.mw[m.idx]
                if m.kind == "rb":
                    for k in ("w0", "w1", "w2"):
                        if k in e:
                            e[k] = ops.split_weight(e[k])
                elif m.kind == "conv3x3" and "w" in e:
                    e["w"] = ops.split_weight(e["w"])
                elif m.kind == "attn":  # the 1x1 QKV / NIN_3 projections (exact fp32 GEMMs before round 5)
                    e["wqkv"] = ops.split_weight(e["wqkv"])
                    e["w3"] = ops.split_weight(e["w3"])

    # ------------------------------------------------------------------ blocks
    # Every activation travels with its per-channel GroupNorm statistics, produced by the
    # epilogue of the GEMM that wrote it, so no separate statistics pass is needed.
    def _conv(self, *a, **kw):
        out_stats = kw.pop("want_stats", True)
        src0 = a[0]
        st = ops.new_stats(src0.shape[0], a[3]) if out_stats else None
        out = ops.conv2d(*a, stats=st, **kw)
        return out, st

    def _resblock(self, m, x0, x1, dense, comb=None, comb_w=None, comb_b=None):
        """x0/x1: (tensor, stats) of the (possibly concatenated) input.
        Where the halo GEMM applies (16-bit, 3x3, H%4 == 0, W%64 == 0) GroupNorm+SiLU is fused
        into the GEMM's halo load; otherwise it is one gn_apply pass (with the FIR for up/down)."""
        e = self.mw[m.idx]
        mode = "up" if m.up else ("down" if m.down else "none")
        (t0, s0), (t1, s1) = x0, (x1 if x1 is not None else (None, None))
        B, H, W, _ = t0.shape
        xs_raw = None
        fused = ops.x3h_ok if self.gemm == "x3" else ops.halo_ok  # GEMMs that take GroupNorm+SiLU in their halo
        if mode == "none" and fused(t0, 3, m.cout):
            gn0 = ops.gn_scale_shift(s0, e["gn0_g"], e["gn0_b"], H * W, sums1=s1)
            h, hs_ = self._conv(t0, e["w0"], 3, m.cout, src1=t1, gn=gn0, bias=e["b0"], temb=dense,
                                temb_off=e["temb_off"])
        elif mode != "none" and t1 is None and ops.resample_ok(t0):
            # one LDS-tiled pass: SiLU(GN(x)) resampled for Conv_0 and the raw FIR of x for Conv_2
            gn0 = ops.gn_scale_shift(s0, e["gn0_g"], e["gn0_b"], H * W)
            a0, xs_raw = ops.gn_resample(t0, *gn0, act=True, mode=mode, want_raw="w2" in e)
            h, hs_ = self._conv(a0, e["w0"], 3, m.cout, bias=e["b0"], temb=dense, temb_off=e["temb_off"])
        else:
            a0 = ops.gn_apply(t0, t1, s0, e["gn0_g"], e["gn0_b"], act=True, mode=mode, sums1=s1)
            h, hs_ = self._conv(a0, e["w0"], 3, m.cout, bias=e["b0"], temb=dense, temb_off=e["temb_off"])
        Hh, Wh = h.shape[1], h.shape[2]
        if fused(h, 3, m.cout):
            src, gn1 = h, ops.gn_scale_shift(hs_, e["gn1_g"], e["gn1_b"], Hh * Wh)
        else:
            src, gn1 = ops.gn_apply(h, None, hs_, e["gn1_g"], e["gn1_b"], act=True), None
        if "w2" in e:
            if mode != "none":
                xs0, xs1 = (ops.fir(t0, mode) if xs_raw is None else xs_raw), None
            else:
                xs0, xs1 = t0, t1
            return self._conv(src, e["w1"], 3, m.cout, gn=gn1, bias=e["b1"], sc=xs0, sc1=xs1, sc_wgt=e["w2"],
                              out_scale=INV_SQRT2, comb=comb, comb_w=comb_w, comb_b=comb_b)
        assert t1 is None
        return self._conv(src, e["w1"], 3, m.cout, gn=gn1, bias=e["b1"], res=t0, out_scale=INV_SQRT2,
                          comb=comb, comb_w=comb_w, comb_b=comb_b)

    def _attn(self, m, x):
        e = self.mw[m.idx]
        t, s = x
        a = ops.gn_apply(t, None, s, e["gn_g"], e["gn_b"], act=False)
        qkv, _ = self._conv(a, e["wqkv"], 1, 3 * m.cout, bias=e["bqkv"], want_stats=False)
        o = ops.attention(qkv, m.cout, split=self.gemm == "x3")
        return self._conv(o, e["w3"], 1, m.cout, bias=e["b3"], res=t, out_scale=INV_SQRT2)

    def _pyramid_head(self, gn_m, conv_m, h, pyr_up):
        g = self.mw[gn_m.idx]
        c = self.mw[conv_m.idx]
        t, s = h
        if ops.head_ok(t, split=self.gemm == "x3"):  # GroupNorm+SiLU fused into the head conv's halo load
            gn = ops.gn_scale_shift(s, g["g"], g["b"], t.shape[1] * t.shape[2])
            return ops.conv2d(t, c["w"], 3, 4, bias=c["b"], res=pyr_up, out_f32=True, gn=gn)
        a = ops.gn_apply(t, None, s, g["g"], g["b"], act=True)
        return ops.conv2d(a, c["w"], 3, 4, bias=c["b"], res=pyr_up, out_f32=True)

    # ------------------------------------------------------------------ forward
    def temb(self, t):
        W = self.W
        temb = ops.temb_mlp(t, W["gfp"], W["l1w"], W["l1b"], W["l2w"], W["l2b"])
        return ops.temb_dense(temb, W["dense_w"], W["dense_b"])

    def pyramid(self, x, y, t):
        """x, y complex64 [B,F,T] (contiguous, device); t [B] f32 -> final pyramid [B,F,T,4] f32
        (ncsnpp.py:389-398 before the division by t and the output layer)."""
        key = torch.cuda.current_stream(x.device).cuda_stream
        arena = self._arenas.get(key)
        if arena is None:
            arena = self._arenas[key] = ops.StatsArena(x.device)
        self._arena = arena
        with arena:
            return self._pyramid(x, y, t)

    def _pyramid(self, x, y, t):
        W = self.W
        dense = self.temb(t)
        if self.dtype in ops.H16 and ops.input_conv_ok(x) and not _NO_FUSED_INPUT:
            ht, hst, pyr_in = ops.input_conv(x, y, W["in_w"], W["in_b"])
            h = (ht, hst)
        elif self.gemm == "x3" and ops.input_conv_x3_ok(x) and not _NO_FUSED_INPUT:
            ht, hst, pyr_in = ops.input_conv_x3(x, y, W["in_w"], W["in_b"])  # (W["in_w"]: split weights)
            h = (ht, hst)
        else:
            col, pyr_in = ops.input_pack(x, y, self.dtype)
            h = self._conv(col, W["in_w"], 1, 128, bias=W["in_b"])
        hs = [h]
        plan = self.plan
        i = 4
        nres = 7
        for lvl in range(nres):
            for _ in range(2):
                h = self._resblock(plan[i], hs[-1], None, dense)
                i += 1
                if plan[i].kind == "attn":
                    h = self._attn(plan[i], h)
                    i += 1
                hs.append(h)
            if lvl != nres - 1:
                rb, cmb = plan[i], plan[i + 1]
                pyr_in = ops.fir(pyr_in, "down")
                ce = self.mw[cmb.idx]
                h = self._resblock(rb, hs[-1], None, dense, comb=pyr_in, comb_w=ce["w"], comb_b=ce["b"])
                i += 2
                hs.append(h)
        h = hs[-1]
        h = self._resblock(plan[i], h, None, dense); i += 1  # noqa: E702
        h = self._attn(plan[i], h); i += 1  # noqa: E702
        h = self._resblock(plan[i], h, None, dense); i += 1  # noqa: E702
        if self.mid_hook is not None:  # one-shot callback between the down and the up path (lane stagger)
            hook, self.mid_hook = self.mid_hook, None
            hook()
        pyr = None
        for lvl in reversed(range(nres)):
            for _ in range(3):
                h = self._resblock(plan[i], h, hs.pop(), dense)
                i += 1
            if plan[i].kind == "attn":
                h = self._attn(plan[i], h)
                i += 1
            pyr_up = None if pyr is None else ops.fir(pyr, "up")
            pyr = self._pyramid_head(plan[i], plan[i + 1], h, pyr_up)
            i += 2
            if lvl != 0:
                h = self._resblock(plan[i], h, None, dense)
                i += 1
        assert i == len(plan) and not hs
        return pyr

    def score(self, x, y, t, score_mode=0):
        """Preconditioned score (ScoreModel.forward, model.py:481-543) as complex64 [B,F,T]."""
        pyr = self.pyramid(x, y, t)
        _, _, sc = ops.score_update(pyr, self.W["out_w"], self.W["out_b"], t, score_mode, x, y, want_score=True)
        return sc

    def dnn(self, x, y, t):
        """Raw NCSNpp.forward output (no sign / preconditioning): complex64 [B,F,T]."""
        return -self.score(x, y, t, score_mode=0)

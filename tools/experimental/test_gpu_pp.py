"""The ping-pong halo GEMM (csrc/conv_pp.hip, conv_variant 6) against the v5 halo GEMM it restructures.

Both accumulate the same K order (32-channel chunks x 9 taps) in fp32 MFMAs and run the same epilogue
arithmetic, so their bf16 outputs are identical; the per-channel GroupNorm statistics differ only in the
order of the f64 atomics.  Cases cover the GroupNorm modes (none / affine / affine + SiLU), temb, residual,
Combine, statistics, concatenated inputs, two Cout tiles per image, the non-temporal store flavour and
tile counts that leave the two halves of a workgroup uneven runs (or one of them nothing).  A 1x1
shortcut falls back to v5 (pp_ok)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _run(ops, variant, kw):
    ops.set_option("conv_variant", variant)
    try:
        st = ops.new_stats(kw["src0"].shape[0], kw["cout"]) if kw.pop("want_stats", False) else None
        out = ops.conv2d(kw["src0"], kw["wgt"], 3, kw["cout"], **{k: v for k, v in kw.items()
                                                                  if k not in ("src0", "wgt", "cout")}, stats=st)
        ran = ops.kernel_name(ops.get_option("last_kernel"))
    finally:
        ops.set_option("conv_variant", 0)
    torch.cuda.synchronize()
    return out, st, ran


CASES = [
    # B, C0, C1, Cout, H, W, gn(0 none / 1 affine / 2 +SiLU), temb, res, comb, stats, tiles/half
    (2, 128, 0, 128, 16, 128, 2, True, False, False, True, 4),    # Conv_0: 16 tiles = 2 WGs x 2 x 4
    (2, 128, 0, 128, 16, 128, 2, False, True, False, True, 4),    # Conv_1 + residual
    (1, 128, 0, 128, 12, 64, 2, True, False, False, True, 4),     # 3 tiles: halves run 2 and 1
    (1, 128, 0, 128, 4, 64, 2, True, False, False, True, 4),      # 1 tile: half 1 idles throughout
    (3, 256, 0, 256, 8, 128, 2, True, False, False, True, 3),     # two Cout tiles per image, runs of 3
    (2, 256, 256, 256, 8, 64, 0, False, True, False, False, 4),   # cat input, no GroupNorm
    (2, 128, 128, 128, 8, 128, 2, True, False, False, True, 2),   # up-path cat Conv_0
    (2, 128, 0, 128, 8, 64, 1, False, False, True, True, 4),      # affine only, Combine term
    (2, 128, 0, 128, 8, 64, 2, False, True, True, False, 1),      # runtime-flag epilogue, 1 tile per half
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("epi_nt", [0, 1])
def test_pp_matches_v5(gpu, case, epi_nt):
    from snrse import ops
    B, C0, C1, Co, H, W, gnm, use_temb, use_res, use_comb, use_st, tpw = case
    g = torch.Generator(device=gpu).manual_seed(sum(case[:6]) + gnm)
    Cin = C0 + C1
    x0 = (torch.randn(B, H, W, C0, device=gpu, generator=g) * 1.3 + 0.1).bfloat16()
    x1 = torch.randn(B, H, W, C1, device=gpu, generator=g).bfloat16() if C1 else None
    w = (torch.randn(Co, 3, 3, Cin, device=gpu, generator=g) / math.sqrt(9 * Cin)).bfloat16()
    kw = dict(src0=x0, wgt=w.reshape(Co, -1).contiguous(), cout=Co, bias=torch.randn(Co, device=gpu, generator=g),
              src1=x1, want_stats=use_st)
    if gnm:
        gam = torch.rand(Cin, device=gpu, generator=g) + 0.5
        bet = torch.randn(Cin, device=gpu, generator=g) * 0.2
        sums = ops.gn_stats(x0, x1)
        kw["gn"] = ops.gn_scale_shift(sums[0], gam, bet, H * W, sums1=sums[1])
        kw["gn_act"] = gnm == 2
    if use_temb:
        kw["temb"] = torch.randn(B, Co + 40, device=gpu, generator=g)
        kw["temb_off"] = 40
    if use_res:
        kw["res"] = torch.randn(B, H, W, Co, device=gpu, generator=g).bfloat16()
        kw["out_scale"] = 1 / math.sqrt(2)
    if use_comb:
        kw["comb"] = torch.randn(B, H, W, 4, device=gpu, generator=g)
        kw["comb_w"] = torch.randn(Co, 4, device=gpu, generator=g)
        kw["comb_b"] = torch.randn(Co, device=gpu, generator=g)
    ops.set_option("epi_nt", epi_nt)
    ops.set_option("pp_tiles", tpw)
    try:
        o5, s5, r5 = _run(ops, 5, dict(kw))
        o6, s6, r6 = _run(ops, 6, dict(kw))
    finally:
        ops.set_option("epi_nt", 2)
        ops.set_option("pp_tiles", 4)
    assert r5 == "conv_halo5_kernel" and r6 == "conv_pp_kernel", (r5, r6)
    # the same MFMA order and epilogue arithmetic: identical up to the compiler's FMA contraction of the
    # epilogue in the two kernels (a last-bit difference on a handful of elements at most)
    mism = float((o6 != o5).float().mean())
    assert mism < 1e-3 and torch.allclose(o6.float(), o5.float(), rtol=1e-2, atol=1e-3), (
        mism, (o6.float() - o5.float()).abs().max().item())
    if use_st:
        f5, f6 = ops.fold_stats(s5), ops.fold_stats(s6)
        assert torch.allclose(f6, f5, rtol=1e-5, atol=1e-2), (f6 - f5).abs().max().item()  # fp32 partial-sum order


def test_pp_vs_fp32_reference_level0(gpu):
    """One C2 level-0 Conv_0 (B=8, 256 x 512, 128 -> 128, GroupNorm+SiLU, temb, statistics, non-temporal
    epilogue) against fp32 torch conv of the same bf16 operands."""
    from snrse import ops
    B, H, W, C = 8, 256, 512, 128
    g = torch.Generator(device=gpu).manual_seed(7)
    x = (torch.randn(B, H, W, C, device=gpu, generator=g) * 1.3 + 0.1).bfloat16()
    w = (torch.randn(C, 3, 3, C, device=gpu, generator=g) / math.sqrt(9 * C)).bfloat16()
    bias = torch.randn(C, device=gpu, generator=g) * 0.1
    gam = torch.rand(C, device=gpu, generator=g) + 0.5
    bet = torch.randn(C, device=gpu, generator=g) * 0.2
    temb = torch.randn(B, C + 40, device=gpu, generator=g)
    sums, _ = ops.gn_stats(x)
    gn = ops.gn_scale_shift(sums, gam, bet, H * W)
    st = ops.new_stats(B, C)
    ops.set_option("conv_variant", 6)
    ops.set_option("epi_nt", 1)
    try:
        out = ops.conv2d(x, w.reshape(C, -1).contiguous(), 3, C, bias=bias, stats=st, gn=gn, temb=temb, temb_off=40)
        assert ops.kernel_name(ops.get_option("last_kernel")) == "conv_pp_kernel"
    finally:
        ops.set_option("conv_variant", 0)
        ops.set_option("epi_nt", 2)
    torch.cuda.synchronize()
    folded = ops.fold_stats(st)
    for b in (0, 5, 7):
        a = F.silu(x[b].float().permute(2, 0, 1)[None] * gn[0][b][None, :, None, None]
                   + gn[1][b][None, :, None, None]).bfloat16().float()
        ref = F.conv2d(a, w.float().permute(0, 3, 1, 2), bias, padding=1)[0] + temb[b, 40:40 + C, None, None]
        got = out[b].float().permute(2, 0, 1)
        err = float((got - ref).pow(2).mean().sqrt() / ref.pow(2).mean().sqrt())
        assert err < 1e-2, (b, err)
        o = out[b].double()
        st_ref = torch.stack([o.sum((0, 1)), (o * o).sum((0, 1))], -1)
        assert float((folded[b] - st_ref).norm() / st_ref.norm()) < 3e-3

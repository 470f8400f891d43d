"""The split-bf16 form of the v10 halo GEMM (csrc/conv_h10x3.hip: the fp32x3 parity mode's ResBlock convs on the
v10 structure, option h10) against a float64 torch reference of the same fp32 operands and against the x3h halo
kernel it replaces (reference ResnetBlockBigGANpp.Conv_0 / Conv_1 + Conv_2, sgmse/backbones/ncsnpp_utils/
layerspp.py:244-276, fp32 as the reference runs, sgmse/model.py:824).  Tolerance 3e-5 relative RMS as every split
conv (tests/test_gpu_x3.py: ~2^-16 relative per product, averaging down over K)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
TOL = 3e-5


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


CASES = [
    # B, C0, C1, Cout, H, W, gn (0 none, 1 affine, 2 affine+SiLU), temb, res, comb, stats, Csc, Csc1
    (2, 128, 0, 128, 64, 128, 2, True, False, False, True, 0, 0),       # Conv_0
    (2, 128, 0, 128, 64, 128, 2, False, True, False, True, 0, 0),       # Conv_1 + residual
    (2, 128, 128, 128, 32, 64, 2, True, False, False, True, 0, 0),      # cat input
    (2, 256, 0, 256, 32, 64, 1, False, False, False, True, 0, 0),       # affine only, two cout tiles
    (1, 128, 0, 128, 16, 96, 0, False, True, True, False, 0, 0),        # no GroupNorm, Combine; 12 tiles
    (2, 128, 0, 128, 64, 128, 2, False, False, False, True, 128, 128),  # up-path Conv_1: 2 shortcut chunks per main
    (2, 256, 0, 256, 32, 64, 2, False, False, False, True, 256, 128),   # 1.5 per main chunk
    (3, 128, 0, 128, 24, 64, 2, False, False, False, True, 128, 0),     # 1 per main chunk; 18 tiles
]


@pytest.mark.parametrize("case", CASES)
def test_h10x3_vs_f64_and_x3h(gpu, case):
    from snrse import ops
    B, C0, C1, Co, H, W, gnm, use_temb, use_res, use_comb, use_st, Csc, Csc1 = case
    g = torch.Generator(device=gpu).manual_seed(sum(case[:6]) + 11)
    Cin = C0 + C1
    x0 = torch.randn(B, H, W, C0, device=gpu, generator=g) * 1.3 + 0.1
    x1 = torch.randn(B, H, W, C1, device=gpu, generator=g) if C1 else None
    w = torch.randn(Co, 3, 3, Cin, device=gpu, generator=g) / math.sqrt(9 * Cin)
    bias = torch.randn(Co, device=gpu, generator=g)
    kw = {}
    if use_temb:
        kw.update(temb=torch.randn(B, Co + 40, device=gpu, generator=g), temb_off=40)
    if use_res:
        kw.update(res=torch.randn(B, H, W, Co, device=gpu, generator=g), out_scale=1 / math.sqrt(2))
    ws = None
    if Csc:
        ws = torch.randn(Co, Csc + Csc1, device=gpu, generator=g) / math.sqrt(Csc + Csc1)
        kw.update(sc=torch.randn(B, H, W, Csc, device=gpu, generator=g),
                  sc1=torch.randn(B, H, W, Csc1, device=gpu, generator=g) if Csc1 else None,
                  sc_wgt=ops.split_weight(ws), out_scale=1 / math.sqrt(2))
    if use_comb:
        kw.update(comb=torch.randn(B, H, W, 4, device=gpu, generator=g), comb_w=torch.randn(Co, 4, device=gpu, generator=g),
                  comb_b=torch.randn(Co, device=gpu, generator=g))
    xin = x0 if x1 is None else torch.cat([x0, x1], -1)
    a = xin.double().permute(0, 3, 1, 2)
    gn = None
    if gnm:
        gam = torch.rand(Cin, device=gpu, generator=g) + 0.5
        bet = torch.randn(Cin, device=gpu, generator=g) * 0.2
        sums = ops.gn_stats(x0, x1)
        gn = ops.gn_scale_shift(sums[0], gam, bet, H * W, sums1=sums[1])
        a = a * gn[0].double()[:, :, None, None] + gn[1].double()[:, :, None, None]
        a = F.silu(a) if gnm == 2 else a
    ref = F.conv2d(a, w.double().permute(0, 3, 1, 2), bias.double(), padding=1)
    if use_temb:
        ref = ref + kw["temb"].double()[:, 40:40 + Co, None, None]
    if Csc:
        xs = kw["sc"] if not Csc1 else torch.cat([kw["sc"], kw["sc1"]], -1)
        ref = (ref + torch.einsum("bhwc,oc->bohw", xs.double(), ws.double())) * kw["out_scale"]
    if use_res:
        ref = (ref + kw["res"].double().permute(0, 3, 1, 2)) * kw["out_scale"]
    if use_comb:
        ref = ref + torch.einsum("bhwi,oi->bohw", kw["comb"].double(), kw["comb_w"].double()) + \
            kw["comb_b"].double()[:, None, None]
    wp = ops.split_weight(w.reshape(Co, -1))

    h10_prev = ops.get_option("h10")

    def run(h10):
        st = ops.new_stats(B, Co) if use_st else None
        ops.set_option("h10", h10)
        ops.set_option("x3_tile", 4)  # (the x3h kernel wherever its shape allows, for the comparison)
        try:
            out = ops.conv2d(x0, wp, 3, Co, bias=bias, src1=x1, stats=st, gn=gn, gn_act=gnm == 2, **kw)
            ran = ops.kernel_name(ops.get_option("last_kernel"))
        finally:
            ops.set_option("h10", h10_prev)
            ops.set_option("x3_tile", 0)
        return out, st, ran

    out10, st10, ran10 = run(1)
    outh, _, ranh = run(0)
    assert ran10 == "conv_halo10x3_kernel" and ranh == "conv_x3h_kernel", (ran10, ranh)
    assert out10.dtype == torch.float32
    assert rel(out10.permute(0, 3, 1, 2), ref) < TOL, rel(out10.permute(0, 3, 1, 2), ref)
    assert rel(out10, outh) < TOL
    if st10 is not None:
        o = out10.double()
        st_ref = torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1)
        assert rel(ops.fold_stats(st10), st_ref) < 1e-5

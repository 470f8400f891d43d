"""The v10 halo GEMM (csrc/conv_h10.hip: persistent, one wave per SIMD, 16 x 32 px x 128 cout tiles, the next
chunk's GroupNorm+SiLU halo prepared between the MFMAs, register-only epilogue) against an fp32 torch reference of
the same bf16 operands and against the v5 halo GEMM, on the ResBlock conv configurations it serves (reference
ResnetBlockBigGANpp.Conv_0 / Conv_1, sgmse/backbones/ncsnpp_utils/layerspp.py:244-276): fused GroupNorm(+SiLU)
prologue, cat inputs, temb, residual x 1/sqrt(2), Combine, statistics; tile counts below, equal to and not a
multiple of the CU count."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


CASES = [
    # B, C0, C1, Cout, H, W, gn (0 none, 1 affine, 2 affine+SiLU), temb, res, comb, stats[, Csc, Csc1]
    (4, 128, 0, 128, 256, 512, 2, True, False, False, True),    # level-0 Conv_0 (1024 tiles)
    (4, 128, 0, 128, 256, 512, 2, False, True, False, True),    # level-0 Conv_1 + residual
    (8, 128, 128, 128, 128, 256, 2, True, False, False, True),  # up-path Conv_0 on cat(h, skip)
    (8, 256, 0, 256, 64, 128, 2, True, False, False, True),     # two cout tiles per image
    (2, 256, 256, 256, 32, 64, 0, False, True, False, False),   # cat input, no GroupNorm
    (3, 128, 0, 128, 48, 96, 1, False, False, False, True),     # GroupNorm affine only; 27 tiles < CUs
    (7, 128, 0, 128, 128, 256, 2, False, True, True, True),     # Combine (run-time epilogue); 448 tiles
    (2, 128, 0, 128, 80, 96, 2, True, False, False, True),      # 30 tiles, H = 80
    # fused 1x1 shortcut (Conv_2 as extra K, layerspp.py:268-274): shortcut chunks before every main chunk
    (4, 128, 0, 128, 256, 512, 2, False, False, False, True, 128, 128),  # up-path Conv_1, level 0: 2 per main chunk
    (4, 256, 0, 256, 64, 128, 2, False, False, False, True, 256, 128),   # 1.5 per main chunk, two cout tiles
    (2, 256, 0, 256, 32, 64, 2, False, False, True, True, 128, 0),       # 0.5 per main chunk, Combine
    (3, 128, 0, 128, 48, 96, 2, False, False, False, True, 128, 128),    # 27 tiles
]


def _case(gpu, case):
    from snrse import ops
    B, C0, C1, Co, H, W, gnm, use_temb, use_res, use_comb, use_st = case[:11]
    Csc, Csc1 = case[11:] if len(case) > 11 else (0, 0)
    g = torch.Generator(device=gpu).manual_seed(sum(case[:6]) + 7)
    Cin = C0 + C1
    x0 = (torch.randn(B, H, W, C0, device=gpu, generator=g) * 1.3 + 0.1).bfloat16()
    x1 = torch.randn(B, H, W, C1, device=gpu, generator=g).bfloat16() if C1 else None
    w = (torch.randn(Co, 3, 3, Cin, device=gpu, generator=g) / math.sqrt(9 * Cin)).bfloat16()
    bias = torch.randn(Co, device=gpu, generator=g)
    kw = {}
    if use_temb:
        kw.update(temb=torch.randn(B, Co + 40, device=gpu, generator=g), temb_off=40)
    if use_res:
        kw.update(res=torch.randn(B, H, W, Co, device=gpu, generator=g).bfloat16(), out_scale=1 / math.sqrt(2))
    if Csc:
        kw.update(sc=torch.randn(B, H, W, Csc, device=gpu, generator=g).bfloat16(),
                  sc1=torch.randn(B, H, W, Csc1, device=gpu, generator=g).bfloat16() if Csc1 else None,
                  sc_wgt=(torch.randn(Co, Csc + Csc1, device=gpu, generator=g) / math.sqrt(Csc + Csc1)).bfloat16(),
                  out_scale=1 / math.sqrt(2))
    if use_comb:
        kw.update(comb=torch.randn(B, H, W, 4, device=gpu, generator=g), comb_w=torch.randn(Co, 4, device=gpu, generator=g),
                  comb_b=torch.randn(Co, device=gpu, generator=g))
    xin = x0 if x1 is None else torch.cat([x0, x1], -1)
    a = xin.float().permute(0, 3, 1, 2)
    gn = None
    if gnm:
        gam = torch.rand(Cin, device=gpu, generator=g) + 0.5
        bet = torch.randn(Cin, device=gpu, generator=g) * 0.2
        sums = ops.gn_stats(x0, x1)
        gn = ops.gn_scale_shift(sums[0], gam, bet, H * W, sums1=sums[1])
        a = a * gn[0][:, :, None, None] + gn[1][:, :, None, None]
        a = (F.silu(a) if gnm == 2 else a).bfloat16().float()
    ref = F.conv2d(a, w.float().permute(0, 3, 1, 2), bias, padding=1)
    if use_temb:
        ref = ref + kw["temb"][:, 40:40 + Co, None, None]
    if Csc:
        xs = kw["sc"] if not Csc1 else torch.cat([kw["sc"], kw["sc1"]], -1)
        ref = (ref + torch.einsum("bhwc,oc->bohw", xs.float(), kw["sc_wgt"].float())) * kw["out_scale"]
    if use_res:
        ref = (ref + kw["res"].float().permute(0, 3, 1, 2)) * kw["out_scale"]
    if use_comb:
        ref = ref + torch.einsum("bhwi,oi->bohw", kw["comb"], kw["comb_w"]) + kw["comb_b"][:, None, None]

    def run(variant):
        st = ops.new_stats(B, Co) if use_st else None
        ops.set_option("conv_variant", variant)
        try:
            out = ops.conv2d(x0, w.reshape(Co, -1).contiguous(), 3, Co, bias=bias, src1=x1, stats=st, gn=gn,
                             gn_act=gnm == 2, **kw)
            ran = ops.kernel_name(ops.get_option("last_kernel"))
        finally:
            ops.set_option("conv_variant", 0)
        return out, st, ran

    return ref, run


@pytest.mark.parametrize("case", CASES)
def test_h10_vs_fp32_and_v5(gpu, case):
    from snrse import ops
    ref, run = _case(gpu, case)
    out10, st10, ran10 = run(10)
    assert ran10 == "conv_halo10_kernel"
    got = out10.float().permute(0, 3, 1, 2)
    assert rel(got, ref) < 1e-2, rel(got, ref)
    if case[5] % 64 == 0:  # (v5 tiles 64-px rows: no v5 leg at W = 96)
        out5, st5, ran5 = run(5)
        assert ran5 == "conv_halo5_kernel"
        # v10 and v5 differ only in the fp32 accumulation order before the bf16 rounding
        assert rel(out10.float(), out5.float()) < 4e-3
    if st10 is not None:
        o = out10.double()
        st_ref = torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1)
        assert rel(ops.fold_stats(st10), st_ref) < 3e-3


def test_h10_repeat_is_deterministic_and_stats_accumulate_once(gpu):
    """Two launches into fresh statistics buffers give bit-identical outputs and equal statistics (every tile
    is computed by exactly one workgroup of the persistent grid, every channel's statistics added once)."""
    from snrse import ops
    _, run = _case(gpu, CASES[6])
    o1, s1, _ = run(10)
    o2, s2, _ = run(10)
    assert torch.equal(o1, o2)
    assert rel(ops.fold_stats(s1), ops.fold_stats(s2)) < 1e-12


@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[8]])
def test_h10_nontemporal_epilogue_matches(gpu, case):
    """The non-temporal form of the 16-B epilogue stores (option epi_nt = 1, which the auto mode takes for outputs
    beyond 256 MB, e.g. every level-0 conv at C2) writes the same bytes as the cached form."""
    from snrse import ops
    _, run = _case(gpu, case)
    outs = []
    for nt in (1, 0):
        ops.set_option("epi_nt", nt)
        try:
            o, st, ran = run(10)
            assert ran == "conv_halo10_kernel" and ops.get_option("last_epi_nt") == nt
        finally:
            ops.set_option("epi_nt", 2)
        outs.append((o, st))
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert rel(ops.fold_stats(outs[0][1]), ops.fold_stats(outs[1][1])) < 1e-12


@pytest.mark.parametrize("h10,case,want", [(3, CASES[8], "conv_halo10_kernel"), (3, CASES[9], "conv_halo5_kernel"),
                                           (2, CASES[8], "conv_halo5_kernel"), (3, CASES[2], "conv_halo10_kernel")])
def test_h10_auto_dispatch(gpu, h10, case, want):
    """Option h10 under conv_variant 0: 2 takes v10 for the concatenated-input convs without a shortcut, 3 also
    for the convs whose shortcut spans twice their input (the up path's Conv_1 over cat(h, skip)); the result is
    the same conv either way."""
    from snrse import ops
    ref, run = _case(gpu, case)
    old = ops.get_option("h10")
    ops.set_option("h10", h10)
    try:
        out, _, ran = run(0)
    finally:
        ops.set_option("h10", old)
    assert ran == want
    assert rel(out.float().permute(0, 3, 1, 2), ref) < 1e-2

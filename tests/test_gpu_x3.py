"""Parity of the split-bf16 fp32 GEMM (snrse_conv2d dtype SNRSE_F32X3, conv_x3_kernel): fp32
activations, weights pre-split by ops.split_weight, three bf16 MFMA products per K-tile.

Tolerances: single convs 3e-5 relative RMS against a float64 torch conv of the same fp32 operands
(the split keeps ~16 significant bits of each operand: ~2^-16 relative per product, averaging down
over K); the network and the N=5 PC loop are held to the north star's 1e-4 absolute RMS on the
complex spectrogram against the reference goldens (CPU emulation of this arithmetic on the PC golden:
6.0e-5, tools/x3_emulate.py)."""
import math

import pytest
import torch
import torch.nn.functional as F

from conftest import fnormal, formula_sd, golden
from test_gpu_kernels import abs_rms, nchw, nhwc, rel

pytestmark = pytest.mark.gpu
TOL = 3e-5


@pytest.mark.parametrize("shape", [(2, 128, 128, 8, 16), (1, 256, 128, 4, 8), (3, 128, 256, 5, 7), (2, 384, 256, 4, 4),
                                   (2, 128, 128, 8, 64), (1, 384, 256, 4, 128), (1, 256, 256, 12, 64),
                                   (2, 64, 128, 16, 32), (1, 128, 128, 8, 100), (2, 256, 256, 4, 59)])
@pytest.mark.parametrize("tile", [0, 4])
def test_x3_conv3x3(gpu, shape, tile):
    """tile: option x3_tile 0 auto (register-staged at these small grids), 4 the halo kernel where
    H % 4 == 0 (W not a multiple of 64: the last tile column cut by the edge; else register-staged)."""
    from snrse import ops
    B, cin, cout, H, W = shape
    x = torch.from_numpy(fnormal("t.conv.x", (B, cin, H, W)))
    w = torch.from_numpy(fnormal("t.conv.w", (cout, cin, 3, 3))) / math.sqrt(9 * cin)
    b = torch.from_numpy(fnormal("t.conv.b", (cout,)))
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1)
    c0 = 256 if cin == 384 else cin
    xg = nhwc(x).to(gpu)
    src0, src1 = (xg[..., :c0].contiguous(), xg[..., c0:].contiguous()) if c0 != cin else (xg, None)
    wp = ops.split_weight(w.permute(0, 2, 3, 1).reshape(cout, -1).to(gpu))
    assert wp.dtype == torch.bfloat16 and wp.shape == (cout, 2 * 9 * cin)
    ops.set_option("x3_tile", tile)
    try:
        out = ops.conv2d(src0, wp, 3, cout, bias=b.to(gpu), src1=src1)
        kern = ops.get_option("last_kernel")
    finally:
        ops.set_option("x3_tile", 0)
    assert kern == (4 if tile == 4 and H % 4 == 0 else 3), kern
    assert out.dtype == torch.float32
    assert rel(nchw(out), ref) < TOL


@pytest.mark.parametrize("tile", [0, 4])
@pytest.mark.parametrize("hw", [(8, 8), (8, 64), (64, 128), (4, 94)])
def test_x3_epilogue_shortcut_temb_comb(gpu, hw, tile):
    """Conv_1 + Conv_2 shortcut (split weights) as extra K, temb, residual scale, Combine, stats; the
    small shapes run split-K (conv_splitk_finalize), the 64 x 128 one (256 tiles) the in-kernel LDS epilogue."""
    from snrse import ops
    B, cin, cout = 2, 128, 256
    H, W = hw
    h = torch.from_numpy(fnormal("t.ep.h", (B, cout, H, W)))
    xs = torch.from_numpy(fnormal("t.ep.xs", (B, cin, H, W)))
    w1 = torch.from_numpy(fnormal("t.ep.w1", (cout, cout, 3, 3))) / 48
    w2 = torch.from_numpy(fnormal("t.ep.w2", (cout, cin, 1, 1))) / 11
    b1 = torch.from_numpy(fnormal("t.ep.b1", (cout,)))
    temb = torch.from_numpy(fnormal("t.ep.temb", (B, 300)))
    pyr = torch.from_numpy(fnormal("t.ep.pyr", (B, 4, H, W)))
    cw = torch.from_numpy(fnormal("t.ep.cw", (cout, 4)))
    cb = torch.from_numpy(fnormal("t.ep.cb", (cout,)))
    ref = (F.conv2d(h.double(), w1.double(), b1.double(), padding=1) + F.conv2d(xs.double(), w2.double())
           + temb[:, 20:20 + cout, None, None].double()) / math.sqrt(2)
    ref = ref + torch.einsum("bihw,oi->bohw", pyr.double(), cw.double()) + cb.double()[None, :, None, None]
    st = ops.new_stats(B, cout)
    ops.set_option("x3_tile", tile)
    try:
        out = ops.conv2d(nhwc(h).to(gpu), ops.split_weight(w1.permute(0, 2, 3, 1).reshape(cout, -1).to(gpu)),
                         3, cout, bias=b1.to(gpu), sc=nhwc(xs).to(gpu),
                         sc_wgt=ops.split_weight(w2.reshape(cout, cin).to(gpu)), temb=temb.to(gpu), temb_off=20,
                         out_scale=1 / math.sqrt(2), comb=nhwc(pyr).to(gpu), comb_w=cw.to(gpu), comb_b=cb.to(gpu),
                         stats=st)
        kern, ksplit = ops.get_option("last_kernel"), ops.get_option("last_ksplit")
    finally:
        ops.set_option("x3_tile", 0)
    halo = tile == 4 or B * (H // 4) * (-(-W // 64)) * 2 >= 256
    assert kern == (4 if halo else 3), kern
    if not halo and H * W <= 512:  # 2 / 16 output tiles of the register-staged kernel split K
        assert ksplit > 1, ksplit
    assert rel(nchw(out), ref) < TOL
    o = out.double()
    st_ref = torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1)
    assert rel(ops.fold_stats(st), st_ref) < 1e-5


def test_x3_residual_and_layout_errors(gpu):
    from snrse import ops
    B, C, H, W = 1, 128, 8, 64
    x = torch.from_numpy(fnormal("t.x3r.x", (B, C, H, W)))
    r = torch.from_numpy(fnormal("t.x3r.r", (B, C, H, W)))
    w = torch.from_numpy(fnormal("t.x3r.w", (C, C, 1, 1))) / 11
    ref = (F.conv2d(x.double(), w.double()) + r.double()) * 0.5
    wp = w.reshape(C, C).to(gpu)
    out = ops.conv2d(nhwc(x).to(gpu), ops.split_weight(wp), 1, C, res=nhwc(r).to(gpu), out_scale=0.5)
    assert rel(nchw(out), ref) < TOL
    with pytest.raises(TypeError):  # split main weights with exact shortcut weights
        ops.conv2d(nhwc(x).to(gpu), ops.split_weight(wp), 1, C, sc=nhwc(x).to(gpu), sc_wgt=wp)
    with pytest.raises(RuntimeError):  # 16 < Cout, Cout % 128 != 0: no split tile
        ops.conv2d(nhwc(x).to(gpu), ops.split_weight(torch.zeros(64, 9 * C, device=gpu)), 3, 64)


@pytest.mark.parametrize("head_small", [1, 0])
def test_x3_pyramid_head(gpu, head_small):
    """Cout = 4 (16 padded rows) with the upsampled pyramid as an fp32 residual at a size the tiled head cannot
    take: the wave-per-8-pixels fp32x3 head (option head_small 1, the default) and the heads' split GEMM (0)."""
    from snrse import ops
    B, cin, H, W = 2, 256, 8, 16
    x = torch.from_numpy(fnormal("t.py.x", (B, cin, H, W)))
    w = torch.from_numpy(fnormal("t.py.w", (4, cin, 3, 3))) / 48
    b = torch.from_numpy(fnormal("t.py.b", (4,)))
    r = torch.from_numpy(fnormal("t.py.r", (B, 4, H, W)))
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1) + r.double()
    wp = torch.cat([w.permute(0, 2, 3, 1).reshape(4, -1), torch.zeros(12, 9 * cin)]).to(gpu)
    ops.set_option("head_small", head_small)
    try:
        out = ops.conv2d(nhwc(x).to(gpu), ops.split_weight(wp), 3, 4, bias=b.to(gpu), res=nhwc(r).to(gpu),
                         out_f32=True)
        assert ops.get_option("last_kernel") == (14 if head_small else 3)
    finally:
        ops.set_option("head_small", 1)
    assert out.dtype == torch.float32
    assert rel(nchw(out), ref) < TOL


@pytest.mark.parametrize("gnm", [0, 1, 2])
@pytest.mark.parametrize("shape", [(2, 128, 8, 32), (1, 256, 16, 64), (2, 128, 24, 96), (1, 64, 8, 32)])
def test_x3_pyramid_head_fused(gpu, shape, gnm):
    """The split-bf16 halo head (conv_head_x3_kernel, H % 8 == 0, W % 32 == 0): conv3x3(act(GN(x)), C -> 4)
    + bias + the upsampled pyramid residual, gnm 0 raw x, 1 GroupNorm, 2 GroupNorm+SiLU (ncsnpp.py:348-366)."""
    from snrse import ops
    B, cin, H, W = shape
    x = torch.from_numpy(fnormal("t.pyf.x", (B, cin, H, W))) * 1.5 + 0.2
    w = torch.from_numpy(fnormal("t.pyf.w", (4, cin, 3, 3))) / math.sqrt(9 * cin)
    b = torch.from_numpy(fnormal("t.pyf.b", (4,)))
    r = torch.from_numpy(fnormal("t.pyf.r", (B, 4, H, W)))
    g = torch.from_numpy(fnormal("t.pyf.g", (cin,))) * 0.1 + 1
    be = torch.from_numpy(fnormal("t.pyf.be", (cin,))) * 0.1
    a = x.double()
    if gnm:
        a = F.group_norm(a, min(cin // 4, 32), g.double(), be.double(), eps=1e-6)
        a = F.silu(a) if gnm == 2 else a
    ref = F.conv2d(a, w.double(), b.double(), padding=1) + r.double()
    xg = nhwc(x).to(gpu)
    gn = None
    if gnm:
        sums, _ = ops.gn_stats(xg)
        gn = ops.gn_scale_shift(sums, g.to(gpu), be.to(gpu), H * W)
    wp = torch.cat([w.permute(0, 2, 3, 1).reshape(4, -1), torch.zeros(12, 9 * cin)]).to(gpu)
    assert ops.head_ok(xg, split=True) and not ops.head_ok(xg)
    out = ops.conv2d(xg, ops.split_weight(wp), 3, 4, bias=b.to(gpu), res=nhwc(r).to(gpu), out_f32=True, gn=gn,
                     gn_act=gnm == 2)
    assert ops.get_option("last_kernel") == 11
    assert out.dtype == torch.float32
    assert rel(nchw(out), ref) < TOL


def test_x3_pyramid_head_level0_vs_exact_fp32(gpu):
    """The level-0 pyramid head at C2 size on two images (256 x 512, 128 -> 4, GroupNorm+SiLU fused, upsampled
    pyramid residual): the split halo head vs the exact-fp32 path (gn_apply pass + register-staged fp32 GEMM)."""
    from snrse import ops
    B, C, H, W = 2, 128, 256, 512
    g = torch.Generator(device=gpu).manual_seed(5)
    x = torch.randn(B, H, W, C, device=gpu, generator=g) * 1.5 + 0.2
    w = torch.cat([torch.randn(4, 9 * C, device=gpu, generator=g) / math.sqrt(9 * C),
                   torch.zeros(12, 9 * C, device=gpu)])
    b = torch.randn(4, device=gpu, generator=g)
    r = torch.randn(B, H, W, 4, device=gpu, generator=g)
    gam = torch.rand(C, device=gpu, generator=g) + 0.5
    bet = torch.randn(C, device=gpu, generator=g) * 0.1
    sums, _ = ops.gn_stats(x)
    exact = ops.conv2d(ops.gn_apply(x, None, sums, gam, bet, act=True), w, 3, 4, bias=b, res=r, out_f32=True)
    assert ops.get_option("last_kernel") == 1
    gn = ops.gn_scale_shift(sums, gam, bet, H * W)
    split = ops.conv2d(x, ops.split_weight(w), 3, 4, bias=b, res=r, out_f32=True, gn=gn)
    assert ops.get_option("last_kernel") == 11
    assert rel(split, exact) < TOL


def test_x3_level0_vs_exact_fp32(gpu):
    """One C2 level-0 shape (256 x 512, 128 -> 128) on two images: the split halo kernel vs the exact-fp32
    kernel."""
    from snrse import ops
    B, C, H, W = 2, 128, 256, 512
    g = torch.Generator(device=gpu).manual_seed(3)
    x = torch.randn(B, H, W, C, device=gpu, generator=g)
    w = torch.randn(C, 9 * C, device=gpu, generator=g) / math.sqrt(9 * C)
    b = torch.randn(C, device=gpu, generator=g)
    st_a, st_b = ops.new_stats(B, C), ops.new_stats(B, C)
    a = ops.conv2d(x, w, 3, C, bias=b, stats=st_a)
    assert ops.get_option("last_kernel") == 1
    s = ops.conv2d(x, ops.split_weight(w), 3, C, bias=b, stats=st_b)
    assert ops.get_option("last_kernel") == 4  # 1,024 tiles: the halo kernel
    assert rel(s, a) < TOL
    assert rel(ops.fold_stats(st_b), ops.fold_stats(st_a)) < 1e-5


@pytest.mark.parametrize("spread", [2, 1, 0])
@pytest.mark.parametrize("act", [True, False])
@pytest.mark.parametrize("shape", [(2, 128, 128, 8, 64), (1, 384, 256, 4, 128), (2, 256, 128, 4, 64),
                                   (1, 128, 128, 8, 72), (1, 384, 256, 8, 64), (1, 96, 128, 8, 32)])
def test_x3h_fused_groupnorm_silu(gpu, shape, act, spread):
    """The halo form consuming SiLU(GN(x)) (act) or GN(x) from raw fp32 x + per-(b, c) scale / shift, with a
    raw 1x1 shortcut as extra K; every other split conv rejects a fused GroupNorm.  spread 2 = the pair schedule
    (two taps per phase) where its tiles apply (8 x 32, an even number of main chunks: the (2, 128, ...) and
    (1, 384, 256, 8, 64) cases; the others fall back to spread 1)."""
    from snrse import ops
    B, cin, cout, H, W = shape
    x = torch.from_numpy(fnormal("t.fg.x", (B, cin, H, W))) * 1.5 + 0.2
    w = torch.from_numpy(fnormal("t.fg.w", (cout, cin, 3, 3))) / math.sqrt(9 * cin)
    g = torch.from_numpy(fnormal("t.fg.g", (cin,))) * 0.1 + 1
    be = torch.from_numpy(fnormal("t.fg.b", (cin,))) * 0.1
    xs = torch.from_numpy(fnormal("t.fg.xs", (B, 128, H, W)))
    w2 = torch.from_numpy(fnormal("t.fg.w2", (cout, 128, 1, 1))) / 11
    a = F.group_norm(x.double(), min(cin // 4, 32), g.double(), be.double(), eps=1e-6)
    a = F.silu(a) if act else a
    ref = F.conv2d(a, w.double(), padding=1) + F.conv2d(xs.double(), w2.double())
    xg = nhwc(x).to(gpu)
    c0 = 256 if cin == 384 else cin
    s0, s1 = (xg[..., :c0].contiguous(), xg[..., c0:].contiguous()) if c0 != cin else (xg, None)
    sums = ops.gn_stats(s0, s1)
    gn = ops.gn_scale_shift(sums[0], g.to(gpu), be.to(gpu), H * W, sums1=sums[1])
    wp = ops.split_weight(w.permute(0, 2, 3, 1).reshape(cout, -1).to(gpu))
    w2p = ops.split_weight(w2.reshape(cout, 128).to(gpu))
    assert not ops.x3h_ok(s0, 3, cout)  # a small grid: the register-staged form, which has no GroupNorm
    with pytest.raises(RuntimeError):
        ops.conv2d(s0, wp, 3, cout, src1=s1, gn=gn, gn_act=act, sc=nhwc(xs).to(gpu), sc_wgt=w2p)
    ops.set_option("x3_tile", 4)
    ops.set_option("x3_spread", spread)  # pair schedule (2), halo stored one piece per tap (1) or in one go (0)
    try:
        assert ops.x3h_ok(s0, 3, cout)
        out = ops.conv2d(s0, wp, 3, cout, src1=s1, gn=gn, gn_act=act, sc=nhwc(xs).to(gpu), sc_wgt=w2p)
        assert ops.get_option("last_kernel") == 4
    finally:
        ops.set_option("x3_tile", 0)
        ops.set_option("x3_spread", 2)
    assert rel(nchw(out), ref) < TOL


@pytest.mark.parametrize("nt", [0, 1])
@pytest.mark.parametrize("gnm", [2, 0])
@pytest.mark.parametrize("flags", ["temb", "res", "comb", "shortcut"])
def test_x3h_specialised_epilogue_matches_runtime_flags(gpu, flags, gnm, nt):
    """The pair schedule's compile-time epilogue variants (option h5_specialise 1, the default: GroupNorm+SiLU or
    none, + temb / residual / Combine / the shortcut as extra K, with statistics, +-NT) against the run-time-flag
    kernel (h5_specialise 0) on the same inputs -- same arithmetic, so equal to 1e-6 -- and against fp64."""
    from snrse import ops
    B, cin, cout, H, W = 2, 128, 128, 8, 64
    x = torch.from_numpy(fnormal("t.xs.x", (B, cin, H, W))) * 1.5 + 0.2
    w = torch.from_numpy(fnormal("t.xs.w", (cout, cin, 3, 3))) / math.sqrt(9 * cin)
    b = torch.from_numpy(fnormal("t.xs.b", (cout,)))
    g = torch.from_numpy(fnormal("t.xs.g", (cin,))) * 0.1 + 1
    be = torch.from_numpy(fnormal("t.xs.be", (cin,))) * 0.1
    a = x.double()
    if gnm:
        a = F.silu(F.group_norm(a, min(cin // 4, 32), g.double(), be.double(), eps=1e-6))
    ref = F.conv2d(a, w.double(), b.double(), padding=1)
    xg = nhwc(x).to(gpu)
    kw = {}
    if gnm:
        sums = ops.gn_stats(xg)
        kw.update(gn=ops.gn_scale_shift(sums[0], g.to(gpu), be.to(gpu), H * W), gn_act=True)
    if flags == "temb":
        temb = torch.from_numpy(fnormal("t.xs.temb", (B, 200)))
        ref = ref + temb[:, 8:8 + cout, None, None].double()
        kw.update(temb=temb.to(gpu), temb_off=8)
    elif flags == "res":
        r = torch.from_numpy(fnormal("t.xs.r", (B, cout, H, W)))
        ref = (ref + r.double()) / math.sqrt(2)
        kw.update(res=nhwc(r).to(gpu), out_scale=1 / math.sqrt(2))
    elif flags == "comb":
        pyr = torch.from_numpy(fnormal("t.xs.pyr", (B, 4, H, W)))
        cw = torch.from_numpy(fnormal("t.xs.cw", (cout, 4)))
        cb = torch.from_numpy(fnormal("t.xs.cb", (cout,)))
        ref = ref + torch.einsum("bihw,oi->bohw", pyr.double(), cw.double()) + cb.double()[None, :, None, None]
        kw.update(comb=nhwc(pyr).to(gpu), comb_w=cw.to(gpu), comb_b=cb.to(gpu))
    else:
        xs = torch.from_numpy(fnormal("t.xs.xs", (B, 64, H, W)))
        w2 = torch.from_numpy(fnormal("t.xs.w2", (cout, 64, 1, 1))) / 8
        ref = ref + F.conv2d(xs.double(), w2.double())
        kw.update(sc=nhwc(xs).to(gpu), sc_wgt=ops.split_weight(w2.reshape(cout, 64).to(gpu)))
    wp = ops.split_weight(w.permute(0, 2, 3, 1).reshape(cout, -1).to(gpu))
    outs, sts = {}, {}
    ops.set_option("x3_tile", 4)
    ops.set_option("epi_nt", nt)
    try:
        for spec in (1, 0):
            ops.set_option("h5_specialise", spec)
            sts[spec] = ops.new_stats(B, cout)
            outs[spec] = ops.conv2d(xg, wp, 3, cout, bias=b.to(gpu), stats=sts[spec], **kw)
            assert ops.get_option("last_kernel") == 4
            assert ops.get_option("last_epi_nt") == nt
    finally:
        ops.set_option("x3_tile", 0)
        ops.set_option("epi_nt", 2)
        ops.set_option("h5_specialise", 1)
    assert rel(outs[1], outs[0]) < 1e-6
    assert rel(ops.fold_stats(sts[1]), ops.fold_stats(sts[0])) < 1e-6
    assert rel(nchw(outs[1]), ref) < TOL
    o = outs[1].double()
    assert rel(ops.fold_stats(sts[1]), torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1)) < 1e-5


@pytest.fixture(scope="module")
def net_x3(gpu):
    from snrse import ncsnpp
    sd = {k: torch.from_numpy(v) for k, v in formula_sd("ncsnpp").items()}
    return ncsnpp.NCSNppHIP(sd, dtype=torch.float32, device=gpu, gemm="x3")


@pytest.fixture(params=[0, 4], ids=["auto", "halo_forced"])
def x3_tile(request):
    """x3_tile 0: at the goldens' [2, 256, 64] grid every split conv is register-staged (+ gn_act);
    4: the halo kernel with the fused GroupNorm wherever W % 64 == 0 (the benched form at C2 sizes)."""
    from snrse import ops
    ops.set_option("x3_tile", request.param)
    yield request.param
    ops.set_option("x3_tile", 0)


def test_x3_ncsnpp_full_golden(gpu, net_x3, x3_tile):
    g = golden("ncsnpp_full.npz")
    x = torch.from_numpy(fnormal("golden.ncsnpp.x", (2, 2, 256, 64), complex_=True)) * 0.5
    t = torch.tensor([0.5, 0.8], device=gpu)
    out = net_x3.dnn(x[:, 0].contiguous().to(gpu), x[:, 1].contiguous().to(gpu), t)
    assert rel(out, g["out"][:, 0]) < 1e-4
    assert abs_rms(out, g["out"][:, 0]) < 1e-4


def test_x3_pc_loop_vs_reference_golden(gpu, net_x3, x3_tile):
    """The benched class (PCEnhancer) in the fp32x3 mode on the reference's N=5 OUVE run."""
    import paritycheck
    r = paritycheck.pc_vs_golden(gpu, net_x3)
    assert r["dtype"] == "fp32x3" and r["nfe"] == 10
    assert r["abs_rms"] < 1e-4, r

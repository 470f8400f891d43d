"""C5: long-form 30 s utterances, T = 3776 frames, fp32.

At T=3776 only the full-resolution level (W=3776) is a multiple of 64; the half-resolution and
smaller levels (1888, 944, 472, 236, 118, 59 frames) take the generic GEMM tiles, the 16-row
attention runs at L = 16*236 = 3776 and the mid-block attention at the ragged L = 4*59 = 236.
The oracle (CPU restatement of NCSNpp.forward, ncsnpp.py:247-404) runs one fp32 NFE at this
size in ~20 s on 16 host threads; the fp32 HIP path is held to the north-star 1e-4 relative
RMS on the complex spectrogram, fp16 (the headline format) to 1e-2, bf16 to 2e-2.
"""
import pytest
import torch

from conftest import fnormal, formula_sd
from oracle import ncsnpp_ref

pytestmark = pytest.mark.gpu

T30 = 3776  # 1 + 480000 // 128 = 3751 frames, padded to a multiple of 64 (util/other.py:83-90)


def rel(a, b):
    a = torch.as_tensor(a).detach().cpu().to(torch.complex128)
    b = torch.as_tensor(b).detach().cpu().to(torch.complex128)
    return float((a - b).abs().pow(2).mean().sqrt() / (b.abs().pow(2).mean().sqrt() + 1e-30))


@pytest.fixture(scope="module")
def longform():
    sd_np = formula_sd("ncsnpp")
    x = torch.from_numpy(fnormal("longform.x", (1, 2, 256, T30), complex_=True)) * 0.5
    t = torch.tensor([0.7])
    torch.set_num_threads(16)
    ref = ncsnpp_ref.ncsnpp_forward(x, t, ncsnpp_ref.state_dict_to_torch(sd_np))[:, 0]
    return {k: torch.from_numpy(v) for k, v in sd_np.items()}, x, t, ref


@pytest.mark.parametrize("dt", ["f32", "fp16", "bf16"])
def test_ncsnpp_longform_30s(gpu, longform, dt):
    from snrse import ncsnpp
    sd, x, t, ref = longform
    net = ncsnpp.NCSNppHIP(sd, dtype={"f32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[dt])
    out = net.dnn(x[:, 0].contiguous().to(gpu), x[:, 1].contiguous().to(gpu), t.to(gpu))
    torch.cuda.synchronize()
    assert torch.isfinite(torch.view_as_real(out)).all()
    err = rel(out, ref)
    assert err < {"f32": 1e-4, "fp16": 1e-2, "bf16": 2e-2}[dt], err


def test_pc_step_longform_30s(gpu, longform):
    """One fused reverse-diffusion step (predictors.py:75-80) at T=3776: x_mean = x - rev_f with
    rev_f = f - G^2 * score; the score is -dnn (model.py:488-489, bbed scoring mode)."""
    from snrse import ncsnpp, ops
    sd, x, t, ref = longform
    net = ncsnpp.NCSNppHIP(sd, dtype=torch.float32)
    xs, ys = x[:, 0].contiguous(), x[:, 1].contiguous()
    pyr = net.pyramid(xs.to(gpu), ys.to(gpu), t.to(gpu))
    coef = torch.tensor([[1.0, 0.0, 0.01, 0.1]], device=gpu)
    xo, xm, _ = ops.score_update(pyr, net.W["out_w"], net.W["out_b"], t.to(gpu), 0, xs.to(gpu), ys.to(gpu),
                                 coef=coef, seed=3)
    torch.cuda.synchronize()
    xm_ref = xs + 0.01 * (-ref)
    assert rel(xm - xs.to(gpu), xm_ref - xs) < 1e-4
    assert torch.isfinite(torch.view_as_real(xo)).all()

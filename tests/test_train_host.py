"""CPU checks of the consistency-training host logic (snrse/train.py): the t grid of model.py:366-367
against the reference-generated golden, the sebridge_v3 preconditioning, and the drop-in API surface."""
import numpy as np
import pytest

from conftest import golden


def test_t_grid_matches_reference_golden():
    from snrse import train
    g = golden("train_step.npz")
    np.testing.assert_allclose(train.t_grid(g["n"]), g["t_n"], rtol=1e-6)
    np.testing.assert_allclose(train.t_grid(g["n"] + 1), g["t_n1"], rtol=1e-6)
    # the inference grid t_30 (model.py:22-23) is the same schedule over n = 1..30
    from sgmse.model import t_30
    np.testing.assert_allclose(train.t_grid(np.arange(1, 31)), t_30, rtol=1e-12)


def test_precond_formula():
    from snrse import train
    t = np.array([0.001, 0.3, 1.0])
    cs, co = train.precond(t)
    np.testing.assert_allclose(cs, 0.25 / ((t - 0.001) ** 2 + 0.25))
    np.testing.assert_allclose(co, 0.5 * (t - 0.001) / np.sqrt(0.25 + t ** 2))
    assert co[0] == 0.0 and cs[0] == 1.0


def test_training_api_surface_and_unsupported_branches():
    import torch
    from sgmse.model import ScoreModel
    m = ScoreModel(backbone="ncsnpp", sde="ouve", model_type="bbed", theta=1.5, sigma_min=0.05, sigma_max=0.5)
    for name in ("_step", "training_step", "configure_optimizers", "optimizer_step"):
        assert callable(getattr(m, name))
    x = torch.zeros(1, 1, 256, 64, dtype=torch.complex64)
    with pytest.raises(NotImplementedError):
        m._step((x, x), 0)


def test_split_weight_layout():
    """ops.split_weight (the SNRSE_F32X3 weight layout): per 32-element K-tile 32 hi then 32 lo bf16,
    hi + lo within 2^-16 of the fp32 weight."""
    import torch
    from snrse import ops
    g = torch.Generator().manual_seed(0)
    w = torch.randn(3, 96, generator=g) * torch.logspace(-3, 3, 96)
    s = ops.split_weight(w)
    assert s.dtype == torch.bfloat16 and s.shape == (3, 192)
    t = s.float().reshape(3, 3, 2, 32)
    hi, lo = t[:, :, 0].reshape(3, 96), t[:, :, 1].reshape(3, 96)
    assert torch.equal(hi, w.to(torch.bfloat16).float())
    assert ((hi + lo - w).abs() <= w.abs() * 2.0 ** -16).all()


def test_resample_shape_contract():
    """ops.resample_ok mirrors snrse_gn_resample's contract: bf16 C % 16 == 0 (row strips / LDS tiles), f32
    C % 4 == 0 with C / 4 dividing 64 (row strips only); other dtypes go through snrse_gn_apply."""
    import torch
    from snrse import ops
    ok = lambda c, dt: ops.resample_ok(torch.empty(1, 2, 2, c, dtype=dt))  # noqa: E731
    assert ok(128, torch.bfloat16) and ok(256, torch.bfloat16) and not ok(8, torch.bfloat16)
    assert ok(4, torch.float32) and ok(128, torch.float32) and ok(256, torch.float32)
    assert not ok(512, torch.float32) and not ok(12, torch.float32) and not ok(6, torch.float32)
    assert ok(128, torch.float16) and not ok(8, torch.float16)  # fp16: the 16-bit path's format since round 6
    assert not ok(128, torch.float64)

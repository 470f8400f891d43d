"""CPU checks of the drop-in `sgmse` package: import surface, state-dict layout identical to
the reference's, registries and SDE scalar math vs golden vectors (no GPU calls)."""
import json

import numpy as np
import pytest
import torch

from conftest import fnormal, golden, state_dict_keys


def test_imports_without_lightning():
    import sgmse.data_module  # noqa: F401
    import sgmse.model  # noqa: F401
    import sgmse.sampling  # noqa: F401
    import sgmse.sdes  # noqa: F401
    import sgmse.snr_estimator  # noqa: F401
    from sgmse.model import ScoreModel, t_30
    assert hasattr(ScoreModel, "enhance") and hasattr(ScoreModel, "load_from_checkpoint")
    np.testing.assert_allclose(t_30[[0, -1]], [0.001, 1.0])


def test_ncsnpp_state_dict_layout_matches_reference():
    from sgmse.backbones import BackboneRegistry
    ref = state_dict_keys()
    m = BackboneRegistry.get_by_name("ncsnpp")()
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == ref["ncsnpp"]
    assert [n for n, p in m.named_parameters() if not p.requires_grad] == ref["ncsnpp_frozen"]
    assert [n for n, p in m.named_parameters() if p.requires_grad] == ref["ncsnpp_trainable_order"]
    from sgmse.backbones import SNRNet
    assert [[k, list(v.shape)] for k, v in SNRNet().state_dict().items()] == ref["snrnet"]


def test_registries():
    from sgmse.sampling import CorrectorRegistry, PredictorRegistry
    from sgmse.sdes import SDERegistry
    assert set(PredictorRegistry.get_all_names()) >= {"reverse_diffusion", "euler_maruyama", "none"}
    assert set(CorrectorRegistry.get_all_names()) >= {"ald", "langevin", "none"}
    assert set(SDERegistry.get_all_names()) >= {"ouve", "bbed", "proposed_1"}
    with pytest.raises(ValueError, match="unknown"):
        PredictorRegistry.get_by_name("nope")


def test_sde_api_matches_golden():
    from sgmse.sdes import BBED, OUVESDE, PROPOSED_1, SDERegistry
    g = golden("sde.npz")
    ts = torch.tensor(g["t"])
    x = torch.from_numpy(fnormal("golden.sde.x", (5, 1, 4, 4), complex_=True))
    y = torch.from_numpy(fnormal("golden.sde.y", (5, 1, 4, 4), complex_=True))
    for nm, s in (("ouve", OUVESDE(1.5, 0.05, 0.5, N=30)), ("ouve_smax1", OUVESDE(1.5, 0.05, 1.0, N=30)),
                  ("bbed", BBED(0.999, 2.6, 0.52, N=30)), ("proposed_1", PROPOSED_1(0.99, 1.0, 2.6, 0.52, N=30)),
                  ("proposed_1b", SDERegistry.get_by_name("proposed_1")(0.99, 0.5, 3.0, 0.53, N=30))):
        np.testing.assert_allclose(s._std(ts).double().numpy(), g[f"{nm}_std"], rtol=2e-6)
        d, gg = s.sde(x, ts[:, None, None, None], y)
        np.testing.assert_allclose(d.numpy(), g[f"{nm}_drift"], rtol=2e-5, atol=1e-5)
        np.testing.assert_allclose(torch.as_tensor(gg).reshape(-1).numpy(), g[f"{nm}_g"], rtol=2e-6)
        np.testing.assert_allclose(s._mean(x, ts, y).numpy(), g[f"{nm}_mean"], rtol=2e-5, atol=1e-6)
        sp = s.spec()
        np.testing.assert_allclose([sp.std(float(t)) for t in ts], g[f"{nm}_std"], rtol=2e-6)
        np.testing.assert_allclose([sp.g(float(t)) for t in ts], g[f"{nm}_g"], rtol=2e-6)
    # BBED works batched here (the reference's drift fails for B>1, sdes.py:276)
    bb = BBED(0.999, 2.6, 0.52)
    d, _ = bb.sde(x, ts, y)
    assert d.shape == x.shape
    assert bb._std(ts).dtype == torch.float32


def test_score_model_construction_and_cpu_refusal():
    from sgmse.model import ScoreModel
    m = ScoreModel(backbone="ncsnpp", sde="ouve", model_type="bbed", theta=1.5, sigma_min=0.05, sigma_max=0.5)
    assert m.sde.N == 1000 and m.t_eps == 0.03 and m.sigma_max == 0.5
    x = torch.zeros(1, 1, 256, 64, dtype=torch.complex64)
    with pytest.raises(RuntimeError, match="no CPU fallback|HIP"):
        m.dnn(torch.cat([x, x], 1), torch.ones(1))


def test_checkpoint_roundtrip_with_ema(tmp_path):
    """A PL-shaped checkpoint (state_dict, hyper_parameters, ema) loads with weights_only=True
    and eval(no_ema=False) swaps the EMA shadow weights in, train() restores them."""
    from sgmse.model import ScoreModel
    hp = dict(backbone="ncsnpp", sde="ouve", model_type="bbed", snr_conditioned="false", theta=1.5,
              sigma_min=0.05, sigma_max=0.5, N=30)
    src = ScoreModel(**hp)
    sd = {k: torch.randn_like(v) if v.is_floating_point() else v for k, v in src.state_dict().items()}
    shadow = [torch.full_like(p, 0.25) for p in src.parameters() if p.requires_grad]
    ckpt = {"state_dict": sd, "hyper_parameters": hp,
            "ema": {"decay": 0.999, "num_updates": 7, "shadow_params": shadow, "collected_params": None}}
    path = tmp_path / "m.ckpt"
    torch.save(ckpt, path)
    m = ScoreModel.load_from_checkpoint(str(path), base_dir="", batch_size=16, num_workers=0,
                                        kwargs=dict(gpu=False))
    w = m.dnn.all_modules[4].Conv_0.weight
    assert torch.equal(w, sd["dnn.all_modules.4.Conv_0.weight"])
    m.eval(no_ema=False)
    assert torch.all(w == 0.25)
    assert torch.equal(m.dnn.all_modules[0].W, sd["dnn.all_modules.0.W"])  # frozen GFP not in EMA
    m.train()
    assert torch.equal(w, sd["dnn.all_modules.4.Conv_0.weight"])


def test_ouve_copy_resets_starting_point():
    """OUVESDE.copy() starts from _T = 1 like the reference (sdes.py:185-186), so eval.py's
    `model.sde._T = reverse_starting_point` (eval.py:105-108) never reaches the PC sampler, which
    always samples from a copy (model.py:552): the schedule starts at t = 1."""
    from sgmse.sdes import OUVESDE
    from snrse import sampler
    sde = OUVESDE(theta=1.5, sigma_min=0.05, sigma_max=0.5, N=30)
    sde._T = 0.5  # eval.py --reverse_starting_point 0.5
    c = sde.copy()
    assert sde.T == 0.5 and c.T == 1 and c.N == 30
    steps, prior, _ = sampler.build_schedule(c.spec(), 15, 0.03, "reverse_diffusion", "ald", 0.5, 1)
    assert steps[0][1] == 1.0
    assert abs(prior[3] - sampler.SDESpec("ouve", theta=1.5, sigma_min=0.05, sigma_max=0.5).std(1.0)) < 1e-12


def test_unsupported_topology_rejected_at_construction():
    from sgmse.backbones import BackboneRegistry
    cls = BackboneRegistry.get_by_name("ncsnpp")
    cls()  # the shipped topology constructs
    for kw in (dict(nf=64), dict(ch_mult=(1, 2, 2, 2)), dict(num_res_blocks=4), dict(attn_resolutions=(8,)),
               dict(image_size=128)):
        with pytest.raises(NotImplementedError):
            cls(**kw)


def test_probability_flow_does_not_change_pc_schedule():
    """The reference's Predictor builds rsde without probability_flow (predictors.py:18): the flag
    changes nothing in the PC updates."""
    from snrse import sampler
    sde = sampler.SDESpec("ouve", theta=1.5, sigma_min=0.05, sigma_max=0.5)
    for pred in ("reverse_diffusion", "euler_maruyama"):
        a = sampler.build_schedule(sde, 7, 0.03, pred, "ald", 0.5, 1, probability_flow=False)
        b = sampler.build_schedule(sde, 7, 0.03, pred, "ald", 0.5, 1, probability_flow=True)
        assert a == b


def test_enhance_follows_data_module_transform():
    """enhance() takes its front / back end from the checkpoint's data-module hparams
    (model.py:749, 612-613): 'exponent' -> fused mode 1, 'none' -> raw mode 0, a configuration the
    HIP kernels are not built for raises before any device work."""
    from sgmse.data_module import SpecsDataModule
    from sgmse.model import ScoreModel
    assert SpecsDataModule().hip_mode() == 1
    assert SpecsDataModule(transform_type="none").hip_mode() == 0
    for kw in (dict(window="sqrthann"), dict(spec_factor=0.3), dict(transform_type="log")):
        with pytest.raises(NotImplementedError):
            SpecsDataModule(**kw).hip_mode()
    m = ScoreModel(backbone="ncsnpp", sde="ouve", model_type="bbed", theta=1.5, sigma_min=0.05, sigma_max=0.5,
                   window="sqrthann")
    with pytest.raises(NotImplementedError):
        m.enhance(torch.zeros(1, 1000), torch.zeros(1, 1000))


def test_enhance_fixed_snr_branch_raises_like_reference():
    """snr_conditioned='fixed' is a training-only mode: the reference's enhance raises
    NotImplementedError("snr fixed is only for experiment purpose, not real inference.")
    (sgmse-bbed/sgmse/model.py:792-793); here it raises the same, before any device work, while the
    model itself still constructs (the 'fixed' consistency-training branch needs it)."""
    from sgmse.model import ScoreModel
    m = ScoreModel(backbone="ncsnpp", sde="ouve", model_type="sebridge_v3", snr_conditioned="fixed",
                   fixed_snr=0.17783, theta=1.5, sigma_min=0.05, sigma_max=0.5)
    with pytest.raises(NotImplementedError, match="snr fixed is only for experiment purpose, not real inference."):
        m.enhance(torch.zeros(1, 16000), torch.zeros(1, 16000))
    m.snr_conditioned = "bogus"
    with pytest.raises(NotImplementedError):
        m.enhance(torch.zeros(1, 16000), torch.zeros(1, 16000))


def test_upfirdn2d_dtype_table():
    """The reference binding dispatches float / double / half (upfirdn2d_kernel.cu:311)."""
    from snrse import _lib, ops
    assert set(ops.UPFIRDN_DTYPES) == {torch.float32, torch.float64, torch.float16, torch.bfloat16}
    assert (_lib.F16, _lib.F64) == (2, 3)

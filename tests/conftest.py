import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "snr-aligned_diffse_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) to run")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def state_dict_keys():
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        return json.load(f)


def formula_sd(kind="ncsnpp", prefix=""):
    """Formula weights for the reference module whose keys were recorded by gen_golden."""
    from snrse import formula
    keys = state_dict_keys()[kind]
    shapes = {prefix + k: tuple(s) for k, s in keys}
    vals = formula.formula_state_dict(shapes)
    return {k[len(prefix):]: v for k, v in vals.items()}


def formula_block_sd(prefix, in_ch, out_ch, up=False, down=False):
    """Formula weights of a standalone ResnetBlockBigGANpp (names as in gen_golden)."""
    from snrse import formula
    shapes = {
        "GroupNorm_0.weight": (in_ch,), "GroupNorm_0.bias": (in_ch,),
        "Conv_0.weight": (out_ch, in_ch, 3, 3), "Conv_0.bias": (out_ch,),
        "Dense_0.weight": (out_ch, 512), "Dense_0.bias": (out_ch,),
        "GroupNorm_1.weight": (out_ch,), "GroupNorm_1.bias": (out_ch,),
        "Conv_1.weight": (out_ch, out_ch, 3, 3), "Conv_1.bias": (out_ch,),
    }
    if in_ch != out_ch or up or down:
        shapes["Conv_2.weight"] = (out_ch, in_ch, 1, 1)
        shapes["Conv_2.bias"] = (out_ch,)
    full = {prefix + k: v for k, v in shapes.items()}
    vals = formula.formula_state_dict(full)
    return {k[len(prefix):]: v for k, v in vals.items()}


def formula_attn_sd(prefix, C=256):
    from snrse import formula
    shapes = {"GroupNorm_0.weight": (C,), "GroupNorm_0.bias": (C,)}
    for i in range(4):
        shapes[f"NIN_{i}.W"] = (C, C)
        shapes[f"NIN_{i}.b"] = (C,)
    full = {prefix + k: v for k, v in shapes.items()}
    vals = formula.formula_state_dict(full)
    return {k[len(prefix):]: v for k, v in vals.items()}


def fnormal(name, shape, complex_=False):
    from snrse import formula
    return formula.normal_tensor(name, shape, complex_)


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not has_gpu():
        pytest.skip("no HIP device")
    import torch
    return torch.device("cuda:0")
